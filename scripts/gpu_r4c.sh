# round 4 profile of the shipped launch shape: kernel trace + stats, PMC passes, stamped timeline
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_clean
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clean -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 > gpurun_out/prof_clean.log 2>&1 || { tail -20 gpurun_out/prof_clean.log; exit 1; }
echo trace ok; grep '^{"metric"' gpurun_out/prof_clean.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms'])"
python scripts/trace_summary.py $(ls gpurun_out/prof_clean/*/run_kernel_trace.csv 2>/dev/null || ls gpurun_out/prof_clean/run_kernel_trace.csv) gpurun_out/r04_trace_summary.json | tail -5
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -30 gpurun_out/pmc.log; exit 1; }
tail -12 gpurun_out/pmc.log
SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_stamps.so timeout -k 10 200 python -u scripts/plane_timeline.py > gpurun_out/r04_timeline.txt 2>&1 || { tail -20 gpurun_out/r04_timeline.txt; exit 1; }
tail -30 gpurun_out/r04_timeline.txt
