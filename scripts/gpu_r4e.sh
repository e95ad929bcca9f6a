# round 4: the full GPU suite (timed), then the profile of the new default shape
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4e_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4e_gpu_tests.log; exit 1; }
tail -22 gpurun_out/r4e_gpu_tests.log
BENCH_EXTRA="--steps 50 --warmup 2" bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -30 gpurun_out/pmc.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pmc_plane_kernel.json'));c=d['counters_per_launch'];print('pmc', d['shape'], d['grid_threads'], 'waves', c['SQ_WAVES'], 'valu', d['valu_insts_per_launch'], 'hbm', d['hbm_bytes_per_launch'], 'waitinst', d['sq_wait_inst_any_share'], 'wait', d['sq_wait_any_share'])"
rm -rf gpurun_out/prof_clean
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clean -o run --output-format csv -- python -u bench.py --steps 50 --warmup 2 --no-cpu --no-extras --latency-boards 0 > gpurun_out/prof_clean.log 2>&1 || { tail -20 gpurun_out/prof_clean.log; exit 1; }
grep '^{"metric"' gpurun_out/prof_clean.log > gpurun_out/r4e_prof_bench.json
python scripts/trace_summary.py gpurun_out/prof_clean/run_kernel_trace.csv gpurun_out/r4e_trace_summary.json | tail -12
