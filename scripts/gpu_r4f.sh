# round 4: profile of the default shape (6 in flight x 1 wave per SIMD, 8 hardware queues) + default bench
mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -30 gpurun_out/pmc.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pmc_plane_kernel.json'));c=d['counters_per_launch'];print('pmc', d['shape'], d['grid_threads'], 'waves', c['SQ_WAVES'], 'valu', d['valu_insts_per_launch'], 'hbm', d['hbm_bytes_per_launch'], 'waitinst', d['sq_wait_inst_any_share'], 'wait', d['sq_wait_any_share'])"
rm -rf gpurun_out/prof_clean
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clean -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 > gpurun_out/prof_clean.log 2>&1 || { tail -20 gpurun_out/prof_clean.log; exit 1; }
grep '^{"metric"' gpurun_out/prof_clean.log > gpurun_out/r4f_prof_bench.json
python scripts/trace_summary.py gpurun_out/prof_clean/run_kernel_trace.csv gpurun_out/r4f_trace_summary.json | tail -12
timeout -k 10 400 python -u bench.py > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || { tail -20 gpurun_out/r4f_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r4f_bench.json').read().strip().splitlines()[-1]);r=d['roofline'];print('value',d['value'],'frac',r['frac'],'useful',r.get('useful_lane_frac'),'traffic',r['traffic'],'kernel_ms',r['kernel_ms'],'shape',r['shape'],'cpu',d['cpu_baseline']['value'])"
