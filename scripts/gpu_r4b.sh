# round 4: search-mode switch parity, then A/B of the switch threshold on the bench
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batches.py -m gpu > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4b_tests.log | tail -2
for k in 0 64 128 256 0 64 128 256; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --mrv-after $k > gpurun_out/r4b_mrv$k.json 2> gpurun_out/r4b_mrv$k.err || { tail -20 gpurun_out/r4b_mrv$k.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r4b_mrv$k.json').read().strip().splitlines()[-1]);print('mrv $k', round(d['value']/1e6,1), 'M/s serial', round(d['serial']['value']/1e6,1), 'passes', round(d['sweeps_per_board'],2), 'guesses', round(d['guesses_per_board'],2))"
done
