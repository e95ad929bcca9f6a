# round 4: multi-batch parity, then the default bench (strong scaling at N=1)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batches.py -m gpu > gpurun_out/r4a_batches.log 2>&1 || { tail -40 gpurun_out/r4a_batches.log; exit 1; }
tail -3 gpurun_out/r4a_batches.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "inflight or grid_waves or refill_extremes or chunk_records or smoke or golden" > gpurun_out/r4a_parity.log 2>&1 || { tail -40 gpurun_out/r4a_parity.log; exit 1; }
tail -3 gpurun_out/r4a_parity.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { tail -20 gpurun_out/r4a_bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4a_bench.json').read().strip().splitlines()[-1])
print({k:d[k] for k in ('value','ms_per_step','guesses_per_board','sweeps_per_board','all_solved_and_checked')})
print('serial',d['serial']); print('roof',{k:d['roofline'].get(k) for k in ('kernel_ms','kernel','shape','pmc_match')})
print('shard_rate',json.dumps(d['side_configs']['shard_rate']))
print('hard_search',d['side_configs']['hard_search']['boards_per_s'], d['side_configs']['hard_search']['inflight'])
print('node', d['side_configs']['node_http']['requests_per_s'], d['side_configs']['node_http_4peer']['requests_per_s'])
PY
