mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stream_probe.py 1048576 20 2>&1 | grep boards
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().split(chr(10))[-1]); print('G/s %.3f' % (d['value']/1e9), 'serial', round(d['serial']['value']/1e9,3)); print(json.dumps(d['side_configs']['e2e'])); print(d['side_configs']['hard_search']['boards_per_s']/1e6)"
WORKLOAD=hard_search bash scripts/gpu_pmc.sh > gpurun_out/pmc_hs.log 2>&1; echo "pmc hs rc=$?"; tail -3 gpurun_out/pmc_hs.log
CFGS="cur:default prio1:default prio2:default prio3:default" R=3 bash scripts/gpu_ab.sh || exit 1
BENCH_ARGS="--inflight 1" CFGS="cur:default prio2:default" R=2 bash scripts/gpu_ab.sh || exit 1
