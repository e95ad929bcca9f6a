mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 200 python -u scripts/e2e_probe.py 2>&1 | grep solve_host; done
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --latency-boards 0 > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/b.json').read().strip().split(chr(10))[-1]); print('G/s %.3f' % (d['value']/1e9), 'serial', round(d['serial']['value']/1e9,3)); print(json.dumps(d['side_configs']['e2e']))"
done
