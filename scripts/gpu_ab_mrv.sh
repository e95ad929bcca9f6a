# A/B of the search-mode switch threshold (bench.py --mrv-after), alternating rounds
mkdir -p gpurun_out; export TMPDIR=/tmp
W=${WORKLOAD:-hard17}
for k in $KS $KS; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --workload $W --mrv-after $k > gpurun_out/ab_mrv$k.json 2> gpurun_out/ab_mrv$k.err || { tail -20 gpurun_out/ab_mrv$k.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_mrv$k.json').read().strip().splitlines()[-1]);print('$W mrv $k', round(d['value']/1e6,1), 'M/s serial', round(d['serial']['value']/1e6,1), 'passes', round(d['sweeps_per_board'],2), 'guesses', round(d['guesses_per_board'],2))"
done
