# A/B of the plane kernel's scheduling knobs ($SDK_PLANE_*), alternating rounds
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial $BENCH_EXTRA"
for r in 1 2; do
for cfg in $CFGS; do
  env $(echo $cfg | tr ',' ' ') timeout -k 10 200 python -u bench.py $B > gpurun_out/ab_k.json 2> gpurun_out/ab_k.err || { tail -20 gpurun_out/ab_k.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_k.json').read().strip().splitlines()[-1]);print('$cfg', round(d['value']/1e6,1))"
done
done
