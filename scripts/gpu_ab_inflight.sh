# A/B of launches in flight x grid waves x hardware queues (GPU_MAX_HW_QUEUES), alternating rounds
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 30 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial"
for r in 1 2 3; do
for cfg in $CFGS; do
  set -- $(echo $cfg | tr ',' ' ')
  GPU_MAX_HW_QUEUES=$3 timeout -k 10 200 python -u bench.py $B --inflight $1 --grid-waves $2 > gpurun_out/ab_i.json 2> gpurun_out/ab_i.err || { tail -20 gpurun_out/ab_i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_i.json').read().strip().splitlines()[-1]);print('inflight $1 grid $2 hwq $3', round(d['value']/1e6,1))"
done
done
