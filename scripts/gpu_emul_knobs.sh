# N=8 rank emulation (2^17-board steps, 20 steps) under knob settings: CFGS of "ENV=V,...;bench flags"
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
for cfg in "$@"; do
  envs=$(echo "$cfg" | cut -d';' -f1 | tr ',' ' '); flags=$(echo "$cfg" | cut -d';' -f2)
  env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial --scaling weak --batch 131072 $flags > gpurun_out/emk.json 2> gpurun_out/emk.err || { tail -20 gpurun_out/emk.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/emk.json').read().strip().splitlines()[-1]);print('[$cfg]', 'rank', round(d['value']/1e6,1), 'x8', round(8*d['value']/1e6,1))"
done
done
