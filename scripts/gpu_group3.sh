# N=1 (2^20-board steps): one step per launch (default) vs two steps per launch, 20 and 50 steps
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
for k in 20 50; do
for cfg in "def;" "L21-gw2;--launch-boards 2097152 --grid-waves 2" "L21-gw1;--launch-boards 2097152 --grid-waves 1"; do
  tag=${cfg%%;*}; flags=${cfg#*;}
  timeout -k 10 200 python -u bench.py --steps $k --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial $flags > gpurun_out/gr.json 2> gpurun_out/gr.err || { tail -20 gpurun_out/gr.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gr.json').read().strip().splitlines()[-1]);print('K=$k $tag', round(d['value']/1e6,1), 'group', d['config']['steps_per_launch'])"
done
done
done
