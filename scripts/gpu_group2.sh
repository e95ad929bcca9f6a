# strong-scaling ranks at N=2/4/8 (20 steps): default grouping vs 2^21-board launches at 2 / 4 waves per SIMD
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
for n in 2 4 8; do
for cfg in "L21-gw1;--launch-boards 2097152 --grid-waves 1" "L21-gw2;--launch-boards 2097152 --grid-waves 2"; do
  tag=${cfg%%;*}; flags=${cfg#*;}
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial --scaling weak --batch $((1048576 / n)) $flags > gpurun_out/gr.json 2> gpurun_out/gr.err || { tail -20 gpurun_out/gr.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gr.json').read().strip().splitlines()[-1]);print('N=$n $tag', round(d['value']/1e6,1), 'xN', round($n*d['value']/1e6,1), 'group', d['config']['steps_per_launch'])"
done
done
done
