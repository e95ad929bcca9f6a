# one N=8 rank (2^17-board steps, 20 steps): launch grouping x grid waves
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
for cfg in "g8-gw1;--launch-boards 1048576 --grid-waves 1" "g5-gw1;--launch-boards 655360 --grid-waves 1" "g10-gw2;--launch-boards 1310720 --grid-waves 2" "g7-gw1;--launch-boards 917504 --grid-waves 1" "g4-gw1;--launch-boards 524288 --grid-waves 1" "g16-gw2;--launch-boards 2097152 --grid-waves 2"; do
  tag=${cfg%%;*}; flags=${cfg#*;}
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial --scaling weak --batch 131072 $flags > gpurun_out/gr.json 2> gpurun_out/gr.err || { tail -20 gpurun_out/gr.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/gr.json').read().strip().splitlines()[-1]);print('$tag', round(d['value']/1e6,1), 'x8', round(8*d['value']/1e6,1), 'group', d['config']['steps_per_launch'])"
done
done
