# the pooled last launches' grid: as the others (1 wave per SIMD) / 2 / full, N=1 at 20 and 50 steps
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
for k in 20 50; do
for cfg in "def;" "last2;--last-grid-waves 2" "last0;--last-grid-waves 0" "last0-pl1;--last-grid-waves 0 --pool-last 1"; do
  tag=${cfg%%;*}; flags=${cfg#*;}
  timeout -k 10 200 python -u bench.py --steps $k --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial $flags > gpurun_out/lg.json 2> gpurun_out/lg.err || { tail -20 gpurun_out/lg.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/lg.json').read().strip().splitlines()[-1]);print('K=$k $tag', round(d['value']/1e6,1))"
done
done
done
