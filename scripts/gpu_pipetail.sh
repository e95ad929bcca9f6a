# pipelined launches' own tail threshold (SDK_PLANE_PIPE_TAIL), N=1 at 50 steps, three rounds
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
for cfg in "X=1" "SDK_PLANE_PIPE_TAIL=6" "SDK_PLANE_PIPE_TAIL=10" "SDK_PLANE_PIPE_TAIL=12"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 50 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial > gpurun_out/pt.json 2> gpurun_out/pt.err || { tail -20 gpurun_out/pt.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/pt.json').read().strip().splitlines()[-1]);print('$cfg', round(d['value']/1e6,1))"
done
done
