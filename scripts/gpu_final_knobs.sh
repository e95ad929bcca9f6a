# final-shape knob check: search switch (SDK_PLANE_MRV) and pooled tail (SDK_PLANE_TAIL), N=1 / back to back / N=8 rank
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 50 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial"
for r in 1 2; do
for cfg in "X=1" "SDK_PLANE_MRV=48" "SDK_PLANE_MRV=96" "SDK_PLANE_TAIL=12" "SDK_PLANE_TAIL=24"; do
  for mode in "n1;" "b2b;--inflight 1" "r8;--steps 20 --scaling weak --batch 131072"; do
    tag=${mode%%;*}; flags=${mode#*;}
    env $cfg timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/fk.json 2> gpurun_out/fk.err || { tail -20 gpurun_out/fk.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/fk.json').read().strip().splitlines()[-1]);print('$cfg $tag', round(d['value']/1e6,1))"
  done
done
done
