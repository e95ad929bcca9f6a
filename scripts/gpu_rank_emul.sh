# one rank of an N-GPU strong-scaling run emulated on one GPU: --scaling weak --batch 2^20/N
# (the rank's shard per step, grouped into 2^20-board launches), K steps as the driver runs
mkdir -p gpurun_out; export TMPDIR=/tmp
K=${K:-20}
B="--steps $K --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial $BENCH_EXTRA"
for r in 1 2; do
for n in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py $B --scaling weak --batch $((1048576 / n)) > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -20 gpurun_out/emu.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/emu.json').read().strip().splitlines()[-1]);print('N=$n rank rate', round(d['value']/1e6,1), 'x N =', round($n*d['value']/1e6,1), 'ms/step', round(d['ms_per_step'],3), 'group', d['config']['steps_per_launch'])"
done
done
