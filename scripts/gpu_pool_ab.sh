# tail pool A/B: "tag:ENV=V,...[;bench flags]" entries (tag = library build, default = in-tree default)
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial $BENCH_EXTRA"
for r in 1 2; do
for cfg in "$@"; do
  t=${cfg%%:*}; rest=${cfg#*:}; envs=$(echo "${rest%%;*}" | tr ',' ' '); flags=""
  case "$rest" in *\;*) flags=${rest#*;};; esac
  if [ "$t" = default ]; then L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip.so; else L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$t.so; fi
  env SDK_LIB=$L $envs timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/ab_p.json 2> gpurun_out/ab_p.err || { tail -20 gpurun_out/ab_p.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_p.json').read().strip().splitlines()[-1]);print('$cfg', round(d['value']/1e6,1), 'passes', round(d['sweeps_per_board'],2))"
done
done
