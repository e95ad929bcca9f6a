# A/B of library builds (SDK_LIB), alternating rounds; LIBS = "tag ..." (default = the in-tree default build)
mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 30 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial $BENCH_EXTRA"
for r in 1 2 3; do
for t in $LIBS; do
  if [ "$t" = default ]; then L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip.so; else L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$t.so; fi
  SDK_LIB=$L timeout -k 10 200 python -u bench.py $B > gpurun_out/ab_l.json 2> gpurun_out/ab_l.err || { tail -20 gpurun_out/ab_l.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_l.json').read().strip().splitlines()[-1]);print('$t', round(d['value']/1e6,1), 'passes', round(d['sweeps_per_board'],2))"
done
done
