#!/bin/bash
# same-box A/B of in-tree builds sudoku_solver_distributed_amd/libsudoku_hip_<name>.so for
# each name in $LIBS ("cur" = libsudoku_hip.so), two rounds, bench workload
mkdir -p gpurun_out
for i in 1 2; do
  for L in ${LIBS:-cur}; do
    if [ $L = cur ]; then unset SDK_LIB; else export SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$L.so; fi
    timeout -k 10 120 python -u bench.py --steps 5 --batch 1048576 --no-cpu --latency-boards 8 --no-extras > gpurun_out/bq.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]);print('$L', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms p50', round(d['p50_single_ms'],4), 'sweeps', round(d['sweeps_per_board'],2))"
  done
done
