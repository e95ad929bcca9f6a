#!/bin/bash
# same-box A/B of two in-tree builds: libsudoku_hip_prev.so vs libsudoku_hip.so
mkdir -p gpurun_out
for i in 1 2; do
  for L in prev cur; do
    if [ $L = prev ]; then export SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_prev.so; else unset SDK_LIB; fi
    timeout -k 10 120 python -u bench.py --steps 5 --batch 1048576 --no-cpu --latency-boards 8 > gpurun_out/bq.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]);print('$L', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms sweeps', round(d['sweeps_per_board'],2))"
  done
done
