#!/bin/bash
# Same-box A/B of in-tree tuning builds: bash scripts/gpu_abtags.sh base w3 r16 ...
# (base = libsudoku_hip.so, T = libsudoku_hip_T.so); two rounds, interleaved.
mkdir -p gpurun_out
D=sudoku_solver_distributed_amd
for round in 1 2; do
  for T in "$@"; do
    if [ "$T" = base ]; then unset SDK_LIB; else export SDK_LIB=$PWD/$D/libsudoku_hip_$T.so; fi
    timeout -k 10 120 python -u bench.py --steps 10 --no-cpu --no-extras --latency-boards 0 > gpurun_out/ab_$T.log 2>&1 || { echo "$T failed"; tail -5 gpurun_out/ab_$T.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_$T.log').read().strip().splitlines()[-1]);print('$T', round(d['value']/1e6,1),'M/s', round(d['roofline']['kernel_ms'],3),'ms sweeps', round(d['sweeps_per_board'],2), 'guesses', round(d['guesses_per_board'],3), 'deferred', d.get('deferred_per_step'))"
  done
done
