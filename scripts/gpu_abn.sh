#!/bin/bash
# same-box A/B/n of in-tree builds: LIBS="prev pf" compares libsudoku_hip_<tag>.so
# for each tag against the default libsudoku_hip.so ("cur"), after a parity subset
# of the default build.
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$NOPAR" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu \
  -k "golden or random_generated or hard17 or edge or duplicate or alternate or frontier or ordered or invalid or plane" > gpurun_out/tq.log 2>&1
rc=$?; [ -n "$NOPAR" ] || tail -2 gpurun_out/tq.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for L in ${LIBS:-prev} cur; do
    if [ $L = cur ]; then unset SDK_LIB; else export SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$L.so; fi
    timeout -k 10 120 python -u bench.py --steps 5 --batch 1048576 --no-cpu --latency-boards 8 --no-extras > gpurun_out/bq.log 2>&1 || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]);print('$L', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms kern', round(d['roofline']['kernel_ms'],3), 'sweeps', round(d['sweeps_per_board'],2))"
  done
done
