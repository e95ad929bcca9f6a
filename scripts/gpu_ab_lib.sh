#!/bin/bash
# A/B of library builds on one box, alternating, R rounds:
#   LIBS="base new" R=3 bash scripts/gpu_ab_lib.sh
# (libsudoku_hip_<tag>.so built with `python -m sudoku_solver_distributed_amd.build --tag <tag> ...`)
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $(seq 1 ${R:-3}); do
  for tag in ${LIBS}; do
    out=$(SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$tag.so timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --latency-boards 0 --no-extras ${BENCH_ARGS} 2>>gpurun_out/ab.err)
    rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; exit $rc; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $tag', 'Mb/s=%.1f' % (d['value']/1e6), 'kern_ms=%.3f' % d['roofline']['kernel_ms'])"
  done
done
