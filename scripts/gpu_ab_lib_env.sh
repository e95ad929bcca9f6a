#!/bin/bash
# A/B of (library build, runtime knobs) pairs on one box, alternating, R rounds:
#   CFGS="new:default pool16:SDK_PLANE_TAIL=4 ..." R=2 bash scripts/gpu_ab_lib_env.sh
# (tag:env, env = comma-joined VAR=value or "default"); BENCH_ARGS adds bench flags.
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $(seq 1 ${R:-2}); do
  for cfg in ${CFGS}; do
    tag=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = default ] && envs=""
    out=$(env $(echo "$envs" | tr ',' ' ') SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$tag.so timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --latency-boards 0 --no-extras ${BENCH_ARGS} 2>>gpurun_out/ab.err)
    rc=$?; [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; exit $rc; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $cfg', 'Mb/s=%.1f' % (d['value']/1e6), 'kern_ms=%.3f' % d['roofline']['kernel_ms'])"
  done
done
