#!/bin/bash
# A/B on one box: (library build, runtime knobs) pairs, alternating, R rounds,
# one short bench per pair in its own process.
#   CFGS="cur:default new:default cur:SDK_PLANE_TAIL=4,SDK_PLANE_REFILL=8" R=3 bash scripts/gpu_ab.sh
# tag: "cur" = the in-tree libsudoku_hip.so, else libsudoku_hip_<tag>.so (built
# with `python -m sudoku_solver_distributed_amd.build --tag <tag> -DNAME=V ...`);
# env: comma-joined VAR=value, or "default".  BENCH_ARGS adds bench flags;
# TRACE=1 runs each bench under rocprofv3 --kernel-trace --stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $(seq 1 ${R:-2}); do
  for cfg in ${CFGS:-cur:default}; do
    tag=${cfg%%:*}; envs=${cfg#*:}; [ "$envs" = default ] && envs=""
    lib=""; [ "$tag" != cur ] && lib="SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$tag.so"
    name=$(echo "r${r}_$cfg" | tr ',=:' '___')
    args="--steps 20 --warmup 3 --no-cpu --latency-boards 0 --no-extras ${BENCH_ARGS}"
    if [ -n "$TRACE" ]; then
      env $(echo "$envs" | tr ',' ' ') $lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$name \
        -o run --output-format csv -- python3 -u bench.py $args > gpurun_out/tr_$name.log 2>&1
      rc=$?; out=$(grep '^{' gpurun_out/tr_$name.log | tail -1)
    else
      out=$(env $(echo "$envs" | tr ',' ' ') $lib timeout -k 10 120 python -u bench.py $args 2>>gpurun_out/ab.err)
      rc=$?
    fi
    [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; exit $rc; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $cfg', 'Mb/s=%.1f' % (d['value']/1e6), 'ms=%.3f' % d['ms_per_step'], 'kern_ms=%.3f' % d['roofline']['kernel_ms'], 'passes=%.2f' % d.get('sweeps_per_board', 0), 'guess=%.3f' % d.get('guesses_per_board', 0))"
  done
done
