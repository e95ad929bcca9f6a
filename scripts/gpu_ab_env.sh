#!/bin/bash
# A/B of runtime knobs: one short bench per setting, each in its own process.
#   AB="SDK_PLANE_TAIL=0 SDK_PLANE_TAIL=8,SDK_PLANE_REFILL=16 ..." bash scripts/gpu_ab_env.sh
# (comma joins several variables in one setting); BENCH_ARGS adds bench flags.
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${AB:-default}; do
  envs=""
  [ "$cfg" != default ] && envs=$(echo "$cfg" | tr ',' ' ')
  extra=""
  for kv in $envs; do case $kv in BATCH=*) extra="--batch ${kv#BATCH=}";; esac; done
  out=$(env $envs timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --latency-boards 0 --no-extras ${BENCH_ARGS} $extra 2>>gpurun_out/ab.err)
  rc=$?
  [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; exit $rc; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'Mb/s=%.1f' % (d['value']/1e6), 'ms=%.3f' % d['ms_per_step'], 'kern_ms=%.3f' % d['roofline']['kernel_ms'], 'passes=%.2f' % d['sweeps_per_board'], 'guess=%.3f' % d['guesses_per_board'], 'defer=%.0f' % d['deferred_per_step'])"
done
