#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench per knob setting
#   AB="SDK_PLANE_TAIL=0 SDK_PLANE_TAIL=8" bash scripts/gpu_trace_ab.sh
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${AB:-default}; do
  tag=$(echo "$cfg" | tr ',=' '__')
  envs=""
  [ "$cfg" != default ] && envs=$(echo "$cfg" | tr ',' ' ')
  for kv in $envs; do export "$kv"; done
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$tag -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu --latency-boards 0 --no-extras ${BENCH_ARGS} > gpurun_out/tr_$tag.log 2>&1
  rc=$?
  for kv in $envs; do unset "${kv%%=*}"; done
  [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; exit $rc; }
  echo "== $cfg"; f=$(find gpurun_out/tr_$tag -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -8
done
