#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench command (solve launches only)
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${BATCH:-1048576}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- \
  python -u bench.py --steps 5 --warmup 1 --batch $B --no-cpu --latency-boards 0 > gpurun_out/trace.log 2>&1 || exit $?
tail -1 gpurun_out/trace.log
head -5 gpurun_out/trace/run_kernel_stats.csv | cut -c1-200
