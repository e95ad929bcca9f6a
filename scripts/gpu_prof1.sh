#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 5 --batch 1048576 --cpu-budget 10 > gpurun_out/b_1m.log 2>&1 || exit $?
tail -3 gpurun_out/b_1m.log
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python -u bench.py --steps 5 --batch 1048576 --no-cpu > gpurun_out/prof_trace.log 2>&1 || exit $?
find gpurun_out/prof_trace -name "*stats*" | head
