#!/bin/bash
# Clean kernel-trace stats (only the 2^20-board solve launches: no side
# configs, no latency boards) + the PMC passes, for profiles/.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clean -o run --output-format csv -- python -u bench.py --no-cpu --no-extras --latency-boards 0 > gpurun_out/prof_clean.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
