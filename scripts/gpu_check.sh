#!/bin/bash
# GPU parity suite + smoke + default bench line (each step time-limited; the
# first failure ends the script).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 150 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/tall.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR|Error" gpurun_out/tall.log | tail -12; step pytest $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -c 1500 gpurun_out/bench.json; step bench $rc
