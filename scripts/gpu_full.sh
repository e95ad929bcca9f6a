#!/bin/bash
# full GPU suite + smoke; stops at the first non-test failure
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/tall.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tall.log | tail -40
echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; echo "smoke rc=$rc"; exit $rc
