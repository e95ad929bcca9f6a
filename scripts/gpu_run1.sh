#!/bin/bash
# GPU pass: parity tests, then a short bench.  Stops on any non-test failure.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -m gpu \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t1.log 2>&1
rc=$?
tail -40 gpurun_out/t1.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if grep -q "Timeout" gpurun_out/t1.log; then exit 124; fi
timeout -k 10 300 python -u bench.py --steps 3 --batch ${BATCH:-65536} --cpu-budget 5 > gpurun_out/b1.log 2>&1
rc2=$?
tail -20 gpurun_out/b1.log
echo "bench rc=$rc2"
exit $rc2
