#!/bin/bash
# First GPU run of the plane kernel: sanity, full parity suite, bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/gpu_sanity.py > gpurun_out/sanity.log 2>&1
rc=$?; cat gpurun_out/sanity.log | grep -v amdgpu.ids; echo "sanity rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/tall.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/tall.log | tail -8; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -c 1500 gpurun_out/bench.json; echo "bench rc=$rc"; exit $rc
