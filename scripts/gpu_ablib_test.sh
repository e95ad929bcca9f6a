#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu \
  -k "golden_gen or random_generated or hard17_vs or edge_cases or duplicate or frontier or ordered or full_size" > gpurun_out/tq.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/tq.log)"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ablib.sh
