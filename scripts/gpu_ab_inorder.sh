#!/bin/bash
# parity subset on the current build, then same-box A/B vs $LIBS builds
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu \
  -k "golden_gen or random_generated or hard17_vs or edge_cases or duplicate or ordered or full_size" > gpurun_out/tio.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/tio.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/tio.log | head -5; exit $rc; }
LIBS="${LIBS:-sync cur}" bash scripts/gpu_abn.sh
