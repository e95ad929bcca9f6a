mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k inflight > gpurun_out/inflight_tests.log 2>&1 || { tail -30 gpurun_out/inflight_tests.log; exit 1; }
tail -5 gpurun_out/inflight_tests.log
