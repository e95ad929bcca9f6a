mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "chunk_records or inflight or solve_host" > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; exit $rc
