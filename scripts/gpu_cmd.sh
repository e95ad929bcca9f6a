mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "inflight or grid_waves" > gpurun_out/grid_tests.log 2>&1 || { tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -4 gpurun_out/grid_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 1500 gpurun_out/bench.json
