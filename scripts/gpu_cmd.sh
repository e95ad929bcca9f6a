mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_blk64.so
SDK_LIB=$L timeout -k 10 60 python -u bench.py --no-cpu --no-extras --latency-boards 0 --steps 4 --warmup 1 > gpurun_out/b.json 2>gpurun_out/b.err; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
SDK_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
CFGS="cur:default blk64:default" R=3 bash scripts/gpu_ab.sh || exit 1
BENCH_ARGS="--inflight 1" CFGS="cur:default blk64:default" R=2 bash scripts/gpu_ab.sh || exit 1
BENCH_ARGS="--inflight 3" CFGS="cur:default blk64:default" R=2 bash scripts/gpu_ab.sh || exit 1
