mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_evt2.so
SDK_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--steps 50" CFGS="cur:default evt2:default evt3:default evt4:default" R=3 bash scripts/gpu_ab.sh || exit 1
BENCH_ARGS="--steps 20 --workload hard_search" CFGS="cur:default evt2:default evt3:default" R=2 bash scripts/gpu_ab.sh || exit 1
