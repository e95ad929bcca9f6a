mkdir -p gpurun_out; export TMPDIR=/tmp
SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_pf.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/pf_parity.log 2>&1 || { tail -20 gpurun_out/pf_parity.log; exit 1; }
tail -2 gpurun_out/pf_parity.log
BENCH_ARGS="--steps 50" CFGS="cur:default pf:default pf:SDK_PLANE_REFILL=2" R=3 bash scripts/gpu_ab.sh || exit 1
