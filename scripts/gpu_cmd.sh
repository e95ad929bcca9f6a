mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_stamps.so timeout -k 10 120 python -u scripts/plane_timeline.py > gpurun_out/timeline.txt 2>&1; echo tl rc=$?; cat gpurun_out/timeline.txt
CFGS="cur:default nohint:default cur:SDK_PLANE_REFILL=4 nohint:SDK_PLANE_REFILL=4 cur:SDK_PLANE_REFILL=3 cur:SDK_PLANE_REFILL=2" R=3 bash scripts/gpu_ab.sh || exit 1
