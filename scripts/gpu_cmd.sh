mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--steps 50" CFGS="cur:default cur:SDK_PLANE_CHUNK=64 cur:SDK_PLANE_CHUNK=80" R=3 bash scripts/gpu_ab.sh || exit 1
