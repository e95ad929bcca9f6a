mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--steps 50" CFGS="cur:default wb2off:default cur:SDK_PLANE_REFILL=2" R=3 bash scripts/gpu_ab.sh || exit 1
BENCH_ARGS="--steps 50 --inflight 3" CFGS="cur:default" R=2 bash scripts/gpu_ab.sh || exit 1
