mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--steps 50" CFGS="cur:default cur:SDK_PLANE_CHUNK=48 cur:SDK_PLANE_CHUNK=32 cur:SDK_PLANE_TAIL=6 cur:SDK_PLANE_TAIL=10 cur:SDK_PLANE_REFILL=2 cur:SDK_PLANE_REFILL=4" R=3 bash scripts/gpu_ab.sh || exit 1
