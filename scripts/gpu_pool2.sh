# tail pool: threshold sweep at N=1 and in the N=8-rank emulation
mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pool_ab.sh "default:SDK_PLANE_TAIL_MODE=1" "default:SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=16" "default:SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=24" "default:SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=32" "default:SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=40" || exit 1
bash scripts/gpu_emul_knobs.sh "SDK_PLANE_TAIL_MODE=1;" "SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=16;" "SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=24;" "SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=32;" "SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=40;"
