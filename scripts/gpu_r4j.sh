# round 4: one-rank strong-scaling emulation with the tail pool default, K = 20 and 100
mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== K=20"; K=20 bash scripts/gpu_rank_emul.sh || exit 1
echo "== K=100"; K=100 bash scripts/gpu_rank_emul.sh
