# round 4 final shape: full GPU suite, the default bench line, one-rank strong-scaling emulation (20 / 100 steps)
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4k_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4k_gpu_tests.log; exit 1; }
tail -16 gpurun_out/r4k_gpu_tests.log
sed -i 's#r4h_bench#r4k_bench#g' scripts/gpu_r4h.sh
bash scripts/gpu_r4h.sh || exit 1
echo "== K=20"; K=20 bash scripts/gpu_rank_emul.sh || exit 1
echo "== K=100"; K=100 bash scripts/gpu_rank_emul.sh
