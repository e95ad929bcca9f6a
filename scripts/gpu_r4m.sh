# round 4 final profiles (pooled tail 12): GPU suite, PMC + trace + default bench, search-heavy PMC + bench, scaling emulation
mkdir -p gpurun_out; export TMPDIR=/tmp
sed -i 's#gpurun_out/r4e_gpu_tests.log#gpurun_out/r4m_gpu_tests.log#g; s#r4e_prof_bench#r4m_prof_bench#; s#r4e_trace_summary#r4m_trace_summary#' scripts/gpu_r4e.sh
bash scripts/gpu_r4e.sh || exit 1
cp gpurun_out/pmc_plane_kernel.json profiles/pmc_plane_kernel.json
sed -i 's#r4h_bench#r4m_bench#g' scripts/gpu_r4h.sh
bash scripts/gpu_r4h.sh || exit 1
bash scripts/gpu_hs.sh || exit 1
echo "== K=20"; K=20 bash scripts/gpu_rank_emul.sh || exit 1
echo "== K=100"; K=100 bash scripts/gpu_rank_emul.sh
