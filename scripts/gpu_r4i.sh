# round 4, tail pool default: the full GPU suite, PMC + trace of the shipped shape, the default bench line
mkdir -p gpurun_out; export TMPDIR=/tmp
sed -i 's#gpurun_out/r4e_gpu_tests.log#gpurun_out/r4i_gpu_tests.log#g; s#r4e_prof_bench#r4i_prof_bench#; s#r4e_trace_summary#r4i_trace_summary#' scripts/gpu_r4e.sh
bash scripts/gpu_r4e.sh || exit 1
sed -i 's#r4h_bench#r4i_bench#g' scripts/gpu_r4h.sh
bash scripts/gpu_r4h.sh
