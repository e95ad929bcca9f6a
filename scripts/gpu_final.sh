# round 4 final tree: the GPU suite and smoke()
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final_gpu_tests.log 2>&1 || { tail -40 gpurun_out/final_gpu_tests.log; exit 1; }
tail -3 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
