# tail pool (tail mode 2): parity first, then the per-wave timeline, then N=1 and N=8-rank A/B against mode 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_plane_tail_paths" tests/test_gpu_batches.py \
  "tests/test_gpu_parity.py::test_hard17_vs_unique_oracle" > gpurun_out/pool_tests.log 2>&1 || { tail -30 gpurun_out/pool_tests.log; exit 1; }
tail -3 gpurun_out/pool_tests.log
bash scripts/gpu_pool_trace.sh || exit 1
bash scripts/gpu_pool_ab.sh "default:SDK_PLANE_TAIL_MODE=1" "default:SDK_PLANE_TAIL_MODE=2" "default:SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=16" || exit 1
bash scripts/gpu_emul_knobs.sh "SDK_PLANE_TAIL_MODE=1;" "SDK_PLANE_TAIL_MODE=2;" "SDK_PLANE_TAIL_MODE=2,SDK_PLANE_TAIL=16;"
