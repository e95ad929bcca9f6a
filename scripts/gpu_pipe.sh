# pipelined launches: parity of the flag, then N=1 at 20 / 100 steps for pool_last 0 (every launch pipelined) / 1 / 3 / 6
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batches.py > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -2 gpurun_out/pipe_tests.log
for K in 20 100; do
  BENCH_EXTRA="--steps $K" bash scripts/gpu_pool_ab.sh "default:X=1;--pool-last 0" "default:X=1;--pool-last 1" "default:X=1;--pool-last 3" "default:X=1;--pool-last 6" || exit 1
done
bash scripts/gpu_emul_knobs.sh "X=1;--pool-last 0" "X=1;"
