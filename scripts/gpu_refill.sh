# pool -> lane refill: parity, then A/B of library builds at N=1 (20 steps, and back to back) and as one N=8 rank
mkdir -p gpurun_out; export TMPDIR=/tmp
REPS=4 timeout -k 10 300 python -u tests/diag_pool.py > gpurun_out/diag.txt 2>&1 || { tail -5 gpurun_out/diag.txt; exit 1; }
grep -v " 0 wrong" gpurun_out/diag.txt | grep -v amdgpu.ids; grep -c " 0 wrong" gpurun_out/diag.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_plane_tail_paths" tests/test_gpu_batches.py \
  "tests/test_gpu_parity.py::test_hard17_vs_unique_oracle" "tests/test_gpu_parity.py::test_hard_search_vs_unique_oracle" > gpurun_out/refill_tests.log 2>&1 || { tail -30 gpurun_out/refill_tests.log; exit 1; }
tail -2 gpurun_out/refill_tests.log
B="--steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial"
for r in 1 2 3; do
for t in default fifo; do
  if [ "$t" = default ]; then L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip.so; else L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_$t.so; fi
  for mode in "n1;" "b2b;--inflight 1" "r8;--scaling weak --batch 131072"; do
    tag=${mode%%;*}; flags=${mode#*;}
    SDK_LIB=$L timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/rf.json 2> gpurun_out/rf.err || { tail -20 gpurun_out/rf.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rf.json').read().strip().splitlines()[-1]);print('$t $tag', round(d['value']/1e6,1), 'passes', round(d['sweeps_per_board'],2))"
  done
done
done
