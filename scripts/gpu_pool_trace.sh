# per-wave timeline of one launch, tail mode 1 vs 2 (stamps build)
mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_stamps.so
for m in 1 2; do
  echo "== tail mode $m"
  SDK_LIB=$L SDK_PLANE_TAIL_MODE=$m timeout -k 10 200 python -u scripts/plane_timeline.py > gpurun_out/pt_$m.txt 2>&1 || { tail -20 gpurun_out/pt_$m.txt; exit 1; }
  cat gpurun_out/pt_$m.txt
done
