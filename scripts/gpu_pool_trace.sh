# per-wave timelines of one launch (stamps build): full grid and 1 wave per SIMD, hard17 and search-heavy
mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_stamps.so
for cfg in "1048576 hard17 0" "1048576 hard17 1" "1048576 hard_search 0"; do
  set -- $cfg
  echo "== $cfg"
  SDK_LIB=$L timeout -k 10 200 python -u scripts/plane_timeline.py $1 $2 $3 > gpurun_out/pt.txt 2>&1 || { tail -20 gpurun_out/pt.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/pt.txt
done
