#!/bin/bash
# Round check on one MI355X: PMC passes for the 1 / 2 / 4 / 8-GPU rank shapes
# (and hard_search at N=1) first -- copied into this box's profiles/ so the
# bench line below quotes counters of the same build -- then the GPU parity
# suite, smoke, the driver's bench line, rocprofv3 kernel-trace stats of the
# same command, and the max-over-ranks strong-scaling emulation.  Every GPU
# step has its own time limit; the first failure ends the script.  Results
# under gpurun_out/ (copy what is judged to profiles/).  PART=pmc runs the
# PMC passes only, PART=rest the rest (two gpurun calls under the 20-minute
# limit: copy the PMC files to profiles/ in between).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
if [ "$PART" != rest ]; then
  for N in 1 2 4 8; do
    WORLD=$N bash scripts/gpu_pmc.sh > gpurun_out/pmc_w$N.log 2>&1
    step pmc_w$N $?
  done
  WORKLOAD=hard_search bash scripts/gpu_pmc.sh > gpurun_out/pmc_w1_hard_search.log 2>&1
  step pmc_w1_hard_search $?
  cp gpurun_out/pmc_plane_kernel_multi_w*.json profiles/
fi
[ "$PART" = pmc ] && exit 0
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/tall.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/tall.log | tail -8; step pytest $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; step smoke $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -c 600 gpurun_out/bench.json; step bench $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras --no-serial --latency-boards 0 > gpurun_out/prof_trace.log 2>&1
step trace $?
python scripts/trace_summary.py gpurun_out/prof_trace/run_kernel_trace.csv gpurun_out/trace_summary.json --steps 20 > /dev/null
timeout -k 10 600 python -u scripts/rank_emul.py --worlds 1,2,4,8 --steps 20 --out gpurun_out/rank_emul_k20.jsonl > gpurun_out/rank_emul_k20.log 2>&1
step rank_emul $?
