#!/bin/bash
# Round check on one MI355X: GPU parity suite, smoke, the driver's bench
# line, rocprofv3 kernel-trace stats of the same command, PMC passes for the
# 1 / 2 / 4 / 8-GPU rank shapes, and the max-over-ranks strong-scaling
# emulation.  Every GPU step has its own time limit; the first failure ends
# the script.  Results under gpurun_out/ (copy what is judged to profiles/).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/tall.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/tall.log | tail -8; step pytest $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; step smoke $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -c 600 gpurun_out/bench.json; step bench $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-extras --no-serial --latency-boards 0 > gpurun_out/prof_trace.log 2>&1
step trace $?
python scripts/trace_summary.py gpurun_out/prof_trace/run_kernel_trace.csv gpurun_out/trace_summary.json --steps 20 > /dev/null
for N in 1 2 4 8; do
  WORLD=$N bash scripts/gpu_pmc.sh > gpurun_out/pmc_w$N.log 2>&1
  step pmc_w$N $?
done
timeout -k 10 600 python -u scripts/rank_emul.py --worlds 1,2,4,8 --steps 20 --out gpurun_out/rank_emul_k20.jsonl > gpurun_out/rank_emul_k20.log 2>&1
step rank_emul $?
