#!/bin/bash
# Round check on one MI355X: GPU parity suite, smoke, default bench line,
# rocprofv3 kernel-trace stats of the same bench command, PMC passes.
# Every GPU step has its own time limit; the first failure ends the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 150 --timeout-method thread -m gpu > gpurun_out/tall.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/tall.log | tail -8; step pytest $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; step smoke $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -c 600 gpurun_out/bench.json; step bench $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python -u bench.py --no-cpu --no-extras --latency-boards 0 > gpurun_out/prof_trace.log 2>&1
step trace $?
python scripts/trace_summary.py gpurun_out/prof_trace/run_kernel_trace.csv gpurun_out/trace_summary.json > /dev/null
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1
step pmc $?
WORKLOAD=hard_search bash scripts/gpu_pmc.sh > gpurun_out/pmc_hs.log 2>&1
step pmc_hard_search $?
