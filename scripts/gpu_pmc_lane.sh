#!/bin/bash
# one PMC pass (instruction mix) for the lane-per-board kernel
mkdir -p gpurun_out
export TMPDIR=/tmp SDK_SOLVE_KERNEL=l
B=${BATCH:-1048576}
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM \
  -d gpurun_out/pmcl_valu -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --batch $B --no-cpu --latency-boards 0 --no-extras > gpurun_out/pmcl_valu.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT \
  -d gpurun_out/pmcl_wait -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --batch $B --no-cpu --latency-boards 0 --no-extras > gpurun_out/pmcl_wait.log 2>&1 || exit $?
PMC_KERNEL=lane_kernel python scripts/pmc_summarize.py gpurun_out/pmc_lane.json $B 2024 gpurun_out/pmcl_valu gpurun_out/pmcl_wait
cat gpurun_out/pmc_lane.json
