#!/bin/bash
# PMC passes of the solve kernel on one bench launch shape (one counter group
# per run, each its own rocprofv3 process) -> gpurun_out/pmc_<kernel>[_<tag>].json,
# which bench.py picks by shape once copied to profiles/.
#   WORLD=8 bash scripts/gpu_pmc.sh      one rank of the driver's 8-GPU run (--steps 20)
#   WORKLOAD=hard_search bash scripts/gpu_pmc.sh
# The profiled bench runs the timed steps only (--warmup 0, --no-serial), so
# per-step counters are the kernel's dispatch totals over STEPS.
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${WORKLOAD:-hard17}
N=${WORLD:-1}
STEPS=${STEPS:-20}
K=${PMC_KERNEL:-plane_kernel_multi}
EMUL=""
[ "$N" -gt 1 ] && EMUL="--emulate-world $N --emulate-rank ${RANK_EMUL:-0}"
CMD="python -u bench.py --steps $STEPS --warmup 0 --no-cpu --latency-boards 0 --no-extras --no-serial --workload $W $EMUL $BENCH_EXTRA"
TAG=${TAG:-w$N}
[ "$W" != hard17 ] && TAG=${TAG}_$W
run() {  # name counters...
  local name=$1; shift
  rm -rf gpurun_out/pmc_${TAG}_$name
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run valu SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM || exit 1
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
D=gpurun_out/pmc_${TAG}
PMC_STEPS=$STEPS PMC_WORKLOAD=$W PMC_KERNEL=$K python scripts/pmc_summarize.py gpurun_out/pmc_${K}_$TAG.json 1048576 2024 ${D}_valu ${D}_wait ${D}_fetch ${D}_write
