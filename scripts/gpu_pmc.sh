#!/bin/bash
# PMC passes for the solve kernel on the bench workload (one counter group per run)
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${BATCH:-1048576}
W=${WORKLOAD:-hard17}
# the bench's default launch shape (BENCH_EXTRA adds flags, e.g. --launch-boards)
CMD="python -u bench.py --steps 6 --warmup 1 --batch $B --no-cpu --latency-boards 0 --no-extras --no-serial --workload $W $BENCH_EXTRA"
run() {  # name counters...
  local name=$1; shift
  rm -rf gpurun_out/pmc_$name
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- $CMD > gpurun_out/pmc_$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
run valu SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM || exit 1
run wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
K=${PMC_KERNEL:-plane_kernel}
OUT=gpurun_out/pmc_$K.json
[ "$W" != hard17 ] && OUT=gpurun_out/pmc_${K}_$W.json
PMC_WORKLOAD=$W PMC_KERNEL=$K python scripts/pmc_summarize.py $OUT $B 2024 gpurun_out/pmc_valu gpurun_out/pmc_wait gpurun_out/pmc_fetch gpurun_out/pmc_write
