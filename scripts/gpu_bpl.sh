#!/bin/bash
# boards-per-lane grid sizing sweep (SDK_PLANE_BPL) + a 4x batch for the drain effect
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # label batch
  timeout -k 10 120 python -u bench.py --steps 5 --batch $2 --no-cpu --latency-boards 0 --no-extras > gpurun_out/bq.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]);print('$1', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms sweeps', round(d['sweeps_per_board'],2))"
}
for i in 1 2; do
  for b in ${BPLS:-0 6 8 12 16}; do SDK_PLANE_BPL=$b run "bpl=$b" 1048576; done
done
SDK_PLANE_BPL=0 run "bpl=0 batch=4M" 4194304
