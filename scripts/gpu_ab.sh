#!/bin/bash
# v2 vs v3 on the bench workload (same box), then the GPU suite on the default kernel
mkdir -p gpurun_out
for v in 2 3 2 3; do
  SDK_SOLVE_KERNEL=$v timeout -k 10 120 python -u bench.py --steps 5 --batch 1048576 --no-cpu --latency-boards 8 > gpurun_out/ab_$v.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('v$v', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms p50', round(d['p50_single_ms'],4))"
done
bash scripts/gpu_full.sh
