#!/bin/bash
# kernel time vs batch at the fixed persistent grid (start-up / drain cost)
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 262144 524288 1048576 2097152 4194304; do
  timeout -k 10 120 python -u bench.py --steps 5 --batch $b --no-cpu --latency-boards 0 --no-extras > gpurun_out/bs.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]);print('batch $b', round(d['value']/1e6,1),'M/s kern', round(d['roofline']['kernel_ms'],3),'ms sweeps', round(d['sweeps_per_board'],2))"
done
