#!/bin/bash
# parity subset under both sweep modes, then interleaved A/B bench
mkdir -p gpurun_out
for m in one both; do
  SDK_SWEEP=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu \
    -k "golden_gen or random_generated or hard17_vs or edge_cases or duplicate or frontier or ordered" > gpurun_out/tq_$m.log 2>&1
  rc=$?; echo "$m: $(tail -1 gpurun_out/tq_$m.log)"; [ $rc -ne 0 ] && exit $rc
done
for m in one both one both; do
  SDK_SWEEP=$m timeout -k 10 120 python -u bench.py --steps 5 --batch 1048576 --no-cpu --latency-boards 8 > gpurun_out/bq.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bq.log').read().strip().splitlines()[-1]);print('$m', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms p50', round(d['p50_single_ms'],4), 'sweeps', round(d['sweeps_per_board'],2))"
done
