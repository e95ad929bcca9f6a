#!/bin/bash
# parity subset + bench for kernel variants given in $VARS (SDK_SOLVE_KERNEL values)
mkdir -p gpurun_out
for v in ${VARS:-2 l}; do
  SDK_SOLVE_KERNEL=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -m gpu \
    -k "golden_gen or random_generated or hard17_vs or edge_cases or duplicate or ordered or full_size" > gpurun_out/tv_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/tv_$v.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/tv_$v.log | head -5; exit $rc; }
done
for i in 1 2; do for v in ${VARS:-2 l}; do
  SDK_SOLVE_KERNEL=$v timeout -k 10 120 python -u bench.py --steps 5 --batch 1048576 --no-cpu --latency-boards 8 --no-extras > gpurun_out/bv.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bv.log').read().strip().splitlines()[-1]);print('$v', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms p50', round(d['p50_single_ms'],4), 'passes', round(d['sweeps_per_board'],2))"
done; done
