# search-heavy workload: PMC of the bench shape, then its bench line (in flight) and back to back
mkdir -p gpurun_out; export TMPDIR=/tmp
WORKLOAD=hard_search BENCH_EXTRA="--steps 50 --warmup 2" bash scripts/gpu_pmc.sh > gpurun_out/pmc_hs.log 2>&1 || { tail -30 gpurun_out/pmc_hs.log; exit 1; }
cp gpurun_out/pmc_plane_kernel_hard_search.json profiles/pmc_plane_kernel_hard_search.json
timeout -k 10 300 python -u bench.py --workload hard_search --no-cpu --no-extras --latency-boards 0 > gpurun_out/hs_bench.json 2> gpurun_out/hs_bench.err || { tail -20 gpurun_out/hs_bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/hs_bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('hard_search value', round(d['value']/1e6,1), 'serial', round(d['serial']['value']/1e6,1), 'frac', r['frac'], 'traffic', r['traffic'], 'pmc_match', r['pmc_match'], 'passes', round(d['sweeps_per_board'],2))
PY
