# round 4 final: smoke(), the search-heavy bench line with its own profile
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --workload hard_search --no-cpu --no-extras --latency-boards 0 > gpurun_out/hs_bench.json 2> gpurun_out/hs_bench.err || { tail -20 gpurun_out/hs_bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/hs_bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('hard_search value', round(d['value']/1e6,1), 'serial', round(d['serial']['value']/1e6,1), 'frac', r['frac'], 'traffic', r['traffic'], 'pmc_match', r['pmc_match'], 'useful', r.get('useful_lane_frac'))
PY
