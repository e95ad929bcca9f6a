# round 4: the default bench line (all side configs), as the driver runs it
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r4h_bench.json 2> gpurun_out/r4h_bench.err || { tail -20 gpurun_out/r4h_bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4h_bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('value',round(d['value']/1e6,1),'ms/step',round(d['ms_per_step'],3),'passes',round(d['sweeps_per_board'],2),'guesses',round(d['guesses_per_board'],2))
print('roof frac',r['frac'],'useful',r.get('useful_lane_frac'),'traffic',r['traffic'],'pmc_match',r['pmc_match'],'kernel_ms',r['kernel_ms'])
print('serial',d['serial'],'cpu',d['cpu_baseline']['value'])
sc=d['side_configs']
print('shard_rate',json.dumps(sc['shard_rate']))
print('hard_search',sc['hard_search']['boards_per_s'],sc['hard_search']['inflight'],'gen100k',sc['gen100k']['boards_per_s'])
print('e2e',sc['e2e']['boards_per_s'],sc['e2e']['pipelined']['boards_per_s'])
for k in ('node_http','node_http_4peer','node_http_1peer_procs','node_http_4peer_procs'): print(k, sc[k].get('requests_per_s'), sc[k].get('p50_ms'))
print('pathological',sc['pathological'])
PY
