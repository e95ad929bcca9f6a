# after the generator / step-input change: two-rank path, default bench (PMC must still match), one N=8 rank
mkdir -p gpurun_out; export TMPDIR=/tmp
T0=$(date +%s); timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial --scaling weak --batch 131072 > gpurun_out/gen_r8.json 2> gpurun_out/gen_r8.err || { tail -20 gpurun_out/gen_r8.err; exit 1; }
echo "rank start-up+run $(( $(date +%s) - T0 )) s"
python -c "import json;d=json.loads(open('gpurun_out/gen_r8.json').read().strip().splitlines()[-1]);print('r8', round(d['value']/1e6,1), 'group', d['config']['steps_per_launch'])"
