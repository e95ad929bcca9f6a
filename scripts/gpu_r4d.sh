# round 4: PMC of the shipped shape (no serial steps), steady-state ceiling, deeper in-flight queues
mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -30 gpurun_out/pmc.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/pmc_plane_kernel.json'));c=d['counters_per_launch'];print('pmc', d['shape'], d['grid_threads'], 'waves', c['SQ_WAVES'], 'valu', d['valu_insts_per_launch'], 'hbm', d['hbm_bytes_per_launch'], 'waitinst', d['sq_wait_inst_any_share'], 'wait', d['sq_wait_any_share'])"
B="--no-cpu --no-extras --latency-boards 0 --no-serial"
timeout -k 10 200 python -u bench.py --batch 8388608 --inflight 1 --steps 3 --warmup 1 $B > gpurun_out/r4d_big.json 2> gpurun_out/r4d_big.err || { tail -20 gpurun_out/r4d_big.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r4d_big.json').read().strip().splitlines()[-1]);print('2^23 per launch, back to back', round(d['value']/1e6,1))"
for cfg in "3 2 4" "4 1 4" "3 2 8" "4 1 8" "4 2 8" "6 1 8" "5 1 8" "3 2 4" "4 1 8" "6 1 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$3 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --inflight $1 --grid-waves $2 $B > gpurun_out/r4d_q.json 2> gpurun_out/r4d_q.err || { tail -20 gpurun_out/r4d_q.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r4d_q.json').read().strip().splitlines()[-1]);print('inflight $1 grid $2 hwq $3', round(d['value']/1e6,1))"
done
