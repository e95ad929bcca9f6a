# kernel trace of the N=8 rank emulation (2^17-board steps x 20, grouped 8 per launch)
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/emu_trace
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/emu_trace -o run --output-format csv -- python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial --scaling weak --batch 131072 > gpurun_out/emu_trace.log 2>&1 || { tail -20 gpurun_out/emu_trace.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/emu_trace/**/run_kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r['Kernel_Name'].startswith('plane_kernel')]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[-3]['Start_Timestamp'])
for r in rows[-6:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(r['Kernel_Name'][:18], 'grid', r['Grid_Size'], 'start %.3f ms end %.3f ms dur %.3f' % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6))
PY
for gw in 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-extras --latency-boards 0 --no-serial --scaling weak --batch 131072 --grid-waves $gw > gpurun_out/emk.json 2> gpurun_out/emk.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/emk.json').read().strip().splitlines()[-1]);print('grid $gw rank', round(d['value']/1e6,1))"
done
