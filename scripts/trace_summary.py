"""Per-launch figures of the plane kernel from a rocprofv3 kernel trace of a
bench.py run (--kernel-trace ... -o run --output-format csv), to check the
bench line's roofline.kernel_ms.  Plan "run" (bench.py's default): the
warm-up steps are one launch and the K timed steps one more (K <= 32), so
the timed launch is the longest plane launch and kernel_ms = its span / K.
Launches that overlap their predecessor (plan "inflight") form one region.

    python scripts/trace_summary.py gpurun_out/prof_trace/run_kernel_trace.csv [out.json] [--steps K]
"""
import csv
import json
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
args = [a for a in args if a != str(steps)] if "--steps" in sys.argv else args
rows = [r for r in csv.DictReader(open(args[0])) if r["Kernel_Name"].startswith("plane_kernel")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
# runs of overlapping launches (each overlaps the one before it)
runs, cur = [], [0]
for i in range(1, len(rows)):
    if st[i] < en[i - 1]:
        cur.append(i)
    else:
        runs.append(cur)
        cur = [i]
runs.append(cur)
spans = [(max(en[i] for i in r) - st[r[0]]) / 1e6 for r in runs]
timed = max(range(len(runs)), key=lambda k: spans[k])
out = {
    "trace": args[0],
    "kernel": rows[runs[timed][0]]["Kernel_Name"].split("(")[0],
    "launches": len(rows),
    "regions_ms": spans,
    "timed": {"launches": len(runs[timed]), "region_ms": spans[timed], "steps": steps,
              "region_ms_per_step": spans[timed] / steps},
}
print(json.dumps(out, indent=1))
if len(args) > 1:
    with open(args[1], "w") as f:
        json.dump(out, f, indent=1)
