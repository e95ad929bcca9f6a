"""Per-launch figures of the plane kernel from a rocprofv3 kernel trace of a
bench.py run (--kernel-trace ... -o run --output-format csv), for checking
the bench line's roofline.kernel_ms: launches that overlap their
predecessor (two in flight) form the timed region, whose span / launches is
kernel_ms; launches that do not are the back-to-back `serial` steps.

    python scripts/trace_summary.py gpurun_out/prof_trace/run_kernel_trace.csv [out.json]
"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith("plane_kernel")]
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
inflight = max(runs, key=len)
region_ms = (max(en[i] for i in inflight) - st[inflight[0]]) / 1e6
serial = [i for r in runs if len(r) == 1 for i in r]
out = {
    "trace": sys.argv[1],
    "launches": len(rows),
    "inflight": {"launches": len(inflight), "region_ms_per_launch": region_ms / len(inflight),
                 "mean_span_ms": sum(en[i] - st[i] for i in inflight) / len(inflight) / 1e6},
    "serial": {"launches": len(serial),
               "mean_span_ms": sum(en[i] - st[i] for i in serial) / max(len(serial), 1) / 1e6},
}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)
