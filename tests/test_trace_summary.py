"""scripts/trace_summary.py (CPU): from a rocprofv3 kernel trace it finds the
run of overlapping launches (bench.py's steps, two in flight) and reports
the timed region per launch that bench.py's roofline.kernel_ms is checked
against, and the back-to-back launches' mean span."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trace_summary_regions(tmp_path):
    rows = []
    t = 1_000_000
    # two overlapping warmup launches, a gap, 4 overlapping launches, 3 serial ones
    spans = [(0, 800), (500, 1500)]
    base = 100_000
    spans += [(base + i * 700, base + i * 700 + 900) for i in range(4)]
    base2 = 200_000
    spans += [(base2 + i * 800, base2 + i * 800 + 750) for i in range(3)]
    for i, (a, b) in enumerate(spans):
        rows.append({"Kernel_Name": "plane_kernel(unsigned char const*)", "Start_Timestamp": t + a * 1000,
                     "End_Timestamp": t + b * 1000, "Queue_Id": 1 + i % 2})
        rows.append({"Kernel_Name": "arm_kernel(unsigned long long*)", "Start_Timestamp": t + a * 1000 - 5,
                     "End_Timestamp": t + a * 1000 - 1, "Queue_Id": 1})
    path = tmp_path / "trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    out = tmp_path / "s.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "trace_summary.py"), str(path), str(out)],
                          stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    assert d["launches"] == 9
    assert d["inflight"]["launches"] == 4
    # region: first start to last end of the 4 overlapping launches, per launch
    assert abs(d["inflight"]["region_ms_per_launch"] - (3 * 700 + 900) / 4 / 1000) < 1e-9
    assert abs(d["inflight"]["mean_span_ms"] - 0.9) < 1e-9
    assert d["serial"]["launches"] == 3 and abs(d["serial"]["mean_span_ms"] - 0.75) < 1e-9
