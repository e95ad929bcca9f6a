"""scripts/trace_summary.py (CPU): from a rocprofv3 kernel trace it finds the
timed launch of a bench.py run -- plan "run": the warm-up steps one launch,
the K timed steps one more, the longest -- and reports its span per step,
which bench.py's roofline.kernel_ms is checked against; launches that
overlap (plan "inflight") count as one region."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(tmp_path, spans):
    rows = []
    t = 1_000_000
    for i, (a, b) in enumerate(spans):
        rows.append({"Kernel_Name": "plane_kernel_multi(PlaneBatches, unsigned long long*)",
                     "Start_Timestamp": t + a * 1000, "End_Timestamp": t + b * 1000, "Queue_Id": 1 + i % 2})
        rows.append({"Kernel_Name": "arm_kernel(unsigned long long*)", "Start_Timestamp": t + a * 1000 - 5,
                     "End_Timestamp": t + a * 1000 - 1, "Queue_Id": 1})
    path = tmp_path / "trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    return path


def test_trace_summary_run_plan(tmp_path):
    # a 5-step warm-up launch, then the 20-step timed launch
    path = _trace(tmp_path, [(0, 8_000), (50_000, 82_000)])
    out = tmp_path / "s.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "trace_summary.py"), str(path), str(out),
                           "--steps", "20"], stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    assert d["launches"] == 2 and d["kernel"] == "plane_kernel_multi"
    assert d["timed"]["launches"] == 1
    assert abs(d["timed"]["region_ms_per_step"] - 32.0 / 20) < 1e-9


def test_trace_summary_overlapping_region(tmp_path):
    # four overlapping launches form one region (plan inflight)
    spans = [(0, 800)] + [(100_000 + i * 700, 100_000 + i * 700 + 900) for i in range(4)]
    path = _trace(tmp_path, spans)
    out = tmp_path / "s.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "scripts", "trace_summary.py"), str(path), str(out),
                           "--steps", "4"], stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    assert d["timed"]["launches"] == 4
    assert abs(d["timed"]["region_ms"] - (3 * 700 + 900) / 1000) < 1e-9
