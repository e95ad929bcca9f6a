"""Summarise rocprofv3 --pmc passes for the solve kernel into
profiles/pmc_<kernel>.json (read by bench.py for the VALU roofline).

    python scripts/pmc_summarize.py OUT.json BATCH SEED DIR [DIR ...]

Each DIR holds one pass's *counter_collection.csv (and DIR.log the profiled
bench's output, whose JSON line gives the launch shape).  Only solve_kernel
dispatches of the full batch are used (largest grid); values are averaged
per dispatch.  FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM (gfx950
reports half of a coalesced stream's bytes); sizes are in KB.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main():
    out, batch, seed, dirs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4:]
    kernel = os.environ.get("PMC_KERNEL", "")
    # PMC_STEPS: the profiled bench's steps (run with --warmup 0): per-step
    # totals over EVERY dispatch of the kernel -- grouped launches (N > 1
    # ranks) hold different numbers of steps, so a per-launch mean would not do
    steps = int(os.environ.get("PMC_STEPS", "0"))
    totals = defaultdict(float)
    vals = defaultdict(list)
    grids = set()
    for d in dirs:
        rows = [r for r in load(d) if r.get("Kernel_Name", "").split("(")[0] in
                ((kernel,) if kernel else ("plane_kernel",))]
        if not rows:
            continue
        # the bench runs only its timed launch shape under the profiler
        # (--no-serial), the deferred-board kernel aside: one grid size
        gmax = max(int(r.get("Grid_Size", 0) or 0) for r in rows)
        grids.add(gmax)
        per = defaultdict(float)
        for r in rows:
            totals[r["Counter_Name"]] += float(r["Counter_Value"])
            if int(r.get("Grid_Size", 0) or 0) != gmax:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, name), v in per.items():
            vals[name].append(v)
    summary = {k: sum(v) / len(v) for k, v in vals.items()}
    # the launch shape the profiled bench ran (its own JSON line, in each
    # pass's log): bench.py uses these counters only for that exact shape
    shape = None
    for d in dirs:
        try:
            with open(d + ".log") as fh:
                for ln in fh:
                    if ln.startswith('{"metric"'):
                        shape = shape or json.loads(ln)["roofline"]["shape"]
        except OSError:
            pass
    res = {"kernel": kernel or "plane_kernel", "batch": batch, "seed": seed, "shape": shape,
           "grid_threads": sorted(grids),
           "workload": os.environ.get("PMC_WORKLOAD", "hard17"),
           "counters_per_launch": summary,
           "valu_insts_per_launch": summary.get("SQ_INSTS_VALU"),
           "hbm_bytes_per_launch": None}
    if "FETCH_SIZE" in summary and "WRITE_SIZE" in summary:
        res["hbm_bytes_per_launch"] = (2 * summary["FETCH_SIZE"] + summary["WRITE_SIZE"]) * 1024
    if steps:
        res["steps"] = steps
        res["counters_per_step"] = {k: v / steps for k, v in totals.items()}
        res["valu_insts_per_step"] = totals.get("SQ_INSTS_VALU", 0.0) / steps or None
        if "FETCH_SIZE" in totals and "WRITE_SIZE" in totals:
            res["hbm_bytes_per_step"] = (2 * totals["FETCH_SIZE"] + totals["WRITE_SIZE"]) * 1024 / steps
    if "SQ_WAVE_CYCLES" in summary:
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in summary:
                res[k.lower() + "_share"] = summary[k] / summary["SQ_WAVE_CYCLES"]
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
