"""Strong-scaling projection from one GPU: every rank of an N-rank job, one
after the other (bench.py --emulate-world N --emulate-rank r: that rank's own
shard_bounds shard of each 2^20-board step, its step rotation and launch
shape), and the job's step time = the SLOWEST rank's wall time, as the real
job's max-over-ranks clock takes it.  RCCL's barrier and max-reduction are
not in these figures.  Tooling, not product.

    python scripts/rank_emul.py [--worlds 1,2,4,8] [--steps 20] [--rounds 2] [--out FILE] [bench flags...]

Prints one JSON line per (world, round) and a summary line; --out appends
them all to FILE.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_rank(world, rank, steps, warmup, extra):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", str(warmup),
           "--no-cpu", "--no-extras", "--no-serial", "--latency-boards", "0"]
    if world > 1:
        cmd += ["--emulate-world", str(world), "--emulate-rank", str(rank)]
    r = subprocess.run(cmd + extra, cwd=ROOT, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"rank {rank}/{world} failed ({r.returncode}): {r.stderr[-2000:]}")
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--ranks", default="all", help="ranks to run per world (comma list; 'all': every rank)")
    ap.add_argument("--label", default="")
    args, extra = ap.parse_known_args()
    batch = 1 << 20
    for a, b in zip(extra, extra[1:]):
        if a == "--batch":
            batch = int(b)
    res = []
    base = None
    for rnd in range(args.rounds):
        for w in (int(x) for x in args.worlds.split(",")):
            ranks = []
            rlist = range(w) if args.ranks == "all" else [int(x) for x in args.ranks.split(",") if int(x) < w]
            for r in rlist:
                t0 = time.time()
                line = run_rank(w, r, args.steps, args.warmup, extra)
                wall = line["ms_per_step"] * args.steps / 1e3
                ranks.append({"rank": r, "wall_s": wall, "rank_boards_per_s": line["value"],
                              "kernel_ms": line["roofline"]["kernel_ms"], "frac": line["roofline"]["frac"],
                              "pmc_match": line["roofline"]["pmc_match"], "shape": line["roofline"]["shape"]})
                print(f"# world {w} rank {r}: {wall * 1e3:.3f} ms ({time.time() - t0:.0f} s)", flush=True)
            slow = max(x["wall_s"] for x in ranks)
            job = batch * args.steps / slow
            if w == 1:
                base = job
            rec = {"label": args.label, "flags": extra, "world": w, "round": rnd, "steps": args.steps, "max_rank_wall_s": slow,
                   "min_rank_wall_s": min(x["wall_s"] for x in ranks),
                   "job_boards_per_s": job, "x_of_1gpu": job / base if base else None,
                   "efficiency": job / base / w if base else None, "ranks": ranks}
            res.append(rec)
            print(json.dumps(rec), flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
