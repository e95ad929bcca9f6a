"""Build the hard 17-clue corpus: sudoku_solver_distributed_amd/data/hard17_classes.txt.

    python scripts/make_hard17.py [--target N] [--two]

Seeds: gen.SEEDS_17 (the six boards bench.py used through round 3) plus
scripts/hard17/recalled17.txt (34 boards of the public 17-clue collection,
written down from memory; every line there passed the certification below,
and the strings that did not -- 53 of 87 -- were dropped).  From the seeds,
scripts/hard17/hard17_search.c runs a {-1, +1} clue exchange search to
closure (drop a clue, enumerate the 16-clue board's completions, add a clue
held by exactly one of them); --two also tries {-2, +2} exchanges through
16-clue boards with <= 64 completions (found nothing new from the six seeds'
18 classes in 3 CPU-minutes x 8 threads).  Boards are deduplicated by
isomorphism class (a cheap invariant while searching, then the exact minlex
form over transposition, band / stack and row / column permutations and
digit relabelling -- the group gen._symmetry_images draws from), and every
class is certified with the oracle's own counter: 17 clues, exactly one
completion (oracle_count_solutions_fast).

Results (round 4): the six seeds close at 18 classes; with the recalled
boards, 80 classes.  Workload tooling only -- it uses the oracle as the
certifier, never as a product path.
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "scripts", "hard17", "hard17_search.c")
RECALLED = os.path.join(ROOT, "scripts", "hard17", "recalled17.txt")
OUT = os.path.join(ROOT, "sudoku_solver_distributed_amd", "data", "hard17_classes.txt")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", type=int, default=5000)
    ap.add_argument("--two", action="store_true", help="also try {-2,+2} exchanges (slow)")
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    from oracle import oracle as O  # the certifier
    from sudoku_solver_distributed_amd.gen import SEEDS_17
    with tempfile.TemporaryDirectory() as tmp:
        exe = os.path.join(tmp, "hard17_search")
        subprocess.run(["gcc", "-O3", "-fopenmp", "-o", exe, SRC], check=True)
        seeds = os.path.join(tmp, "seeds.txt")
        with open(RECALLED) as f:
            recalled = [ln.strip() for ln in f if len(ln.strip()) == 81]
        with open(seeds, "w") as f:
            f.write("\n".join(list(SEEDS_17) + recalled) + "\n")
        found = subprocess.run([exe, seeds, str(args.target), "100000", "1" if args.two else "0"],
                               check=True, capture_output=True, text=True).stdout
        classes = subprocess.run([exe, "--canon"], input=found, check=True, capture_output=True,
                                 text=True).stdout.split()
    for s in classes:
        b = np.array([int(c) for c in s], dtype=np.uint8)
        if (b > 0).sum() != 17 or O.count_solutions(b, 2) != 1:
            raise SystemExit(f"not a unique 17-clue board: {s}")
    with open(args.out, "w") as f:
        f.write("# hard 17-clue corpus: one isomorphism class per line (minlex form), each certified\n"
                "# 17 clues + exactly one completion by the oracle's counter; made by\n"
                "# scripts/make_hard17.py ({-1,+1} exchange closure of gen.SEEDS_17 and\n"
                "# scripts/hard17/recalled17.txt).  gen.hard17_batch draws symmetry images of these.\n")
        f.write("\n".join(classes) + "\n")
    print(f"{len(classes)} classes -> {os.path.relpath(args.out, ROOT)}")


if __name__ == "__main__":
    main()
