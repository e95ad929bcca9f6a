"""Build the search-heavy seed set (sudoku_solver_distributed_amd/data/hard_search_seeds.txt).

    python scripts/make_hard_search.py [N_SEEDS] [CANDIDATES]

1. Full grids the way gen.py:31-52 makes them: three random diagonal boxes,
   then gen.py:6-28's walk fills the rest (the oracle's literal walk).
2. Each grid is reduced to a MINIMAL puzzle: cells are emptied in a random
   order, and an emptying is kept only while the puzzle keeps exactly one
   completion (oracle_count_solutions_fast, limit 2).
3. The plane solver (plane_solver.h compiled for the host) solves each
   minimal puzzle in gen order; puzzles that need at least MIN_GUESSES
   guesses beyond naked / hidden singles are kept, hardest first.

Uses the oracle (test infrastructure) as a build tool only; the product
reads the committed seed file.  Deterministic for a given argv.
"""
import ctypes
import os
import random
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

MIN_GUESSES = 2
OUT = os.path.join(ROOT, "sudoku_solver_distributed_amd", "data", "hard_search_seeds.txt")


def host_plane():
    so = os.path.join(tempfile.mkdtemp(), "libplane_host.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-o", so,
                           os.path.join(ROOT, "tests", "native", "plane_host.cpp")])
    lib = ctypes.CDLL(so)
    lib.plane_solve_stats.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int] + [ctypes.c_void_p] * 3
    return lib


def full_grid(rng):
    g = np.zeros(81, np.uint8)
    for n in range(0, 9, 3):
        nums = rng.sample(range(1, 10), 9)
        for i in range(3):
            for j in range(3):
                g[(n + i) * 9 + n + j] = nums.pop()
    ok, g = O.solve(g)
    assert ok
    return g


def minimal(grid, rng):
    p = grid.copy()
    for c in rng.sample(range(81), 81):
        v = p[c]
        p[c] = 0
        if O.count_solutions(p, 2) != 1:
            p[c] = v
    return p


def main():
    n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    cand = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    rng = random.Random(20261016)
    puzzles = np.array([minimal(full_grid(rng), rng) for _ in range(cand)], dtype=np.uint8)
    lib = host_plane()
    passes, guesses, depth = (np.zeros(cand, np.int32) for _ in range(3))
    lib.plane_solve_stats(puzzles.ctypes.data, cand, 0, passes.ctypes.data, guesses.ctypes.data, depth.ctypes.data)
    keep = np.nonzero(guesses >= MIN_GUESSES)[0]
    keep = keep[np.argsort(-guesses[keep], kind="stable")][:n_seeds]
    with open(OUT, "w") as f:
        f.write("# minimal unique 9x9 puzzles needing >= %d guesses on the plane solver (gen order);\n"
                "# made by scripts/make_hard_search.py from gen.py-style grids; one per line:\n"
                "# board guesses passes max_depth clues\n" % MIN_GUESSES)
        for i in keep:
            f.write("%s %d %d %d %d\n" % ("".join(map(str, puzzles[i])), guesses[i], passes[i], depth[i],
                                        int((puzzles[i] != 0).sum())))
    print(f"{cand} minimal puzzles, {int((guesses >= 1).sum())} need a guess, "
          f"{int((guesses >= MIN_GUESSES).sum())} need >= {MIN_GUESSES}; kept {len(keep)}; "
          f"guesses mean {guesses[keep].mean():.1f} max {guesses[keep].max()}, "
          f"passes mean {passes[keep].mean():.1f}, depth max {depth[keep].max()}")


if __name__ == "__main__":
    main()
