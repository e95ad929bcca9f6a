"""Fixture for test_gpu_parity.py::test_random_generated_vs_oracle
(tests/golden/random_generated.npz).

    python tests/golden/make_random_generated.py

The test's six seeded batches, generate_batch(n, e, seed=1234 + e) for
(e, n) in CASES, made on the CPU exactly as make_configs1.py makes its batch
(gen.generate_batch's `random` draws, each fill solved by the oracle's
literal gen.py:6-28 walk), then every puzzle solved by the oracle's literal
walk in both orders: gen.py:6-28 and node.py:62-74.  Stored: the puzzles and,
per order, the walk's answers and statuses.  A handful of these boards keep
the literal walk busy for 15-45 s each (random 64- and 70-empty boards with no
or many completions), which made this one GPU test 60 % of the -m gpu suite;
the GPU test now diffs against the stored answers, and
tests/test_oracle.py::test_random_generated_fixture re-runs the oracle over
the fixture on the CPU suite, so the fixture stays pinned to the oracle (and
the oracle to the reference's own outputs, test_oracle.py).
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, "random_generated.npz")
CASES = ((30, 256), (50, 256), (58, 256), (64, 128), (70, 64), (81, 4))
SEED0 = 1234


def puzzles_for(empties: int, n: int) -> np.ndarray:
    """generate_batch(n, empties, seed=SEED0 + empties) on the CPU."""
    from oracle import oracle as O
    from sudoku_solver_distributed_amd.gen import _draw_diagonal, _draw_removals
    rng = random.Random(SEED0 + empties)
    diag = np.zeros((n, 81), dtype=np.uint8)
    removals = []
    for k in range(n):  # gen.generate_batch's draw order
        diag[k] = np.asarray(_draw_diagonal(rng), dtype=np.uint8).reshape(81)
        removals.append(_draw_removals(rng, empties, [True] * 81))
    full, st = O.solve_batch_parallel(diag, order="gen", workers=os.cpu_count() or 8, chunk=1)
    assert (st == 1).all()
    p = full.copy()
    np.put_along_axis(p, np.asarray(removals, dtype=np.int64), 0, axis=1)
    return p


def main():
    from oracle import oracle as O
    out = {}
    for e, n in CASES:
        p = puzzles_for(e, n)
        out[f"puzzles_{e}"] = p
        for order in ("gen", "node"):
            sols, st = O.solve_batch_parallel(p, order=order, workers=os.cpu_count() or 8, chunk=1)
            out[f"{order}_solutions_{e}"] = sols
            out[f"{order}_status_{e}"] = st.astype(np.int8)
            print(f"e={e} n={n} {order}: {int((st == 1).sum())} solved", flush=True)
    np.savez_compressed(OUT, cases=np.asarray(CASES, dtype=np.int32), seed0=SEED0, **out)
    print(OUT)


if __name__ == "__main__":
    main()
