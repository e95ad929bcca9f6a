"""Fixture for BASELINE.json configs[1] at full size (tests/golden/configs1_100k.npz).

    python tests/golden/make_configs1.py

generate_batch(100_000, 50, seed=7) made on the CPU: the same `random` draws
as gen.generate_batch (gen.py:31-52 -- three diagonal boxes, the walk's fill,
50 removals), with each fill and then each puzzle solved by the oracle's
literal gen.py:6-28 walk.  Stored per board: an 8-byte blake2b digest of the
puzzle and of the walk's answer, and the walk's status.  The GPU test
(test_gpu_parity.py::test_configs1_full_size) diffs every board's answer
against these digests instead of re-running 100k literal walks on the GPU
box's host (which took most of the -m gpu suite's time).  The oracle itself is
pinned to the reference's own outputs by tests/test_oracle.py.
"""
import hashlib
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
OUT = os.path.join(HERE, "configs1_100k.npz")
N, EMPTY, SEED = 100_000, 50, 7


def digests(boards: np.ndarray) -> np.ndarray:
    return np.array([int.from_bytes(hashlib.blake2b(b.tobytes(), digest_size=8).digest(), "little")
                     for b in boards], dtype=np.uint64)


def main():
    from oracle import oracle as O
    from sudoku_solver_distributed_amd.gen import _draw_diagonal, _draw_removals
    rng = random.Random(SEED)
    diag = np.zeros((N, 81), dtype=np.uint8)
    removals = []
    for k in range(N):  # gen.generate_batch's draw order
        diag[k] = np.asarray(_draw_diagonal(rng), dtype=np.uint8).reshape(81)
        removals.append(_draw_removals(rng, EMPTY, [True] * 81))
    threads = os.cpu_count() or 8
    full, st = O.solve_batch_parallel(diag, order="gen", workers=threads)
    assert (st == 1).all()
    puzzles = full.copy()
    idx = np.asarray(removals, dtype=np.int64)
    np.put_along_axis(puzzles, idx, 0, axis=1)
    sols, wst = O.solve_batch_parallel(puzzles, order="gen", workers=threads)
    np.savez_compressed(OUT, puzzle_digest=digests(puzzles), solution_digest=digests(sols),
                        status=wst.astype(np.int8), n=N, empty=EMPTY, seed=SEED)
    print(f"{OUT}: {N} boards, {int((wst == 1).sum())} solved")


if __name__ == "__main__":
    main()
