"""Drop-in for the reference's ``gen.py`` plus the batch workloads.

* ``solve_sudoku(board)``      -- gen.py:6-28: same signature and result (the
  board is filled in place with the walk's first solution, True/False
  returned); the walk itself runs in the HIP kernel.
* ``generate_sudoku(empty)``   -- gen.py:31-52: same random-call sequence on
  the ``random`` module, so under the same ``random.seed`` it returns the same
  puzzle as the reference.
* ``generate_batch(n, empty, seed)`` -- n calls of generate_sudoku under one
  seed, with every fill solved in ONE GPU batch (identical boards).
* ``hard17_batch(n, seed)``    -- the benchmark's hard set: 17-clue boards with
  a unique solution, made by validity-preserving symmetries (digit relabeling,
  row/column permutations inside bands/stacks, band/stack permutations,
  transposition) of the 80 certified isomorphism classes in
  data/hard17_classes.txt (scripts/make_hard17.py).
* ``hard_search_batch(n, seed)`` -- the search-heavy set: the same symmetries
  applied to 256 minimal puzzles that need real search (data/).
"""
from __future__ import annotations

import os
import random as _random
import sys
from typing import List, Optional

import numpy as np
import torch

from .solver import SDK_SOLVED, as_boards, get_solver
from .sudoku import Sudoku

# 17-clue boards with exactly one solution (certified by
# tests/test_oracle.py::test_seeds_unique with the oracle's counter); the last
# one is the "brute-force resistant" board whose solution's first row is
# 987654321 -- a worst case for the walk.  Through round 3 hard17_batch made
# every benchmark board from these six (six isomorphism classes); they now
# seed the corpus search (scripts/make_hard17.py -> data/hard17_classes.txt),
# and bench.py also reports a search-heavy side set (hard_search_batch).
SEEDS_17 = (
    "000000010400000000020000000000050407008000300001090000300400200050100000000806000",
    "000000010400000000020000000000050604008000300001090000300400200050100000000807000",
    "000000012000035000000600070700000300000400800100000000000120000080000040050000600",
    "000000012003600000000007000410020000000500300700000600280000040000300500000000000",
    "000000012008030000000000040120500000000004700060000000507000300000620000000100000",
    "000000000000003085001020000000507000004000100090000000500000073002010000000040009",
)
PATHOLOGICAL = SEEDS_17[5]
# a 21-clue unique board that naked + hidden singles cannot finish: needs
# real search under either walk order (frontier-split tests / latency bench)
SEARCH_HEAVY = "800000000003600000070090200050007000000045700000100030001000068008500010090000400"


def _board_from_flat(flat) -> List[List[int]]:
    flat = list(flat)
    return [flat[r * 9:(r + 1) * 9] for r in range(9)]


def solve_sudoku(board) -> bool:
    """gen.py:6-28 on the GPU: fills `board` (9x9 list of lists) in place."""
    sols, st = get_solver().solve(as_boards(board))
    if int(st[0].item()) != SDK_SOLVED:
        return False
    flat = sols[0].cpu().tolist()
    for r in range(9):
        board[r][:] = flat[r * 9:(r + 1) * 9]
    return True


def _draw_diagonal(rng) -> List[List[int]]:
    # gen.py:33-40
    board = [[0] * 9 for _ in range(9)]
    for n in range(0, 9, 3):
        nums = rng.sample(range(1, 10), 9)
        for i in range(3):
            for j in range(3):
                board[n + i][n + j] = nums.pop()
    return board


def _draw_removals(rng, empty_boxes, full_mask) -> List[int]:
    # gen.py:46-50, on the zero pattern only (the walk fills every cell of a
    # diagonal-seeded board, so the pattern does not depend on the digits)
    zero = [not f for f in full_mask]
    out = []
    for _ in range(empty_boxes):
        row, col = rng.randint(0, 8), rng.randint(0, 8)
        while zero[row * 9 + col]:
            row, col = rng.randint(0, 8), rng.randint(0, 8)
        zero[row * 9 + col] = True
        out.append(row * 9 + col)
    return out


def generate_sudoku(empty_boxes=0, rng=None) -> Sudoku:
    """gen.py:31-52 (uses the global `random` module unless rng is given)."""
    rng = rng if rng is not None else _random
    board = _draw_diagonal(rng)
    solve_sudoku(board)
    full = [v != 0 for row in board for v in row]
    for cell in _draw_removals(rng, empty_boxes, full):
        board[cell // 9][cell % 9] = 0
    return Sudoku(board)


def generate_batch(n: int, empty_boxes: int, seed: Optional[int] = None, device=None,
                   return_solutions: bool = False):
    """Exactly [generate_sudoku(empty_boxes) for _ in range(n)] after
    random.seed(seed), with the n fills solved as one GPU batch.
    Returns a (n, 81) uint8 tensor on the device (and the full grids)."""
    rng = _random.Random(seed)
    # The reference interleaves per board: 3 samples, solve, removals.  The
    # removal draws depend only on the zero pattern, so drawing board by board
    # here yields the same sequence as long as every fill succeeds (checked).
    diag = np.zeros((n, 81), dtype=np.uint8)
    removals = []
    for k in range(n):
        b = _draw_diagonal(rng)
        diag[k] = np.asarray(b, dtype=np.uint8).reshape(81)
        removals.append(_draw_removals(rng, empty_boxes, [True] * 81))
    solver = get_solver(device)
    full, st = solver.solve(torch.from_numpy(diag))
    if not bool((st == SDK_SOLVED).all().item()):
        raise RuntimeError("a diagonal-seeded board had no completion; "
                           "generate these boards one by one with generate_sudoku")
    puzzles = full.clone()
    if empty_boxes:
        idx = torch.as_tensor(np.asarray(removals, dtype=np.int64).reshape(n, empty_boxes),
                              device=puzzles.device)
        puzzles.scatter_(1, idx, 0)
    return (puzzles, full) if return_solutions else puzzles


# ------------------------------------------------------------ hard 17-clue set
def _perms(rng: np.random.Generator, shape, k: int) -> np.ndarray:
    """Uniform random permutations of range(k), vectorised over `shape`."""
    return np.argsort(rng.random(tuple(shape) + (k,)), axis=-1)


def _symmetry_images(base: np.ndarray, n: int, seed: int) -> np.ndarray:
    """n random validity-preserving images of the (k, 81) boards `base`:
    digit relabeling, row / column permutations inside bands / stacks,
    band / stack permutations, transposition.  Clue count, number of
    completions and logical difficulty are invariants; the walk's cell
    order sees a different board each time."""
    rng = np.random.default_rng(seed)
    base = base.reshape(-1, 9, 9)
    which = rng.integers(len(base), size=n)
    relabel = np.zeros((n, 10), dtype=np.uint8)
    relabel[:, 1:] = _perms(rng, (n,), 9) + 1
    rows = (_perms(rng, (n,), 3)[:, :, None] * 3 + _perms(rng, (n, 3), 3)).reshape(n, 9)
    cols = (_perms(rng, (n,), 3)[:, :, None] * 3 + _perms(rng, (n, 3), 3)).reshape(n, 9)
    trans = rng.integers(2, size=n).astype(bool)
    # one flat source cell per output cell, then 1-D takes in blocks (the same
    # draws and bytes as transposing and gathering rows, columns and digits
    # in turn, in a third of the time): out(r, c) = base(rows[r], cols[c]), or
    # base(cols[c], rows[r]) when transposed
    out = np.empty((n, 81), dtype=np.uint8)
    flat = base.reshape(len(base), 81)
    for lo in range(0, n, 1 << 16):
        sl = slice(lo, min(n, lo + (1 << 16)))
        m = sl.stop - lo
        r, c = rows[sl, :, None].astype(np.int32), cols[sl, None, :].astype(np.int32)
        src = np.where(trans[sl, None, None], c * 9 + r, r * 9 + c).reshape(m, 81)
        cell = np.take(flat, which[sl, None].astype(np.int64) * 81 + src)
        out[sl] = np.take(relabel[sl].ravel(), np.arange(m, dtype=np.int64)[:, None] * 10 + cell)
    return out


_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def hard17_classes() -> List[str]:
    """The hard 17-clue corpus: one board per isomorphism class (minlex
    form), each certified 17 clues + one completion (data/hard17_classes.txt,
    made by scripts/make_hard17.py from SEEDS_17 by clue exchanges)."""
    with open(os.path.join(_DATA, "hard17_classes.txt")) as f:
        return [ln.split()[0] for ln in f if ln.strip() and not ln.startswith("#")]


def hard17_batch(n: int, seed: int = 0, seeds=None, device=None) -> torch.Tensor:
    """n 17-clue unique-solution boards (symmetry images of `seeds`, default
    the hard17_classes() corpus), as a (n, 81) uint8 tensor on `device`
    (host if device is None)."""
    seeds = hard17_classes() if seeds is None else seeds
    base = np.array([[int(c) for c in s] for s in seeds], dtype=np.uint8)
    t = torch.from_numpy(np.ascontiguousarray(_symmetry_images(base, n, seed)))
    return t.to(device) if device is not None else t


_HARD_SEARCH = os.path.join(_DATA, "hard_search_seeds.txt")


def hard_search_seeds() -> List[str]:
    """The search-heavy seed boards (data/hard_search_seeds.txt, made by
    scripts/make_hard_search.py): minimal unique puzzles from gen.py-style
    grids that naked + hidden singles cannot finish (>= 2 guesses)."""
    with open(_HARD_SEARCH) as f:
        return [ln.split()[0] for ln in f if ln.strip() and not ln.startswith("#")]


def hard_search_batch(n: int, seed: int = 0, device=None) -> torch.Tensor:
    """n search-heavy unique-solution boards (symmetry images of
    hard_search_seeds()), as a (n, 81) uint8 tensor."""
    base = np.array([[int(c) for c in s] for s in hard_search_seeds()], dtype=np.uint8)
    t = torch.from_numpy(np.ascontiguousarray(_symmetry_images(base, n, seed)))
    return t.to(device) if device is not None else t


if __name__ == "__main__":  # gen.py:55-66
    empty_boxes = int(sys.argv[1])
    new_puzzle = generate_sudoku(empty_boxes)
    print(new_puzzle)
    print(
        "curl http://localhost:8001/solve -X POST -H 'Content-Type: application/json' -d '{\"sudoku\": %s}'"
        % (new_puzzle.grid)
    )
