"""Drop-in for the reference's ``sudoku.py`` ``Sudoku`` class.

Same constructor, attributes and methods as sudoku.py:5-140 (grid, rate
limiter, ``__str__``, ``update_row``/``update_column``, ``check_is_valid``,
``check_row``/``check_column``/``check_square``, ``check``), with the
board-level entry points on the GPU:

* ``check()``  -> ``sdk_check_batch`` mode 0 (sudoku.py:119-140)
* ``solve()``  -> ``sdk_solve_batch`` (gen.py:6-28's walk; new entry point
  the reference reaches through gen.solve_sudoku)

and batch forms ``Sudoku.check_many`` / ``Sudoku.solve_many`` for whole
tensors of boards.  The per-unit helpers stay host-side: they touch 9 cells.
"""
from __future__ import annotations

import time
from collections import deque

import torch

from .solver import SDK_SOLVED, as_boards, get_solver


class Sudoku:
    def __init__(self, sudoku, base_delay=0.01, interval=10, threshold=5):
        self.grid = sudoku
        self.recent_requests = deque()
        self.base_delay = base_delay
        self.interval = interval
        self.threshold = threshold

    # sudoku.py:13-30 -- same arithmetic, same defaults
    def _limit_calls(self, base_delay=0.01, interval=10, threshold=5):
        if base_delay is None:
            base_delay = self.base_delay
        if interval is None:
            interval = self.interval
        if threshold is None:
            threshold = self.threshold
        now = time.time()
        self.recent_requests.append(now)
        num_requests = sum(1 for t in self.recent_requests if now - t < interval)
        if num_requests > threshold:
            time.sleep(base_delay * (num_requests - threshold + 1))

    # sudoku.py:32-49
    def __str__(self):
        out = "| - - - - - - - - - - - |\n"
        for i in range(9):
            out += "| "
            for j in range(9):
                v = self.grid[i][j]
                out += str(v) if v != 0 else f"\033[93m{v}\033[0m"
                out += " | " if j % 3 == 2 else " "
            if i % 3 == 2:
                out += "\n| - - - - - - - - - - - |"
            out += "\n"
        return out

    # sudoku.py:51-58
    def update_row(self, row, values):
        self.grid[row] = values

    def update_column(self, col, values):
        for row in range(9):
            self.grid[row][col] = values[row]

    # sudoku.py:60-78
    def check_is_valid(self, row, col, num, base_delay=None, interval=None, threshold=None):
        self._limit_calls(base_delay, interval, threshold)
        g = self.grid
        for i in range(9):
            if g[row][i] == num or g[i][col] == num:
                return False
        sr, sc = 3 * (row // 3), 3 * (col // 3)
        for i in range(3):
            for j in range(3):
                if g[sr + i][sc + j] == num:
                    return False
        return True

    # sudoku.py:80-117
    def check_row(self, row, base_delay=None, interval=None, threshold=None):
        self._limit_calls(base_delay, interval, threshold)
        r = self.grid[row]
        return not (sum(r) != 45 or len(set(r)) != 9)

    def check_column(self, col, base_delay=None, interval=None, threshold=None):
        self._limit_calls(base_delay, interval, threshold)
        c = [self.grid[row][col] for row in range(9)]
        return not (sum(c) != 45 or len(set(c)) != 9)

    def check_square(self, row, col, base_delay=None, interval=None, threshold=None):
        self._limit_calls(base_delay, interval, threshold)
        s = [self.grid[row + i][col + j] for i in range(3) for j in range(3)]
        return not (sum(s) != 45 or len(set(s)) != 9)

    # sudoku.py:119-140 -- whole-board verdict on the GPU.  The reference
    # charges _limit_calls once per unit it inspects (rows, columns, squares,
    # stopping at the first bad one); with a non-zero delay we charge the same.
    # Any byte value goes to the kernel (it does the reference's sum / set
    # arithmetic on bytes); a cell that is not a byte at all (negative, > 255,
    # not an int) cannot be a GPU operand, and the reference's own unit
    # helpers give the verdict -- a False unless that unit arithmetic says so,
    # never an exception (sudoku.py:85 returns False).
    def check(self, base_delay=None, interval=None, threshold=None):
        if not self._byte_grid():
            return self._units_until_failure() == 28
        ok = bool(Sudoku.check_many([self.grid])[0].item())
        delay = self.base_delay if base_delay is None else base_delay
        if delay:
            for _ in range(min(27, self._units_until_failure())):
                self._limit_calls(base_delay, interval, threshold)
        return ok

    def _byte_grid(self) -> bool:
        try:
            return len(self.grid) == 9 and all(
                len(r) == 9 and all(type(v) is int and 0 <= v <= 255 for v in r) for r in self.grid)
        except TypeError:
            return False

    def _units_until_failure(self) -> int:
        """1-based index of the first unit (rows, columns, squares) failing
        sudoku.py:85's test, 28 if none does."""
        g = self.grid
        units = [g[r] for r in range(9)]
        units += [[g[r][c] for r in range(9)] for c in range(9)]
        units += [[g[3 * i + a][3 * j + b] for a in range(3) for b in range(3)]
                  for i in range(3) for j in range(3)]
        for k, u in enumerate(units):
            if sum(u) != 45 or len(set(u)) != 9:
                return k + 1
        return 28

    # ----------------------------------------------------------- GPU batch
    def solve(self) -> bool:
        """Fill self.grid in place with the walk's first solution
        (gen.py:6-28); return False and leave the grid untouched if none."""
        solver = get_solver()
        sols, st = solver.solve(as_boards(self.grid))
        st_h = int(st[0].item())
        if st_h == SDK_SOLVED:
            flat = sols[0].cpu().tolist()
            for r in range(9):
                self.grid[r][:] = flat[r * 9:(r + 1) * 9]
            return True
        return False

    @staticmethod
    def check_many(grids, mode: int = 0) -> torch.Tensor:
        return get_solver().check(grids, mode)

    @staticmethod
    def solve_many(puzzles, ordered: bool = False):
        return get_solver().solve(as_boards(puzzles), ordered=ordered)
