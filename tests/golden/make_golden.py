"""Generate golden vectors by running the REFERENCE's own Python code.

Run only in the build container (the reference is mounted read-only at
/root/reference there; it does not exist on the GPU box):

    python tests/golden/make_golden.py [/root/reference]

It imports the reference's gen.py, sudoku.py and node.py and records
inputs + outputs as JSON data (no reference source is copied):

* golden_gen.json     -- gen.generate_sudoku(e) under random.seed(s)
                         (gen.py:31-52), its gen.solve_sudoku result
                         (gen.py:6-28) and Sudoku(...).check() (sudoku.py:119-140)
* golden_solve.json   -- gen.solve_sudoku on named boards: README puzzle,
                         two 17-clue puzzles, duplicate-given and
                         unsolvable boards, the empty board
* golden_check.json   -- Sudoku.check / check_is_valid (sudoku.py) and
                         node.SudokuSolver.check (node.py:82-116) on grids
* golden_node.json    -- node.SudokuSolver.solve_sudoku_destributed
                         (node.py:76-80) tasks and solve_sudoku_recursive
                         (node.py:62-74) on small boards
"""
from __future__ import annotations

import contextlib
import io
import json
import logging
import os
import random
import signal
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


class _Timeout(Exception):
    pass


def _alarm(_s, _f):
    raise _Timeout()


def s81(board):
    return "".join(str(v) for row in board for v in row)


def b81(s):
    return [[int(s[r * 9 + c]) for c in range(9)] for r in range(9)]


def run_limited(fn, seconds):
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(seconds)
    try:
        return fn()
    finally:
        signal.alarm(0)


NAMED = {
    # README.md:21 curl example (8 clues, many solutions)
    "readme": "000100000000320000000009000000000070000000000000900000000000900000000003000000000",
    # 17-clue puzzles with a unique solution (certified by the oracle's counter)
    "c17_a": "000000012003600000000007000410020000000500300700000600280000040000300500000000000",
    "c17_b": "000000012008030000000000040120500000000004700060000000507000300000620000000100000",
    "empty": "0" * 81,
    # full valid grid: sudoku.py:144-156 example
    "full_valid": "897124635531679284642385179154293867289716453376458912923867541765941328418532796",
    # duplicate givens (two 5s in row 0) -- the reference never tests givens
    "dup_row": "550000000000000000000000000000000000000000000000000000000000000000000000000000000",
    # duplicate givens in a column and box, many empties
    "dup_col": "300000000300000000000000000000000000000000000000000000000000000000000000000000000",
    # cell (0,8) has no candidate: row 0 holds 1..8, column 8 holds 9
    "dead_cell": "123456780000000009000000000000000000000000000000000000000000000000000000000000000",
    # unsolvable without a dead cell at the start: a digit has no place in box 0
    "no_place": "000000000000000000000000000100000000010000000001000000000100000000010000000001000",
}


def main(ref_dir):
    sys.path.insert(0, ref_dir)
    import gen  # noqa: E402  (reference)
    import sudoku as ref_sudoku  # noqa: E402  (reference)

    logging.disable(logging.CRITICAL)
    with contextlib.redirect_stdout(io.StringIO()):
        import node  # noqa: E402  (reference; prints at import-time paths)

    # ---------------------------------------------------------------- gen
    gen_cases = []
    for seed in range(12):
        for empties in (0, 5, 20, 40, 50, 58, 64, 81):
            random.seed(seed * 1000 + empties)
            puzzle = gen.generate_sudoku(empties)
            board = [row[:] for row in puzzle.grid]
            p = s81(board)
            try:
                ok = run_limited(lambda: gen.solve_sudoku(board), 60)
            except _Timeout:
                continue
            gen_cases.append({
                "seed": seed * 1000 + empties, "empty_boxes": empties,
                "puzzle": p, "solved": bool(ok), "solution": s81(board),
                "check": bool(ref_sudoku.Sudoku([r[:] for r in board]).check()),
            })
    with open(os.path.join(HERE, "golden_gen.json"), "w") as f:
        json.dump(gen_cases, f, indent=0)

    # -------------------------------------------------------------- solve
    solve_cases = []
    for name, p in NAMED.items():
        board = b81(p)
        try:
            ok = run_limited(lambda: gen.solve_sudoku(board), 600)
        except _Timeout:
            print("timeout", name)
            continue
        solve_cases.append({"name": name, "puzzle": p, "solved": bool(ok),
                            "solution": s81(board)})
        print("solve", name, ok, flush=True)
    with open(os.path.join(HERE, "golden_solve.json"), "w") as f:
        json.dump(solve_cases, f, indent=0)

    # -------------------------------------------------------------- check
    rng = random.Random(7)
    grids = [c["solution"] for c in gen_cases if c["solved"]][:40]
    grids += [NAMED["full_valid"], "5" * 81, "0" * 81, NAMED["readme"]]
    mutated = []
    for g in grids[:20]:
        cells = list(g)
        i, j = rng.randrange(81), rng.randrange(81)
        cells[i], cells[j] = cells[j], cells[i]
        mutated.append("".join(cells))
        cells = list(g)
        cells[rng.randrange(81)] = str(rng.randrange(10))
        mutated.append("".join(cells))
    # row-permuted rows keep row sums/sets, break columns only if rows swap across bands
    g = NAMED["full_valid"]
    mutated.append(g[9:18] + g[0:9] + g[18:])
    mutated.append(g[27:54] + g[0:27] + g[54:])
    check_cases = []
    solver = node.SudokuSolver(0)
    for g in grids + mutated:
        board = b81(g)
        valid_tests = []
        for _ in range(6):
            r, c, n = rng.randrange(9), rng.randrange(9), rng.randrange(1, 10)
            valid_tests.append([r, c, n, bool(ref_sudoku.Sudoku(b81(g)).check_is_valid(r, c, n))])
        check_cases.append({
            "grid": g,
            "check": bool(ref_sudoku.Sudoku(board).check()),
            "node_check": bool(solver.check(b81(g))),
            "is_valid": valid_tests,
        })
    with open(os.path.join(HERE, "golden_check.json"), "w") as f:
        json.dump(check_cases, f, indent=0)

    # --------------------------------------------------------------- node
    node_cases = {"first_candidate": [], "solve_recursive": []}
    small = [c for c in gen_cases if c["empty_boxes"] in (5, 20) and c["solved"]]
    for c in small[:12]:
        board = b81(c["puzzle"])
        for i in range(81):
            if c["puzzle"][i] == "0":
                r, col = divmod(i, 9)
                s = node.SudokuSolver(0)
                with contextlib.redirect_stdout(io.StringIO()):
                    num = s.solve_sudoku_destributed(board, r, col)
                node_cases["first_candidate"].append(
                    {"grid": c["puzzle"], "row": r, "col": col, "num": num})
    for name in ("dup_row",):
        board = b81(NAMED[name])
        node_cases["first_candidate"].append(
            {"grid": NAMED[name], "row": 0, "col": 2,
             "num": node.SudokuSolver(0).solve_sudoku_destributed(board, 0, 2)})
    # a sums-45 board with an empty cell: node.py's short-circuit fires
    quirk = "5" * 80 + "0"
    with contextlib.redirect_stdout(io.StringIO()):
        num = node.SudokuSolver(0).solve_sudoku_destributed(b81(quirk), 8, 8)
    node_cases["first_candidate"].append({"grid": quirk, "row": 8, "col": 8, "num": num})
    for c in [c for c in gen_cases if c["empty_boxes"] == 5][:6]:
        board = b81(c["puzzle"])
        s = node.SudokuSolver(0)
        with contextlib.redirect_stdout(io.StringIO()):
            out = s.solve_sudoku(board)
        node_cases["solve_recursive"].append(
            {"puzzle": c["puzzle"], "solved": out is not None,
             "solution": s81(board), "solved_puzzles": s.solved_puzzles})
    with open(os.path.join(HERE, "golden_node.json"), "w") as f:
        json.dump(node_cases, f, indent=0)
    print("gen", len(gen_cases), "solve", len(solve_cases), "check", len(check_cases),
          "node", {k: len(v) for k, v in node_cases.items()})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
