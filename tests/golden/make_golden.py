"""Generate golden vectors by running the REFERENCE's own Python code.

Run only in the build container (the reference is mounted read-only at
/root/reference there; it does not exist on the GPU box):

    python tests/golden/make_golden.py [/root/reference] [--gen] [--solve] [--check] [--node]

It imports the reference's gen.py, sudoku.py and node.py and records
inputs + outputs as JSON data (no reference source is copied):

* golden_gen.json     -- gen.generate_sudoku(e) under random.seed(s)
                         (gen.py:31-52), its gen.solve_sudoku result
                         (gen.py:6-28) and Sudoku(...).check() (sudoku.py:119-140)
* golden_solve.json   -- gen.solve_sudoku on named boards: README puzzle,
                         two 17-clue puzzles, the empty board, full boards,
                         clashing givens, a dead first cell
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
    # 17-clue puzzles with a unique solution (certified by the oracle's counter);
    # gen.py's walk needs ~4e7-7e7 candidate tests on these (minutes in Python)
    "c17_a": "000000012003600000000007000410020000000500300700000600280000040000300500000000000",
    "c17_b": "000000012008030000000000040120500000000004700060000000507000300000620000000100000",
    "empty": "0" * 81,
    # full valid grid: sudoku.py:144-156 example
    "full_valid": "897124635531679284642385179154293867289716453376458912923867541765941328418532796",
    # full board of one digit: no empty cell, so the walk returns True at once
    "full_fives": "5" * 81,
    # clashing givens (two 8s in row 0) with three blanks: still completable,
    # the walk never tests givens
    "clash_completable": None,  # built below from full_valid
    # the walk's first cell (row 8 col 8) has no candidate: False at once
    "dead_first": "0" * 71 + "9" + "123456780",
}
_FULL = NAMED["full_valid"]
NAMED["clash_completable"] = ("88" + _FULL[2:30] + "0" + _FULL[31:50] + "0" + _FULL[51:70] + "0"
                              + _FULL[71:])
assert all(len(v) == 81 for v in NAMED.values())

def main(ref_dir, stages):
    sys.path.insert(0, ref_dir)
    import gen  # noqa: E402  (reference)
    import sudoku as ref_sudoku  # noqa: E402  (reference)

    logging.disable(logging.CRITICAL)
    with contextlib.redirect_stdout(io.StringIO()):
        import node  # noqa: E402  (reference; prints at import-time paths)

    # ---------------------------------------------------------------- gen
    gen_path = os.path.join(HERE, "golden_gen.json")
    if "gen" not in stages:
        with open(gen_path) as f:
            gen_cases = json.load(f)
    gen_cases = [] if "gen" in stages else gen_cases
    for seed in (range(12) if "gen" in stages else ()):
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
    if "gen" in stages:
        with open(gen_path, "w") as f:
            json.dump(gen_cases, f, indent=0)

    # -------------------------------------------------------------- solve
    solve_cases = []
    only = os.environ.get("GOLDEN_ONLY")  # comma list: recompute these, keep the rest
    solve_path = os.path.join(HERE, "golden_solve.json")
    if only and os.path.exists(solve_path):
        with open(solve_path) as f:
            solve_cases = [c for c in json.load(f) if c["name"] not in only.split(",")]
    for name, p in (NAMED.items() if "solve" in stages else ()):
        if only and name not in only.split(","):
            continue
        board = b81(p)
        try:
            ok = run_limited(lambda: gen.solve_sudoku(board), 600)
        except _Timeout:
            print("timeout", name)
            continue
        solve_cases.append({"name": name, "puzzle": p, "solved": bool(ok),
                            "solution": s81(board)})
        print("solve", name, ok, flush=True)
    if "solve" in stages:
        order = {k: i for i, k in enumerate(NAMED)}
        solve_cases.sort(key=lambda c: order.get(c["name"], 99))
        with open(solve_path, "w") as f:
            json.dump(solve_cases, f, indent=0)

    # -------------------------------------------------------------- check
    if "check" in stages:
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
        g = NAMED["full_valid"]
        mutated.append(g[9:18] + g[0:9] + g[18:])   # rows swapped inside a band
        mutated.append(g[27:54] + g[0:27] + g[54:])  # bands swapped
        check_cases = []
        solver = node.SudokuSolver(0)
        for g in grids + mutated:
            valid_tests = []
            for _ in range(6):
                r, c, n = rng.randrange(9), rng.randrange(9), rng.randrange(1, 10)
                valid_tests.append([r, c, n, bool(ref_sudoku.Sudoku(b81(g)).check_is_valid(r, c, n))])
            check_cases.append({
                "grid": g,
                "check": bool(ref_sudoku.Sudoku(b81(g)).check()),
                "node_check": bool(solver.check(b81(g))),
                "is_valid": valid_tests,
            })
        with open(os.path.join(HERE, "golden_check.json"), "w") as f:
            json.dump(check_cases, f, indent=0)

    # --------------------------------------------------------------- node
    if "node" in stages:
        node_cases = {"first_candidate": [], "solve_recursive": []}
        small = [c for c in gen_cases if c["empty_boxes"] in (5, 20) and c["solved"]]
        for c in small[:12]:
            board = b81(c["puzzle"])
            for i in range(81):
                if c["puzzle"][i] == "0":
                    r, col = divmod(i, 9)
                    with contextlib.redirect_stdout(io.StringIO()):
                        num = node.SudokuSolver(0).solve_sudoku_destributed(board, r, col)
                    node_cases["first_candidate"].append(
                        {"grid": c["puzzle"], "row": r, "col": col, "num": num})
        # clashing givens, and a sums-45 board with an empty cell (node.py's
        # is_valid_move short-circuit fires: node.py:44-45)
        for grid, r, col in (("550000000" + "0" * 72, 0, 2), ("5" * 80 + "0", 8, 8),
                             (NAMED["dead_first"], 8, 8)):
            with contextlib.redirect_stdout(io.StringIO()):
                num = node.SudokuSolver(0).solve_sudoku_destributed(b81(grid), r, col)
            node_cases["first_candidate"].append({"grid": grid, "row": r, "col": col, "num": num})
        for c in [c for c in gen_cases if c["empty_boxes"] == 5][:6] + \
                 [c for c in gen_cases if c["empty_boxes"] == 20][:2]:
            board = b81(c["puzzle"])
            s = node.SudokuSolver(0)
            with contextlib.redirect_stdout(io.StringIO()):
                out = s.solve_sudoku(board)
            node_cases["solve_recursive"].append(
                {"puzzle": c["puzzle"], "solved": out is not None,
                 "solution": s81(board), "solved_puzzles": s.solved_puzzles})
        with open(os.path.join(HERE, "golden_node.json"), "w") as f:
            json.dump(node_cases, f, indent=0)
    print("done", stages)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    st = [a[2:] for a in sys.argv[1:] if a.startswith("--")] or ["gen", "solve", "check", "node"]
    main(args[0] if args else "/root/reference", set(st))
