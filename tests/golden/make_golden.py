"""Generate golden vectors by running the REFERENCE's own Python code.

Run only in the build container (the reference is mounted read-only at
/root/reference there; it does not exist on the GPU box):

    python tests/golden/make_golden.py [/root/reference] [--gen] [--solve] [--check] [--node] [--sc] [--peer]

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
* golden_sc.json      -- node.SudokuSolver.solve_sudoku (node.py:31-40, 62-74)
                         on boards where is_valid_move's short-circuit
                         (node.py:44-45: every unit sums to 45) can fire:
                         a full grid with one cell emptied and three cells
                         shifted so every unit still sums to 45, plus 0-5
                         extra blanks.  `sc_fires` marks the boards whose
                         answer differs from a walk without the short-circuit
                         (the build container's oracle decides; the expected
                         output is the reference's).
* golden_peer.json    -- node.P2PNode.peer_sudoku_solve (node.py:534-557), the
                         reference's HTTP /solve path, on a fresh single node
                         with handicap 0 (no peers: every cell task runs
                         locally, node.py:443-449): README puzzle + gen boards.
                         Its answer can be partial or invalid; a 3 s alarm
                         records the boards on which it never returns.
* golden_peer_seq.json -- the same /solve path on ONE node serving several
                         requests in a row.  P2PNode keeps partial_solution
                         and tried_numbers_by_position (node.py:149, 167)
                         across requests (peer_sudoku_solve resets neither,
                         node.py:534-552), so a later answer can depend on
                         earlier ones; `fresh` is the answer of a new node,
                         `validations` the node's counter after each request.
                         A sequence ends at the first request the reference
                         never returns from (the node would spin forever).
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


def b81s(s):
    return [int(x) for x in s]


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

def _sc_board(full, rng, extra):
    """Empty cell A=(r,c) (value v), add v to B=(r,c2) and C=(r3,c), subtract
    v from D=(r3,c2), c2 in A's box column: every unit still sums to 45."""
    g = [int(x) for x in full]
    for _ in range(1000):
        r, c = rng.randrange(9), rng.randrange(9)
        c2, r3 = 3 * (c // 3) + rng.randrange(3), rng.randrange(9)
        if c2 == c or r3 == r:
            continue
        A, B, C, D = r * 9 + c, r * 9 + c2, r3 * 9 + c, r3 * 9 + c2
        v = g[A]
        if g[B] + v <= 9 and g[C] + v <= 9 and g[D] - v >= 0:
            g[A], g[B], g[C], g[D] = 0, g[B] + v, g[C] + v, g[D] - v
            for e in rng.sample([i for i in range(81) if g[i]], extra):
                g[e] = 0
            return "".join(map(str, g))
    return None


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
    # ------------------------------------------------------ short-circuit
    if "sc" in stages:
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        import numpy as np
        from oracle import oracle as O  # filter only: which boards the short-circuit changes
        fulls = [c["solution"] for c in gen_cases if c["empty_boxes"] == 0]
        rng = random.Random(2026)
        sc_cases, fires = [], 0
        while len(sc_cases) < 64:
            p = _sc_board(fulls[len(sc_cases) % len(fulls)], rng, rng.choice([0, 0, 1, 2, 3, 5]))
            if p is None:
                continue
            plain, pst = O.solve_batch(np.array([b81s(p)], dtype=np.uint8), order="node")
            board = b81(p)
            s_ = node.SudokuSolver(0)
            try:
                with contextlib.redirect_stdout(io.StringIO()):
                    out = run_limited(lambda: s_.solve_sudoku(board), 30)
            except _Timeout:
                continue
            sol = s81(board)
            differs = (out is not None) != bool(pst[0]) or sol != "".join(map(str, plain[0].tolist()))
            if not differs and fires * 2 < len(sc_cases):
                continue  # keep at least half the fixture on boards where it fires
            fires += differs
            sc_cases.append({"puzzle": p, "solved": out is not None, "solution": sol, "sc_fires": differs})
        with open(os.path.join(HERE, "golden_sc.json"), "w") as f:
            json.dump(sc_cases, f, indent=0)
        print("sc", len(sc_cases), "fires", fires)

    # --------------------------------------------------------------- peer
    if "peer" in stages:
        boards = [("readme", NAMED["readme"])]
        boards += [(f"gen{c['seed']}", c["puzzle"]) for c in gen_cases
                   if c["empty_boxes"] in (5, 20, 40, 50, 58, 64)]
        sc_path = os.path.join(HERE, "golden_sc.json")
        if os.path.exists(sc_path):
            with open(sc_path) as f:
                boards += [(f"sc{k}", c["puzzle"]) for k, c in enumerate(json.load(f)[:16])]
        peer_cases = []
        for name, p in boards:
            with contextlib.redirect_stdout(io.StringIO()):
                n = node.P2PNode("127.0.0.1", 0, handicap=0)
                try:
                    out = run_limited(lambda: n.peer_sudoku_solve(b81(p)), 3)
                    res = s81(out) if out else None
                except _Timeout:
                    res = "TIMEOUT"
            peer_cases.append({"name": name, "puzzle": p, "returned": res,
                               "validations": n.solver.validations,
                               "solved_puzzles": n.solver.solved_puzzles})
        with open(os.path.join(HERE, "golden_peer.json"), "w") as f:
            json.dump(peer_cases, f, indent=0)
        print("peer", len(peer_cases))
    # ----------------------------------------------------------- peer-seq
    if "peerseq" in stages:
        with open(os.path.join(HERE, "golden_peer.json")) as f:
            fresh = {c["puzzle"]: c["returned"] for c in json.load(f)}
        pool = [p for p, r in fresh.items() if r != "TIMEOUT"]
        rng = random.Random(3)
        seqs, differing, tries = [], 0, 0
        while len(seqs) < 24 and tries < 2000:
            tries += 1
            k = rng.choice([2, 3, 4, 5])
            boards = [rng.choice(pool) for _ in range(k)]
            if rng.random() < 0.2:
                boards[1] = boards[0]  # the same board twice in a row
            steps = []
            with contextlib.redirect_stdout(io.StringIO()):
                n = node.P2PNode("127.0.0.1", 0, handicap=0)
                for p in boards:
                    try:
                        out = run_limited(lambda: n.peer_sudoku_solve(b81(p)), 3)
                        res = s81(out) if out else None
                    except _Timeout:
                        res = "TIMEOUT"
                    steps.append({"puzzle": p, "returned": res, "fresh": fresh[p],
                                  "validations": n.solver.validations,
                                  "solved_puzzles": n.solver.solved_puzzles})
                    if res == "TIMEOUT":
                        break
            d = any(st["returned"] != st["fresh"] for st in steps)
            if not d and differing * 2 < len(seqs) + 1:
                continue  # keep at least half the fixture on sequences where the state shows
            differing += d
            seqs.append({"requests": steps, "state_matters": d})
        with open(os.path.join(HERE, "golden_peer_seq.json"), "w") as f:
            json.dump(seqs, f, indent=0)
        print("peerseq", len(seqs), "state matters in", differing, "tries", tries)
    print("done", stages)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    st = [a[2:] for a in sys.argv[1:] if a.startswith("--")] or ["gen", "solve", "check", "node", "sc", "peer"]
    main(args[0] if args else "/root/reference", set(st))
