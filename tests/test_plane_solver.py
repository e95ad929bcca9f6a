"""CPU checks of the digit-plane lane solver (csrc/plane_solver.h, the
default GPU solve kernel): the same header compiled for the host with g++
(tests/native/plane_host.cpp), compared with the oracle on the goldens,
generated boards in both walk orders, clashing givens, hard 17-clue boards,
and its board loader against a plain per-byte loader."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import b81, load_golden
from oracle import oracle as O

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
# extra compiler flags for the host builds, e.g. SDK_HOST_CFLAGS="-DSDK_PLANE_LC=7"
# to check a rule-D variant against its restatement
HOST_FLAGS = os.environ.get("SDK_HOST_CFLAGS", "").split()


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    out = os.path.join(str(tmp_path_factory.mktemp("plane")), "libplane_host.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", *HOST_FLAGS, "-o", out,
                           os.path.join(NATIVE, "plane_host.cpp")])
    lib = ctypes.CDLL(out)
    lib.plane_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    lib.plane_check_load.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.plane_check_load.restype = ctypes.c_int64
    lib.plane_set_mrv_after.argtypes = [ctypes.c_uint32]
    lib.plane_set_mrv_after(0)
    return lib


@pytest.fixture(params=[0, 1, 24, 128], ids=lambda k: f"mrv{k}")
def mrv_after(request, host):
    """plane::solve's search-mode switch (M_WALK -> M_COUNT after k passes,
    0 = never): results never depend on it."""
    host.plane_set_mrv_after(request.param)
    yield request.param
    host.plane_set_mrv_after(0)


def _solve(lib, boards, node_order=0, max_depth=81, stats=None):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
    out = np.zeros_like(boards)
    st = np.zeros(len(boards), dtype=np.int32)
    g, p = ctypes.c_uint64(), ctypes.c_uint64()
    lib.plane_solve_batch(boards.ctypes.data, out.ctypes.data, st.ctypes.data, len(boards), node_order,
                          max_depth, ctypes.byref(g), ctypes.byref(p))
    if stats is not None:
        stats.update(guesses=g.value, passes=p.value)
    return out, st


def _s(row):
    return "".join(map(str, row.tolist()))


def test_plane_golden_gen(host):
    cases = load_golden("golden_gen.json")
    boards = np.array([b81(c["puzzle"]) for c in cases], dtype=np.uint8)
    out, st = _solve(host, boards)
    for c, o, s in zip(cases, out, st):
        assert s in (0, 1), c["seed"]
        assert bool(s) == c["solved"], c["seed"]
        assert _s(o) == c["solution"], c["seed"]


def test_plane_golden_solve_and_node(host):
    for c in load_golden("golden_solve.json"):
        out, st = _solve(host, np.array([b81(c["puzzle"])]))
        if st[0] == 2:  # clashing givens: the wave kernel's job
            continue
        assert bool(st[0]) == c["solved"] and _s(out[0]) == c["solution"], c["name"]
    for c in load_golden("golden_node.json")["solve_recursive"]:
        out, st = _solve(host, np.array([b81(c["puzzle"])]), node_order=1)
        if st[0] == 2:
            continue
        assert bool(st[0]) == c["solved"] and _s(out[0]) == c["solution"]


@pytest.mark.parametrize("order", ["gen", "node"])
def test_plane_generated_vs_literal_walk(host, order, mrv_after):
    from sudoku_solver_distributed_amd.gen import hard17_batch
    # gen.py-style boards on the CPU: complete grids with 55 cells erased
    grids, _ = O.solve_unique_batch(hard17_batch(200, seed=4321).numpy())
    rng = np.random.default_rng(4321)
    for g in grids:
        g[rng.choice(81, 55, replace=False)] = 0
    full = "897124635531679284642385179154293867289716453376458912923867541765941328418532796"
    dup = "88" + full[2:30] + "0" + full[31:50] + "0" + full[51:70] + "0" + full[71:]
    edge = np.array([b81(x) for x in (full, "5" * 81, dup, "0" * 81)], dtype=np.uint8)
    puzzles = np.concatenate([grids, edge])
    out, st = _solve(host, puzzles, node_order=int(order == "node"))
    want, wst = O.solve_batch(puzzles, order=order)
    mine = st != 2
    assert st[-3] == 2 and st[-2] == 2  # "5"*81 and dup have clashing givens
    assert np.array_equal(st[mine], wst[mine])
    assert np.array_equal(out[mine], want[mine])


@pytest.mark.parametrize("order", ["gen", "node"])
def test_plane_hard17_vs_oracle(host, order, mrv_after):
    from sudoku_solver_distributed_amd.gen import hard17_batch
    boards = hard17_batch(256, seed=7).numpy()
    stats = {}
    out, st = _solve(host, boards, node_order=int(order == "node"), stats=stats)
    want, cnt = O.solve_unique_batch(boards)  # unique completions: every walk finds it
    assert (cnt == 1).all()
    assert (st == 1).all()
    assert (out == want).all()
    print(order, "passes/board", stats["passes"] / len(boards), "guesses/board", stats["guesses"] / len(boards))


@pytest.mark.parametrize("order", ["gen", "node"])
def test_plane_count_mode_unsolvable_and_multi(host, order, mrv_after):
    """Boards the completion count sees no completion on: 17-clue boards
    with one more (wrong) clue -- no completion, or clashing givens left to
    the wave kernel."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    rng = np.random.default_rng(11)
    b = hard17_batch(300, seed=12).numpy()
    sols, _ = O.solve_unique_batch(b)
    for i in range(len(b)):
        c = rng.choice(np.nonzero(b[i] == 0)[0])
        b[i, c] = 1 + (sols[i, c] + rng.integers(0, 8)) % 9  # a digit the completion does not hold
    out, st = _solve(host, b, node_order=int(order == "node"))
    # no completion by construction: one would also complete the unique
    # 17-clue board, whose completion does not hold the added digit
    mine = st != 2
    assert mine.sum() > 50 and (st[mine] == 0).all() and np.array_equal(out[mine], b[mine])
    # (boards with many completions: test_plane_generated_vs_literal_walk,
    # where at mrv1 every board starts counting and goes back to the walk)


def test_plane_depth_overflow_defers(host):
    out, st = _solve(host, np.zeros((1, 81), np.uint8), max_depth=3)
    assert st[0] == 2
    out, st = _solve(host, np.zeros((1, 81), np.uint8))
    want, wst = O.solve_batch(np.zeros((1, 81), np.uint8), order="gen")
    assert st[0] == 1 and np.array_equal(out, want)


def test_plane_loader_matches_byte_loader(host):
    rng = np.random.default_rng(3)
    n = 2000
    boards = rng.integers(0, 10, size=(n, 81), dtype=np.uint8)
    boards[rng.random((n, 81)) < 0.6] = 0
    boards[::7, rng.integers(0, 81)] = rng.integers(10, 256)  # some invalid bytes
    boards[1] = 0
    boards[2] = 9
    boards[3, 80] = 10
    for v in range(10, 256):  # every invalid byte value, at positions of every word and byte lane
        boards[100 + v, (7 * v) % 81] = v
    assert host.plane_check_load(boards.ctypes.data, n) == 0


def test_pass_matches_previous_formulation(host):
    """The full-rate pass (v_bitop3 forms, plane_solver.h) leaves the same
    state and verdict as the previous formulation after every pass: along
    the search of hard 17-clue and generated boards, and from random plane
    states (tests/native/plane_host.cpp plane_check_pass)."""
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    grids, _ = O.solve_unique_batch(hard17_batch(200, seed=13).numpy())
    rng = np.random.default_rng(13)
    for g in grids:  # gen.py-style: complete grids with 50 cells erased
        g[rng.choice(81, 50, replace=False)] = 0
    host.plane_check_pass.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64]
    host.plane_check_pass.restype = ctypes.c_int64
    boards = np.ascontiguousarray(np.concatenate([hard17_batch(300, seed=11).numpy(),
                                                  hard_search_batch(300, seed=12).numpy(),
                                                  grids]))
    assert host.plane_check_pass(boards.ctypes.data, len(boards), 200_000, 99) == 0


# ---- the wave-wide tail solver (csrc/plane_wide.h) over an emulated wave

@pytest.fixture(scope="module")
def wide(tmp_path_factory):
    out = os.path.join(str(tmp_path_factory.mktemp("wide")), "libwide_host.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", *HOST_FLAGS, "-o", out,
                           os.path.join(NATIVE, "wide_host.cpp")])
    lib = ctypes.CDLL(out)
    lib.wide_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
    lib.wide_check_fixpoint.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32]
    lib.wide_check_fixpoint.restype = ctypes.c_int64
    lib.wide_set_mrv_after.argtypes = [ctypes.c_uint32]
    lib.wide_set_mrv_after(0)
    return lib


def _wide(lib, boards, node_order=0, lane_guesses=0, max_depth=81, stats=None):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
    out = np.zeros_like(boards)
    st = np.zeros(len(boards), dtype=np.int32)
    g, pl, pw = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.wide_solve_batch(boards.ctypes.data, out.ctypes.data, st.ctypes.data, len(boards), node_order,
                         max_depth, lane_guesses, ctypes.byref(g), ctypes.byref(pl), ctypes.byref(pw))
    if stats is not None:
        stats.update(guesses=g.value, passes_lane=pl.value, passes_wide=pw.value)
    return out, st


def _mixed_boards(n=150, seed=21):
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    grids, _ = O.solve_unique_batch(hard17_batch(n, seed=seed).numpy())
    rng = np.random.default_rng(seed)
    for g in grids:
        g[rng.choice(81, 56, replace=False)] = 0
    return np.ascontiguousarray(np.concatenate([hard17_batch(n, seed=seed + 1).numpy(),
                                                hard_search_batch(n, seed=seed + 2).numpy(), grids,
                                                np.zeros((1, 81), np.uint8)]))


def test_wide_fixpoint_matches_lane_pass(wide):
    """Jacobi hidden singles over the wave reach the lane pass's fixpoint
    (same verdict, same planes, same undetermined cells), from each board and
    from 20 random mid-search states per board; the only admitted
    disagreements are states holding two determined cells with one digit in
    a unit (wide_host.cpp wide_check_fixpoint)."""
    boards = _mixed_boards()
    assert wide.wide_check_fixpoint(boards.ctypes.data, len(boards), 20, 5) == 0


@pytest.mark.parametrize("order", ["gen", "node"])
@pytest.mark.parametrize("lane_guesses", [0, 1, 3])
def test_wide_continuation_vs_lane_solver(host, wide, order, lane_guesses, mrv_after):
    """Hand a board from the lane solver to the wave-wide solver after
    `lane_guesses` guesses (0: the whole search wide): identical answers and
    statuses.  The wide pass eliminates this pass's hidden singles at once,
    so it meets contradictions (a duplicated determined digit) no later than
    the lane pass: never more guesses, up to 1 % noise."""
    boards = _mixed_boards()
    no = int(order == "node")
    s_lane, s_wide = {}, {}
    want, wst = _solve(host, boards, node_order=no, stats=s_lane)
    wide.wide_set_mrv_after(mrv_after)  # the board's search mode is handed over too
    try:
        got, gst = _wide(wide, boards, node_order=no, lane_guesses=lane_guesses, stats=s_wide)
    finally:
        wide.wide_set_mrv_after(0)
    assert np.array_equal(gst, wst)
    assert np.array_equal(got, want)
    # (the completion count walks whole subtrees, contradictory states
    # included, where the two passes may part for a pass: a little more noise)
    assert s_wide["guesses"] <= (1.01 if mrv_after == 0 else 1.05) * s_lane["guesses"]
    if lane_guesses == 0:
        assert s_wide["passes_wide"] > 0 and s_wide["passes_lane"] == 0


def test_wide_edge_cases(wide):
    full = "897124635531679284642385179154293867289716453376458912923867541765941328418532796"
    boards = np.array([b81(x) for x in (full, "0" * 81, full[:40] + "0" + full[41:])], dtype=np.uint8)
    got, st = _wide(wide, boards)
    want, wst = O.solve_batch(boards, order="gen")
    assert np.array_equal(st, wst) and np.array_equal(got, want)
    # an unsolvable board: cell (8, 8) has no candidate (row 8 holds 2..9,
    # column 8 a 1); the gen.py walk starts there, so the oracle ends at once
    dead = np.zeros((1, 81), np.uint8)
    dead[0, 72:80] = [2, 3, 4, 5, 6, 7, 8, 9]
    dead[0, 63 + 8] = 1
    got, st = _wide(wide, dead)
    want, wst = O.solve_batch(dead, order="gen")
    assert st[0] == wst[0] == 0 and np.array_equal(got, want)
    # depth overflow hands the board on
    _, st = _wide(wide, np.zeros((1, 81), np.uint8), max_depth=3)
    assert st[0] == 2


# ---- other pass variants

@pytest.mark.parametrize("flags,group", [(0, 1), (1, 1), (5, 1), (7, 1), (3, 2), (3, 3), (3, 9), (7, 2)])
def test_pass_variants_match_their_restatement(tmp_path, flags, group):
    """Every SDK_PLANE_LC rule-D variant (0 none, 1 box -> column, 2 box ->
    row -- 3, both, is the default, covered above --, 4 column -> box) and every
    SDK_PLANE_GROUP grouping of rule C's hidden singles (1 Gauss-Seidel, the
    default; 2 and 3 digits per group; 9 Jacobi) keeps the pass equal to its
    plain-loop restatement (plane_host.cpp v1::pass) after every pass, and
    the wave-wide pass reaches its fixpoints (wide_host.cpp), so a build with
    other flags stays exact."""
    defines = ["-DSDK_PLANE_LC=%d" % flags, "-DSDK_PLANE_GROUP=%d" % group]
    libs = {}
    for name in ("plane_host", "wide_host"):
        out = str(tmp_path / ("lib%s_%d_%d.so" % (name, flags, group)))
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", *defines, "-o", out,
                               os.path.join(NATIVE, name + ".cpp")])
        libs[name] = ctypes.CDLL(out)
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    boards = np.ascontiguousarray(np.concatenate([hard17_batch(150, seed=21).numpy(),
                                                  hard_search_batch(150, seed=22).numpy()]))
    chk = libs["plane_host"].plane_check_pass
    chk.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64]
    chk.restype = ctypes.c_int64
    assert chk(boards.ctypes.data, len(boards), 50_000, 5) == 0
    f = libs["wide_host"].wide_check_fixpoint
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_uint32]
    f.restype = ctypes.c_int64
    assert f(boards[:100].ctypes.data, 100, 5, 3) == 0
    if group > 1:  # and the solver's answers are the oracle's
        lib = libs["plane_host"]
        lib.plane_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        lib.plane_set_mrv_after.argtypes = [ctypes.c_uint32]
        lib.plane_set_mrv_after(64)
        sols, st = _solve(lib, boards)
        want, cnt = O.solve_unique_batch(boards)
        assert (cnt == 1).all() and (st == 1).all() and np.array_equal(sols, want)


def test_open_root_rule_same_answers_fewer_passes(tmp_path):
    """SDK_PLANE_ROOT_OPEN (plane_solver.h): a board whose propagated root
    keeps >= 58 open cells counts its completions from the root at once.
    Same answers and statuses as without the rule (the count's one
    completion is the walk's answer), fewer passes on the 17-clue corpus."""
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    boards = np.ascontiguousarray(np.concatenate([hard17_batch(1500, seed=31).numpy(),
                                                  hard_search_batch(300, seed=32).numpy()]))
    res = {}
    for t in (0, 58):
        out = str(tmp_path / ("libplane_root%d.so" % t))
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-DSDK_PLANE_ROOT_OPEN=%d" % t,
                               "-o", out, os.path.join(NATIVE, "plane_host.cpp")])
        lib = ctypes.CDLL(out)
        lib.plane_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        lib.plane_set_mrv_after.argtypes = [ctypes.c_uint32]
        lib.plane_set_mrv_after(64)
        stats = {}
        sols, st = _solve(lib, boards, stats=stats)
        hard = {}
        _solve(lib, boards[:1500], stats=hard)
        res[t] = (sols, st, hard["passes"])
    assert np.array_equal(res[0][0], res[58][0]) and np.array_equal(res[0][1], res[58][1])
    assert res[58][2] < 0.95 * res[0][2], (res[0][2], res[58][2])
