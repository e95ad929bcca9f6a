"""HIP path vs oracle / reference golden vectors (runs on an MI355X).

Bar: bit-exact boards and statuses.  The full-size cases (BASELINE.json's 1M
hard batch, every board against the oracle, and the bench's exact launch
shape) are in test_gpu_full_size.py.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, b81, load_golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _s(row):
    return "".join(str(int(v)) for v in row)


def test_library_is_native(solver):
    from sudoku_solver_distributed_amd import _lib
    assert solver.lib is _lib.load()
    assert b"gfx950" in solver.lib.sdk_version()
    assert solver.lib.sdk_device_cu_count() > 0


def test_golden_gen(solver):
    cases = load_golden("golden_gen.json")
    p = torch.tensor([b81(c["puzzle"]) for c in cases], dtype=torch.uint8)
    sols, st = solver.solve(p)
    sols, st = sols.cpu().numpy(), st.cpu().numpy()
    for c, o, s in zip(cases, sols, st):
        assert (s == 1) == c["solved"], c["seed"]
        assert _s(o) == c["solution"], (c["seed"], c["empty_boxes"])


def test_golden_named(solver):
    for c in load_golden("golden_solve.json"):
        sols, st = solver.solve(torch.tensor([b81(c["puzzle"])], dtype=torch.uint8))
        assert (int(st[0]) == 1) == c["solved"], c["name"]
        assert _s(sols[0].cpu()) == c["solution"], c["name"]


@pytest.mark.parametrize("order", ["gen", "node"])
def test_random_generated_vs_oracle(solver, order):
    """Seeded generate_batch boards, 30-81 empties, against the oracle's
    literal walk in each order.  The walk's answers are the committed fixture
    (tests/golden/make_random_generated.py; a few of these boards keep the
    literal walk busy for up to a minute each, so the fixture is pinned to
    the oracle on the CPU suite: test_oracle.py::test_random_generated_fixture)."""
    from sudoku_solver_distributed_amd.gen import generate_batch
    z = np.load(os.path.join(GOLDEN, "random_generated.npz"))
    for empties, n in z["cases"]:
        empties, n = int(empties), int(n)
        puzzles = generate_batch(n, empties, seed=int(z["seed0"]) + empties)
        assert np.array_equal(puzzles.cpu().numpy(), z[f"puzzles_{empties}"]), empties
        sols, st = solver.solve(puzzles, order=order)
        assert np.array_equal(st.cpu().numpy(), z[f"{order}_status_{empties}"]), empties
        assert np.array_equal(sols.cpu().numpy(), z[f"{order}_solutions_{empties}"]), empties


def test_generate_batch_matches_sequential(solver):
    import random
    from sudoku_solver_distributed_amd.gen import generate_batch, generate_sudoku
    batch = generate_batch(6, 45, seed=99).cpu().numpy()
    random.seed(99)
    seq = [generate_sudoku(45) for _ in range(6)]
    for b, s in zip(batch, seq):
        assert _s(b) == "".join(str(v) for r in s.grid for v in r)


def test_generate_matches_reference_golden(solver):
    import random
    from sudoku_solver_distributed_amd.gen import generate_sudoku
    for c in load_golden("golden_gen.json")[:24]:
        random.seed(c["seed"])
        s = generate_sudoku(c["empty_boxes"])
        assert "".join(str(v) for r in s.grid for v in r) == c["puzzle"]


def test_hard17_vs_unique_oracle(solver):
    from sudoku_solver_distributed_amd.gen import hard17_batch
    p = hard17_batch(384, seed=5)
    sols, st = solver.solve(p)
    want, cnt = O.solve_unique_batch(p.numpy())
    assert (cnt == 1).all()
    assert (st.cpu().numpy() == 1).all()
    assert np.array_equal(sols.cpu().numpy(), want)


def test_seeds_vs_literal_walk(solver):
    """17-clue seeds against the literal row-major walk (seconds each)."""
    from sudoku_solver_distributed_amd.gen import SEEDS_17
    p = np.array([b81(s) for s in SEEDS_17], dtype=np.uint8)
    sols, st = solver.solve(torch.from_numpy(p), order="node")
    want, wst = O.solve_batch(p, order="node")
    assert np.array_equal(sols.cpu().numpy(), want)
    assert np.array_equal(st.cpu().numpy(), wst)


@pytest.mark.parametrize("order", ["gen", "node"])
def test_edge_cases(solver, order):
    full = "897124635531679284642385179154293867289716453376458912923867541765941328418532796"
    bad_full = "5" * 81
    dead = "123456780000000009" + "0" * 63
    # clash in row 0 (cells 0 and 1 both 8) plus three blanks: completable
    dup = "88" + full[2:30] + "0" + full[31:50] + "0" + full[51:70] + "0" + full[71:]
    boards = [full, bad_full, dup, "0" * 81, dead]
    p = np.array([b81(s) for s in boards], dtype=np.uint8)
    sols, st = solver.solve(torch.from_numpy(p), order=order)
    sols, st = sols.cpu().numpy(), st.cpu().numpy()
    # the literal walk is tractable on all but `dead` in gen order (it would
    # enumerate rows 8..1 before reaching the dead cell in row 0)
    k = len(boards) if order == "node" else len(boards) - 1
    want, wst = O.solve_batch(p[:k], order=order)
    assert np.array_equal(st[:k], wst)
    assert np.array_equal(sols[:k], want)
    # `dead` has no completion (counter), so the walk's verdict is False and
    # the board is returned unchanged
    assert O.count_solutions(p[4], 1) == 0 and O.count_solutions(p[2], 1) >= 1
    assert st[4] == 0 and np.array_equal(sols[4], p[4])
    # empty batch
    s0, t0 = solver.solve(torch.empty((0, 81), dtype=torch.uint8), order=order)
    assert s0.shape == (0, 81) and t0.shape == (0,)


def test_invalid_bytes_rejected(solver):
    from sudoku_solver_distributed_amd.solver import as_boards
    with pytest.raises(ValueError):
        as_boards([10] + [0] * 80)
    # raw ABI path: status SDK_INVALID, output = input
    raw = torch.zeros((2, 81), dtype=torch.uint8, device=solver.device)
    raw[1, 5] = 12
    sols, st = solver.solve(raw)
    assert st.cpu().tolist() == [1, -1]
    assert int(sols[1, 5]) == 12


@pytest.mark.parametrize("kernel", ["auto", "plane", "packed"])
@pytest.mark.parametrize("order", ["gen", "node"])
def test_duplicate_givens_vs_oracle(solver, order, kernel):
    """Clashing givens: the walk never tests givens, so such boards can still
    be completed (e.g. nearly full boards); compare where a completion exists
    and the board is otherwise unchanged-False.  `plane` forces the
    lane-per-board kernel, which tests for clashing givens only once a search
    ends without a completion and then defers the board.  Node order is
    checked against the literal node.py walk (is_valid_move included)."""
    from sudoku_solver_distributed_amd import _lib
    prev = solver.lib.sdk_set_solve_kernel(_lib.SDK_KERNELS[kernel])
    try:
        _duplicate_givens_case(solver, order)
    finally:
        solver.lib.sdk_set_solve_kernel(prev)


def _duplicate_givens_case(solver, order):
    rng = np.random.default_rng(3)
    from sudoku_solver_distributed_amd.gen import generate_batch
    full = generate_batch(300, 0, seed=77).cpu().numpy()
    base = full.copy()
    for k, b in enumerate(base):
        b[rng.choice(81, (5, 10, 20)[k % 3], replace=False)] = 0
        i, j = rng.choice(81, 2, replace=False)
        if b[i] == 0:
            b[i] = rng.integers(1, 10)
        b[j] = b[i]
    sols, st = solver.solve(torch.from_numpy(base), order=order)
    sols, st = sols.cpu().numpy(), st.cpu().numpy()
    cnt = np.array([O.count_solutions(b, 1) for b in base])
    dead = cnt == 0
    assert (st[dead] == 0).all() and np.array_equal(sols[dead], base[dead])
    live = np.nonzero(~dead)[0]
    assert live.size > 100
    want, wst = O.solve_batch(base[live], order="node_literal" if order == "node" else order)
    assert np.array_equal(st[live], wst)
    assert np.array_equal(sols[live], want)


@pytest.mark.parametrize("kernel", ["auto", "plane", "packed"])
def test_short_circuit_goldens(solver, kernel):
    """node.py:44-45 (is_valid_move accepts any digit once every unit sums to
    45): the reference's SudokuSolver.solve_sudoku outputs on boards where it
    fires (tests/golden/golden_sc.json), in a small batch, and tiled into a
    batch large enough for the plane kernel (auto) -- whose clash test hands
    these boards to the wave kernel."""
    from sudoku_solver_distributed_amd import _lib
    cases = load_golden("golden_sc.json")
    p = torch.tensor([b81(c["puzzle"]) for c in cases], dtype=torch.uint8)
    want = [c["solution"] for c in cases]
    prev = solver.lib.sdk_set_solve_kernel(_lib.SDK_KERNELS[kernel])
    try:
        for reps in (1, 160):  # 64 and 10240 boards
            sols, st = solver.solve(p.repeat(reps, 1), order="node")
            sols, st = sols.cpu().numpy(), st.cpu().numpy()
            for k in range(len(cases) * reps):
                c = cases[k % len(cases)]
                assert (st[k] == 1) == c["solved"], (k, c["puzzle"])
                assert _s(sols[k]) == want[k % len(cases)], (k, c["puzzle"])
    finally:
        solver.lib.sdk_set_solve_kernel(prev)


def test_short_circuit_frontier(solver):
    """Frontier split in node order on short-circuit boards: the lowest
    solved frontier node is node.py's answer."""
    for c in load_golden("golden_sc.json")[:16]:
        ok, grid = solver.solve_one_split(torch.tensor([b81(c["puzzle"])], dtype=torch.uint8), target=64,
                                          order="node")
        assert ok == c["solved"], c["puzzle"]
        assert _s(grid.cpu()) == c["solution"], c["puzzle"]


def test_check_batch(solver):
    cases = load_golden("golden_check.json")
    g = torch.tensor([b81(c["grid"]) for c in cases], dtype=torch.uint8)
    ok0 = solver.check(g, 0).cpu().tolist()
    ok1 = solver.check(g, 1).cpu().tolist()
    assert ok0 == [int(c["check"]) for c in cases]
    assert ok1 == [int(c["node_check"]) for c in cases]


def test_first_candidate(solver):
    cases = load_golden("golden_node.json")["first_candidate"]
    g = torch.tensor([b81(c["grid"]) for c in cases], dtype=torch.uint8)
    cells = [c["row"] * 9 + c["col"] for c in cases]
    got = solver.first_candidate(g, cells).cpu().tolist()
    assert got == [c["num"] or 0 for c in cases]


# cell sequence of each walk (gen.py scans rows 8..0 in effect; node.py 0..8)
WALK = {"gen": [r * 9 + c for r in range(8, -1, -1) for c in range(9)],
        "node": list(range(81))}


@pytest.mark.parametrize("order", ["gen", "node"])
def test_frontier_order_and_split(solver, order):
    from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY
    root = torch.tensor([b81(SEARCH_HEAVY)], dtype=torch.uint8)
    nodes = solver.frontier(root, target=512, order=order)
    assert nodes.shape[0] >= 64
    # frontier nodes are in the walk's order: lexicographically increasing
    # along the walk's cell sequence
    a = nodes.cpu().numpy()[:, WALK[order]]
    for i in range(a.shape[0] - 1):
        d = np.nonzero(a[i] != a[i + 1])[0]
        assert d.size and 0 < a[i, d[0]] < a[i + 1, d[0]]
    ok, grid = solver.solve_one_split(root, target=2048, order=order)
    want, cnt = O.solve_unique_batch(np.array([b81(SEARCH_HEAVY)], dtype=np.uint8))
    assert ok and cnt[0] == 1
    assert np.array_equal(grid.cpu().numpy(), want[0])


def test_ordered_mode_picks_lowest(solver):
    from sudoku_solver_distributed_amd.gen import hard17_batch
    p = hard17_batch(64, seed=11)
    p[:10, :] = torch.tensor(b81("123456780000000009" + "0" * 63), dtype=torch.uint8)  # dead boards
    sols, st = solver.solve(p, ordered=True)
    st = st.cpu().numpy()
    assert (st[:10] == 0).all()
    assert st[10] == 1
    assert set(np.unique(st[11:])) <= {1, -2}
    assert solver.stats()["best"] == 10


def test_sudoku_class_api(solver):
    from sudoku_solver_distributed_amd.sudoku import Sudoku
    from sudoku_solver_distributed_amd.gen import solve_sudoku
    c = load_golden("golden_solve.json")[0]
    board = [[int(c["puzzle"][r * 9 + k]) for k in range(9)] for r in range(9)]
    assert solve_sudoku(board) == c["solved"]
    assert "".join(str(v) for r in board for v in r) == c["solution"]
    assert Sudoku(board).check() is True
    board[0][0], board[0][1] = board[0][1], board[0][0]
    assert Sudoku(board).check() is False
    # sudoku.py:85 answers False (no exception) for cells outside 1..9
    for bad in (10, 200, -3, 1000):
        b2 = [r[:] for r in board]
        b2[4][4] = bad
        assert Sudoku(b2).check() is False


def test_distributed_single_rank_gpu(solver):
    """distributed.py on the product backend (HIP kernels), world of one."""
    from sudoku_solver_distributed_amd.distributed import solve_shard, solve_split
    from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY, hard17_batch
    want, cnt = O.solve_unique_batch(np.array([b81(SEARCH_HEAVY)], dtype=np.uint8))
    for order in ("gen", "node"):
        st = {}
        ok, grid = solve_split(torch.tensor([b81(SEARCH_HEAVY)], dtype=torch.uint8), order=order,
                               target=256, chunk=16, stats=st)
        assert ok and np.array_equal(grid.cpu().numpy(), want[0]), st
    b = hard17_batch(1000, seed=9)
    (lo, hi), sols, sts = solve_shard(b)
    assert (lo, hi) == (0, 1000) and bool((sts == 1).all())
    w, c = O.solve_unique_batch(b.numpy())
    assert np.array_equal(sols.cpu().numpy(), w)


@pytest.mark.parametrize("kernel", ["packed", "plane"])
def test_alternate_kernels_parity(solver, kernel):
    """The non-default solve kernels (sdk_set_solve_kernel): goldens, generated
    boards in both walks, clashing givens, invalid bytes, ordered mode and
    hard 17-clue boards -- bit-identical to the oracle like the default."""
    from sudoku_solver_distributed_amd import _lib
    from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch
    prev = solver.lib.sdk_set_solve_kernel(_lib.SDK_KERNELS[kernel])
    assert prev > 0
    try:
        assert kernel.encode() in solver.lib.sdk_version()
        cases = load_golden("golden_gen.json")
        sols, st = solver.solve(torch.tensor([b81(c["puzzle"]) for c in cases], dtype=torch.uint8))
        for c, o, s in zip(cases, sols.cpu().numpy(), st.cpu().numpy()):
            assert (s == 1) == c["solved"] and _s(o) == c["solution"], c["seed"]
        for order in ("gen", "node"):
            full = "897124635531679284642385179154293867289716453376458912923867541765941328418532796"
            dup = "88" + full[2:30] + "0" + full[31:50] + "0" + full[51:70] + "0" + full[71:]
            edge = np.array([b81(x) for x in (full, "5" * 81, dup, "0" * 81)], dtype=np.uint8)
            puzzles = np.concatenate([generate_batch(96, 55, seed=4321).cpu().numpy(), edge])
            sols, st = solver.solve(torch.from_numpy(puzzles), order=order)
            want, wst = O.solve_batch(puzzles, order=order)
            assert np.array_equal(st.cpu().numpy(), wst), order
            assert np.array_equal(sols.cpu().numpy(), want), order
        raw = torch.zeros((3, 81), dtype=torch.uint8, device=solver.device)
        raw[1, 80] = 10
        raw[2, 0] = 255
        sols, st = solver.solve(raw)
        assert st.cpu().tolist() == [1, -1, -1] and int(sols[1, 80]) == 10
        p = hard17_batch(2000, seed=5)
        sols, st = solver.solve(p)
        want, cnt = O.solve_unique_batch(p.numpy())
        assert (st.cpu().numpy() == 1).all() and np.array_equal(sols.cpu().numpy(), want)
        p = hard17_batch(64, seed=11)
        p[:10, :] = torch.tensor(b81("123456780000000009" + "0" * 63), dtype=torch.uint8)
        solver.stats(reset=True)
        sols, st = solver.solve(p, ordered=True)
        st = st.cpu().numpy()
        assert (st[:10] == 0).all() and st[10] == 1 and set(np.unique(st[11:])) <= {1, -2}
        assert solver.stats()["best"] == 10
    finally:
        solver.lib.sdk_set_solve_kernel(prev)


def test_stats_agree_between_kernels(solver):
    """sdk_read_stats: every board counted once (the plane kernel's per-lane
    counters are summed over the wave).  Both kernels walk the same branch
    order (sdk_set_plane_search(0)), but the plane pass also applies rule D
    (plane_solver.h: box -> column locked candidates), which the wave kernel
    does not: stronger fixpoints, fewer branch nodes (~40 % fewer on this
    set).  Without rule D the plane kernel was within a few % above the wave
    kernel (it notices two equal determined cells in a unit some passes
    late).  The default search-mode switch needs fewer still."""
    from sudoku_solver_distributed_amd import _lib
    from sudoku_solver_distributed_amd.gen import hard17_batch
    p = hard17_batch(20000, seed=3).to(solver.device)
    got = {}
    for kernel in ("packed", "plane", "plane_count"):
        prev = solver.lib.sdk_set_solve_kernel(_lib.SDK_KERNELS[kernel.split("_")[0]])
        # the walk's own branch order for the like-for-like count; then the
        # default search-mode switch (heavy boards count completions on
        # fewest-candidates cells: fewer guesses)
        solver.lib.sdk_set_plane_search(-1 if kernel == "plane_count" else 0)
        try:
            solver.stats(reset=True)
            sols, st = solver.solve(p)
            torch.cuda.synchronize()
            got[kernel] = solver.stats(reset=True)
            assert bool((st == 1).all())
        finally:
            solver.lib.sdk_set_solve_kernel(prev)
            solver.lib.sdk_set_plane_search(-1)
    for k in ("packed", "plane", "plane_count"):
        assert got[k]["finished"] == 20000 and got[k]["solved"] == 20000, got
    assert got["plane_count"]["guesses"] < got["plane"]["guesses"], got
    # the plane kernel hands the last boards of sparse waves to the wave kernel
    assert got["packed"]["deferred"] == 0 and got["plane"]["deferred"] < 20000, got
    assert got["packed"]["guesses"] > 20000 * 0.3, got
    # rule D prunes: 144100 vs 237435 branch nodes when first measured
    assert got["plane"]["guesses"] < got["packed"]["guesses"] * 0.8, got
    assert got["plane"]["sweeps"] > 20000 * 5, got


def test_configs1_full_size(solver):
    """BASELINE.json configs[1] at its full size: 100k gen.py-generated
    boards (generate_sudoku(50) x 100k under one seed, gen.py:31-52), solved
    in one batch and diffed board by board against the literal gen.py:6-28
    walk: per-board digests of the oracle's walk over the same 100k boards,
    made on the CPU by tests/golden/make_configs1.py (configs1_100k.npz) --
    the puzzles' digests first, so the inputs are the fixture's."""
    import os
    from conftest import GOLDEN
    from sudoku_solver_distributed_amd.gen import generate_batch
    sys_path = os.path.join(GOLDEN, "make_configs1.py")
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_configs1", sys_path)
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    fx = np.load(os.path.join(GOLDEN, "configs1_100k.npz"))
    puzzles = generate_batch(int(fx["n"]), int(fx["empty"]), seed=int(fx["seed"]), device=solver.device)
    assert np.array_equal(mk.digests(puzzles.cpu().numpy()), fx["puzzle_digest"])
    sols, st = solver.solve(puzzles)
    assert np.array_equal(st.cpu().numpy(), fx["status"].astype(np.int32))
    assert np.array_equal(mk.digests(sols.cpu().numpy()), fx["solution_digest"])


@pytest.mark.parametrize("order", ["gen", "node"])
def test_hard_search_vs_unique_oracle(solver, order):
    """The search-heavy set (minimal puzzles that need ~10 guesses): unique
    completions, so every walk's answer is the oracle's completion."""
    from sudoku_solver_distributed_amd.gen import hard_search_batch
    p = hard_search_batch(4096, seed=21)
    sols, st = solver.solve(p, order=order)
    want, cnt = O.solve_unique_batch(p.numpy())
    assert (cnt == 1).all()
    assert (st.cpu().numpy() == 1).all()
    assert np.array_equal(sols.cpu().numpy(), want)


def test_hard_search_4m(solver):
    """4M search-heavy boards in one call: every board solved (status and the
    GPU Sudoku.check), givens kept, 256 sampled boards equal to the oracle,
    and no board handed to the wave kernel for depth (the stack holds 32
    levels; this set needs <= 13)."""
    from sudoku_solver_distributed_amd.gen import hard_search_batch
    n = 1 << 22
    p = hard_search_batch(n, seed=2025, device=solver.device)
    solver.stats(reset=True)
    sols, st = solver.solve(p)
    stats = solver.stats(reset=True)
    assert bool((st == 1).all())
    assert bool((solver.check(sols, 0) == 1).all())
    givens = p != 0
    assert bool((sols[givens] == p[givens]).all())
    assert stats["finished"] == n and stats["deferred"] == 0, stats
    assert stats["guesses"] > 5 * n, stats
    idx = torch.randint(0, n, (256,), generator=torch.Generator().manual_seed(2))
    want, cnt = O.solve_unique_batch(p[idx.to(p.device)].cpu().numpy())
    assert np.array_equal(sols[idx.to(p.device)].cpu().numpy(), want)


@pytest.mark.parametrize("tail,mode", [(40, 1), (0, 1), (40, 2), (8, 2)])
def test_plane_tail_paths(solver, tail, mode):
    """The plane kernel's drained-wave tail (sdk_set_plane_tuning): with 40
    the most boards of every wave end on the tail solver -- wave-wide
    continuation (mode 1, plane_wide.h) or through the XCD pool (2); 0
    switches the tail off.  Search-heavy and hard boards against their
    unique completion, generated multi-solution boards against the literal
    walk in both orders, clashing givens (deferred from the tail), an empty
    board deeper than the stack (deferred), ordered mode."""
    from sudoku_solver_distributed_amd import _lib
    from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch, hard_search_batch
    lib = solver.lib
    prev = lib.sdk_set_solve_kernel(_lib.SDK_KERNELS["plane"])
    assert lib.sdk_set_plane_tuning(-1, tail, mode, -1) == 0
    try:
        for order in ("gen", "node"):
            hs = np.concatenate([hard_search_batch(6144, seed=31).numpy(), hard17_batch(2048, seed=32).numpy()])
            sols, st = solver.solve(torch.from_numpy(hs), order=order)
            want, cnt = O.solve_unique_batch(hs)
            assert (cnt == 1).all() and (st.cpu().numpy() == 1).all()
            assert np.array_equal(sols.cpu().numpy(), want)
            gen = generate_batch(8192, 50, seed=33).cpu().numpy()
            gen[:16] = 0  # empty boards: searches deeper than the stack in gen order
            sols, st = solver.solve(torch.from_numpy(gen), order=order)
            want, wst = O.solve_batch(gen, order=order)
            assert np.array_equal(st.cpu().numpy(), wst)
            assert np.array_equal(sols.cpu().numpy(), want)
            _duplicate_givens_case(solver, order)
        # ordered mode: the lowest solvable index wins, later boards solved or cancelled
        p = hard_search_batch(8192, seed=34)
        p[:100, :] = torch.tensor(b81("123456780000000009" + "0" * 63), dtype=torch.uint8)  # dead boards
        sols, st = solver.solve(p, ordered=True)
        st = st.cpu().numpy()
        assert (st[:100] == 0).all() and st[100] == 1
        assert set(np.unique(st[101:])) <= {1, -2}
        assert solver.stats()["best"] == 100
        want, _ = O.solve_unique_batch(p[100:101].numpy())
        assert np.array_equal(sols[100].cpu().numpy(), want[0])
    finally:
        lib.sdk_set_plane_tuning(-1, -1, -1, -1)
        lib.sdk_set_solve_kernel(prev)


def test_solve_host_pipelined(solver):
    """BatchSolver.solve_host (chunks overlapping H2D / solve / D2H on three
    streams) returns exactly what solve() returns, for ragged chunking."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    boards = torch.cat([hard17_batch(20000, seed=41), torch.zeros((3, 81), dtype=torch.uint8)])
    want, wst = solver.solve(boards.to(solver.device))
    got, gst = solver.solve_host(boards.pin_memory(), chunk=8192)
    assert got.device.type == "cpu" and gst.device.type == "cpu"
    assert torch.equal(got, want.cpu()) and torch.equal(gst, wst.cpu())
    got, gst = solver.solve_host(boards[:5])  # pageable, one chunk
    assert torch.equal(got, want[:5].cpu())


def test_pool_overflow_keeps_boards_local(solver):
    """The XCD tail pool full: a full grid (512 waves per XCD) handing over
    up to 40 boards each reserves more than the pool's 8192 slots per XCD,
    and the boards past them stay in their wave's LDS for its own wide
    solver.  2^19 hard 17-clue boards against their unique completion, the
    kernel's finished count, and the same batch with the pool off."""
    from sudoku_solver_distributed_amd import _lib
    from sudoku_solver_distributed_amd.gen import hard17_batch
    lib = solver.lib
    prev = lib.sdk_set_solve_kernel(_lib.SDK_KERNELS["plane"])
    p = hard17_batch(1 << 19, seed=91)
    want, cnt = O.solve_unique_batch(p.numpy())
    assert (cnt == 1).all()
    try:
        assert lib.sdk_set_plane_tuning(-1, 40, 2, -1) == 0
        solver.stats(reset=True)
        sols, st = solver.solve(p)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 1).all() and np.array_equal(sols.cpu().numpy(), want)
        assert solver.stats()["finished"] == p.shape[0]
        assert lib.sdk_set_plane_tuning(-1, 40, 1, -1) == 0
        s1, t1 = solver.solve(p)
        torch.cuda.synchronize()
        assert torch.equal(s1, sols) and torch.equal(t1, st)
    finally:
        lib.sdk_set_plane_tuning(-1, -1, -1, -1)
        lib.sdk_set_solve_kernel(prev)


@pytest.mark.parametrize("refill,chunk", [(1, 0), (64, 64)])
def test_plane_refill_extremes(solver, refill, chunk):
    """The plane kernel's I/O at extreme knobs (sdk_set_plane_tuning):
    refill at every free lane with one queue claim per refill, and refill only
    when the whole wave is idle with the largest claims -- on a batch larger
    than the grid, so static hand-out, claims, outbox flushes and the tail
    all run.  Every board solved, passing Sudoku.check, givens kept, and a
    sample equal to its unique completion."""
    from sudoku_solver_distributed_amd import _lib
    from sudoku_solver_distributed_amd.gen import hard17_batch
    lib = solver.lib
    prev = lib.sdk_set_solve_kernel(_lib.SDK_KERNELS["plane"])
    assert lib.sdk_set_plane_tuning(refill, -1, -1, chunk) == 0
    try:
        boards = hard17_batch(300_000, seed=51)
        d = boards.to(solver.device)
        sols, st = solver.solve(d)
        assert bool((st == 1).all())
        assert bool((solver.check(sols, 0) == 1).all())
        given = d != 0
        assert bool((sols[given] == d[given]).all())
        idx = np.random.default_rng(51).choice(boards.shape[0], 2000, replace=False)
        want, cnt = O.solve_unique_batch(boards[idx].numpy())
        assert (cnt == 1).all() and np.array_equal(sols[idx].cpu().numpy(), want)
    finally:
        lib.sdk_set_plane_tuning(-1, -1, -1, -1)
        lib.sdk_set_solve_kernel(prev)


def test_solve_inflight_matches_solve(solver):
    """Launches in flight on separate streams / workspaces (the bench's
    steps): every batch's bytes and statuses equal solve()'s, batches of
    different sizes and walk orders interleaved, counters summed over slots."""
    from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch, hard_search_batch
    batches = [hard17_batch(40000, seed=5, device="cuda:0"), generate_batch(3000, 55, seed=6).cuda(),
               hard_search_batch(20000, seed=7, device="cuda:0"), hard17_batch(9000, seed=8, device="cuda:0"),
               generate_batch(50, 60, seed=9).cuda()]
    for order in ("gen", "node"):
        want = [solver.solve(b, order=order) for b in batches]
        want = [(s.clone(), t.clone()) for s, t in want]
        outs = [torch.empty_like(b) for b in batches]
        sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in batches]
        ev = []
        solver.inflight_stats(reset=True)
        got = solver.solve_inflight(batches, outs, sts, inflight=2, order=order, launch_events=ev)
        torch.cuda.synchronize()
        for (ws, wt), (gs, gt) in zip(want, got):
            assert torch.equal(ws, gs) and torch.equal(wt, gt)
        assert len(ev) == len(batches)
        st = solver.inflight_stats()
        assert st["finished"] == sum(b.shape[0] for b in batches)
    with pytest.raises(ValueError):
        solver.solve_inflight(batches, outs[:1], sts, inflight=2)


def test_solve_inflight_ragged_three_slots(solver):
    """Three launches in flight over ragged batches -- empty, one board, an
    invalid byte, clashing givens (the deferred kernel on a slot's own
    workspace), an all-empty board -- equal solve()'s bytes and statuses;
    ordered mode through the slots keeps each batch's own early-exit word."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    one = hard17_batch(1, seed=31)
    bad = hard17_batch(700, seed=32).clone()
    bad[3, 40] = 12
    bad[5, 0], bad[5, 1] = 7, 7  # givens repeating a digit in a row
    if bad[5, 2] == 7:
        bad[5, 2] = 0
    blank = torch.zeros((3, 81), dtype=torch.uint8)
    batches = [b.cuda() for b in (torch.empty((0, 81), dtype=torch.uint8), one, bad, blank,
                                  hard17_batch(30000, seed=33), one)]
    want = [tuple(t.clone() for t in solver.solve(b)) for b in batches]
    outs = [torch.empty_like(b) for b in batches]
    sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in batches]
    got = solver.solve_inflight(batches, outs, sts, inflight=3)
    torch.cuda.synchronize()
    for (ws, wt), (gs, gt) in zip(want, got):
        assert torch.equal(ws, gs) and torch.equal(wt, gt)
    st_bad = got[2][1].cpu().numpy()
    assert st_bad[3] == -1 and np.array_equal(got[2][0][3].cpu().numpy(), bad[3].numpy())  # SDK_INVALID, input back
    # ordered: board 0 of every batch solved, later ones solved or cancelled
    # with their input back
    big = [hard17_batch(20000, seed=40 + i).cuda() for i in range(3)]
    outs = [torch.empty_like(b) for b in big]
    sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in big]
    got = solver.solve_inflight(big, outs, sts, inflight=3, ordered=True)
    torch.cuda.synchronize()
    for b, (s, t) in zip(big, got):
        t = t.cpu().numpy()
        assert t[0] == 1 and set(np.unique(t).tolist()) <= {1, -2}
        canc = np.nonzero(t == -2)[0]
        assert np.array_equal(s.cpu().numpy()[canc], b.cpu().numpy()[canc])


def test_grid_waves_same_results(solver):
    """A launch's grid capped at 1 / 2 waves per SIMD (sdk_solve_batch_grid,
    solve_inflight's co-resident launches) changes only how many lanes share
    the batch: bytes and statuses equal the full grid's, in both orders, on a
    batch several times the capped grid's lanes."""
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    p = torch.cat([hard17_batch(200_000, seed=51), hard_search_batch(60_000, seed=52)]).cuda()
    p[7, 3] = 11  # an invalid byte past the static hand-out of the smallest grid
    for order in ("gen", "node"):
        want = [t.clone() for t in solver.solve(p, order=order)]
        for gw in (1, 2):
            got = solver.solve(p, order=order, grid_waves=gw)
            torch.cuda.synchronize()
            assert torch.equal(want[0], got[0]) and torch.equal(want[1], got[1]), (order, gw)
    with pytest.raises(RuntimeError):
        solver.solve(p[:1], grid_waves=-1)


def test_chunk_records_invalid_and_clashing(solver):
    """Boards that reach lanes through claimed chunks (past the static first
    hand-out of one board per lane) come from the lane-parallel chunk-record
    conversion: its invalid-byte flag (every value 10..255, in every byte
    lane of a word), clashing givens (deferred to the wave kernel) and a
    batch whose byte length is not a multiple of 4 -- statuses and bytes as
    the oracle / the raw-input rule say."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    n = 300_001  # > one board per lane of the persistent grid; 81 n % 4 != 0
    p = hard17_batch(n, seed=17).clone()
    nt = solver.lib.sdk_plane_grid_lanes() if hasattr(solver.lib, "sdk_plane_grid_lanes") else 262_144
    rng = np.random.default_rng(5)
    bad_idx = rng.choice(np.arange(nt, n), size=246, replace=False)
    for v, i in zip(range(10, 256), bad_idx):
        p[i, (7 * v) % 81] = v
    full = "897124635531679284642385179154293867289716453376458912923867541765941328418532796"
    dup = "88" + full[2:30] + "0" + full[31:50] + "0" + full[51:70] + "0" + full[71:]
    clash_idx = rng.choice(np.setdiff1d(np.arange(nt, n), bad_idx), size=40, replace=False)
    for i in clash_idx:
        p[i] = torch.tensor(b81(dup), dtype=torch.uint8)
    p[n - 1] = torch.tensor(b81("0" * 81), dtype=torch.uint8)
    sols, st = solver.solve(p.cuda())
    sols, st = sols.cpu().numpy(), st.cpu().numpy()
    pn = p.numpy()
    assert (st[bad_idx] == -1).all() and np.array_equal(sols[bad_idx], pn[bad_idx])
    want, wst = O.solve_batch(pn[clash_idx[:8]])
    assert np.array_equal(st[clash_idx[:8]], wst) and np.array_equal(sols[clash_idx[:8]], want)
    assert (st[clash_idx] == st[clash_idx[0]]).all()
    want_last, wst_last = O.solve_batch(pn[n - 1:])
    assert st[n - 1] == wst_last[0] and np.array_equal(sols[n - 1], want_last[0])
    rest = np.setdiff1d(np.arange(n - 1), np.concatenate([bad_idx, clash_idx]))
    assert (st[rest] == 1).all()
    sample = rng.choice(rest, size=512, replace=False)
    w, cnt = O.solve_unique_batch(pn[sample])
    assert np.array_equal(sols[sample], w)


def test_chunk_records_ordered_mode(solver):
    """Ordered mode (the frontier split's solve) on a batch large enough that
    most boards arrive through chunk records: once board 0 is solved every
    later board is either solved or cancelled with its input back, and the
    lowest solved index is 0."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    n = 300_000
    p = hard17_batch(n, seed=23)
    solver.stats(reset=True)
    sols, st = solver.solve(p.cuda(), ordered=True)
    sols, st = sols.cpu().numpy(), st.cpu().numpy()
    assert st[0] == 1 and solver.stats()["best"] == 0
    assert set(np.unique(st).tolist()) <= {1, -2}
    canc = np.nonzero(st == -2)[0]
    assert np.array_equal(sols[canc], p.numpy()[canc])
    done = np.nonzero(st == 1)[0]
    rng = np.random.default_rng(3)
    sample = rng.choice(done, size=min(256, len(done)), replace=False)
    w, cnt = O.solve_unique_batch(p.numpy()[sample])
    assert np.array_equal(sols[sample], w)
