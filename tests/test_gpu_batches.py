"""Several batches per launch (sdk_solve_batches / BatchSolver.solve_batches,
the strong-scaling steps): every batch's bytes and statuses equal what
solve() gives it alone -- the queue runs over the batches laid end to end, so
claims, static hand-out windows, staged spans, the outbox, the wave-wide
tails, the XCD pool and the deferred list all cross batch boundaries here."""
import numpy as np
import pytest
import torch

from conftest import b81
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FULL = "897124635531679284642385179154293867289716453376458912923867541765941328418532796"
# givens repeating a digit in a row (rules B/C unsound: the deferred list)
CLASH = "88" + FULL[2:30] + "0" + FULL[31:50] + "0" + FULL[51:70] + "0" + FULL[71:]


def _mixed(seed):
    from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch, hard_search_batch
    bad = hard17_batch(701, seed=seed).clone()
    bad[3, 40] = 12                     # an invalid byte
    bad[500] = torch.tensor(b81(CLASH), dtype=torch.uint8)
    blank = torch.zeros((3, 81), dtype=torch.uint8)
    return [b.contiguous().cuda() for b in (
        hard17_batch(40_001, seed=seed + 1), generate_batch(3000, 55, seed=seed + 2).cpu(),
        torch.empty((0, 81), dtype=torch.uint8), hard_search_batch(20_000, seed=seed + 3),
        hard17_batch(1, seed=seed + 4), bad, blank, hard17_batch(9_003, seed=seed + 5))]


def _check_same(solver, batches, order="gen", grid_waves=0):
    want = [tuple(t.clone() for t in solver.solve(b, order=order)) for b in batches]
    outs = [torch.full_like(b, 0xEE) for b in batches]
    sts = [torch.full((b.shape[0],), 77, dtype=torch.int32, device=b.device) for b in batches]
    solver.stats(reset=True)
    got = solver.solve_batches(batches, outs, sts, order=order, grid_waves=grid_waves)
    torch.cuda.synchronize()
    for i, ((ws, wt), (gs, gt)) in enumerate(zip(want, got)):
        assert torch.equal(ws, gs) and torch.equal(wt, gt), (order, grid_waves, i)
    assert solver.stats()["finished"] == sum(b.shape[0] for b in batches)


@pytest.mark.parametrize("order", ["gen", "node"])
def test_solve_batches_matches_solve(solver, order):
    batches = _mixed(100)
    for gw in (0, 1):
        _check_same(solver, batches, order, gw)


def test_solve_batches_sixteen_unaligned(solver):
    """16 batches of odd sizes (byte offsets of every batch boundary mod 4
    differ), a grid of 1 wave per SIMD so most boards arrive by claims that
    straddle batch boundaries, and views into one buffer at odd offsets."""
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    big = torch.cat([hard17_batch(200_000, seed=7), hard_search_batch(30_000, seed=8)]).cuda()
    sizes = [1, 63, 65, 8191, 13, 20_011, 3, 40_000, 127, 1, 12_345, 77, 30_001, 5, 64, 50_000]
    offs = np.cumsum([0] + sizes)
    batches = [big[offs[i] + 3 * i: offs[i + 1] + 3 * i] for i in range(16)]
    _check_same(solver, batches, "gen", 1)
    _check_same(solver, batches, "node", 2)


def test_solve_batches_widest_tail(solver):
    """The widest tail (40 boards per wave, on the wave itself and through the
    XCD pool) and one-board claims, through several batches."""
    lib = solver.lib
    try:
        assert lib.sdk_set_plane_tuning(-1, 40, 2, -1) == 0
        _check_same(solver, _mixed(200), "gen", 1)
        assert lib.sdk_set_plane_tuning(-1, 40, 1, 1) == 0   # one-board claims
        _check_same(solver, _mixed(300), "node", 0)
    finally:
        lib.sdk_set_plane_tuning(-1, -1, -1, -1)


def test_solve_batches_vs_oracle(solver):
    """Independent of solve(): hard boards split over 5 batches equal the
    oracle's unique completions; generated boards the literal walk."""
    from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch
    h = hard17_batch(12_000, seed=61)
    g = generate_batch(2_000, 50, seed=62).cpu()
    parts = [h[:5000], g[:1000], h[5000:11_000], g[1000:], h[11_000:]]
    batches = [p.contiguous().cuda() for p in parts]
    outs = [torch.empty_like(b) for b in batches]
    sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in batches]
    got = solver.solve_batches(batches, outs, sts, grid_waves=1)
    torch.cuda.synchronize()
    wh, cnt = O.solve_unique_batch(h.numpy())
    wg, wgs = O.solve_batch(g.numpy())
    want = [wh[:5000], wg[:1000], wh[5000:11_000], wg[1000:], wh[11_000:]]
    for (s, t), w in zip(got, want):
        assert np.array_equal(s.cpu().numpy(), w)
    assert (cnt == 1).all() and all(bool((t == 1).all()) for _, t in got[::2])


def test_solve_inflight_grouped(solver):
    """solve_inflight(group=G): G consecutive batches per launch, launches in
    flight on three slots -- the bench's strong-scaling steps -- equal solve()."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    steps = [hard17_batch(16_384 + 7 * i, seed=70 + i, device="cuda:0") for i in range(11)]
    want = [tuple(t.clone() for t in solver.solve(b)) for b in steps]
    outs = [torch.empty_like(b) for b in steps]
    sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in steps]
    ev = []
    got = solver.solve_inflight(steps, outs, sts, inflight=3, group=4, launch_events=ev)
    torch.cuda.synchronize()
    assert len(ev) == 3  # 4 + 4 + 3 batches
    for (ws, wt), (gs, gt) in zip(want, got):
        assert torch.equal(ws, gs) and torch.equal(wt, gt)
    with pytest.raises(ValueError):
        solver.solve_inflight(steps, outs, sts, group=33)
    with pytest.raises(ValueError):
        solver.solve_inflight(steps, outs, sts, group=2, ordered=True)
    with pytest.raises(ValueError):
        solver.solve_batches(steps[:1] * 33, outs[:1] * 33, sts[:1] * 33)


@pytest.mark.parametrize("order", ["gen", "node"])
def test_search_mode_switch_same_results(solver, order):
    """sdk_set_plane_search: boards still searching after k passes restart
    from their root counting completions (plane::search_step).  Bytes and
    statuses never depend on k -- walk only (0), every board counting from
    its first pass (1), and thresholds in between -- on hard 17-clue boards,
    generated boards with many completions (the count's second completion
    sends them back to the walk), search-heavy boards, no-completion boards
    (one wrong clue added to a unique board), invalid bytes and clashing
    givens; in the lane loop, in the wave-wide tail (tail 40) and across
    batches (sdk_solve_batches)."""
    from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch, hard_search_batch
    lib = solver.lib
    rng = np.random.default_rng(21)
    nosol = hard17_batch(3000, seed=22).numpy()
    sols, _ = O.solve_unique_batch(nosol[:300])
    for i in range(300):  # one wrong clue: no completion (it would complete the unique board)
        c = rng.choice(np.nonzero(nosol[i] == 0)[0])
        nosol[i, c] = 1 + (sols[i, c] + rng.integers(0, 8)) % 9
    parts = [hard17_batch(30_000, seed=23), generate_batch(1000, 52, seed=24).cpu(),
             hard_search_batch(8000, seed=25), torch.from_numpy(nosol)]
    p = torch.cat(parts).cuda()
    p[11, 5] = 13
    p[40_000] = torch.tensor(b81(CLASH), dtype=torch.uint8)
    try:
        assert lib.sdk_set_plane_search(0) == 128  # the default in effect before
        want = [t.clone() for t in solver.solve(p, order=order)]
        torch.cuda.synchronize()
        # the generated boards (many completions) against the literal walk
        g0, g1 = 30_000, 31_000
        w, ws = O.solve_batch(p[g0:g1].cpu().numpy(), order=order)
        assert np.array_equal(want[0][g0:g1].cpu().numpy(), w) and np.array_equal(want[1][g0:g1].cpu().numpy(), ws)
        for k in (1, 8, 48, 128):
            assert lib.sdk_set_plane_search(k) >= 0
            for tail, mode in ((8, 1), (16, 2), (40, 2)):  # own tail / XCD pool
                assert lib.sdk_set_plane_tuning(-1, tail, mode, -1) == 0
                got = solver.solve(p, order=order)
                torch.cuda.synchronize()
                assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1]), (k, tail, mode)
        # across batches, and ordered mode (frontier split semantics)
        assert lib.sdk_set_plane_search(1) >= 0
        cut = [0, 7_000, 30_500, 36_000, p.shape[0]]
        bs = [p[a:b] for a, b in zip(cut, cut[1:])]
        outs = [torch.empty_like(b) for b in bs]
        sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in bs]
        solver.solve_batches(bs, outs, sts, order=order, grid_waves=1)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(outs), want[0]) and torch.equal(torch.cat(sts), want[1])
        h = hard17_batch(20_000, seed=26).cuda()
        s1, t1 = solver.solve(h, ordered=True, order=order)
        torch.cuda.synchronize()
        t1 = t1.cpu().numpy()
        assert t1[0] == 1 and set(np.unique(t1).tolist()) <= {1, -2}
        done = np.nonzero(t1 == 1)[0][:256]
        wu, cnt = O.solve_unique_batch(h[done].cpu().numpy())
        assert np.array_equal(s1[done].cpu().numpy(), wu)
    finally:
        lib.sdk_set_plane_search(-1)
        lib.sdk_set_plane_tuning(-1, -1, -1, -1)


def test_pipelined_flag_same_results(solver):
    """SDK_GRID_PIPELINED (a launch with another queued behind it: drained
    waves keep to their own tails) against the default launch (the XCD tail
    pool): the same bytes and statuses, single- and multi-batch, and through
    solve_inflight with every launch pipelined / none."""
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    p = torch.cat([hard17_batch(40_000, seed=61), hard_search_batch(20_000, seed=62)]).cuda()
    a = [t.clone() for t in solver.solve(p)]
    b = solver.solve(p, pipelined=True)
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and bool((a[1] == 1).all())
    parts = [p[:25_000], p[25_000:]]
    for pipe in (False, True):
        outs = [torch.empty_like(x) for x in parts]
        sts = [torch.empty(x.shape[0], dtype=torch.int32, device=x.device) for x in parts]
        solver.solve_batches(parts, outs, sts, grid_waves=1, pipelined=pipe)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(outs), a[0]) and torch.equal(torch.cat(sts), a[1])
    steps = [p[i * 10_000:(i + 1) * 10_000] for i in range(6)]
    for last in (0, 2, 6):
        outs = [torch.empty_like(x) for x in steps]
        sts = [torch.empty(x.shape[0], dtype=torch.int32, device=x.device) for x in steps]
        solver.solve_inflight(steps, outs, sts, inflight=3, pool_last=last)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(outs), a[0]) and torch.equal(torch.cat(sts), a[1]), last
    with pytest.raises(ValueError):
        solver.solve(p[:10], grid_waves=1 << 16)
