"""BASELINE.json configs[2] at full size on one MI355X, against the oracle
board by board, and the workspace's own accounting of answered boards.

* all 2^20 boards of the bench's batch (hard17_batch(2^20, seed 2024)) solved
  by one call, and by the EXACT launch shape bench.py times (bench.run_plan,
  bench.step_inputs: the driver's 20 steps, each the batch rotated by 7919 j
  boards, as ONE sdk_solve_batches launch on a full grid, two launches in
  flight, the XCD pool on the last), at N = 1 (20 x 2^20 boards) and for
  rank 7 of the 8-GPU run (20 x 2^17): every board of every step equal to
  the oracle's unique completion of the same global board
  (oracle_solve_unique_prop: 17-clue boards have one completion, which is
  therefore the walk's first, gen.py:6-28);
* a pool consumer that gives up waiting on a record (forced: zero polls)
  makes sdk_verify_workspace raise, and a flag the abandoned launch left set
  never leaks into the next launch on the same workspace (generation-tagged
  ready flags).
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 20


@pytest.fixture(scope="module")
def full_batch():
    """The bench's batch and the oracle's answers for it (~10-20 s of CPU)."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    p = hard17_batch(N, seed=2024)
    want, cnt = O.solve_unique_batch(p.numpy())
    assert (cnt == 1).all()
    return p, want


def test_full_size_vs_oracle(solver, full_batch):
    """One call over 2^20 hard 17-clue boards: every board the oracle's."""
    p, want = full_batch
    d = p.cuda()
    solver.stats(reset=True)
    sols, st = solver.solve(d)
    assert bool((st == 1).all())
    assert np.array_equal(sols.cpu().numpy(), want)
    assert bool((solver.check(sols, 0) == 1).all())
    v = solver.verify()
    assert v["assigned"] == v["finished"] == N and v["error"] == 0


def _timed_shape_vs_oracle(solver, full_batch, world, rank, steps=20):
    """bench.py's timed launch shape, verbatim (bench.run_plan / step_inputs,
    the calls bench.main makes): `steps` steps, step j = this rank's
    shard_bounds slice of the 2^20 batch rotated by 7919 j boards, one
    sdk_solve_batches launch over all of them (group = steps), two in
    flight, full grid, the pool on the last launch.  Every board of every
    step equal to the oracle's answer for the same global board, every
    status SOLVED, every board answered exactly once."""
    import bench
    from sudoku_solver_distributed_amd.distributed import shard_bounds
    p, want = full_batch
    lo, hi = shard_bounds(N, rank, world)
    shard = hi - lo
    plan = bench.run_plan(steps)
    assert plan == {"group": steps, "inflight": 2, "grid_waves": 0, "pool_last": 1}
    g = plan["group"]
    dev = torch.device("cuda", 0)
    inputs = bench.step_inputs(p, lo, hi, g, dev)
    nb = plan["inflight"] * g
    outs = [torch.full((shard, 81), 0xEE, dtype=torch.uint8, device=dev) for _ in range(nb)]
    sts = [torch.full((shard,), 77, dtype=torch.int32, device=dev) for _ in range(nb)]
    solver._slot_solvers(plan["inflight"])
    solver.inflight_stats(reset=True)
    solver.verify_inflight()
    solver.solve_inflight([inputs[i % g] for i in range(steps)], [outs[i % nb] for i in range(steps)],
                          [sts[i % nb] for i in range(steps)], inflight=plan["inflight"],
                          grid_waves=plan["grid_waves"], group=g, pool_last=plan["pool_last"])
    torch.cuda.synchronize()
    v = solver.verify_inflight()
    assert v["assigned"] == v["finished"] == steps * shard and v["error"] == 0
    assert solver.inflight_stats()["finished"] == steps * shard
    want_d = torch.from_numpy(want).to(dev)
    for i in range(steps):
        idx = (torch.arange(lo, hi, device=dev) + bench.ROTATION * (i % g)) % N
        assert bool((sts[i] == 1).all()), i
        assert torch.equal(outs[i], want_d[idx]), i
    # the bench's own check of the same buffers agrees
    ok = bench.check_steps(solver, inputs, [(outs[i], sts[i]) for i in range(nb)], steps, g, lo, N)
    assert all(ok.values()), ok
    for i in range(steps, nb):  # buffers no step wrote stay untouched
        assert bool((sts[i] == 77).all())


def test_bench_timed_shape_vs_oracle(solver, full_batch):
    """The driver's N = 1 command (--steps 20): 20 rotated copies of the 2^20
    batch, 21 M boards through ONE plane_kernel_multi launch, diffed board by
    board against the oracle (gen.py:6-28's first completion of each)."""
    _timed_shape_vs_oracle(solver, full_batch, world=1, rank=0)


def test_bench_rank_shape_vs_oracle(solver, full_batch):
    """One rank of the 8-GPU strong-scaling run: rank 7's 2^17-board shard
    of each of the 20 rotated steps in one launch, against the oracle."""
    _timed_shape_vs_oracle(solver, full_batch, world=8, rank=7)


_TIMEOUT_CHILD = r"""
import os, sys
os.environ["SDK_PLANE_TAIL_MODE"] = "2"     # the XCD pool (tail mode 1 is the default)
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
from sudoku_solver_distributed_amd.gen import hard17_batch
from sudoku_solver_distributed_amd.solver import BatchSolver, SudokuHipError
from oracle import oracle as O
s = BatchSolver("cuda:0")
p = hard17_batch(1 << 17, seed=31)
d = p.cuda()
os.environ["SDK_PLANE_POOL_POLLS"] = "0"    # every pool consumer gives up at once
sols, st = s.solve(d)
torch.cuda.synchronize()
try:
    s.verify()
    print("NO-RAISE")
    sys.exit(1)
except SudokuHipError as e:
    msg = str(e)
    assert "pool" in msg and "answered" in msg, msg
    print("RAISED", msg)
assert s.verify()["error"] == 0             # reported once, then re-synced
del os.environ["SDK_PLANE_POOL_POLLS"]     # the default bound again
sols, st = s.solve(d)                       # same workspace: stale flags must not read as set
torch.cuda.synchronize()
v = s.verify()
want, cnt = O.solve_unique_batch(p[:20000].numpy())
assert bool((st == 1).all()) and np.array_equal(sols[:20000].cpu().numpy(), want), "after recovery"
print("RECOVERED", v)
"""


def test_pool_wait_timeout_is_loud():
    """A pool consumer that gives up (SDK_PLANE_POOL_POLLS=0) leaves boards
    unanswered: sdk_verify_workspace raises, naming the pool; the next solve
    on the same workspace is exact again."""
    r = subprocess.run([sys.executable, "-u", "-c", _TIMEOUT_CHILD, ROOT], cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "RAISED" in r.stdout and "RECOVERED" in r.stdout
