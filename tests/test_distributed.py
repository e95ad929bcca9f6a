"""Multi-rank orchestration: world_size 2 over gloo.

CPU tests: the per-rank compute is the oracle (test-side backend).  The GPU
test runs the product backend (GpuBackend, HIP kernels) in both ranks, both
on cuda:0, through the same orchestration code
(sudoku_solver_distributed_amd/distributed.py); RCCL replaces gloo on a
multi-GPU node (bench.py --gpus N under torchrun).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WALK = {"gen": [r * 9 + c for r in range(8, -1, -1) for c in range(9)], "node": list(range(81))}


class OracleBackend:
    """Frontier without propagation (plain walk levels) + the literal walk."""

    def frontier(self, board, target, order):
        nodes = [board[0].numpy().copy()]
        for _ in range(81):
            if len(nodes) >= target:
                break
            nxt = []
            grew = False
            for g in nodes:
                empties = [c for c in WALK[order] if g[c] == 0]
                if not empties:
                    nxt.append(g)
                    continue
                cell = empties[0]
                r, c = divmod(cell, 9)
                for d in range(1, 10):
                    if O.is_valid(g, r, c, d):
                        ch = g.copy()
                        ch[cell] = d
                        nxt.append(ch)
                grew = True
            nodes = nxt
            if not grew or not nodes:
                break
        return torch.from_numpy(np.array(nodes, dtype=np.uint8).reshape(-1, 81))

    def solve(self, boards, order, ordered):
        sols, st = O.solve_batch(boards.numpy(), order=order)
        return torch.from_numpy(sols), torch.from_numpy(st)


def _batch(board, order):
    """5 boards: the board, its solution (no empty cell), an empty board..."""
    batch = np.array([board] * 5, dtype=np.uint8)
    batch[1:] = O.solve_batch(np.array([board], dtype=np.uint8), order=order)[0][0]
    batch[3] = 0
    return batch


def _worker(rank, world, port, board, order, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sudoku_solver_distributed_amd.distributed import solve_shard, solve_split
        be = OracleBackend()
        st = {}
        ok, grid = solve_split(torch.tensor([board], dtype=torch.uint8), order=order, target=64, chunk=3,
                               backend=be, stats=st)
        batch = torch.from_numpy(_batch(board, order))
        (lo, hi), sols, sts = solve_shard(batch, order=order, backend=be, gather=True)
        results[rank] = (ok, grid.numpy().tolist(), st, (lo, hi), sols.numpy().tolist(), sts.numpy().tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("order", ["gen", "node"])
def test_two_rank_split_and_shards(order):
    import json
    from conftest import load_golden
    # a generated board with many empty cells (several completions)
    case = [c for c in load_golden("golden_gen.json") if c["empty_boxes"] == 58][0]
    board = [int(x) for x in case["puzzle"]]
    want, wst = O.solve_batch(np.array([board], dtype=np.uint8), order=order)
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), board, order, results), nprocs=2, join=True)
    for r in range(2):
        ok, grid, st, (lo, hi), sols, sts = results[r]
        assert ok and wst[0] == 1
        assert grid == want[0].tolist(), (r, st)
        assert st["frontier"] > 2 and st["rounds"] >= 1
        # gathered shard results equal the oracle on the whole batch
        wb, wbs = O.solve_batch(_batch(board, order), order=order)
        assert (lo, hi) == (0, 5)
        assert sols == wb.tolist() and sts == wbs.tolist()


def test_shard_bounds():
    from sudoku_solver_distributed_amd.distributed import shard_bounds
    for n in (0, 1, 7, 8, 1 << 20):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def _gpu_worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from sudoku_solver_distributed_amd.distributed import GpuBackend, solve_shard, solve_split
        from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY, hard17_batch
        be = GpuBackend("cuda:0")
        batch = hard17_batch(1 << 16, seed=31)
        (lo, hi), sols, sts = solve_shard(batch, order="gen", backend=be, gather=True)
        out = {"span": (lo, hi), "sols": sols.cpu().numpy(), "st": sts.cpu().numpy(), "split": {}}
        board = torch.tensor([[int(c) for c in SEARCH_HEAVY]], dtype=torch.uint8)
        for order in ("gen", "node"):
            st = {}
            ok, grid = solve_split(board, order=order, target=512, chunk=16, backend=be, stats=st)
            out["split"][order] = (ok, grid.cpu().numpy(), st)
        results[rank] = out
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_gpu_backend():
    """solve_shard (gather) on 2^16 hard boards and solve_split on a
    search-heavy board, both ranks on the HIP backend: every rank ends with
    the oracle's answers (unique completions = the walk's, gen.py:6-28)."""
    from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY, hard17_batch
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_gpu_worker, args=(2, _free_port(), results), nprocs=2, join=True)
    want, cnt = O.solve_unique_batch(hard17_batch(1 << 16, seed=31).numpy())
    assert (cnt == 1).all()
    hw, hc = O.solve_unique_batch(np.array([[int(c) for c in SEARCH_HEAVY]], dtype=np.uint8))
    for r in range(2):
        res = results[r]
        assert res["span"] == (0, 1 << 16)
        assert (res["st"] == 1).all() and np.array_equal(res["sols"], want)
        for order in ("gen", "node"):
            ok, grid, st = res["split"][order]
            assert ok and np.array_equal(grid, hw[0]), (r, order, st)
            assert st["frontier"] > 16, st
