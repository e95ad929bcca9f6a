"""Multi-GPU execution: one process per GPU (torchrun), RCCL over xGMI.

The reference spreads ONE board over its UDP peers cell by cell
(node.py:419-449 `solve_sudoku`: a `solve` message per empty cell, a
`solution` message back, node.py:384-406).  Here the unit of distribution is
re-designed around the GPU:

* **batches** -- boards are independent, so each rank solves a contiguous
  shard (`shard_bounds`) of the batch on its own GPU.  No data-path
  collective: weak scaling; an optional all-gather returns every result.
* **one hard board** -- the walk's search tree is cut into a frontier of
  subtrees that stays in walk order (`BatchSolver.frontier`, built
  identically on every rank).  Chunks of that frontier are dealt round-robin
  to ranks; each rank solves its chunk in ordered mode (the lowest solved
  index inside a chunk wins), then one all-reduce(MIN) of the lowest solved
  frontier index -- the early-exit word -- tells every rank whether a lower
  chunk can still hold the walk's answer.  The owner broadcasts the grid.

Backends are pluggable (`GpuBackend` by default) so the orchestration is
exercised on CPU with gloo in the test-suite; the product path always uses
the HIP kernels.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from .solver import SDK_SOLVED, as_boards, get_solver

NONE = 1 << 62  # "no board solved yet" in the early-exit word


def rank_world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of n items for `rank` of `world`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _comm_device() -> torch.device:
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class GpuBackend:
    """The product backend: the HIP kernels of this rank's GPU."""

    def __init__(self, device=None):
        self.solver = get_solver(device)

    def frontier(self, board: torch.Tensor, target: int, order: str) -> torch.Tensor:
        return self.solver.frontier(board, target=target, order=order)

    def solve(self, boards: torch.Tensor, order: str, ordered: bool):
        return self.solver.solve(boards, order=order, ordered=ordered)


def solve_shard(boards, order: str = "gen", backend=None, gather: bool = False):
    """Solve this rank's shard of `boards` (every rank passes the same batch,
    or a generator that builds it).  Returns ((lo, hi), solutions, status);
    with gather=True, every rank gets the full (solutions, status)."""
    rank, world = rank_world()
    be = backend or GpuBackend()
    b = as_boards(boards)
    lo, hi = shard_bounds(b.shape[0], rank, world)
    sols, st = be.solve(b[lo:hi], order, False)
    if not gather or world == 1:
        return (lo, hi), sols, st
    dev = _comm_device()
    counts = [shard_bounds(b.shape[0], r, world) for r in range(world)]
    m = max(h - l for l, h in counts)
    pad_s = torch.zeros((m, 81), dtype=torch.uint8, device=dev)
    pad_t = torch.full((m,), -9, dtype=torch.int32, device=dev)
    pad_s[: hi - lo] = sols.to(dev)
    pad_t[: hi - lo] = st.to(dev)
    all_s = [torch.empty_like(pad_s) for _ in range(world)]
    all_t = [torch.empty_like(pad_t) for _ in range(world)]
    dist.all_gather(all_s, pad_s)
    dist.all_gather(all_t, pad_t)
    sols_full = torch.cat([s[: h - l] for s, (l, h) in zip(all_s, counts)])
    st_full = torch.cat([t[: h - l] for t, (l, h) in zip(all_t, counts)])
    return (0, b.shape[0]), sols_full, st_full


def solve_split(board, order: str = "gen", target: Optional[int] = None, chunk: Optional[int] = None,
                backend=None, stats: Optional[dict] = None) -> Tuple[bool, torch.Tensor]:
    """One board, split over every rank's GPU.  Returns (solved, grid81) on
    every rank -- bit-identical to the walk `order` on that board."""
    rank, world = rank_world()
    be = backend or GpuBackend()
    root = as_boards(board)
    if root.shape[0] != 1:
        raise ValueError("solve_split takes exactly one board")
    nodes = be.frontier(root, target or 4096 * world, order)
    k = nodes.shape[0]
    if k == 0:
        return False, root[0].clone()
    chunk = chunk or max(1, math.ceil(k / (world * 4)))
    nchunks = math.ceil(k / chunk)
    best = NONE
    mine = None
    rounds = 0
    dev = _comm_device() if world > 1 else torch.device("cpu")
    while True:
        j = rounds * world + rank
        local = NONE
        if j < nchunks and j * chunk < best:
            lo, hi = j * chunk, min(k, (j + 1) * chunk)
            sols, st = be.solve(nodes[lo:hi], order, True)
            hit = torch.nonzero(st == SDK_SOLVED)
            if hit.numel():
                i = int(hit[0, 0].item())
                local = lo + i
                mine = (local, sols[i].clone())
        rounds += 1
        if world > 1:
            w = torch.tensor([local], dtype=torch.int64, device=dev)
            dist.all_reduce(w, op=dist.ReduceOp.MIN)  # the early-exit word
            local = int(w.item())
        best = min(best, local)
        # every chunk below rounds*world has been handled: stop once the best
        # solved index lies below that line, or nothing is left
        if best < rounds * world * chunk or rounds * world >= nchunks:
            break
    if stats is not None:
        stats.update({"frontier": k, "chunk": chunk, "rounds": rounds, "best": best})
    if best == NONE:
        return False, root[0].clone()
    owner = (best // chunk) % world
    if world == 1:
        return True, mine[1]
    grid = torch.zeros(81, dtype=torch.uint8, device=dev)
    if rank == owner:
        assert mine is not None and mine[0] == best
        grid.copy_(mine[1].to(dev))
    dist.broadcast(grid, src=owner)
    return True, grid
