"""Two launches in flight per GPU (each on its own stream and workspace):
how much of a launch's end-of-batch drain does the next launch's start fill?

    python scripts/overlap_probe.py [BATCH] [STEPS]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import BatchSolver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
boards = hard17_batch(n, seed=2024, device=dev)
solvers = [BatchSolver(dev), BatchSolver(dev)]
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
outs = [torch.empty_like(boards) for _ in range(2)]
sts = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]


def run(m):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        k = i % m
        solvers[k].solve(boards, out=outs[k], status=sts[k], stream=streams[k])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


for m in (1, 2, 1, 2):
    run(m)
    ms = run(m) * 1e3
    ok = all(bool((sts[k] == 1).all()) for k in range(m))
    print(f"in flight {m}: {ms:.3f} ms/step, {n / ms / 1e6:.3f} G boards/s, all solved {ok}", flush=True)
print("outputs identical:", bool(torch.equal(outs[0], outs[1])))

# the same through BatchSolver.solve_inflight (the bench's path)
solver = solvers[0]
solver._slots = [(solvers[0], streams[0]), (solvers[1], streams[1])]


def run_api(m):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    solver.solve_inflight([boards] * steps, [outs[i % m] for i in range(steps)], [sts[i % m] for i in range(steps)],
                          inflight=m)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


for m in (1, 2, 1, 2):
    run_api(m)
    ms = run_api(m) * 1e3
    print(f"solve_inflight {m}: {ms:.3f} ms/step, {n / ms / 1e6:.3f} G boards/s", flush=True)


def run_bench_like(m, stats=False, events=False):
    if stats:
        solver.inflight_stats(reset=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if events:
        e0.record(torch.cuda.current_stream())
    solver.solve_inflight([boards] * steps, [outs[i % m] for i in range(steps)], [sts[i % m] for i in range(steps)],
                          inflight=m)
    if events:
        e1.record(torch.cuda.current_stream())
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


for kw in ({}, {"stats": True}, {"events": True}, {"stats": True, "events": True}, {}):
    ms = run_bench_like(2, **kw) * 1e3
    print(f"bench-like {kw}: {ms:.3f} ms/step, {n / ms / 1e6:.3f} G boards/s", flush=True)
    ms = run_bench_like(2, **kw) * 1e3
    print(f"bench-like {kw} again: {ms:.3f} ms/step, {n / ms / 1e6:.3f} G boards/s", flush=True)
