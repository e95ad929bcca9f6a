"""Where a single-board solve's time goes: wall time of solver.solve(1 board)
+ synchronize (bench.py's p50_single_ms), the GPU span of the call between
HIP events, and the floor of one trivial launch + synchronize."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

s = get_solver("cuda:0")
boards = hard17_batch(256, seed=2024, device="cuda:0")
x = torch.zeros(1, device="cuda:0")
for _ in range(20):
    s.solve(boards[:1])
torch.cuda.synchronize()


def med(f, n=200):
    t = []
    for i in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f(i)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(t)


print("trivial launch + sync us", round(med(lambda i: x.add_(1)), 1))
print("solve(1 board) + sync us", round(med(lambda i: s.solve(boards[i % 256:i % 256 + 1])), 1))
out = torch.empty((1, 81), dtype=torch.uint8, device="cuda:0")
st = torch.empty(1, dtype=torch.int32, device="cuda:0")
print("solve(1, preallocated) + sync us", round(med(lambda i: s.solve(boards[i % 256:i % 256 + 1], out=out, status=st)), 1))
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g = []
for i in range(200):
    ev0.record()
    s.solve(boards[i % 256:i % 256 + 1], out=out, status=st)
    ev1.record()
    torch.cuda.synchronize()
    g.append(ev0.elapsed_time(ev1) * 1e3)
print("GPU span of one solve (events) us", round(statistics.median(g), 1))
