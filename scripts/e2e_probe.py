"""PCIe-inclusive solve (BatchSolver.solve_host) with different stream
layouts, after solve_inflight has created its slot streams (the bench's
order).  Which streams share a hardware queue decides whether the copies
overlap the kernel.

    python scripts/e2e_probe.py [BATCH]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
dev = torch.device("cuda", 0)
solver = get_solver(dev)
boards = hard17_batch(n, seed=2024, device=dev)
host = boards.cpu().pin_memory()
out_h = torch.empty_like(host).pin_memory()
st_h = torch.empty(n, dtype=torch.int32).pin_memory()


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


print("before slots: solve_host %.3f ms" % t(lambda: solver.solve_host(host, out=out_h, status=st_h)), flush=True)
outs = [torch.empty_like(boards) for _ in range(2)]
sts = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
solver.solve_inflight([boards] * 4, [outs[i % 2] for i in range(4)], [sts[i % 2] for i in range(4)])
torch.cuda.synchronize()
print("after slots: solve_host %.3f ms" % t(lambda: solver.solve_host(host, out=out_h, status=st_h)), flush=True)
print("all solved", bool((st_h == 1).all()))
