"""PCIe-inclusive rate of BatchSolver.solve_host by chunk size (pinned host
boards in and out, 2^20 hard boards), next to the serial copy-solve-copy."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

s = get_solver("cuda:0")
host = hard17_batch(1 << 20, seed=2024).pin_memory()
out = torch.empty_like(host).pin_memory()
st = torch.empty(host.shape[0], dtype=torch.int32).pin_memory()
want, _ = s.solve(host.to("cuda:0"))
want = want.cpu()
for chunk in (1 << 20, 1 << 19, 1 << 18, 1 << 17, 1 << 16):
    best = 1e9
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.solve_host(host, chunk=chunk, out=out, status=st)
        best = min(best, time.perf_counter() - t0)
    ok = torch.equal(out, want) and bool((st == 1).all())
    print(f"chunk {chunk:8d}: {best * 1e3:.3f} ms  {host.shape[0] / best / 1e6:.1f} M boards/s  identical={ok}", flush=True)
