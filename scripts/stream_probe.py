"""Is a launch on the default (null) stream slower than on a created one?
Back-to-back solves of one batch, timed on each, alternating.

    python scripts/stream_probe.py [BATCH] [STEPS]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
solver = get_solver(dev)
own = torch.cuda.Stream(dev)
for name, make in (("hard17", hard17_batch), ("hard_search", hard_search_batch)):
    boards = make(n, seed=2024, device=dev)
    out, st = torch.empty_like(boards), torch.empty(n, dtype=torch.int32, device=dev)
    for rep in range(3):
        for sname, s in (("default", None), ("created", own)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                solver.solve(boards, out=out, status=st, stream=s)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            print(f"{name} {sname:8s} {ms:.3f} ms/step {n / ms / 1e6:.3f} G boards/s", flush=True)
