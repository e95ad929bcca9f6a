"""Status histogram of one 2^20-board solve (debugging aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
s = get_solver("cuda:0")
p = hard17_batch(n, seed=2024, device="cuda:0")
for rep in range(3):
    st = torch.full((n,), 77, dtype=torch.int32, device="cuda:0")
    sols, st = s.solve(p, status=st)
    torch.cuda.synchronize()
    v, c = torch.unique(st, return_counts=True)
    bad = torch.nonzero(st != 1).flatten()
    b = bad.cpu()
    print("rep", rep, dict(zip(v.tolist(), c.tolist())), "first bad", b[:6].tolist(),
          "bad<262144", int((b < 262144).sum()), "lane hist(mod 64) top", torch.bincount(b % 64, minlength=64).topk(4).indices.tolist(),
          "stats", s.stats(reset=True))
