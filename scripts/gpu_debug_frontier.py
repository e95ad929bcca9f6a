import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from sudoku_solver_distributed_amd.solver import get_solver
from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY, hard17_batch
s = get_solver()
root = torch.tensor([[int(c) for c in SEARCH_HEAVY]], dtype=torch.uint8)
for order in ("gen", "node"):
    nodes = root.cuda()
    for lvl in range(6):
        ch = s.expand(nodes, order=order)
        print(order, lvl, "in", nodes.shape[0], "out", ch.shape[0], flush=True)
        for r in ch[:3].cpu().numpy():
            print("   ", "".join(map(str, r)), int((r == 0).sum()))
        if ch.shape[0] == 0:
            break
        nodes = ch
sol, st = s.solve(root, order="gen"); print("direct", st.tolist(), "".join(map(str, sol[0].cpu().tolist())), s.stats(reset=True))
