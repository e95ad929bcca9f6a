import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from sudoku_solver_distributed_amd.solver import get_solver
from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY
s = get_solver()
root = torch.tensor([[int(c) for c in SEARCH_HEAVY]], dtype=torch.uint8)
nodes = s._dev(root)
for lvl in range(8):
    ch = s.expand(nodes, order="gen")
    eq = ch.shape[0] == nodes.shape[0] and torch.equal(ch, nodes)
    print(lvl, nodes.shape, nodes.device, "->", ch.shape, "equal", eq, flush=True)
    if lvl == 0:
        print("root ", "".join(map(str, nodes[0].cpu().tolist())))
        for r in ch.cpu().numpy(): print("child", "".join(map(str, r)))
    nodes = ch
print("frontier()", s.frontier(root, target=512, order="gen").shape)
print("frontier(cuda)", s.frontier(root.cuda(), target=512, order="gen").shape)
