"""Tiny GPU sanity pass: a few boards per order, compared with the oracle."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle as O
from sudoku_solver_distributed_amd.solver import get_solver
from sudoku_solver_distributed_amd.gen import hard17_batch, SEEDS_17
s = get_solver()
easy = np.array([[int(c) for c in "000000050000500000008206400040900600980610000071800035507040308802305040000709060"]], dtype=np.uint8)
for order in ("gen", "node"):
    t = time.time()
    sol, st = s.solve(torch.from_numpy(easy), order=order); torch.cuda.synchronize()
    want, wst = O.solve_batch(easy, order=order)
    print(order, "easy", st.cpu().tolist(), np.array_equal(sol.cpu().numpy(), want), f"{time.time()-t:.3f}s", flush=True)
h = hard17_batch(8, seed=1)
for order in ("gen", "node"):
    t = time.time()
    sol, st = s.solve(h, order=order); torch.cuda.synchronize()
    want, cnt = O.solve_unique_batch(h.numpy())
    print(order, "hard8", st.cpu().tolist(), np.array_equal(sol.cpu().numpy(), want), f"{time.time()-t:.3f}s", s.stats(reset=True), flush=True)
