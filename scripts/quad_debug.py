"""Diagnostic (not product): the four-board tail solver (tail mode 3) on the
pool-heavy setting of test_plane_tail_paths, checked against the oracle;
prints the stall diagnostics the kernel leaves in the workspace."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from sudoku_solver_distributed_amd import _lib  # noqa: E402
from sudoku_solver_distributed_amd.gen import generate_batch, hard17_batch, hard_search_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import SudokuHipError, get_solver  # noqa: E402

tail, mode = int(sys.argv[1]), int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
s = get_solver("cuda:0")
lib = s.lib
lib.sdk_set_solve_kernel(_lib.SDK_KERNELS["plane"])
assert lib.sdk_set_plane_tuning(-1, tail, mode, -1) == 0
hs = np.concatenate([hard_search_batch(n * 3 // 4, seed=31).numpy(), hard17_batch(n // 4, seed=32).numpy()])
want, cnt = O.solve_unique_batch(hs)
for order in ("gen", "node"):
    s.stats(reset=True)
    t = time.time()
    sols, st = s.solve(torch.from_numpy(hs), order=order)
    torch.cuda.synchronize()
    el = time.time() - t
    try:
        v = s.verify()
    except SudokuHipError as e:
        v = str(e)
    diag = s.workspace[16 * 8:24 * 8].view(torch.int64).cpu().numpy()
    ok = bool((st == 1).all()) and np.array_equal(sols.cpu().numpy(), want)
    print(order, "tail", tail, "mode", mode, "ok", ok, "s", round(el, 3), v, [hex(int(x)) for x in diag], flush=True)
    if not ok:
        bad = np.nonzero((sols.cpu().numpy() != want).any(1) | (st.cpu().numpy() != 1))[0]
        print("bad boards", len(bad), bad[:10], st.cpu().numpy()[bad[:10]], flush=True)

gen = generate_batch(n, 50, seed=33).cpu().numpy()
gen[:16] = 0  # empty boards: deeper than the stack in gen order
for order in ("gen", "node"):
    s.stats(reset=True)
    sols, st = s.solve(torch.from_numpy(gen), order=order)
    torch.cuda.synchronize()
    try:
        v = s.verify()
    except SudokuHipError as e:
        v = str(e)
    want, wst = O.solve_batch(gen, order=order)
    print("generated", order, "ok", np.array_equal(st.cpu().numpy(), wst) and np.array_equal(sols.cpu().numpy(), want),
          v, flush=True)
