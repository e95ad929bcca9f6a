"""Diagnostic: solve unique-solution boards several ways and classify every
board whose answer differs from its unique completion (oracle), to locate a
tail-pool handoff bug: another board's answer (id mix-up), an invalid grid
(stale planes), a valid grid other than the unique one (impossible for sound
search), or a wrong status."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import oracle as O  # noqa: E402
from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

solver = get_solver("cuda:0")
big = torch.cat([hard17_batch(200_000, seed=7), hard_search_batch(30_000, seed=8)])
want, cnt = O.solve_unique_batch(big.numpy())
assert (cnt == 1).all()
index = {w.tobytes(): i for i, w in enumerate(want)}


def valid(g):
    g = g.reshape(9, 9)
    ok = all(sorted(g[r]) == list(range(1, 10)) for r in range(9))
    ok = ok and all(sorted(g[:, c]) == list(range(1, 10)) for c in range(9))
    return ok and all(sorted(g[3 * (b // 3):3 * (b // 3) + 3, 3 * (b % 3):3 * (b % 3) + 3].ravel()) == list(range(1, 10))
                      for b in range(9))


def classify(tag, sols, st, lo=0):
    sols, st = sols.cpu().numpy(), st.cpu().numpy()
    bad = np.nonzero((sols != want[lo:lo + len(sols)]).any(1) | (st != 1))[0]
    kinds = {}
    for i in bad[:2000]:
        g = sols[i]
        j = index.get(g.tobytes())
        if st[i] != 1:
            k = f"status {st[i]}"
        elif j is not None:
            k = "another board's answer"
        elif not valid(g):
            k = "invalid grid" + ("" if ((big[lo + i].numpy() == 0) | (g == big[lo + i].numpy())).all() else ", givens changed")
        else:
            k = "a different valid grid"
        kinds[k] = kinds.get(k, 0) + 1
    print(f"{tag}: {len(bad)} wrong of {len(sols)} {kinds}", flush=True)


p = big.cuda()
for order in ("node", "gen"):
    for gw in (0, 1, 2):
        for rep in range(int(os.environ.get("REPS", "2"))):
            s, t = solver.solve(p, order=order, grid_waves=gw)
            torch.cuda.synchronize()
            classify(f"solve {order} grid {gw} #{rep}", s, t)
    sizes = [1, 63, 65, 8191, 13, 20_011, 3, 40_000, 127, 1, 12_345, 77, 30_001, 5, 64, 50_000]
    offs = np.cumsum([0] + sizes)
    bs = [p[offs[i]:offs[i + 1]] for i in range(16)]
    outs = [torch.empty_like(b) for b in bs]
    sts = [torch.empty(b.shape[0], dtype=torch.int32, device=b.device) for b in bs]
    for gw in (1, 2):
        for rep in range(int(os.environ.get("REPS", "2"))):
            solver.solve_batches(bs, outs, sts, order=order, grid_waves=gw)
            torch.cuda.synchronize()
            classify(f"batches {order} grid {gw} #{rep}", torch.cat(outs), torch.cat(sts))
