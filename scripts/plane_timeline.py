"""Per-wave timeline of one plane_kernel launch (diagnostic build with
SDK_PLANE_STAMPS=1, loaded with SDK_LIB=...libsudoku_hip_stamps.so).

    SDK_LIB=$PWD/sudoku_solver_distributed_amd/libsudoku_hip_stamps.so python scripts/plane_timeline.py [BATCH [hard_search]]

Prints, in microseconds from the first wave's start: when waves saw the
queue drained and when they exited (percentiles over waves), and the loop
iterations waves ran after the drain."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch  # noqa: E402
from sudoku_solver_distributed_amd.solver import get_solver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
solver = get_solver("cuda:0")
lib = solver.lib
make = hard_search_batch if (len(sys.argv) > 2 and sys.argv[2] == "hard_search") else hard17_batch
gw = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # waves per SIMD in the grid (0: full)
boards = make(n, seed=2024, device="cuda:0")
for _ in range(3):
    solver.solve(boards, grid_waves=gw)
torch.cuda.synchronize()
ws = solver.workspace
ws[24 * 8:30 * 8].zero_()
solver.stats(reset=True)
solver.solve(boards, grid_waves=gw)
torch.cuda.synchronize()
v = solver.verify()
print(f"boards answered {v['finished']} of {v['assigned']}")
pd = ws[24 * 8:30 * 8].view(torch.int64).cpu().numpy()
if pd[0] or pd[1]:
    print(f"tail pool: {pd[0]} claims, {pd[1]} failed claims, {pd[2]} flag polls; kcycles claiming {pd[3] / 1e3:.0f}, waiting {pd[4] / 1e3:.0f}, solving {pd[5] / 1e3:.0f}")
cap = 1 << 20
total = int(lib.sdk_workspace_bytes())
pool_bytes = 8 * (32 + 16384 * 37) * 4  # PLANE_POOL_BYTES (common.h, round 6 layout), after the deferred list
list_off = total - pool_bytes - cap * 8
waves = (min(n, 256 * 4 * 64 * (gw or 4))) // 64
st = ws[list_off + (cap // 2) * 8: list_off + (cap // 2) * 8 + waves * 256].view(torch.int64).cpu().numpy().reshape(-1, 32)
t0 = st[:, 0].min()
us = lambda x: (x - t0) / 100.0  # 100 MHz
q = [0, 10, 50, 90, 99, 100]
print(f"batch {n}, waves {waves}")
print("start   pct", q, np.percentile(us(st[:, 0]), q).round(1).tolist())
print("drained pct", q, np.percentile(us(st[:, 1]), q).round(1).tolist())
print("exit    pct", q, np.percentile(us(st[:, 2]), q).round(1).tolist())
print("iters after drain pct", q, np.percentile(st[:, 3], q).round(0).tolist())
ex = np.sort(us(st[:, 2]))
for frac in (0.25, 0.5, 0.75, 0.9, 0.99):
    print(f"  {frac:.0%} of waves exited by {ex[int(frac * (len(ex) - 1))]:.1f} us")
life = (st[:, 2] - st[:, 0]) / 100.0
cyc = st[:, 4] + st[:, 5] + st[:, 6]
print(f"wave lifetime us: mean {life.mean():.1f}; loop iterations: mean {st[:, 7].mean():.1f}")
for k, name in ((4, "pass"), (5, "store+refill+control"), (8, "  of which queue atomic"), (9, "  of which span DMA"),
                (10, "  of which deposit"), (11, "  of which store"),
                (6, "tail (wide / restart)")):
    print(f"  {name:22s} {st[:, k].sum() / cyc.sum():.3f} of stamped cycles, {st[:, k].mean() / 1e3:.1f} kcycles per wave")
loop_end = us(st[:, 12])
print("lane loop end pct", q, np.percentile(loop_end, q).round(1).tolist())
print("post-drain lane phase us pct", q, np.percentile(loop_end - us(st[:, 1]), q).round(1).tolist())
print("tail us pct", q, np.percentile(us(st[:, 2]) - loop_end, q).round(1).tolist())
print("tail boards pct", q, np.percentile(st[:, 13], q).round(1).tolist(), " tail passes pct",
      np.percentile(st[:, 14], q).round(1).tolist())
late = us(st[:, 2]) >= np.percentile(us(st[:, 2]), 90)
print(f"latest 10% of waves: drained at {us(st[late, 1]).mean():.1f} us (all: {us(st[:, 1]).mean():.1f}), "
      f"lane phase {(loop_end - us(st[:, 1]))[late].mean():.1f} us, tail {(us(st[:, 2]) - loop_end)[late].mean():.1f} us, "
      f"{st[late, 13].mean():.1f} boards / {st[late, 14].mean():.1f} passes")
claims, last = st[:, 15] & 0xFFFFFFFF, st[:, 15] >> 32
print(f"claims per wave mean {claims.mean():.1f}; last claim size: latest 10% {last[late].mean():.1f}, all {last.mean():.1f}")
ld = us(st[:, 1]) >= np.percentile(us(st[:, 1]), 90)
print(f"latest-drained 10% of waves: last claim size {last[ld].mean():.1f}, claims {claims[ld].mean():.1f}")
print(f"  stamped kcycles per wave {cyc.mean() / 1e3:.1f} (shader clock; lifetime {life.mean():.1f} us)")
piters, lanes = st[:, 16].sum(), st[:, 17].sum()
print(f"pass iterations {piters / len(st):.0f} per wave, active lanes per pass iteration {lanes / max(piters, 1):.1f} of 64; "
      f"search step {st[:, 18].sum() / max(st[:, 4].sum(), 1):.3f} of the pass+step cycles; iterations with a guess "
      f"{st[:, 19].sum() / max(piters, 1):.2f}, with a backtrack {st[:, 20].sum() / max(piters, 1):.2f}")
