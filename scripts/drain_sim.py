"""Event model of plane_kernel's scheduling (not product code): which end-of-
batch policy is worth building?  Lanes are boards with a pass count drawn
from the host plane solver's per-board counts (tests/native/plane_host.cpp
plane_board_passes); a wave's iteration is one pass over its active lanes
plus, when SDK_PLANE_REFILL lanes are idle, a refill.  A SIMD shares its
issue among its live waves: a pass takes max(T1, T4 * w / 4) for w live waves
(T1, T4: plane::pass at 1 and 4 waves per SIMD, profiles/r03_mask_probe.json,
scaled to the kernel's measured time).

    python scripts/drain_sim.py [hard17|search] [policy ...]

policies: base (today: wide tail at <= 8), tail0, donate<D> (drained waves at
<= D active boards hand them to a live wave of their workgroup through LDS)."""
import ctypes
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 1 << 20
SIMDS = 1024
WPS = 4                      # waves per SIMD
# pass cycles at 4 live waves per SIMD: the stamped timeline's 14.8 k per loop
# iteration (profiles/r02_plane_timeline.txt); at 1 wave the mask probe's ratio
T4 = 14800.0
T1 = T4 * 5277.0 / 10680.0
CLK = 2.13e3                 # shader cycles per us (stamped cycles / wave lifetime)
CTRL = 2200.0                # loop control per iteration
IO_FIX, IO_PER, ST_PER = 3000.0, 960.0, 290.0  # refill: claim + span DMA, deposit per board, store per board
WIDE_PASS = 0.75 * CLK       # wave-wide tail: cycles per pass of one board
REFILL = 6


def pass_counts(kind):
    so = "/tmp/libplane_host_sim.so"
    if not os.path.exists(so):
        import subprocess
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-o", so,
                               os.path.join(ROOT, "tests/native/plane_host.cpp")])
    lib = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    lib.plane_board_passes.argtypes = [vp, ctypes.c_int64, ctypes.c_int, vp, vp]
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    b = (hard17_batch if kind == "hard17" else hard_search_batch)(1 << 15, seed=2024).cpu().numpy()
    b = np.ascontiguousarray(b, dtype=np.uint8).reshape(-1, 81)
    p = np.zeros(len(b), np.uint32)
    g = np.zeros(len(b), np.uint32)
    lib.plane_board_passes(b.ctypes.data, len(b), 0, p.ctypes.data, g.ctypes.data)
    return p.astype(np.int64)


def simulate(passes, policy):
    rng = np.random.default_rng(1)
    work = rng.choice(passes, N)
    tail = 8
    if "_t" in policy:
        policy, tail = policy.split("_t")
        tail = int(tail)
    donate = int(policy[6:]) if policy.startswith("donate") else (64 if policy == "fit" else -1)
    fit = policy == "fit"
    nw = SIMDS * WPS
    rem = np.zeros((nw, 64), np.int64)      # remaining passes per lane (0 idle)
    live = np.ones(nw, bool)
    simd_live = np.full(SIMDS, WPS)
    head = 0
    # static first hand-out: 64 boards per wave
    for w in range(nw):
        rem[w] = work[head:head + 64]
        head += 64
    mail = {}   # workgroup -> list of donated remaining-pass counts
    ev = [(0.0, w) for w in range(nw)]
    heapq.heapify(ev)
    issued = 0.0          # lane slots issued in lane passes
    useful = 0.0
    t_end = 0.0
    exits = []
    while ev:
        t, w = heapq.heappop(ev)
        s = w // WPS
        wg = (s // 4, w % WPS)   # CU, slot: the workgroup's 4 waves sit on the CU's 4 SIMDs
        r = rem[w]
        act = r > 0
        na = int(act.sum())
        dt = CTRL
        drained = head >= N
        if 64 - na >= REFILL or na == 0:
            k = 64 - na
            if not drained:
                kk = min(k, N - head)
                idle = np.nonzero(~act)[0][:kk]
                r[idle] = work[head:head + kk]
                head += kk
                dt += IO_FIX + (IO_PER + ST_PER) * kk
            elif donate >= 0 and mail.get(wg):
                box = mail[wg]
                kk = min(k, len(box))
                idle = np.nonzero(~act)[0][:kk]
                r[idle] = box[:kk]
                del box[:kk]
                dt += IO_FIX + 200.0 * kk
            act = r > 0
            na = int(act.sum())
        drained = head >= N
        gave = False
        if drained and donate >= 0 and 0 < na <= donate:
            cu = s // 4
            peer_waves = [(cu * 4 + i) * WPS + w % WPS for i in range(4)]
            others = [p for p in peer_waves if live[p] and p != w]
            room = sum(64 - int((rem[p] > 0).sum()) for p in others) - len(mail.get(wg, []))
            if others and (not fit or room >= na):
                mail.setdefault(wg, []).extend(r[act].tolist())
                r[:] = 0
                na = 0
                gave = True
                dt += 500.0
        if na and drained and na <= tail:
            # wave-wide tail: each board in turn
            dt += WIDE_PASS * float(r[r > 0].sum())
            r[:] = 0
            na = 0
        if gave or (na == 0 and drained and not (donate >= 0 and mail.get(wg))):
            live[w] = False
            simd_live[s] -= 1
            exits.append(t + dt)
            t_end = max(t_end, t + dt)
            continue
        if na:
            wl = max(simd_live[s], 1)
            dt += max(T1, T4 * wl / 4.0)
            issued += 64
            useful += na
            r[act] -= 1
        heapq.heappush(ev, (t + dt, w))
    return t_end / CLK, useful / max(issued, 1), np.percentile(np.array(exits) / CLK, [0, 50, 100])


if __name__ == "__main__":
    kind = sys.argv[1] if len(sys.argv) > 1 else "hard17"
    pols = sys.argv[2:] or ["base", "tail0", "donate16", "donate24", "donate32"]
    pc = pass_counts(kind)
    print(f"{kind}: mean passes {pc.mean():.2f}")
    for pol in pols:
        t, uf, ex = simulate(pc, pol)
        print(f"{pol:10s} end {t:7.1f} us  ({N / t / 1e3:.2f} G boards/s)  lane use {uf:.3f}  exits {ex.round(0).tolist()}")
