"""Would a heavy-first board order shorten the end of a launch?  (Tooling,
not product code)

    python scripts/order_sim.py [--boards 2621440] [--out profiles/r06/order_model.json]

1. Host model (scripts/native/root_features.cpp over plane_solver.h): per
   board of hard17_batch(2^16, seed=2024), the passes and branch nodes of the
   kernel's search (switch at 64), and features at the root fixpoint and
   after 1..4 passes.  Fits log(passes) on them (least squares): how much of
   a board's cost is predictable, and how early.
2. Event model of one plane_kernel launch (4096 waves of 64 lanes, 4 per
   SIMD sharing issue: 11.5 us per lane-loop iteration at four live waves,
   half that alone; a wave refills at 3 idle lanes; once the queue is empty
   a wave with <= 6 boards hands them to its XCD's pool, solved one at a time
   wave-wide at 0.8 us per pass), for an 8-GPU rank's 2.6 M boards, with the
   queue in random order (today), sorted by true cost, by the root-fixpoint
   predictor, by the root's open cells; and the only order a kernel could
   produce without solving every board twice: every board's root phase
   first (the boards the root solves end there), then the others' remaining
   passes (+1 to resume) in predicted-heavy-first buckets.
"""
import argparse
import ctypes
import heapq
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS, WPS, XCDS = 1024, 4, 8
T4, WIDE, TAIL, REFILL = 11.5, 0.8, 6, 3
T1 = T4 * 0.5


def features(n=1 << 16):
    so = "/tmp/libroot_features.so"
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-o", so,
                           os.path.join(ROOT, "scripts/native/root_features.cpp")])
    lib = ctypes.CDLL(so)
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd.gen import hard17_batch
    b = np.ascontiguousarray(hard17_batch(n, seed=2024).cpu().numpy(), dtype=np.uint8)
    out = np.zeros((len(b), 18), np.int32)
    lib.root_features(b.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(len(b)), ctypes.c_uint32(64),
                      out.ctypes.data_as(ctypes.c_void_p))
    return out


def fit(X, y):
    X = np.c_[np.ones(len(y)), X]
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    pred = X @ coef
    return pred, float(1 - ((y - pred) ** 2).sum() / ((y - y.mean()) ** 2).sum())


def launch_end(w):
    """Event model of one launch over work items w (passes each), in order."""
    nb = len(w)
    nw = SIMDS * WPS
    rem = np.zeros((nw, 64), np.int64)
    head = 0
    for i in range(nw):
        k = min(64, nb - head)
        rem[i, :k] = w[head:head + k]
        head += k
    simd_live = np.full(SIMDS, WPS)
    pool = [[] for _ in range(XCDS)]
    ev = [(0.0, i) for i in range(nw)]
    heapq.heapify(ev)
    t_end, t_empty = 0.0, None
    while ev:
        t, i = heapq.heappop(ev)
        s = i // WPS
        r = rem[i]
        act = r > 0
        na = int(act.sum())
        if 64 - na >= REFILL and head < nb:
            k = min(64 - na, nb - head)
            r[np.nonzero(~act)[0][:k]] = w[head:head + k]
            head += k
            act = r > 0
            na = int(act.sum())
            if head >= nb and t_empty is None:
                t_empty = t
        live = max(simd_live[s], 1)
        if head >= nb and na <= TAIL:
            if na:
                pool[s % XCDS].extend(r[act].tolist())
                r[:] = 0
            if pool[s % XCDS]:
                heapq.heappush(ev, (t + pool[s % XCDS].pop() * WIDE * max(1.0, live / 2.0), i))
                continue
            simd_live[s] -= 1
            t_end = max(t_end, t)
            continue
        r[act] -= 1
        heapq.heappush(ev, (t + max(T1, T4 * live / 4.0), i))
    return t_end, t_empty


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=2621440)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles/r06/order_model.json"))
    a = ap.parse_args()
    F = features()
    P, rp, U = F[:, 0].astype(np.int64), F[:, 2].astype(np.int64), F[:, 3]
    y = np.log(P)
    res = {"boards_modelled": len(P), "passes_mean": float(P.mean()),
           "passes_pct_50_90_99_999_max": np.percentile(P, [50, 90, 99, 99.9, 100]).round(1).tolist(),
           "root": {"passes_to_fixpoint_mean": float(rp.mean()), "solved_at_root_frac": float((U == 0).mean()),
                    "solved_at_root_passes_max": int(P[U == 0].max())}}
    pred_root, r2_root = fit(np.c_[F[:, 2:6], U >= 58], y)
    res["r2_log_passes"] = {"root_fixpoint": round(r2_root, 3)}
    for k in range(1, 5):
        res["r2_log_passes"][f"after_{k}_passes"] = round(fit(F[:, 6:6 + 3 * k], y)[1], 3)
    rng = np.random.default_rng(1)
    idx = rng.integers(0, len(P), a.boards)
    Pb, rpb, Ub, prb = P[idx], rp[idx], U[idx], pred_root[idx]
    ends = {}
    for name, key in [("random (today)", None), ("true cost, heaviest first", Pb), ("root predictor, heaviest first", prb),
                      ("root open cells, most first", Ub)]:
        w = Pb if key is None else Pb[np.argsort(-key, kind="stable")]
        ends[name] = launch_end(w)
        print(name, ends[name], flush=True)
    heavy = Ub > 0
    rest = (Pb - rpb + 1)[heavy]
    order = np.argsort(-prb[heavy], kind="stable")
    w = np.concatenate([np.where(heavy, rpb, Pb), rest[order]])
    ends["roots first, then the rest heaviest first"] = launch_end(w)
    print(ends, flush=True)
    base = ends["random (today)"][0]
    res["launch_end_us"] = {k: {"end": round(v[0], 1), "queue_empty": round(v[1], 1),
                                "vs_random": round(v[0] / base - 1, 4)} for k, v in ends.items()}
    res["model"] = {"waves": SIMDS * WPS, "us_per_iteration_4_waves": T4, "wide_us_per_pass": WIDE,
                    "tail": TAIL, "refill": REFILL, "boards": a.boards}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
