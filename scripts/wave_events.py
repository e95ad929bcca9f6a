"""Wave-level event model of plane_kernel's lane loop (tooling, not product):
per-board pass outcome sequences from the host lane solver
(scripts/native/pass_trace.cpp), replayed on waves of 64 lanes with the
kernel's refill rule (refill once >= REFILL lanes are idle, from the wave's
own stream of boards; a wave drains when its share runs out).  Counts, per
wave iteration (one pass over the active lanes), how often the wave-wide
push path (some lane guesses) and pop path (some lane backtracks) run and
the mean active lanes -- the VALU the kernel issues beyond pass work.

    python scripts/wave_events.py [hard17|hard_search] [boards]
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MAXLEN = 2048


def traces(boards):
    so = "/tmp/libpass_trace.so"
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-o", so,
                           os.path.join(ROOT, "scripts", "native", "pass_trace.cpp")])
    lib = ctypes.CDLL(so)
    n = boards.shape[0]
    tr = np.zeros((n, MAXLEN), dtype=np.uint8)
    ln = np.zeros(n, dtype=np.uint32)
    vp = ctypes.c_void_p
    lib.pass_trace.argtypes = [vp, ctypes.c_int64, ctypes.c_int, vp, ctypes.c_int, vp]
    b = np.ascontiguousarray(boards, dtype=np.uint8)
    lib.pass_trace(b.ctypes.data, n, 0, tr.ctypes.data, MAXLEN, ln.ctypes.data)
    return tr, ln


def simulate(tr, ln, per_wave=256, refill=3, tail=8):
    n = len(ln)
    waves = n // per_wave
    it = push_it = pop_it = refill_ev = act_sum = lane_passes = tail_boards = 0
    for w in range(waves):
        q = list(range(w * per_wave, (w + 1) * per_wave))
        lane_b = [q.pop(0) for _ in range(64)]
        pos = [0] * 64
        while True:
            act = [i for i in range(64) if lane_b[i] is not None]
            if not q and len(act) <= tail:
                tail_boards += len(act)
                break
            if not act:
                break
            it += 1
            act_sum += len(act)
            pu = po = False
            for i in act:
                b = lane_b[i]
                r = tr[b, pos[i]]
                pos[i] += 1
                lane_passes += 1
                if r == 3:
                    pu = True
                elif r == 1:
                    po = True
                if pos[i] >= ln[b]:
                    lane_b[i] = None
            push_it += pu
            pop_it += po
            idle = [i for i in range(64) if lane_b[i] is None]
            if q and len(idle) >= refill:
                refill_ev += 1
                for i in idle:
                    if q:
                        lane_b[i] = q.pop(0)
                        pos[i] = 0
    return {"wave_iterations": it, "mean_active_lanes": act_sum / max(it, 1),
            "push_path_frac": push_it / max(it, 1), "pop_path_frac": pop_it / max(it, 1),
            "refills_per_iteration": refill_ev / max(it, 1), "tail_boards_per_wave": tail_boards / max(waves, 1),
            "passes_per_board": ln.mean(), "guesses_per_board": float((tr == 3).sum()) / n}


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "hard17"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 15
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    boards = (hard17_batch if kind == "hard17" else hard_search_batch)(n, seed=2024).numpy()
    tr, ln = traces(boards)
    r = simulate(tr, ln)
    # VALU per wave iteration (ISA counts): pass 1270, push path ~95, pop ~68
    it = r["wave_iterations"]
    pass_valu = it * 1270
    extra = it * (r["push_path_frac"] * 95 + r["pop_path_frac"] * 68)
    r["useful_lane_frac_of_pass_issue"] = r["mean_active_lanes"] / 64
    r["push_pop_valu_over_pass_valu"] = extra / pass_valu
    print(kind, {k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()})


if __name__ == "__main__":
    main()
