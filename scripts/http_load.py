"""HTTP load generator for node.py peers (BASELINE.json configs[4]): POST
/solve with 17-clue boards from `procs` worker processes x `clients` threads
each, spread round-robin over the peers' URLs.  Runs in its own process(es),
so the peers under test share nothing with it (bench.py node_load_procs).

    python scripts/http_load.py URL [URL ...] [--requests N] [--clients C] [--procs P]

Prints one JSON line: requests/s over the timed requests (after a warm-up of
64), p50 / p99 latency, and whether every answer is a valid completion that
keeps the board's givens.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time
import urllib.request
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _valid(board, sol) -> bool:
    flat = [v for row in sol for v in row]
    if len(flat) != 81 or any(b and b != s for b, s in zip(board, flat)):
        return False
    units = [[9 * r + c for c in range(9)] for r in range(9)] + [[9 * r + c for r in range(9)] for c in range(9)]
    units += [[9 * (3 * (b // 3) + i) + 3 * (b % 3) + j for i in range(3) for j in range(3)] for b in range(9)]
    return all(sorted(flat[i] for i in u) == list(range(1, 10)) for u in units)


def _worker(args):
    urls, boards, clients, start_evt, ready_q, res_q = args
    bodies = [json.dumps({"sudoku": [b[9 * r:9 * r + 9] for r in range(9)]}).encode() for b in boards]

    def one(i):
        t0 = time.perf_counter()
        req = urllib.request.Request(urls[i % len(urls)], data=bodies[i], headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=120) as r:
            sol = json.loads(r.read())
        return time.perf_counter() - t0, _valid(boards[i], sol)

    with ThreadPoolExecutor(max_workers=clients) as ex:
        list(ex.map(one, range(min(16, len(boards)))))  # warm-up (connections, first batches)
        ready_q.put(1)
        start_evt.wait()
        t0 = time.perf_counter()
        res = list(ex.map(one, range(len(boards))))
        t1 = time.perf_counter()
    res_q.put((t0, t1, [r[0] for r in res], all(r[1] for r in res)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("urls", nargs="+")
    ap.add_argument("--requests", type=int, default=2000)
    ap.add_argument("--clients", type=int, default=64, help="client threads in all")
    ap.add_argument("--procs", type=int, default=4, help="load-generator processes")
    ap.add_argument("--seed", type=int, default=77)
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd.gen import hard17_batch
    boards = [list(map(int, b)) for b in hard17_batch(args.requests, seed=args.seed).numpy()]
    ctx = mp.get_context("spawn")
    start_evt, ready_q, res_q = ctx.Event(), ctx.Queue(), ctx.Queue()
    per = [boards[i::args.procs] for i in range(args.procs)]
    procs = [ctx.Process(target=_worker, args=((args.urls, p, max(1, args.clients // args.procs), start_evt, ready_q,
                                            res_q),))
             for p in per]
    for p in procs:
        p.start()
    for _ in procs:
        ready_q.get(timeout=300)  # every worker warmed up
    start_evt.set()
    out = [res_q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join()
    t0, t1 = min(o[0] for o in out), max(o[1] for o in out)
    lat = sorted(x for o in out for x in o[2])
    print(json.dumps({"requests": args.requests, "clients": args.clients, "load_procs": args.procs,
                      "requests_per_s": args.requests / (t1 - t0), "p50_ms": lat[len(lat) // 2] * 1e3,
                      "p99_ms": lat[int(len(lat) * 0.99)] * 1e3, "all_valid": all(o[3] for o in out)}), flush=True)


if __name__ == "__main__":
    main()
