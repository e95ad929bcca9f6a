"""Headline benchmark: hard 17-clue 9x9 boards solved per second (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

One process per GPU (torchrun for N > 1, RCCL for the barrier / max-time
reduction only: boards are independent, each rank solves its own shard, no
data-path collective).  A step = the hot path over one batch of B boards
(default 2^20 = BASELINE.json's "1M hard 17-clue" batch) already resident in
HBM.  --scaling strong (the default; BASELINE configs[2]: "1M ... sharded
across 1/2/4/8 MI355X"): B boards per step over ALL ranks, rank r solving
its shard_bounds share (B/N boards) of every step's batch; weak: B boards per
GPU per step.  Launch plan "run" (the default): a rank's K timed steps are
ceil(K / 32) sdk_solve_batches launches -- one queue over up to 32 steps'
batches that drains once, on a full grid, the next launch queued behind the
running one -- each step keeping its own input (the batch rotated by 7919 j
boards for step j) and output buffers.  value = all ranks' boards /
max-over-ranks wall time.  Beside it, labelled: `serial` = the same K steps
as K one-step launches back to back, `single_batch` = one step's batch in
one solve() call (the "1M batch" alone), `output_checks` = every timed
step's output checked (SOLVED, Sudoku.check, givens kept, equal across the
rotated steps).

Rank 0 prints ONE JSON line with the contract fields plus:
  roofline     -- the solve kernel against the INT32 VALU roofline (VALU
                  instructions per launch from the committed rocprofv3 PMC
                  profile of this exact workload, over kernel_ms = the
                  timed GPU region per launch, HIP events; launch_ms = a
                  launch's own start-to-end span, overlapped with its
                  neighbours, which rocprofv3's kernel trace reports) and,
                  as `hbm`, its algorithmic bytes per launch against HBM;
  cpu_baseline -- the oracle's literal reference walk (gen.py:6-28 restated in
                  C, oracle/) on a time-bounded sample of the same boards, one
                  walk per host core (affinity, capped by $OMP_NUM_THREADS),
                  rank 0 at N = 1 only;
  p50_single_ms -- single-board latency (one board per launch, frontier
                  split off), median over the first boards of the batch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# hardware queues per process (HIP's default is 4), read when HIP starts:
# each launch in flight has its own stream, and streams past the queues
# share one and serialise (six launches in flight need 8)
if not os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() or int(os.environ["GPU_MAX_HW_QUEUES"]) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"  # (the GPU boxes export HIP's default, 4)

PEAK_VALU_OPS = 256 * 4 * 32 * 2.4e9   # lane-ops/s: 256 CU x 4 SIMD32 x 2.4 GHz
PEAK_HBM = 8.0e12                       # B/s (MI355X_MICROARCH.md)
BYTES_PER_BOARD = 81 + 81 + 4           # board in, board out, status
PMC_DIR = os.path.join(ROOT, "profiles")   # pmc_<kernel symbol>.json (scripts/gpu_pmc.sh)


def cpu_baseline(boards, budget_s: float):
    """Literal reference walk (gen.py:6-28 restated in C, oracle/) on every
    host core this process may use, one walk per core over its own slice of
    the sample; boards completed within the budget."""
    from oracle import oracle as O  # checker only: bench's cpu_baseline leg
    threads = O.host_threads()
    t0 = time.perf_counter()
    done = O.solve_batch_timed_parallel(boards, budget_s, threads)
    return done, time.perf_counter() - t0, threads


ROTATION = 7919  # step j's batch is the synthetic batch rotated by ROTATION * j boards


def run_plan(steps: int) -> dict:
    """Launch plan "run" (the default) for `steps` timed steps: ceil(K / 32)
    sdk_solve_batches launches of equal step counts on full grids, the
    running launch and the next one queued behind it (two in flight), the
    last launch sharing its tail through the XCD pool.  tests/test_gpu_full_size.py
    diffs exactly this shape against the oracle."""
    from sudoku_solver_distributed_amd._lib import SDK_MAX_BATCHES
    n_launch = -(-steps // SDK_MAX_BATCHES)
    return {"group": -(-steps // n_launch), "inflight": 2, "grid_waves": 0, "pool_last": 1}


def step_inputs(full, lo: int, hi: int, group: int, dev):
    """One input per step of a launch group: step j's boards are this rank's
    [lo, hi) of the batch rotated by ROTATION * j boards."""
    import torch
    n = full.shape[0]
    return [full[(torch.arange(lo, hi) + ROTATION * j) % n].contiguous().to(dev) for j in range(group)]


def check_steps(solver, inputs, bufs, steps, group, lo, batch):
    """Every buffer the timed steps wrote, against the reference's contract
    (gen.py:6-28's first completion of every board): every board SOLVED and
    passing Sudoku.check (sudoku.py:119-140), the givens kept, and -- step j
    being the batch rotated by 7919 j boards -- board for board equal to the
    answer another step gave the same global board (buffer b holds the last
    step i < steps with i % len(bufs) == b)."""
    import torch
    nb = len(bufs)
    shard = inputs[0].shape[0]
    held = [max(i for i in range(steps) if i % nb == b) for b in range(min(nb, steps))]
    ok = {"solved": True, "checked": True, "givens_kept": True, "rotations_agree": True}
    ref_b = 0
    j_ref = held[ref_b] % group
    ar = torch.arange(shard, device=inputs[0].device)
    for b, i in enumerate(held):
        out, st = bufs[b]
        inp = inputs[i % group]
        ok["solved"] &= bool((st == 1).all())
        ok["checked"] &= bool((solver.check(out, 0) == 1).all())
        ok["givens_kept"] &= bool(((inp == 0) | (out == inp)).all())
        # position k of step i is global board (lo + k + 7919 j) % batch; in
        # the reference buffer it sits at (global - lo - 7919 j_ref) % batch
        j = i % group
        g = (lo + ar + ROTATION * j) % batch
        k_ref = (g - lo - ROTATION * j_ref) % batch
        sel = k_ref < shard
        ok["rotations_agree"] &= bool(torch.equal(out[sel], bufs[ref_b][0][k_ref[sel]]))
    return ok


def _time(fn, reps=3):
    import torch
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return best, out


def node_load(dev, requests: int = 2000, clients: int = 32, peers: int = 1, solvers: int = 1):
    """BASELINE.json configs[4] serving figure: `peers` in-process peers
    (node.py mirror; each a GpuSolverBackend with `solvers` solvers on this
    GPU -- the shape of "2 MI355X per peer" on one device) connected through
    the first one, answering concurrent HTTP POST /solve from `clients`
    client threads spread over their ports; requests/s and latency."""
    import urllib.request
    from concurrent.futures import ThreadPoolExecutor

    from sudoku_solver_distributed_amd.gen import hard17_batch
    from sudoku_solver_distributed_amd.node import GpuSolverBackend, P2PNode, make_http_server
    nodes, servers, urls = [], [], []
    for i in range(peers):
        node = P2PNode("127.0.0.1", 0, anchor_node=nodes[0].id if nodes else None, handicap=0,
                       backend=GpuSolverBackend([dev.index] * solvers))
        node.bind()
        httpd = make_http_server(node, "127.0.0.1", 0)
        threading.Thread(target=httpd.serve_forever, daemon=True).start()
        threading.Thread(target=node.run, daemon=True).start()
        nodes.append(node)
        servers.append(httpd)
        urls.append(f"http://127.0.0.1:{httpd.server_address[1]}/solve")
    boards = hard17_batch(requests, seed=77).numpy()
    bodies = [json.dumps({"sudoku": b.reshape(9, 9).tolist()}).encode() for b in boards]

    def one(i):
        t0 = time.perf_counter()
        req = urllib.request.Request(urls[i % peers], data=bodies[i], headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=60) as r:
            sol = json.loads(r.read())
        return time.perf_counter() - t0, sum(sum(row) for row in sol) == 405
    try:
        with ThreadPoolExecutor(max_workers=clients) as ex:
            list(ex.map(one, range(min(64, requests))))  # warm-up
            b0 = sum(n.solver.batcher.batches for n in nodes)
            t0 = time.perf_counter()
            res = list(ex.map(one, range(requests)))
            el = time.perf_counter() - t0
        lat = sorted(r[0] for r in res)
        return {"requests": requests, "clients": clients, "peers": peers, "solvers_per_peer": solvers,
                "requests_per_s": requests / el,
                "p50_ms": lat[len(lat) // 2] * 1e3, "p99_ms": lat[int(len(lat) * 0.99)] * 1e3,
                "gpu_batches": sum(n.solver.batcher.batches for n in nodes) - b0,
                "all_solved": all(r[1] for r in res)}
    finally:
        for node, httpd in zip(nodes, servers):
            node.shutdown()
            httpd.shutdown()


def _free_ports(k: int):
    import socket
    socks, ports = [], []
    for _ in range(k):
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        socks.append(sk)
        ports.append(sk.getsockname()[1])
    for sk in socks:
        sk.close()
    return ports


def node_load_procs(dev, peers: int = 4, solvers: int = 2, requests: int = 4000, clients: int = 64,
                    load_procs: int = 4, startup_s: float = 240.0):
    """BASELINE.json configs[4] in its process shape (README.md: one node.py
    per peer): `peers` node.py processes (python -m
    sudoku_solver_distributed_amd.node -h 0 --gpus <dev> x solvers; the
    first is the others' anchor), and the HTTP load in `load_procs` more
    processes (scripts/http_load.py).  Nothing of the bench process is on
    the request path.  Requests/s, p50 / p99, every answer validated."""
    import subprocess
    import tempfile
    import urllib.request
    ports = _free_ports(2 * peers)
    http, p2p = ports[:peers], ports[peers:]
    procs, logs = [], []
    try:
        for i in range(peers):
            cmd = [sys.executable, "-u", "-m", "sudoku_solver_distributed_amd.node", "-p", str(http[i]),
                   "-s", str(p2p[i]), "-h", "0", "--gpus", ",".join([str(dev.index)] * solvers)]
            if i:
                cmd += ["-a", f"127.0.0.1:{p2p[0]}"]
            log = tempfile.TemporaryFile(mode="w+")
            logs.append(log)
            procs.append(subprocess.Popen(cmd, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT))
        deadline = time.time() + startup_s
        for i, p in enumerate(procs):  # each peer answers /stats
            while True:
                if p.poll() is not None:
                    logs[i].seek(0)
                    raise RuntimeError(f"peer {i} exited ({p.returncode}): {logs[i].read()[-1500:]}")
                try:
                    with urllib.request.urlopen(f"http://127.0.0.1:{http[i]}/stats", timeout=5) as r:
                        r.read()
                    break
                except OSError:
                    if time.time() > deadline:
                        raise RuntimeError(f"peer {i} did not come up in {startup_s} s")
                    time.sleep(0.5)
        urls = [f"http://127.0.0.1:{h}/solve" for h in http]
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "http_load.py"), *urls,
                            "--requests", str(requests), "--clients", str(clients), "--procs", str(load_procs)],
                           cwd=ROOT, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"load generator failed: {r.stderr[-1500:]}")
        res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        res.update({"peers": peers, "solvers_per_peer": solvers, "peer_processes": peers})
        return res
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for log in logs:
            log.close()


def e2e_rate(solver, boards, reps: int = 3):
    """PCIe-inclusive rate: pinned host boards in, host solutions and
    statuses out (the serving path's view; `value` is device-resident).
    `serial`: copy in, solve, copy out back to back; `pipelined`:
    BatchSolver.solve_host, chunks overlapping both copy directions with the
    solve."""
    import torch
    host = boards.cpu().pin_memory()
    out_h = torch.empty_like(host).pin_memory()
    st_h = torch.empty(host.shape[0], dtype=torch.int32).pin_memory()

    def serial():
        d = host.to(solver.device, non_blocking=True)
        sols, st = solver.solve(d)
        out_h.copy_(sols, non_blocking=True)
        st_h.copy_(st, non_blocking=True)
        return st_h

    def pipelined():
        return solver.solve_host(host, out=out_h, status=st_h)[1]
    t, st = _time(serial, reps)
    res = {"boards": host.shape[0], "ms": t * 1e3, "boards_per_s": host.shape[0] / t,
           "all_solved": bool((st == 1).all())}
    t, st = _time(pipelined, reps)
    res["pipelined"] = {"ms": t * 1e3, "boards_per_s": host.shape[0] / t, "chunk": 1 << 18,
                        "all_solved": bool((st == 1).all())}
    return res


# waves per SIMD of the grouped (multi-step) launches of sharded steps
GRID_WAVES_GROUPED = 2


def shard_rates(solver, boards, launch_boards: int = 1 << 21, reps: int = 3):
    """configs[2]'s per-GPU regime under strong scaling, on one GPU: steps of
    B/2, B/4, B/8 boards (a rank's shard of the B-board step at N = 2, 4, 8),
    either one step per launch (`ungrouped`) or
    consecutive steps' shards in one sdk_solve_batches launch of
    `launch_boards` boards (`grouped`, the bench's strong-scaling steps);
    launches in flight as the bench's (solver.default_inflight).
    8 B boards per measurement, best of `reps`; every step checked SOLVED."""
    import torch
    n = boards.shape[0]
    out = {}
    for div in (2, 4, 8):
        sh = n // div
        parts = [boards[j * sh:(j + 1) * sh] for j in range(div)]
        k = 8 * div
        res = {"boards_per_step": sh, "steps": k}
        from sudoku_solver_distributed_amd.solver import default_inflight
        m = default_inflight()[0]
        for name, g in (("ungrouped", 1), ("grouped", max(1, min(32, -(-launch_boards // sh))))):
            nb = m * max(g, div)
            bufs = [(torch.empty_like(parts[0]), torch.empty(sh, dtype=torch.int32, device=boards.device))
                    for _ in range(nb)]

            def run(kk):
                solver.solve_inflight([parts[i % div] for i in range(kk)], [bufs[i % nb][0] for i in range(kk)],
                                      [bufs[i % nb][1] for i in range(kk)], inflight=m, group=g,
                                      grid_waves=GRID_WAVES_GROUPED if g > 1 else None)
            run(2 * g)
            best = None
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(k)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                best = el if best is None else min(best, el)
            ok = all(bool((b[1] == 1).all()) for b in bufs[:min(nb, k)])
            res[name] = {"steps_per_launch": g, "boards_per_s": sh * k / best, "all_solved": ok}
        out[f"1/{div}"] = res
    return out


def side_configs(solver, dev, world, rank, boards, serving: bool = True):
    """BASELINE.json configs[1], [2]'s per-GPU shard regime, [3] and [4], a
    search-heavy batch and the PCIe-inclusive rate, outside the timed region.

    configs[1]: 100k gen.py-style boards (generate_sudoku(50) under one seed,
    same random calls as gen.py:31-52) solved in one batch on one GPU.
    configs[3]: one search-heavy board, the walk's direct single-wave solve
    vs the frontier split (over every rank's GPU when N > 1, RCCL
    all-reduce(MIN) early-exit word).
    configs[4]: concurrent HTTP /solve against one peer, and against four
    peers with two solvers each (node_load).
    hard_search: 2^20 boards that need real search (gen.hard_search_batch).
    e2e: the timed batch with host buffers on both sides.
    Every result is checked.
    """
    import torch
    from sudoku_solver_distributed_amd.distributed import solve_split
    from sudoku_solver_distributed_amd.gen import SEARCH_HEAVY, generate_batch, hard_search_batch
    out = {}
    if rank == 0 and world == 1:
        out["shard_rate"] = shard_rates(solver, boards)
    if rank == 0:
        gen = generate_batch(100_000, 50, seed=7, device=dev)
        t, (sols, st) = _time(lambda: solver.solve(gen))
        ok = bool((st == 1).all()) and bool((solver.check(sols, 0) == 1).all())
        out["gen100k"] = {"boards": 100_000, "empty_boxes": 50, "seconds": t, "boards_per_s": 100_000 / t,
                          "all_solved_and_checked": ok}
        hs = hard_search_batch(boards.shape[0], seed=5, device=dev)
        solver.solve(hs)
        solver.stats(reset=True)
        t, (sols, st) = _time(lambda: solver.solve(hs))
        s3 = solver.stats(reset=True)
        ok = bool((st == 1).all()) and bool((solver.check(sols, 0) == 1).all())
        out["hard_search"] = {"boards": hs.shape[0], "seconds": t, "boards_per_s": hs.shape[0] / t,
                              "guesses_per_board": s3["guesses"] / max(s3["finished"], 1),
                              "passes_per_board": s3["sweeps"] / max(s3["finished"], 1),
                              "deferred_per_call": s3["deferred"] / 3, "all_solved_and_checked": ok}
        # the same batch as steps with launches in flight (the headline's method)
        from sudoku_solver_distributed_amd.solver import default_inflight
        m = default_inflight()[0]
        k = 3 * m
        hb = [(torch.empty_like(hs), torch.empty(hs.shape[0], dtype=torch.int32, device=dev)) for _ in range(m)]
        solver.solve_inflight([hs] * m, [b[0] for b in hb], [b[1] for b in hb], inflight=m)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        solver.solve_inflight([hs] * k, [hb[i % m][0] for i in range(k)], [hb[i % m][1] for i in range(k)], inflight=m)
        torch.cuda.synchronize()
        ti = (time.perf_counter() - t0) / k
        out["hard_search"]["inflight"] = {"steps": k, "boards_per_s": hs.shape[0] / ti,
                                          "identical": all(bool(torch.equal(b[0], sols)) for b in hb)}
        out["e2e"] = e2e_rate(solver, boards)
    if rank == 0 and serving:
        # configs[4]: peers in THIS process (GIL-bound, labelled so) and
        # peers as their own node.py processes (the reference's shape)
        out["node_http"] = node_load(dev)
        out["node_http_4peer"] = node_load(dev, requests=2000, clients=64, peers=4, solvers=2)
        out["node_http_4peer"]["shape"] = "four peers and the client threads in the bench process"
        for name, peers in (("node_http_1peer_procs", 1), ("node_http_4peer_procs", 4)):
            try:
                out[name] = node_load_procs(dev, peers=peers, solvers=2)
            except Exception as e:  # a side figure: report, never fail the bench
                out[name] = {"error": repr(e)[:800]}
    board = torch.tensor([[int(c) for c in SEARCH_HEAVY]], dtype=torch.uint8, device=dev)
    t_direct, (g1, s1) = _time(lambda: solver.solve(board))
    st = {}
    t_split, (ok2, g2) = _time(lambda: solve_split(board, order="gen", target=4096, stats=st))
    same = bool(int(s1[0]) == 1 and ok2 and torch.equal(g1[0].cpu(), g2.cpu()))
    out["pathological"] = {"board": SEARCH_HEAVY, "direct_ms": t_direct * 1e3, "split_ms": t_split * 1e3,
                           "ranks": world, "frontier": st.get("frontier"), "rounds": st.get("rounds"),
                           "identical": same}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the driver's own K / W (BENCH_r05's command): a run with no flags is the
    # launch shape profiles/pmc_plane_kernel_multi_w1.json was counted on, so
    # its line carries roofline.frac too
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 20,
                    help="boards per step: over all GPUs (--scaling strong) or per GPU (weak)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: --batch boards per step sharded over the ranks (BASELINE configs[2]); "
                         "weak: --batch boards per GPU per step")
    ap.add_argument("--launch-boards", type=int, default=-1,
                    help="a launch solves consecutive steps' shards together (sdk_solve_batches, <= 32 steps) "
                         "until it holds this many boards; 0 = one step per launch; -1: 2^21 when a rank's "
                         "shard is below 2^20 boards (strong scaling, N > 1), else one step per launch")
    ap.add_argument("--plan", choices=("run", "inflight"), default="run",
                    help="run (default): the timed steps as few launches as sdk_solve_batches allows (<= 32 steps "
                         "each), each on a full grid, the next queued behind the current one -- one drain per "
                         "launch, one launch for K <= 32; inflight: round 4's plan, one step (or --launch-boards "
                         "boards of steps) per launch, --inflight launches kept in flight at --grid-waves each")
    ap.add_argument("--launches", type=int, default=0,
                    help="split the timed steps' shards into this many launches of equal step counts "
                         "(sdk_solve_batches, <= SDK_MAX_BATCHES steps each) instead of --launch-boards")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--workload", choices=("hard17", "hard_search"), default="hard17",
                    help="timed boards: BASELINE's hard 17-clue set (default, the metric's config) or the "
                         "search-heavy set (profiling / A/B only)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--latency-boards", type=int, default=32,
                    help="boards timed one per launch for p50_single_ms (0 = skip; profiling runs)")
    ap.add_argument("--inflight", type=int, default=-1,
                    help="launches in flight per GPU (BatchSolver.solve_inflight: each on its own stream and "
                         "workspace, so one launch's drain overlaps the next ones); 1 = back to back; "
                         "-1: solver.default_inflight() (6 with >= 8 hardware queues, else 3)")
    ap.add_argument("--grid-waves", type=int, default=-1,
                    help="waves per SIMD in each launch's grid (sdk_solve_batch_grid; -1: the default for the "
                         "launches in flight, a full grid at --inflight 1; 0: a full grid)")
    ap.add_argument("--pool-last", type=int, default=-1,
                    help="launches at the end of the timed sequence that run unpipelined, their drained waves "
                         "sharing the last boards through the XCD tail pool (-1: solve_inflight's default, "
                         "half the launches in flight)")
    ap.add_argument("--launch-events", action="store_true",
                    help="also time each launch's own span with events on its slot stream (launch_ms)")
    ap.add_argument("--mrv-after", type=int, default=-1,
                    help="passes on a board before its search switches to the completion count "
                         "(sdk_set_plane_search; -1: the library default, 0: the walk's order only) -- A/B only")
    ap.add_argument("--no-serial", action="store_true",
                    help="skip the one-launch-per-step and single-batch figures (profiling runs: only the timed "
                         "launch shape runs)")
    ap.add_argument("--no-serving", action="store_true",
                    help="skip the configs[4] HTTP serving figures (peers in this process and as processes)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the configs[1] / configs[3] side measurements")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="process group for N > 1 (nccl = RCCL, the product; gloo = rehearsal of the "
                         "multi-rank path with every rank on one GPU)")
    ap.add_argument("--device-index", type=int, default=None,
                    help="put every rank on cuda:<index> instead of cuda:<LOCAL_RANK> (rehearsal of the "
                         "multi-rank path on a one-GPU box)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one process on one GPU runs rank --emulate-rank of a strong-scaling job of this many "
                         "ranks: that rank's own shard_bounds shard, step rotation and launch shape, no "
                         "collectives; the line reports that rank's wall time (scripts/rank_emul.py runs every "
                         "rank and takes the max).  Diagnostic: not the metric")
    ap.add_argument("--emulate-rank", type=int, default=0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    emulated = args.emulate_world > 0
    if emulated and (world != 1 or args.scaling != "strong" or not 0 <= args.emulate_rank < args.emulate_world):
        raise SystemExit("--emulate-world: one process, --scaling strong, 0 <= --emulate-rank < --emulate-world")
    # the job whose shard this process runs: the real one, or the emulated rank's
    job_world, job_rank = (args.emulate_world, args.emulate_rank) if emulated else (world, rank)
    gpu = local if args.device_index is None else args.device_index
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    comm_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    from sudoku_solver_distributed_amd.distributed import shard_bounds
    from sudoku_solver_distributed_amd.gen import hard17_batch, hard_search_batch
    from sudoku_solver_distributed_amd.solver import get_solver

    solver = get_solver(dev)
    if args.mrv_after >= 0:
        solver.lib.sdk_set_plane_search(args.mrv_after)
    make = hard17_batch if args.workload == "hard17" else hard_search_batch
    if args.scaling == "strong":
        lo, hi = shard_bounds(args.batch, job_rank, job_world)
    else:
        lo, hi = 0, args.batch
    shard = hi - lo  # this rank's boards per step
    if shard <= 0:
        raise SystemExit("--batch too small for the number of ranks")
    # steps per launch: enough consecutive steps' shards to fill a launch
    # (--plan inflight; the default plan "run" sets the group below).
    # Sharded steps (N > 1) go 2^21 boards to a launch at 2 waves per SIMD:
    # fewer launches, so fewer drains at the end of the run (one rank of
    # N = 2 / 4 / 8 at 20 steps: +6 / +6 / +5 % over 2^20 at 1 wave)
    from sudoku_solver_distributed_amd._lib import SDK_MAX_BATCHES
    launch_boards = args.launch_boards if args.launch_boards >= 0 else (1 << 21 if shard < (1 << 20) else 0)
    group = 1 if launch_boards <= shard else min(SDK_MAX_BATCHES, -(-launch_boards // shard))
    plan_run = args.plan == "run" and args.launches <= 0 and args.launch_boards < 0
    if plan_run:
        # the whole run's steps in ceil(K / 32) launches of equal step counts
        group = run_plan(args.steps)["group"]
    if args.launches > 0:
        group = min(SDK_MAX_BATCHES, -(-args.steps // args.launches))
    # one input per step of a launch group (each step its own boards): step
    # j's batch is the synthetic batch rotated by 7919 j boards (one
    # generation however many steps a launch holds); strong: this rank's
    # [lo, hi) of it (the same global batch on every rank), weak: per-rank seeds
    full = make(args.batch, seed=args.seed + (rank if args.scaling == "weak" else 0))
    inputs = step_inputs(full, lo, hi, group, dev)
    del full
    boards = inputs[0]
    from sudoku_solver_distributed_amd.solver import default_inflight
    m_def, gw_def = default_inflight()
    m = m_def if args.inflight < 0 else max(1, args.inflight)
    if plan_run and args.inflight < 0:
        m = run_plan(args.steps)["inflight"]  # the running launch and the next one queued behind it
    # one (solutions, status) pair per step that can be in flight: step i
    # reads inputs[i % group] and writes pair i % (m * group)
    nb = m * group
    bufs = [(torch.empty_like(boards), torch.empty(shard, dtype=torch.int32, device=dev)) for _ in range(nb)]
    out, status = bufs[0]
    stream = torch.cuda.current_stream(dev)
    solver._slot_solvers(m)  # slot workspaces allocated before any timing
    if args.grid_waves >= 0:
        grid_waves = args.grid_waves
    elif m == 1 or plan_run:
        grid_waves = 0
    elif group > 1 and args.inflight < 0:
        grid_waves = GRID_WAVES_GROUPED
    else:
        grid_waves = gw_def if args.inflight < 0 else (1 if m >= 5 else 2)
    grid_waves_used = grid_waves

    # the launches that share their tails through the XCD pool (unpipelined):
    # plan run: the last (nothing is queued behind it); inflight: half the
    # launches in flight (solve_inflight's default)
    pool_last_arg = args.pool_last if args.pool_last >= 0 else (run_plan(args.steps)["pool_last"] if plan_run else None)

    def steps(k, events=None, inflight=m):
        solver.solve_inflight([inputs[i % group] for i in range(k)], [bufs[i % nb][0] for i in range(k)],
                              [bufs[i % nb][1] for i in range(k)], inflight=inflight, launch_events=events,
                              grid_waves=grid_waves if inflight > 1 else 0, group=group,
                              pool_last=pool_last_arg)

    steps(args.warmup)
    torch.cuda.synchronize(dev)
    if not all(bool((bufs[i][1] == 1).all()) for i in range(min(nb, args.warmup))):
        raise SystemExit("warmup: not every board solved")

    solver.inflight_stats(reset=True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    launches = [] if args.launch_events else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    steps(args.steps, launches)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    # the launches overlap (m in flight): a launch's share of the timed GPU
    # region, and separately each launch's own start-to-end span
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    launch_ms = sum(a.elapsed_time(b) for a, b in launches) / len(launches) if launches else None
    st = solver.inflight_stats()
    # every board of every timed step answered exactly once: the kernels'
    # own accounting (sdk_verify_workspace raises on a board a kernel took
    # and could not finish, e.g. a tail-pool record never published) and
    # the finished count against the boards the steps handed out
    solver.verify_inflight()
    if st["finished"] != args.steps * shard:
        raise SystemExit(f"timed steps: {st['finished']} boards answered, {args.steps * shard} handed out")
    t = torch.tensor([wall], dtype=torch.float64, device=comm_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    checks = check_steps(solver, inputs, bufs, args.steps, group, lo, args.batch)
    solved_ok = all(checks.values())

    # the same K steps as K one-step launches back to back (each its own
    # full grid and its own drain): what a run costs without plan "run"'s
    # one queue over the steps
    serial = None
    if not args.no_serial:
        torch.cuda.synchronize(dev)
        s0 = time.perf_counter()
        solver.solve_inflight([inputs[i % group] for i in range(args.steps)], [bufs[i % nb][0] for i in range(args.steps)],
                              [bufs[i % nb][1] for i in range(args.steps)], inflight=1, grid_waves=0, group=1)
        torch.cuda.synchronize(dev)
        s_wall = time.perf_counter() - s0
        solver.verify_inflight()
        serial = {"what": "the same steps, one launch per step, back to back (full grid each)",
                  "value": shard * args.steps / s_wall, "ms_per_step": s_wall / args.steps * 1e3,
                  "outputs_checked": all(check_steps(solver, inputs, bufs, args.steps, group, lo, args.batch).values())}

    # one step's batch alone: one device-resident solve() call (this rank's
    # shard of step 0, 2^20 boards at N = 1), best of 3
    single = None
    if not args.no_serial:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = None
        for _ in range(3):
            torch.cuda.synchronize(dev)
            s0 = time.perf_counter()
            e0.record(stream)
            solver.solve(inputs[0], out=bufs[0][0], status=bufs[0][1])
            e1.record(stream)
            torch.cuda.synchronize(dev)
            w_ms = (time.perf_counter() - s0) * 1e3
            k_ms = e0.elapsed_time(e1)
            best = (w_ms, k_ms) if best is None or w_ms < best[0] else best
        solver.verify()
        single = {"what": "one batch alone: one solve() call of one step's boards, best of 3",
                  "boards": shard, "wall_ms": best[0], "kernel_ms": best[1], "boards_per_s": shard / best[0] * 1e3,
                  "all_solved": bool((bufs[0][1] == 1).all())}

    # single-board latency (p50 over 32 boards, one launch each)
    lat = []
    for i in range(args.latency_boards):
        b = boards[i:i + 1]
        torch.cuda.synchronize(dev)
        s0 = time.perf_counter()
        solver.solve(b)
        torch.cuda.synchronize(dev)
        lat.append((time.perf_counter() - s0) * 1e3)
    lat.sort()
    p50 = lat[len(lat) // 2] if lat else None

    extras = (None if args.no_extras or emulated
              else side_configs(solver, dev, world, rank, boards, serving=not args.no_serving))

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    total = (args.batch if args.scaling == "strong" else args.batch * world) * args.steps
    if emulated:
        total = shard * args.steps  # this rank's boards (the job's value is the max over ranks)
    value = total / wall_max
    kern_s = kern_ms / 1e3  # this GPU's share of the timed region per step
    # pool_last: the launches at the end that share their tails through the
    # XCD pool (solve_inflight's default: half the launches in flight; -1 all)
    pool_last = pool_last_arg if pool_last_arg is not None else ((m + 1) // 2 if m > 1 else -1)
    # (hw_queues: the process's hardware queues, which decide whether the
    # launches in flight run side by side -- bench.py sets 8, HIP's default is 4)
    shape = {"boards_per_step": shard, "group": group, "inflight": m, "grid_waves": grid_waves_used,
             "pool_last": pool_last, "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])}
    roof = {"bound": "valu", "achieved": None, "peak": PEAK_VALU_OPS / 1e12, "unit": "TOP/s",
            "frac": None, "traffic": None, "kernel_ms": kern_ms, "launch_ms": launch_ms, "shape": shape,
            "hbm": {"achieved_GBps": BYTES_PER_BOARD * shard / kern_s / 1e9,
                    "peak_GBps": PEAK_HBM / 1e9,
                    "frac": BYTES_PER_BOARD * shard / kern_s / PEAK_HBM}}
    from sudoku_solver_distributed_amd import _lib
    kname = _lib.KERNEL_SYMBOLS.get(_lib.active_kernel(), "?")
    if group > 1 and kname == "plane_kernel":
        kname = "plane_kernel_multi"  # sdk_solve_batches' kernel
    roof["kernel"] = kname
    # the committed PMC summaries of this kernel (scripts/gpu_pmc.sh: one per
    # workload and launch shape, e.g. pmc_plane_kernel_multi_w8.json for the
    # N = 8 rank's grouped launches); the counters count only if they were
    # taken on EXACTLY this workload and launch shape
    import glob
    pmc, PMC_FILE = None, None
    for f_ in sorted(glob.glob(os.path.join(PMC_DIR, f"pmc_{kname}*.json"))):
        with open(f_) as f:
            cand = json.load(f)
        if (cand.get("kernel") == kname and cand.get("seed") == args.seed
                and cand.get("workload", "hard17") == args.workload and cand.get("shape") == shape):
            pmc, PMC_FILE = cand, f_
            break
    roof["pmc_match"] = pmc is not None
    if pmc is not None:
        # per step: the profiled run's dispatches summed over its steps
        # (grouped launches hold different step counts), else per launch
        valu_step = pmc.get("valu_insts_per_step") or pmc["valu_insts_per_launch"] / group
        ops = valu_step * 64
        roof["achieved"] = ops / kern_s / 1e12
        roof["frac"] = roof["achieved"] / roof["peak"]
        roof["valu_insts_per_step"] = valu_step
        hbm_step = pmc.get("hbm_bytes_per_step") or (pmc["hbm_bytes_per_launch"] / group
                                                    if pmc.get("hbm_bytes_per_launch") is not None else None)
        if hbm_step is not None:
            roof["traffic"] = hbm_step
            roof["traffic_over_algorithmic"] = roof["traffic"] / (BYTES_PER_BOARD * shard)
        for k in ("sq_wait_inst_any_share", "sq_wait_any_share"):
            if k in pmc:
                roof[k] = pmc[k]
        roof["pmc_source"] = os.path.relpath(PMC_FILE, ROOT)
        # lanes doing pass work: passes x VALU per pass (ISA count of
        # plane::pass) over every lane slot the kernel issued
        isa = os.path.join(PMC_DIR, "isa_plane_pass.json")
        if kname.startswith("plane_kernel") and os.path.exists(isa):
            with open(isa) as f:
                vpp = json.load(f)["valu_per_pass"]
            useful = st["sweeps"] / args.steps * vpp
            roof["valu_per_pass"] = vpp
            roof["useful_lane_frac"] = useful / ops
            roof["useful_frac_of_peak"] = useful / kern_s / 1e12 / roof["peak"]
        # the pass's own ceiling at the kernel's occupancy (microbenchmark)
        ceil = os.path.join(PMC_DIR, "r06_pass_ceiling.json")
        if kname.startswith("plane_kernel") and os.path.exists(ceil):
            with open(ceil) as f:
                c = json.load(f)
            cp = c["by_waves_per_simd"][str(c["plane_kernel_waves_per_simd"])]["passes_per_s"]
            roof["pass_ceiling_passes_per_s"] = cp
            roof["pass_ceiling_frac"] = st["sweeps"] / args.steps / kern_s / cp

    cpu = None
    if world == 1 and not args.no_cpu and not emulated:
        sample = boards[:8192].cpu().numpy()
        done, el, threads = cpu_baseline(sample, args.cpu_budget)
        cpu = {"value": done / el, "unit": "boards/s", "cores": threads, "kind": "port",
               "sample": f"{done} boards of the same hard-17 batch (first 8192, split into {threads} "
                         f"contiguous slices) completed in {el:.1f} s by {threads} host threads, one "
                         f"literal gen.py:6-28 walk each (oracle/sudoku_oracle.c)"}

    line = {
        "metric": "puzzles solved/sec (node), 1M hard 9x9 batch @1/2/4/8 GPU; single-puzzle p50 ms"
                  + (f" [EMULATED rank {job_rank} of {job_world} on one GPU: value = that rank's boards/s]"
                     if emulated else ""),
        "value": value,
        "unit": "boards/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: 17-clue unique-solution boards (symmetry images of 80 certified isomorphism "
                "classes, data/hard17_classes.txt)" if args.workload == "hard17" else
                "synthetic: search-heavy minimal boards (symmetry images of data/hard_search_seeds.txt)",
        "config": {"workload": (f"{'hard 17-clue' if args.workload == 'hard17' else 'search-heavy minimal'} 9x9 "
                                f"batch, {args.batch} boards per step "
                                f"{'over all GPUs' if args.scaling == 'strong' else 'per GPU'}"),
                   "global_batch": args.batch if args.scaling == "strong" else args.batch * world,
                   "boards_per_gpu_per_step": shard, "parallelism": f"shard{world}",
                   "steps_per_launch": group, "inflight_per_gpu": m, "grid_waves_per_simd": grid_waves_used or None,
                   "dist_backend": args.dist_backend if world > 1 else None,
                   **({"emulated_rank": job_rank, "emulated_world": job_world, "rank_wall_s": wall_max}
                      if emulated else {})},
        "serial": serial,  # this GPU's steps as one launch each, back to back (rank 0's boards / s)
        "single_batch": single,  # one step's batch in one solve() call (rank 0)
        "output_checks": checks,
        "p50_single_ms": p50,
        "all_solved_and_checked": solved_ok,
        "guesses_per_board": st["guesses"] / max(st["finished"], 1),
        "sweeps_per_board": st["sweeps"] / max(st["finished"], 1),
        "deferred_per_step": st.get("deferred", 0) / args.steps,
        "roofline": roof,
        "cpu_baseline": cpu,
        "side_configs": extras,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
