"""Drop-in for the reference's ``node.py``: a peer with an HTTP front
(`/solve`, `/stats`, `/network`) and a UDP JSON protocol between peers,
whose Sudoku work runs on the GPU(s) the peer owns.

    python -m sudoku_solver_distributed_amd.node -p 8000 -s 7000 [-a host:port] [-h 0]
           [--host 127.0.0.1] [--gpus 0,1] [--forward-threshold N]

What changed against node.py (and why):

* ``SudokuSolver`` (node.py:21-131) keeps its methods and counters; the
  walk (`solve_sudoku`, `solve_sudoku_recursive`, node.py:31-40/62-74), the
  check (node.py:82-116) and the per-cell task (`solve_sudoku_destributed`,
  node.py:76-80) are HIP kernels.  `validations`: the
  reference adds one per SudokuSolver.check call (node.py:87), and its walk
  calls check once per candidate test (is_valid_move, node.py:44, 68) --
  ~1e7-1e8 per hard board, a number only the literal walk itself can count.
  Here a check() / is_valid_move / cell task still adds one each; a walk
  solve on the GPU adds the kernel's propagation passes over the board (one
  pass tests every empty cell against its row, column and box once), and a
  solve in "reference" mode adds exactly the reference's count.
* Every board a peer is asked to solve -- HTTP `/solve` (node.py:672-690),
  a UDP `solve` message, `SudokuSolver.solve_sudoku` -- goes through one
  ``BoardBatcher`` per peer: concurrent requests are coalesced into one GPU
  launch per tick (``max_wait`` after the first pending board, or
  ``max_batch`` boards), sharded over the peer's GPUs (``GpuSolverBackend``),
  and each request gets its own board back.  This is what makes a peer
  serve many clients at once (BASELINE.json configs[4]).
* ``P2PNode.peer_sudoku_solve`` (node.py:534-557) no longer deals one
  board's empty cells to peers one UDP message each (node.py:419-475): a
  board is a few microseconds of GPU work, so the unit of distribution is a
  whole board.  A peer whose batcher queue holds ``forward_threshold`` boards
  or more hands new boards to its peers (round robin, UDP `solve` with a
  `task` id, answered by a `solution` message) and solves locally if a peer
  does not answer in time.  The answer is node.py's recursive walk
  (node.py:62-74), bit-identical.  The reference's HTTP path answers with its
  greedy task loop instead, which differs on some boards; solve_mode
  "reference" reproduces that loop, including the state a reference node
  carries from one request to the next (INTEGRATION.md §3,
  tests/golden/golden_peer.json, golden_peer_seq.json).
* The UDP `solve` / `solution` messages (node.py:384-406) are kept: with
  `row`/`col` they are the reference's cell task; without them a peer hands
  a whole board (`sudoku`) or a batch (`sudokus`, 81-character strings, at
  most MAX_UDP_BOARDS per datagram).  Every `solve` is answered, with an
  `error` field if it could not be served.
* Membership and statistics messages (`connect`, `connected`, `all_peers`,
  `disconnect`, `stats`; node.py:193-382) keep their JSON shape.
* The HTTP server binds a configurable host (node.py:708 hard-codes a LAN IP)
  and serves requests on threads.
"""
from __future__ import annotations

import argparse
import itertools
import json
import logging
import socket
import threading
import time
from collections import deque
from concurrent.futures import Future, ThreadPoolExecutor
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import List, Optional

import torch

from .solver import SDK_NO_RETURN, SDK_SOLVED, BatchSolver, SudokuHipError, as_boards, get_solver

logger = logging.getLogger(__name__)

# boards per UDP `sudokus` message: 81 characters + JSON punctuation each, so
# the request (and the reply, which adds a status per board) stays well inside
# one datagram (65 507 bytes of payload)
MAX_UDP_BOARDS = 256
BATCH_ORDERS = ("gen", "node")


def is_grid9(board) -> bool:
    """Exactly the reference's board type: 9 lists of 9 integers."""
    return (isinstance(board, list) and len(board) == 9
            and all(isinstance(r, list) and len(r) == 9 and all(isinstance(v, int) and not isinstance(v, bool)
                                                                for v in r) for r in board))


class GpuSolverBackend:
    """Kernels of one or more local GPUs; a batch is split over `devices`.

    Each entry of `devices` is one solver with its own workspace and its own
    stream, so a device listed twice ([0, 0]) runs two solvers side by side
    on one GPU (the first uses the process-wide solver of that device).  A
    batch goes host -> pinned staging -> every solver's stream (copy in,
    solve, copy out, all asynchronous), then one wait on all of them: the
    devices work at the same time.  A solver's op_lock is held only while
    its launches are enqueued; the pass count of this batch comes from two
    stream-ordered counter snapshots around the solve (sdk_snapshot_stats),
    so another peer sharing the device neither interleaves with the bracket
    nor leaks into the count, and nothing synchronises under the lock."""

    def __init__(self, devices=None):
        if devices is None:
            devices = [torch.cuda.current_device()] if torch.cuda.is_available() else [None]
        self.solvers = []
        for d in devices:
            s = get_solver(d)
            if any(t is s for t in self.solvers):
                s = BatchSolver(s.device)  # another workspace on the same GPU
            self.solvers.append(s)
        # created once per solver: each stream takes one of the process's few
        # hardware queues (solver.py solve_host)
        self.streams = [torch.cuda.Stream(s.device) for s in self.solvers]
        self._lock = threading.Lock()  # one batch at a time on these streams

    def solve(self, boards: torch.Tensor, order: str):
        """(n,81) host boards -> (host solutions, host status, passes)."""
        boards = as_boards(boards)
        n = boards.shape[0]
        if n == 0:
            return torch.empty((0, 81), dtype=torch.uint8), torch.empty(0, dtype=torch.int32), 0
        k = len(self.solvers)
        pin = torch.empty((n, 81), dtype=torch.uint8, pin_memory=True)
        pin.copy_(boards)
        out = torch.empty((n, 81), dtype=torch.uint8, pin_memory=True)
        st = torch.empty(n, dtype=torch.int32, pin_memory=True)
        counts = torch.zeros((k, 6), dtype=torch.int64, pin_memory=True)
        events = []
        with self._lock:
            for i, (s, stream) in enumerate(zip(self.solvers, self.streams)):
                lo, hi = i * n // k, (i + 1) * n // k
                if lo == hi:
                    continue
                with torch.cuda.device(s.device), torch.cuda.stream(stream):
                    d_in = pin[lo:hi].to(s.device, non_blocking=True)
                    d_out = torch.empty_like(d_in)
                    d_st = torch.empty(hi - lo, dtype=torch.int32, device=s.device)
                    with s.op_lock:  # enqueue only: snapshot, solve, snapshot in stream order
                        before = s.stats_snapshot(stream)
                        s.solve(d_in, out=d_out, status=d_st, order=order, stream=stream)
                        after = s.stats_snapshot(stream)
                    out[lo:hi].copy_(d_out, non_blocking=True)
                    st[lo:hi].copy_(d_st, non_blocking=True)
                    counts[i].copy_(after - before, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    events.append(ev)
            for ev in events:
                ev.synchronize()
        # every board of the batch answered: the stream-ordered count of
        # finished boards around each solver's launch equals its share
        for i in range(k):
            want = (i + 1) * n // k - i * n // k
            if want and int(counts[i, 0]) != want:
                # verify() raises its own error (and clears the workspace's
                # error word): keep its text and this batch's shortfall together
                try:
                    detail = f"workspace: {self.solvers[i].verify()}"
                except SudokuHipError as e:
                    detail = str(e)
                raise SudokuHipError(f"solver {i}: {int(counts[i, 0])} of {want} boards answered ({detail})")
        return out, st, int(counts[:, 3].sum())

    def peer_solve(self, boards: torch.Tensor):
        """The reference's /solve loop per board on a fresh node each
        (sdk_peer_solve_batch): (boards it leaves, status, validations)."""
        s, stream = self.solvers[0], self.streams[0]
        with torch.cuda.device(s.device), torch.cuda.stream(stream):
            out, st, val = s.peer_solve(as_boards(boards), stream=stream)
            res = out.cpu(), st.cpu(), val.cpu()
        return res

    def new_peer_state(self):
        """A new node's persistent /solve state (node.py:149, 167), zeroed on
        the stream peer_solve_seq runs on (streams[0] is a non-blocking pool
        stream: a memset on the caller's stream would not be ordered before
        the first request)."""
        s, stream = self.solvers[0], self.streams[0]
        with torch.cuda.device(s.device), torch.cuda.stream(stream):
            return s.new_peer_state()

    def peer_solve_seq(self, boards: torch.Tensor, state):
        """The reference's /solve loop on ONE node serving `boards` as
        requests in order, from and into `state` (sdk_peer_solve_seq)."""
        s, stream = self.solvers[0], self.streams[0]
        with torch.cuda.device(s.device), torch.cuda.stream(stream):
            out, st, val = s.peer_solve_seq(as_boards(boards), state, stream=stream)
            res = out.cpu(), st.cpu(), val.cpu()
        return res

    def check(self, boards, mode: int):
        return self.solvers[0].check(as_boards(boards, max_value=255), mode).cpu()

    def first_candidate(self, boards, cells):
        return self.solvers[0].first_candidate(as_boards(boards, max_value=255), cells).cpu()


class BoardBatcher:
    """Coalesces concurrent solve requests into one backend call per tick.

    submit() queues (n, 81) boards with a walk order ("gen", "node", or
    "peer" for the reference's /solve loop) and returns a Future of
    (solutions, status); one thread drains the queue: it waits for the first
    board, then up to ``max_wait`` seconds (or until ``max_batch`` boards are
    queued) for more, and solves each order's boards in one call.

    "peer" boards are requests to this batcher's node, in arrival order:
    they run as one sequence from the node's persistent /solve state
    (``peer_state``: the reference P2PNode's partial_solution and
    tried_numbers_by_position, node.py:149, 167), as the reference's
    single-threaded HTTP server would take them one after the other."""

    def __init__(self, backend, max_batch: int = 1 << 16, max_wait: float = 0.0005, on_batch=None):
        self.backend = backend
        self.max_batch = max_batch
        self.max_wait = max_wait
        self.on_batch = on_batch  # callback(boards, passes) after each backend call
        self._q = deque()
        self._queued = 0
        self._cv = threading.Condition()
        self._stop = False
        self.batches = 0
        self.boards = 0
        self.peer_state = None  # created on the first "peer" batch
        self._thread = threading.Thread(target=self._run, name="BoardBatcher", daemon=True)
        self._thread.start()

    def pending(self) -> int:
        return self._queued

    def submit(self, boards: torch.Tensor, order: str = "node") -> Future:
        boards = as_boards(boards)
        fut: Future = Future()
        with self._cv:
            if self._stop:
                raise RuntimeError("BoardBatcher is closed")
            self._q.append((boards, order, fut))
            self._queued += boards.shape[0]
            self._cv.notify()
        return fut

    def reset_peer_state(self):
        """Forget the node's /solve state (a restarted reference node)."""
        with self._cv:
            self.peer_state = None

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout=5)

    def _take(self):
        with self._cv:
            while not self._q and not self._stop:
                self._cv.wait()
            if self._stop and not self._q:
                return None
            deadline = time.monotonic() + self.max_wait
            while self._queued < self.max_batch and not self._stop:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                self._cv.wait(left)
            items, n = [], 0
            while self._q and (n == 0 or n + self._q[0][0].shape[0] <= self.max_batch):
                it = self._q.popleft()
                items.append(it)
                n += it[0].shape[0]
            self._queued -= n
            return items

    def _run(self):
        while True:
            items = self._take()
            if items is None:
                return
            for order in sorted({it[1] for it in items}):
                group = [it for it in items if it[1] == order]
                try:
                    boards = torch.cat([it[0] for it in group])
                    if order == "peer":
                        with self._cv:
                            if self.peer_state is None:
                                self.peer_state = self.backend.new_peer_state()
                            state = self.peer_state
                        sols, st, val = self.backend.peer_solve_seq(boards, state)
                        passes = int(val.sum())
                    else:
                        sols, st, passes = self.backend.solve(boards, order)
                    self.batches += 1
                    self.boards += boards.shape[0]
                    if self.on_batch is not None:
                        self.on_batch(boards.shape[0], int(passes))
                    lo = 0
                    for b, _, fut in group:
                        hi = lo + b.shape[0]
                        fut.set_result((sols[lo:hi], st[lo:hi]))
                        lo = hi
                except Exception as e:  # every waiter hears about it
                    for _, _, fut in group:
                        if not fut.done():
                            fut.set_exception(e)


class PeerError(RuntimeError):
    """A peer answered a forwarded board with an error."""


class ReferenceNoReturn(RuntimeError):
    """The reference's /solve loop (node.py:427-475) never returns on this board."""


def _flat(board):
    return [v for row in board for v in row]


def _copy_into(board, flat):
    for r in range(9):
        board[r][:] = [int(v) for v in flat[r * 9:(r + 1) * 9]]


class SudokuSolver:
    """node.py:21-131 with the walk, check and cell task on the GPU."""

    def __init__(self, base_delay=0.01, backend=None, max_wait: float = 0.0005):
        logger.info("Initializing Sudoku solver")
        self.sudoku_board = None
        self.recent_requests = deque()
        self.solved_puzzles = 0
        self.validations = 0
        self.base_delay = base_delay
        self.backend = backend if backend is not None else GpuSolverBackend()
        self.lock = threading.Lock()
        self.batcher = BoardBatcher(self.backend, max_wait=max_wait, on_batch=self._count_passes)

    def _count_passes(self, boards, passes):
        with self.lock:
            self.validations += passes

    # node.py:31-40 (returns the caller's board object, which node.py keeps
    # in self.sudoku_board -- under concurrent requests that attribute is the
    # latest request's, so it is not read back)
    def solve_sudoku(self, sudoku):
        self.sudoku_board = sudoku
        if self.solve_sudoku_recursive(sudoku):
            with self.lock:
                self.solved_puzzles += 1
            return sudoku
        logger.error("Failed to solve Sudoku puzzle")
        return None

    # node.py:42-60 (host-side accessor: one cell, one digit)
    def is_valid_move(self, board, row, col, num):
        if self.check(board):
            return True
        for i in range(9):
            if board[row][i] == num or board[i][col] == num:
                return False
        sr, sc = 3 * (row // 3), 3 * (col // 3)
        for i in range(3):
            for j in range(3):
                if board[sr + i][sc + j] == num:
                    return False
        return True

    # node.py:62-74 -- the walk in node order, on the GPU, board filled in place
    def solve_sudoku_recursive(self, board):
        sols, st = self.batcher.submit(as_boards(_flat(board)), "node").result()
        if int(st[0]) != SDK_SOLVED:
            return False
        _copy_into(board, sols[0].tolist())
        return True

    # node.py:76-80 -- the UDP "solve" cell task
    def solve_sudoku_destributed(self, board, row, col):
        num = int(self.backend.first_candidate(as_boards(_flat(board), max_value=255), [row * 9 + col])[0])
        with self.lock:
            self.validations += 1
        return num if num > 0 else None

    def solve_many(self, boards, order="node"):
        """Batch entry point (no reference counterpart): (n,81) -> (sols, status)."""
        sols, st = self.batcher.submit(as_boards(boards), order).result()
        with self.lock:
            self.solved_puzzles += int((st == SDK_SOLVED).sum())
        return sols, st

    # node.py:82-116 -- validations counter, rate limiter, sums-only check
    def check(self, board, interval=10, threshold=5):
        with self.lock:
            self.validations += 1
            now = time.time()
            self.recent_requests.append(now)
            while self.recent_requests and now - self.recent_requests[0] >= interval:
                self.recent_requests.popleft()
            n = len(self.recent_requests)
        if n > threshold and self.base_delay:
            time.sleep(self.base_delay * (n - threshold + 1))
        return bool(int(self.backend.check(as_boards(_flat(board), max_value=255), 1)[0]))

    # node.py:118-131
    def __str__(self, board=None):
        board = board if board is not None else self.sudoku_board
        out = "| - - - - - - - - - - - |\n"
        for i in range(9):
            out += "| "
            for j in range(9):
                out += str(board[i][j])
                out += " | " if j % 3 == 2 else " "
            if i % 3 == 2:
                out += "\n| - - - - - - - - - - - |"
            out += "\n"
        return out

    def close(self):
        self.batcher.close()


def _s81(board) -> str:
    return "".join(str(int(v)) for v in (_flat(board) if isinstance(board[0], list) else board))


class P2PNode:
    """node.py:134-657: UDP JSON peer + statistics; solving on local GPUs."""

    def __init__(self, host, port, anchor_node=None, handicap=0.001, backend=None,
                 forward_threshold: Optional[int] = None, forward_timeout: float = 5.0,
                 max_wait: float = 0.0005, solve_mode: str = "walk"):
        if solve_mode not in ("walk", "reference"):
            raise ValueError("solve_mode must be 'walk' or 'reference'")
        self.solve_mode = solve_mode
        self.solver = SudokuSolver(handicap, backend=backend, max_wait=max_wait)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.settimeout(0.2)
        self.id = f"{host}:{port}"
        self.host, self.port = host, port
        self.anchor_node = anchor_node
        self.shutdown_flag = False
        self.peers_out = set()   # peers this node connected to
        self.peers_in = set()    # peers that connected to this node
        self.all_peers = {}      # {peer: [peers connected to it]}
        self.total_peers = []
        self.stats_solved = {}
        self.all_stats = {"all": {"solved": 0, "validations": 0}, "nodes": []}
        self.forward_threshold = forward_threshold
        self.forward_timeout = forward_timeout
        self.forwarded = 0       # boards this peer handed to others
        self.served = 0          # boards this peer solved for others
        self._rr = itertools.count()
        self._tasks = {}         # task id -> [threading.Event, reply]
        self._task_ids = itertools.count(1)
        self._stats_timer = None
        self.lock = threading.RLock()
        # UDP `solve` messages are served off the receive loop by a bounded pool
        self._pool = ThreadPoolExecutor(max_workers=32, thread_name_prefix="udp-solve")

    # ---------------------------------------------------------- transport
    def send(self, address, msg):
        if isinstance(address, str):
            h, p = address.split(":")
            address = (h, int(p))
        self.sock.sendto(json.dumps(msg).encode(), address)

    def recv(self):
        try:
            payload, addr = self.sock.recvfrom(1 << 16)
            return (payload or None), addr
        except socket.timeout:
            return None, None
        except OSError:
            return None, None

    def connected_peers(self):
        with self.lock:
            return sorted(self.peers_out | self.peers_in)

    def broadcast(self, msg):
        for peer in self.connected_peers():
            self.send(peer, msg)

    def broadcast_all_peers(self):
        with self.lock:
            msg = {"type": "all_peers", "all_peers": {k: list(v) for k, v in self.all_peers.items()}}
        self.broadcast(msg)

    def broadcast_stats_soon(self, delay: float = 0.02):
        """broadcast_stats at most once per `delay` under load: one gossip
        round covers every request finished meanwhile."""
        with self.lock:
            if self._stats_timer is not None:
                return
            self._stats_timer = threading.Timer(delay, self._stats_tick)
            self._stats_timer.daemon = True
            self._stats_timer.start()

    def _stats_tick(self):
        with self.lock:
            self._stats_timer = None
        if not self.shutdown_flag:
            self.broadcast_stats()

    def broadcast_stats(self):
        stats = self.get_stats()
        with self.solver.lock:
            solved, validations = self.solver.solved_puzzles, self.solver.validations
        self.broadcast({"type": "stats", "origin": self.id, "solved": solved,
                        "stats": {"address": self.id, "validations": validations},
                        "all_stats": stats})

    def _refresh_total_peers(self):
        peers = set(self.all_peers)
        for kids in self.all_peers.values():
            peers.update(kids)
        peers.discard(self.id)
        self.total_peers = sorted(peers)

    # ----------------------------------------------------------- messages
    def handle_message(self, msg):
        t = msg.get("type")
        if t == "solve":  # GPU work off the receive loop
            self._pool.submit(self._handle_solve_safe, msg)
            return
        rebroadcast = False
        with self.lock:
            if t == "connect":  # node.py:195-199
                self.peers_out.add(msg["address"])
                self.send(msg["address"], {"type": "connected", "address": self.id})
            elif t == "connected":  # node.py:201-210
                self.peers_in.add(msg["address"])
                self.all_peers[msg["address"]] = sorted(set(self.all_peers.get(msg["address"], [])) | {self.id})
                self._refresh_total_peers()
                rebroadcast = True
            elif t == "all_peers":  # node.py:213-260 (merge, re-broadcast on change)
                for peer, kids in msg["all_peers"].items():
                    merged = sorted(set(self.all_peers.get(peer, [])) | set(kids))
                    if merged != self.all_peers.get(peer):
                        self.all_peers[peer] = merged
                        rebroadcast = True
                self._refresh_total_peers()
            elif t == "stats":  # node.py:264-331 (max-merge per node)
                addr = msg["stats"]["address"]
                changed = self._merge_solved(addr, msg.get("solved", 0))
                changed |= self._merge_node(addr, msg["stats"]["validations"])
                for node in msg.get("all_stats", {}).get("nodes", []):
                    if node["address"] != self.id:
                        changed |= self._merge_node(node["address"], node["validations"])
                for node in msg.get("all_stats", {}).get("solved_by", []):
                    if node["address"] != self.id:
                        changed |= self._merge_solved(node["address"], node["solved"])
                if changed:  # pass news on (peers are not all connected to each other)
                    self.broadcast_stats_soon()
            elif t == "disconnect":  # node.py:334-381
                a = msg["address"]
                self.peers_in.discard(a)
                self.peers_out.discard(a)
                self.all_peers.pop(a, None)
                for peer in list(self.all_peers):
                    kids = [k for k in self.all_peers[peer] if k != a]
                    if kids:
                        self.all_peers[peer] = kids
                    else:
                        del self.all_peers[peer]
                self._refresh_total_peers()
            elif t == "solution":
                task = self._tasks.get(msg.get("task"))
                if task is not None:
                    task[1] = msg
                    task[0].set()
        if rebroadcast:
            self.broadcast_all_peers()
            self.broadcast_stats()

    def _merge_node(self, addr, validations) -> bool:
        for node in self.all_stats["nodes"]:
            if node["address"] == addr:
                if validations > node["validations"]:
                    node["validations"] = validations
                    return True
                return False
        self.all_stats["nodes"].append({"address": addr, "validations": validations})
        return True

    def _merge_solved(self, addr, solved) -> bool:
        if solved and solved > self.stats_solved.get(addr, 0):
            self.stats_solved[addr] = solved
            return True
        return False

    def _handle_solve_safe(self, msg):
        """Serve one UDP `solve`; whatever goes wrong, the requester gets a
        `solution` with an `error` field instead of waiting for its timeout."""
        try:
            self._handle_solve(msg)
        except Exception as e:  # noqa: BLE001 -- reported to the requester
            logger.error("solve request failed: %s", e)
            if isinstance(msg.get("address"), str):
                reply = {"type": "solution", "error": str(e), "address": self.id}
                if "task" in msg:
                    reply["task"] = msg["task"]
                for k in ("row", "col"):
                    if k in msg:
                        reply[k] = msg[k]
                try:
                    self.send(msg["address"], reply)
                except OSError as e2:
                    logger.error("could not report the failure to %s: %s", msg["address"], e2)

    def _handle_solve(self, msg):
        sudoku = msg.get("sudoku")
        if not is_grid9(sudoku) and "sudokus" not in msg:
            raise ValueError("sudoku must be 9 lists of 9 integers")
        if "row" in msg and "col" in msg:  # node.py:384-406: the cell task
            num = self.solver.solve_sudoku_destributed(sudoku, msg["row"], msg["col"])
            reply = {"type": "solution", "sudoku": sudoku, "row": msg["row"], "col": msg["col"],
                     "solution": num, "address": self.id}
        elif "sudokus" in msg:  # a batch handed over by a peer (81-character strings)
            order = msg.get("order", "node")
            if order not in BATCH_ORDERS:
                raise ValueError(f"unknown order {order!r}")
            if len(msg["sudokus"]) > MAX_UDP_BOARDS:
                raise ValueError(f"more than {MAX_UDP_BOARDS} boards in one message")
            if not all(isinstance(b, str) and len(b) == 81 and b.isdigit() for b in msg["sudokus"]):
                raise ValueError("boards must be 81-digit strings")
            boards = torch.tensor([[int(c) for c in s] for s in msg["sudokus"]], dtype=torch.uint8).reshape(-1, 81)
            sols, st = self.solver.solve_many(boards, order=order)
            with self.lock:
                self.served += boards.shape[0]
            reply = {"type": "solution", "sudokus": ["".join(map(str, r.tolist())) for r in sols],
                     "status": st.tolist(), "address": self.id}
        elif msg.get("mode") == "reference":  # a whole board, the reference's /solve loop
            board = [row[:] for row in sudoku]
            try:
                out = self._reference_solve(board)
                reply = {"type": "solution", "sudoku": out, "solved": True, "address": self.id}
            except ReferenceNoReturn:
                reply = {"type": "solution", "sudoku": board, "solved": False, "no_return": True,
                         "address": self.id}
            with self.lock:
                self.served += 1
        else:  # a whole board handed over by a peer
            board = [row[:] for row in sudoku]
            out = self.solver.solve_sudoku(board)
            with self.lock:
                self.served += 1
            reply = {"type": "solution", "sudoku": board, "solved": out is not None, "address": self.id}
        if "task" in msg:
            reply["task"] = msg["task"]
        self.send(msg["address"], reply)
        self.broadcast_stats_soon()

    def request_solve(self, peer, sudoku, timeout=10.0, mode=None):
        """Hand a whole board to `peer` over UDP and wait for its solution
        (mode "reference": the peer runs the reference's /solve loop)."""
        msg = {"type": "solve", "sudoku": sudoku}
        if mode:
            msg["mode"] = mode
        return self._request(peer, msg, timeout)

    def request_solve_many(self, peer, boards81: List[str], order="node", timeout=10.0):
        """Hand a batch of boards (81-character strings) to `peer`, in
        messages of at most MAX_UDP_BOARDS boards; returns one reply with all
        `sudokus` and `status` in order (or the first reply with an error)."""
        boards81 = list(boards81)
        sols, status = [], []
        for lo in range(0, max(len(boards81), 1), MAX_UDP_BOARDS):
            rep = self._request(peer, {"type": "solve", "sudokus": boards81[lo:lo + MAX_UDP_BOARDS],
                                       "order": order}, timeout)
            if rep.get("error"):
                return rep
            sols += rep["sudokus"]
            status += rep["status"]
        return {"type": "solution", "sudokus": sols, "status": status, "address": peer}

    def _request(self, peer, msg, timeout):
        tid = next(self._task_ids)
        ev = threading.Event()
        self._tasks[tid] = [ev, None]
        try:
            msg = dict(msg, task=tid, address=self.id)
            self.send(peer, msg)
            if not ev.wait(timeout):
                raise TimeoutError(f"peer {peer} did not answer task {tid}")
            return self._tasks[tid][1]
        finally:
            self._tasks.pop(tid, None)

    # ------------------------------------------------------------- solving
    def _forward_target(self):
        if self.forward_threshold is None or self.solver.batcher.pending() < self.forward_threshold:
            return None
        with self.lock:
            peers = list(self.total_peers)
        if not peers:
            return None
        return peers[next(self._rr) % len(peers)]

    def _reference_solve(self, board):
        """node.py:534-557 exactly (solve_mode "reference"): the greedy cell
        loop on the GPU (sdk_peer_solve_seq) from this node's persistent
        state -- the reference P2PNode keeps partial_solution and
        tried_numbers_by_position across requests (node.py:149, 167), so its
        answer to a request can depend on the requests before it
        (tests/golden/golden_peer_seq.json).  Returns the board it leaves,
        valid or not, and counts one solved puzzle either way (node.py:467-
        474); raises ReferenceNoReturn where node.py never returns (the
        reference node would spin forever; this one goes on serving from the
        state the loop spun in)."""
        sols, st = self.solver.batcher.submit(as_boards(_flat(board)), "peer").result()
        if int(st[0]) == SDK_NO_RETURN:
            raise ReferenceNoReturn("the reference's /solve loop never returns on this board (node.py:429-464)")
        with self.solver.lock:
            self.solver.solved_puzzles += 1
        _copy_into(board, sols[0].tolist())
        return board

    def peer_sudoku_solve(self, sudoku):
        """node.py:534-557: solve one board for an HTTP client -- on this
        peer's GPUs, or on a peer's when this one is overloaded.  solve_mode
        "walk" (default) answers with node.py's recursive walk
        (SudokuSolver.solve_sudoku) or None; "reference" reproduces the
        reference's greedy /solve loop."""
        board = [row[:] for row in sudoku]
        peer = self._forward_target()
        mode = "reference" if self.solve_mode == "reference" else None
        out = None
        if peer is not None:
            try:
                rep = self.request_solve(peer, board, timeout=self.forward_timeout, mode=mode)
                if rep.get("error"):
                    raise PeerError(rep["error"])
                with self.lock:
                    self.forwarded += 1
                self.broadcast_stats_soon()
                if rep.get("no_return"):
                    raise ReferenceNoReturn("the reference's /solve loop never returns on this board")
                if rep.get("solved"):
                    _copy_into(board, _flat(rep["sudoku"]))
                    out = board
                return out
            except (TimeoutError, PeerError) as e:
                logger.warning("peer %s failed (%s), solving locally", peer, e)
        try:
            if mode:
                out = self._reference_solve(board)
            else:
                out = self.solver.solve_sudoku(board)
        finally:
            self.broadcast_stats_soon()
        return out

    def reset_solve_state(self):
        """Forget the reference-mode /solve state (what restarting a
        reference node does: a new P2PNode starts with both dicts empty)."""
        self.solver.batcher.reset_peer_state()

    def get_stats(self):
        """node.py:598-620: {"all": {...}, "nodes": [...]} (plus "solved_by",
        the per-node solved counts that the totals sum)."""
        with self.solver.lock:
            solved, validations = self.solver.solved_puzzles, self.solver.validations
        with self.lock:
            if solved:
                self.stats_solved[self.id] = max(self.stats_solved.get(self.id, 0), solved)
            self._merge_node(self.id, validations)
            self.all_stats["all"]["solved"] = sum(self.stats_solved.values())
            self.all_stats["all"]["validations"] = sum(n["validations"] for n in self.all_stats["nodes"])
            out = json.loads(json.dumps(self.all_stats))
            out["solved_by"] = [{"address": a, "solved": v} for a, v in sorted(self.stats_solved.items())]
            return out

    def network(self):
        with self.lock:
            return dict(self.all_peers) if self.all_peers else {self.id: []}

    # ---------------------------------------------------------- lifecycle
    def bind(self):
        self.sock.bind((self.host, self.port))
        if self.port == 0:
            self.port = self.sock.getsockname()[1]
            self.id = f"{self.host}:{self.port}"

    def connect_to_anchor_node(self):
        if self.anchor_node:
            self.send(self.anchor_node, {"type": "connect", "address": self.id})

    def run(self):
        logger.info("P2P node %s listening", self.id)
        self.connect_to_anchor_node()
        while not self.shutdown_flag:
            payload, _ = self.recv()
            if payload is None:
                continue
            try:
                self.handle_message(json.loads(payload.decode()))
            except Exception as e:  # node.py:642-644: keep serving
                logger.error("Error handling message: %s", e)

    def shutdown(self):
        self.broadcast_stats()
        self.broadcast({"type": "disconnect", "address": self.id})
        self.shutdown_flag = True
        self._pool.shutdown(wait=False)
        self.solver.close()


class SudokuHTTPServer(BaseHTTPRequestHandler):
    """node.py:661-704: POST /solve, GET /stats, GET /network."""

    p2p_node: P2PNode = None  # set by make_http_server
    protocol_version = "HTTP/1.1"  # keep-alive: load clients reuse connections

    def log_message(self, fmt, *args):
        logger.debug(fmt, *args)

    def _send_response(self, content, status=200):
        body = json.dumps(content).encode()
        self.send_response(status)
        self.send_header("Content-type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_POST(self):
        n = int(self.headers.get("Content-Length") or 0)
        data = self.rfile.read(n)
        if self.path != "/solve":
            return self._send_response({"error": "Invalid endpoint"}, 404)
        try:
            sudoku = json.loads(data.decode("utf-8"))["sudoku"]
            if not is_grid9(sudoku):
                raise ValueError("sudoku must be 9 lists of 9 integers")
            as_boards(sudoku)  # range validation
        except Exception as e:
            return self._send_response({"error": f"bad request: {e}"}, 400)
        t0 = time.time()
        try:
            solution = self.p2p_node.peer_sudoku_solve(sudoku)
        except ReferenceNoReturn as e:  # node.py would never answer
            return self._send_response({"error": str(e), "solution": None}, 500)
        logger.info("Execution time: %s", time.time() - t0)
        if solution:
            self._send_response(solution)
        else:
            self._send_response({"error": "No solution found", "solution": solution}, 400)

    def do_GET(self):
        if self.path == "/stats":
            self._send_response(self.p2p_node.get_stats())
        elif self.path == "/network":
            self._send_response(self.p2p_node.network())
        else:
            self._send_response({"error": "Invalid endpoint"}, 404)


class _Server(ThreadingHTTPServer):
    daemon_threads = True
    request_queue_size = 1024  # socketserver's default listen backlog (5) resets concurrent clients


def make_http_server(p2p_node: P2PNode, host: str, port: int) -> ThreadingHTTPServer:
    handler = type("BoundSudokuHTTPServer", (SudokuHTTPServer,), {"p2p_node": p2p_node})
    return _Server((host, port), handler)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Sudoku Solver Node", conflict_handler="resolve")
    ap.add_argument("-p", type=int, default=8001, help="HTTP port")
    ap.add_argument("-s", type=int, default=7000, help="P2P port")
    ap.add_argument("-a", help="Anchor node address (host:port)")
    ap.add_argument("-h", type=float, default=1, help="Handicap (delay in ms) for validation")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--gpus", default=None, help="comma list of local GPU indices (default: current)")
    ap.add_argument("--forward-threshold", type=int, default=None,
                    help="hand new boards to peers while this many wait for the local GPUs")
    ap.add_argument("--solve-mode", choices=("walk", "reference"), default="walk",
                    help="/solve answer: node.py's recursive walk (default) or the reference's greedy "
                         "peer_sudoku_solve loop, bit for bit (INTEGRATION.md §3)")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    devices = [int(x) for x in args.gpus.split(",")] if args.gpus else None
    node = P2PNode(args.host, args.s, anchor_node=args.a, handicap=args.h / 100,
                   backend=GpuSolverBackend(devices), forward_threshold=args.forward_threshold,
                   solve_mode=args.solve_mode)
    node.bind()
    httpd = make_http_server(node, args.host, args.p)
    threading.Thread(target=httpd.serve_forever, daemon=True).start()
    try:
        node.run()
    except KeyboardInterrupt:
        node.shutdown()
    finally:
        httpd.shutdown()


if __name__ == "__main__":
    main()
