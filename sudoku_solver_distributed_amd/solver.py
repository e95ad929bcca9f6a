"""Device-side batch API over the C ABI (include/sudoku_hip.h).

PyTorch is plumbing here: it owns device memory, streams and
``torch.distributed``; all Sudoku work runs in libsudoku_hip.so.  Nothing in
this module falls back to a CPU path -- without a GPU or without the library
every call raises.

Boards are ``uint8`` tensors of shape ``(n, 81)`` (row-major, 0 = empty).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import SDK_CANCELLED, SDK_INVALID, SDK_NO_RETURN, SDK_SOLVED, SDK_UNSOLVABLE, SudokuHipError

__all__ = [
    "BatchSolver", "get_solver", "as_boards", "SDK_SOLVED", "SDK_UNSOLVABLE",
    "SDK_INVALID", "SDK_CANCELLED", "SDK_NO_RETURN", "SudokuHipError",
]


def _require_gpu(device) -> torch.device:
    if not torch.cuda.is_available():
        raise SudokuHipError("no ROCm GPU visible: the Sudoku solver runs only on the HIP path")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise SudokuHipError(f"device {dev} is not a GPU device")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def as_boards(x, device=None, max_value: int = 9) -> torch.Tensor:
    """Anything board-like -> contiguous (n, 81) uint8 tensor (host or device).

    Accepts a 9x9 list of lists (the reference's board type), a list of such
    boards, an 81-char string, numpy arrays and tensors.  Raises ValueError on
    a cell outside 0..max_value: solving takes 0..9 (the reference's walk
    would silently compare other values), the check kernels take any byte
    (0..255, the reference's sum / set arithmetic on them)."""
    if isinstance(x, str):
        x = [int(c) for c in x]
    if isinstance(x, torch.Tensor):
        t = x
    else:
        a = np.asarray(x)
        if a.dtype == object:
            raise ValueError("ragged board")
        if a.size and (a.min() < 0 or a.max() > max_value):
            raise ValueError(f"board cells must be integers 0..{max_value}")
        t = torch.from_numpy(np.ascontiguousarray(a.astype(np.uint8)))
    if t.numel() % 81 != 0:
        raise ValueError(f"board data of {t.numel()} cells is not a multiple of 81")
    t = t.reshape(-1, 81)
    if t.dtype != torch.uint8:
        if t.numel() and (int(t.min()) < 0 or int(t.max()) > max_value):
            raise ValueError(f"board cells must be integers 0..{max_value}")
        t = t.to(torch.uint8)
    if device is not None:
        t = t.to(device, non_blocking=True)
    return t.contiguous()


# Launches in flight and waves per SIMD in each launch's grid
# (solve_inflight's defaults).  A full grid (4 waves per SIMD) leaves a
# launch's drain to the next launch only as its waves exit; smaller grids
# keep several launches resident together.  Each launch in flight has its
# own stream, and streams beyond the process's hardware queues
# ($GPU_MAX_HW_QUEUES, HIP's default 4) share one and serialise: with 8 or
# more queues six launches at 1 wave per SIMD (four resident, two queued),
# else three at 2 (585-593 against 534-537 M boards/s).
GRID_WAVES_INFLIGHT = 2


def default_inflight():
    """(launches in flight, grid waves per SIMD) for this process's hardware
    queue count."""
    try:
        hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        hwq = 4
    return (6, 1) if hwq >= 8 else (3, GRID_WAVES_INFLIGHT)


def pipelined_launches(n_launches: int, inflight: int, pool_last: Optional[int] = None):
    """solve_inflight's per-launch SDK_GRID_PIPELINED flags: every launch
    but the last `pool_last` (default: half the launches in flight, rounded
    up; with one in flight none -- nothing can take a drained launch's
    slots, so each shares its tail through the XCD pool)."""
    if pool_last is None:
        last = n_launches if inflight == 1 else (inflight + 1) // 2
    else:
        last = max(0, pool_last)
    return [i < n_launches - last for i in range(n_launches)]


def _grid_arg(grid_waves: int, pipelined: bool) -> int:
    """sdk_solve_batch_grid / sdk_solve_batches' grid argument: waves per
    SIMD, | SDK_GRID_PIPELINED for a launch with another queued behind it."""
    g = int(grid_waves)
    if g >= _lib.SDK_GRID_PIPELINED:
        raise ValueError("grid_waves must be below 65536")
    return g | (_lib.SDK_GRID_PIPELINED if pipelined and g >= 0 else 0)  # (negative: the library's -2)


class BatchSolver:
    """One per device.  Holds the device workspace of the C ABI.

    Thread-safe: the workspace is single-stream (include/sudoku_hip.h), so
    every call that uses it (solve, stats) runs under one lock, and a call on
    a different stream than the previous one first makes its stream wait for
    the previous stream's work."""

    def __init__(self, device=None):
        self.device = _require_gpu(device)
        self.lib = _lib.load()
        self._lock = threading.Lock()
        self._last_stream = None
        # held by callers that need solve + stats as one step (node.py's backend)
        self.op_lock = threading.RLock()
        self._pool = None  # the solver's streams (_stream_pool)
        self._slots = None  # solve_inflight's (solver, stream) slots (_slot_solvers)
        self._pool_lock = threading.Lock()  # builds _pool / _slots once across threads
        with torch.cuda.device(self.device):
            self.workspace = torch.zeros(int(self.lib.sdk_workspace_bytes()), dtype=torch.uint8,
                                         device=self.device)

    # ------------------------------------------------------------ helpers
    def _stream(self, stream) -> int:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return int(s.cuda_stream)

    def _ws_stream(self, stream) -> int:
        """Stream handle for a workspace call (caller holds self._lock)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if self._last_stream is not None and self._last_stream != s:
            ev = torch.cuda.Event()
            ev.record(self._last_stream)
            s.wait_event(ev)
        self._last_stream = s
        return int(s.cuda_stream)

    def _dev(self, t: torch.Tensor) -> torch.Tensor:
        if t.device != self.device:
            t = t.to(self.device)
        return t.contiguous()

    # -------------------------------------------------------------- solve
    def solve(self, puzzles, out: Optional[torch.Tensor] = None, status: Optional[torch.Tensor] = None,
              ordered: bool = False, order="gen", stream=None, grid_waves: int = 0, pipelined: bool = False
              ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Solve every board with the reference walk `order` ("gen":
        gen.py:6-28, "node": node.py:62-74).  Asynchronous on the stream;
        returns (solutions uint8 (n,81), status int32 (n,)).  grid_waves > 0
        caps the lane-per-board kernel's grid at that many waves per SIMD
        (sdk_solve_batch_grid; solve_inflight's co-resident launches).
        pipelined: another launch follows on the device (SDK_GRID_PIPELINED:
        drained waves exit instead of sharing the last boards); results never
        depend on it."""
        p = self._dev(as_boards(puzzles))
        n = p.shape[0]
        if out is None:
            out = torch.empty_like(p)
        if status is None:
            status = torch.empty(n, dtype=torch.int32, device=self.device)
        if out.shape != p.shape or out.dtype != torch.uint8 or not out.is_contiguous():
            raise ValueError("out must be a contiguous (n, 81) uint8 tensor")
        if status.shape != (n,) or status.dtype != torch.int32:
            raise ValueError("status must be an (n,) int32 tensor")
        with self._lock, torch.cuda.device(self.device):
            rc = self.lib.sdk_solve_batch_grid(p.data_ptr(), out.data_ptr(), status.data_ptr(), n,
                                               self.workspace.data_ptr(), _lib.order_code(order),
                                               1 if ordered else 0, self._ws_stream(stream),
                                               _grid_arg(grid_waves, pipelined))
        _lib.check(rc, "sdk_solve_batch_grid")
        return out, status

    def solve_batches(self, batches, outs, statuses, order="gen", stream=None, grid_waves: int = 0,
                      pipelined: bool = False):
        """Several device batches solved by ONE launch sequence
        (sdk_solve_batches): the lane-per-board kernel's queue runs over the
        batches laid end to end and drains once, so batches too small to fill
        the GPU on their own (a multi-GPU shard of one step) keep every lane
        busy.  Each batch's outputs are exactly solve()'s.  At most
        SDK_MAX_BATCHES (32) batches; unordered only."""
        if not (len(batches) == len(outs) == len(statuses)) or not 1 <= len(batches) <= _lib.SDK_MAX_BATCHES:
            raise ValueError(f"1..{_lib.SDK_MAX_BATCHES} batches, one out and one status tensor each")
        ps = [self._dev(as_boards(b)) for b in batches]
        for p, o, st in zip(ps, outs, statuses):
            if o.shape != p.shape or o.dtype != torch.uint8 or not o.is_contiguous() or o.device != self.device:
                raise ValueError("each out must be a contiguous (n, 81) uint8 tensor on the solver's device")
            if st.shape != (p.shape[0],) or st.dtype != torch.int32 or st.device != self.device:
                raise ValueError("each status must be an (n,) int32 tensor on the solver's device")
        k = len(ps)
        arr = ctypes.c_void_p * k
        ins = arr(*[p.data_ptr() for p in ps])
        out_p = arr(*[o.data_ptr() for o in outs])
        st_p = arr(*[st.data_ptr() for st in statuses])
        ns = (ctypes.c_int64 * k)(*[p.shape[0] for p in ps])
        with self._lock, torch.cuda.device(self.device):
            rc = self.lib.sdk_solve_batches(ins, out_p, st_p, ns, k, self.workspace.data_ptr(), _lib.order_code(order),
                                            self._ws_stream(stream), _grid_arg(grid_waves, pipelined))
        _lib.check(rc, "sdk_solve_batches")
        return list(zip(outs, statuses))

    def _stream_pool(self, k: int):
        """The solver's own streams, created once and shared by solve_host
        (compute, copy-in) and solve_inflight (one per slot): a process has
        few hardware queues (4), and streams past them share a queue and
        serialise."""
        with self._pool_lock:
            if self._pool is None:
                self._pool = []
            while len(self._pool) < k:
                self._pool.append(torch.cuda.Stream(self.device))
            return self._pool[:k]

    def _slot_solvers(self, inflight: int):
        """[self] + inflight - 1 more solvers on this device, each with its
        own workspace (~1.1 GB: per-lane stacks) and its own stream."""
        streams = self._stream_pool(inflight)
        with self._pool_lock:
            if self._slots is None:
                self._slots = [(self, streams[0])]
            while len(self._slots) < inflight:
                self._slots.append((BatchSolver(self.device), streams[len(self._slots)]))
            return self._slots[:inflight]

    def solve_inflight(self, batches, outs, statuses, inflight: Optional[int] = None, order="gen",
                       ordered: bool = False, launch_events=None, grid_waves: Optional[int] = None, group: int = 1,
                       pool_last: Optional[int] = None):
        """Solve a sequence of device batches with up to `inflight` launches
        in flight on this GPU: batch i runs on slot i % inflight (its own
        workspace and stream), so a launch's end -- its last boards draining
        while most lanes idle -- overlaps the next launches instead of
        idling the GPU.  inflight / grid_waves (waves per SIMD in each
        launch's grid; 0 = a full grid): default_inflight() -- six launches
        at 1 wave per SIMD with >= 8 hardware queues, else three at 2.  Each
        launch is a whole sdk_solve_batch_grid; results are those of solve().  outs[i] / statuses[i] receive batch i (buffers of
        batches that may be in flight together must not alias).  The
        caller's current stream waits for every batch; nothing synchronises
        the host.  launch_events: optional list that receives a (start, end)
        timing-event pair per launch, recorded on its slot's stream.
        group > 1: each launch solves `group` consecutive batches at once
        (solve_batches, one queue over them; unordered only) -- the
        strong-scaling steps, where one GPU's share of a step is too small to
        fill the GPU alone.  The last `pool_last` launches run unpipelined
        -- little is queued behind them, so their drained waves share the last
        boards through the XCD tail pool; every earlier launch is pipelined
        (its drained waves leave their slots to the launches on the other
        streams).  Default: half the launches in flight, rounded up (three of
        six: +1.3 % over six and over none at 20 steps, equal at 100; the
        N = 8 rank's 20 steps +12 %); with one launch in flight
        nothing can use the slots, so every launch shares its tail."""
        if inflight is None:
            inflight, gw = default_inflight()
            grid_waves = gw if grid_waves is None else grid_waves
        if inflight < 1:
            raise ValueError("inflight must be >= 1")
        if not 1 <= group <= _lib.SDK_MAX_BATCHES or (group > 1 and ordered):
            raise ValueError(f"group must be 1..{_lib.SDK_MAX_BATCHES} (and 1 in ordered mode)")
        if not (len(batches) == len(outs) == len(statuses)):
            raise ValueError("one out and one status tensor per batch")
        if grid_waves is None:
            grid_waves = GRID_WAVES_INFLIGHT if inflight > 1 else 0
        slots = self._slot_solvers(inflight)
        caller = torch.cuda.current_stream(self.device)
        # every batch in its final form (contiguous uint8 on this device)
        # BEFORE `ready` is recorded: a conversion enqueued on the caller
        # stream after it would race the slot stream's kernel
        batches = [self._dev(as_boards(b)) for b in batches]
        ready = torch.cuda.Event()
        ready.record(caller)
        for _, s in slots:
            s.wait_event(ready)
        pipes = pipelined_launches((len(batches) + group - 1) // group, inflight, pool_last)
        for i, lo in enumerate(range(0, len(batches), group)):
            solver, s = slots[i % inflight]
            pipe = pipes[i]
            bs, os_, sts = batches[lo:lo + group], outs[lo:lo + group], statuses[lo:lo + group]
            if launch_events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
            if group == 1:
                solver.solve(bs[0], out=os_[0], status=sts[0], order=order, ordered=ordered, stream=s,
                             grid_waves=grid_waves, pipelined=pipe)
            else:
                solver.solve_batches(bs, os_, sts, order=order, stream=s, grid_waves=grid_waves, pipelined=pipe)
            if launch_events is not None:
                e1.record(s)
                launch_events.append((e0, e1))
            for t in (*bs, *os_, *sts):  # caller-stream allocations used on the slot's stream
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(s)
        for _, s in slots:
            caller.wait_stream(s)
        return list(zip(outs, statuses))

    def inflight_stats(self, reset: bool = False) -> dict:
        """stats() summed over the solve_inflight slots' workspaces."""
        tot = None
        for solver, s in (self._slots or [(self, None)]):
            st = solver.stats(reset=reset, stream=s)
            tot = st if tot is None else {k: (tot[k] + v if k != "best" else min(tot[k], v)) for k, v in st.items()}
        return tot

    def solve_host(self, puzzles: torch.Tensor, order="gen", chunk: int = 1 << 18,
                   out: Optional[torch.Tensor] = None, status: Optional[torch.Tensor] = None
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Host boards in, host solutions and statuses out (the serving
        path), pipelined: chunk i+1 is copied in on one stream and chunk i-1
        copied out on another while chunk i is solved, so both PCIe
        directions overlap the kernel.  Give pinned host tensors (`out` /
        `status` are allocated pinned when omitted); pageable input is copied
        synchronously.  Same results as solve(); returns when all is back."""
        p = as_boards(puzzles)
        if p.device.type != "cpu":
            raise ValueError("solve_host takes host boards; use solve() for device tensors")
        n = p.shape[0]
        if out is None:
            out = torch.empty((n, 81), dtype=torch.uint8).pin_memory()
        if status is None:
            status = torch.empty(n, dtype=torch.int32).pin_memory()
        if out.shape != (n, 81) or out.dtype != torch.uint8 or out.device.type != "cpu":
            raise ValueError("out must be a host (n, 81) uint8 tensor")
        if status.shape != (n,) or status.dtype != torch.int32 or status.device.type != "cpu":
            raise ValueError("status must be a host (n,) int32 tensor")
        if n == 0:
            return out, status
        d_in = torch.empty((n, 81), dtype=torch.uint8, device=self.device)
        d_out = torch.empty_like(d_in)
        d_st = torch.empty(n, dtype=torch.int32, device=self.device)
        caller = torch.cuda.current_stream(self.device)
        # three streams in all: the solver's two (shared with solve_inflight's
        # slots, created once) and the caller's for the copies out.  A
        # process has few hardware queues (4); past them streams share one,
        # and a copy queued behind a solve serialises the pipeline.
        compute, h2d = self._stream_pool(2)
        d2h = caller
        compute.wait_stream(caller)
        h2d.wait_stream(caller)  # the device buffers are caller-stream allocations
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            with torch.cuda.stream(h2d):
                d_in[lo:hi].copy_(p[lo:hi], non_blocking=True)
            compute.wait_stream(h2d)
            self.solve(d_in[lo:hi], out=d_out[lo:hi], status=d_st[lo:hi], order=order, stream=compute)
            d2h.wait_stream(compute)
            with torch.cuda.stream(d2h):
                out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
                status[lo:hi].copy_(d_st[lo:hi], non_blocking=True)
        for t in (d_in, d_out, d_st):
            t.record_stream(h2d)
            t.record_stream(compute)
        d2h.synchronize()
        return out, status

    def check(self, grids, mode: int = 0, stream=None) -> torch.Tensor:
        """mode 0: Sudoku.check (sudoku.py:119-140); mode 1: node.py:82-116."""
        g = self._dev(as_boards(grids, max_value=255))
        ok = torch.empty(g.shape[0], dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.sdk_check_batch(g.data_ptr(), ok.data_ptr(), g.shape[0], mode, self._stream(stream))
        _lib.check(rc, "sdk_check_batch")
        return ok

    def first_candidate(self, grids, cells, stream=None) -> torch.Tensor:
        """node.py:76-80 per (board, cell) task; 0 means None."""
        g = self._dev(as_boards(grids, max_value=255))
        c = self._dev(torch.as_tensor(cells, dtype=torch.int32).reshape(-1))
        if c.shape[0] != g.shape[0]:
            raise ValueError("one cell index per board")
        num = torch.empty(g.shape[0], dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.sdk_first_candidate_batch(g.data_ptr(), c.data_ptr(), num.data_ptr(), g.shape[0],
                                                    self._stream(stream))
        _lib.check(rc, "sdk_first_candidate_batch")
        return num

    def peer_solve(self, boards, stream=None):
        """node.py:534-557 P2PNode.peer_sudoku_solve (the reference's HTTP
        /solve greedy loop) per board: (boards it leaves (n,81), status (n,),
        validations (n,)); status SDK_SOLVED / SDK_UNSOLVABLE (check passed /
        failed) or SDK_NO_RETURN (node.py never returns on that board)."""
        g = self._dev(as_boards(boards))
        n = g.shape[0]
        out = torch.empty_like(g)
        st = torch.empty(n, dtype=torch.int32, device=self.device)
        val = torch.empty(n, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.sdk_peer_solve_batch(g.data_ptr(), out.data_ptr(), st.data_ptr(), val.data_ptr(), n,
                                               self._stream(stream))
        _lib.check(rc, "sdk_peer_solve_batch")
        return out, st, val

    def new_peer_state(self) -> torch.Tensor:
        """A new P2PNode's persistent /solve state (partial_solution and
        tried_numbers_by_position, node.py:149, 167) for peer_solve_seq."""
        return torch.zeros(_lib.SDK_PEER_STATE_BYTES, dtype=torch.uint8, device=self.device)

    def peer_solve_seq(self, boards, state: torch.Tensor, stream=None):
        """The same /solve loop on ONE node serving the boards as requests in
        order (sdk_peer_solve_seq): each request starts from the node state
        the previous one left; `state` (new_peer_state()) is updated in place.
        Returns (boards left, status, validations per request)."""
        g = self._dev(as_boards(boards))
        if state.device != self.device or state.dtype != torch.uint8 or state.numel() != _lib.SDK_PEER_STATE_BYTES:
            raise ValueError("state must be a new_peer_state() tensor on this device")
        n = g.shape[0]
        out = torch.empty_like(g)
        st = torch.empty(n, dtype=torch.int32, device=self.device)
        val = torch.empty(n, dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.sdk_peer_solve_seq(g.data_ptr(), out.data_ptr(), st.data_ptr(), val.data_ptr(), n,
                                             state.data_ptr(), self._stream(stream))
        _lib.check(rc, "sdk_peer_solve_seq")
        return out, st, val

    def expand(self, nodes, order="gen", stream=None) -> torch.Tensor:
        """One frontier level (sdk_expand_frontier); synchronises to size it."""
        nd = self._dev(as_boards(nodes))
        n = nd.shape[0]
        tmp = torch.empty_like(nd)
        offsets = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        cap = 9 * n
        children = torch.empty((max(cap, 1), 81), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.sdk_expand_frontier(nd.data_ptr(), n, tmp.data_ptr(), offsets.data_ptr(),
                                              children.data_ptr(), cap, _lib.order_code(order),
                                              self._stream(stream))
        _lib.check(rc, "sdk_expand_frontier")
        total = int(offsets[n].item()) if n else 0
        if total > cap:
            raise SudokuHipError(f"frontier overflow: {total} > {cap}")
        return children[:total]

    def stats(self, reset: bool = False, stream=None) -> dict:
        out = (ctypes.c_int64 * 6)()
        with self._lock, torch.cuda.device(self.device):
            rc = self.lib.sdk_read_stats(self.workspace.data_ptr(), out, 1 if reset else 0, self._ws_stream(stream))
        _lib.check(rc, "sdk_read_stats")
        return {"finished": out[0], "solved": out[1], "guesses": out[2], "sweeps": out[3], "best": out[4],
                "deferred": out[5]}

    def verify(self, stream=None) -> dict:
        """Every board handed to this workspace's solve kernels since the last
        stats(reset=True) has its answer, and no kernel reported an error
        (sdk_verify_workspace; synchronises the stream).  Returns {"assigned",
        "finished", "error"}; raises SudokuHipError otherwise -- a board a
        kernel took but could not finish (a tail-pool record never published,
        DESIGN.md §3) is never a silent stale output."""
        out = (ctypes.c_int64 * 4)()
        with self._lock, torch.cuda.device(self.device):
            rc = self.lib.sdk_verify_workspace(self.workspace.data_ptr(), out, self._ws_stream(stream))
        if rc == -3:
            raise SudokuHipError(self.lib.sdk_last_error().decode(errors="replace"))
        _lib.check(rc, "sdk_verify_workspace")
        return {"assigned": out[0], "finished": out[1], "error": out[2]}

    def verify_inflight(self) -> dict:
        """verify() over the solve_inflight slots' workspaces (summed)."""
        tot = {"assigned": 0, "finished": 0, "error": 0}
        for solver, s in (self._slots or [(self, None)]):
            for k, v in solver.verify(stream=s).items():
                tot[k] += v
        return tot

    def stats_snapshot(self, stream=None) -> torch.Tensor:
        """The counters of stats() as a device int64 (6,) tensor, copied
        asynchronously in stream order with this workspace's solves
        (sdk_snapshot_stats): the difference of two snapshots around a solve
        is that solve's own work, with no host synchronisation."""
        out = torch.empty(6, dtype=torch.int64, device=self.device)
        with self._lock, torch.cuda.device(self.device):
            rc = self.lib.sdk_snapshot_stats(self.workspace.data_ptr(), out.data_ptr(), self._ws_stream(stream))
        _lib.check(rc, "sdk_snapshot_stats")
        return out

    # ------------------------------------------------------ frontier split
    def frontier(self, board, target: int = 4096, max_levels: int = 81, order="gen") -> torch.Tensor:
        """Expand one board's search tree level by level (in the walk's
        order) until the frontier holds >= target nodes, or the next level
        would be narrower (dead branches outnumber new ones), or nothing is
        left to split.  Returns the frontier, in walk order."""
        nodes = self._dev(as_boards(board))
        for _ in range(max_levels):
            if nodes.shape[0] >= target or nodes.shape[0] == 0:
                break
            children = self.expand(nodes, order=order)
            if children.shape[0] == nodes.shape[0] and torch.equal(children, nodes):
                break  # every node already solved: nothing left to split
            if 0 < children.shape[0] < nodes.shape[0]:
                break  # narrowing: keep the wider level
            nodes = children
        return nodes

    def solve_one_split(self, board, target: int = 4096, order="gen") -> Tuple[bool, torch.Tensor]:
        """Single hard board: frontier split over all waves of this GPU, then
        an ordered solve; returns (solved, grid81)."""
        root = self._dev(as_boards(board))
        if root.shape[0] != 1:
            raise ValueError("solve_one_split takes exactly one board")
        nodes = self.frontier(root, target, order=order)
        if nodes.shape[0] == 0:
            return False, root[0].clone()
        sols, st = self.solve(nodes, ordered=True, order=order)
        hit = torch.nonzero(st == SDK_SOLVED)
        if hit.numel() == 0:
            return False, root[0].clone()
        return True, sols[int(hit[0, 0].item())].clone()


_SOLVERS = {}
_SOLVERS_LOCK = threading.Lock()


def get_solver(device=None) -> BatchSolver:
    dev = _require_gpu(device)
    with _SOLVERS_LOCK:
        s = _SOLVERS.get(dev.index)
        if s is None:
            s = _SOLVERS[dev.index] = BatchSolver(dev)
        return s
