"""ctypes binding of libsudoku_hip.so (the C ABI declared in include/sudoku_hip.h).

There is no fallback: if the library is missing or fails to load, every entry
point raises.  Build it with ``python -m sudoku_solver_distributed_amd.build``
(or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SDK_LIB selects another in-tree build of the same ABI (A/B experiments)
LIB_PATH = os.environ.get("SDK_LIB") or os.path.join(_HERE, "libsudoku_hip.so")

SDK_UNSOLVABLE = 0
SDK_SOLVED = 1
SDK_INVALID = -1
SDK_CANCELLED = -2
SDK_NO_RETURN = -4   # sdk_peer_solve_batch: node.py's /solve loop never returns
SDK_PEER_STATE_BYTES = 1600  # sdk_peer_solve_seq: one node's partial_solution + tried sets
SDK_ORDER_GEN = 0    # gen.py:6-28's walk (last row with an empty cell first)
SDK_ORDER_NODE = 1   # node.py:62-74's walk (row-major)
ORDERS = {"gen": SDK_ORDER_GEN, "node": SDK_ORDER_NODE}

# every symbol include/sudoku_hip.h declares
EXPORTS = (
    "sdk_workspace_bytes",
    "sdk_solve_batch",
    "sdk_solve_batch_grid",
    "sdk_solve_batches",
    "sdk_check_batch",
    "sdk_first_candidate_batch",
    "sdk_peer_solve_batch",
    "sdk_peer_solve_seq",
    "sdk_expand_frontier",
    "sdk_read_stats",
    "sdk_snapshot_stats",
    "sdk_verify_workspace",
    "sdk_last_error",
    "sdk_version",
    "sdk_device_cu_count",
    "sdk_set_solve_kernel",
    "sdk_set_plane_tuning",
    "sdk_set_plane_search",
)
SDK_KERNELS = {"auto": 1, "packed": 5, "plane": 6}
SDK_MAX_BATCHES = 32  # sdk_solve_batches: batches per launch
SDK_GRID_PIPELINED = 0x10000  # grid_waves flag: another launch is queued behind this one
# device symbol of each solve kernel (rocprofv3 Kernel_Name, profiles/pmc_<symbol>.json)
KERNEL_SYMBOLS = {1: "plane_kernel", 5: "solvep_kernel", 6: "plane_kernel"}

_lib = None


class SudokuHipError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load the HIP library (raises SudokuHipError if it is absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SudokuHipError(
            f"{LIB_PATH} not found: build it with `python -m sudoku_solver_distributed_amd.build`"
        )
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, i32, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_size_t
    L.sdk_workspace_bytes.restype = sz
    L.sdk_workspace_bytes.argtypes = []
    L.sdk_solve_batch.restype = i32
    L.sdk_solve_batch.argtypes = [vp, vp, vp, i64, vp, i32, i32, vp]
    L.sdk_solve_batch_grid.restype = i32
    L.sdk_solve_batch_grid.argtypes = [vp, vp, vp, i64, vp, i32, i32, vp, i32]
    pp = ctypes.POINTER(ctypes.c_void_p)
    L.sdk_solve_batches.restype = i32
    L.sdk_solve_batches.argtypes = [pp, pp, pp, ctypes.POINTER(ctypes.c_int64), i32, vp, i32, vp, i32]
    L.sdk_check_batch.restype = i32
    L.sdk_check_batch.argtypes = [vp, vp, i64, i32, vp]
    L.sdk_first_candidate_batch.restype = i32
    L.sdk_first_candidate_batch.argtypes = [vp, vp, vp, i64, vp]
    L.sdk_peer_solve_batch.restype = i32
    L.sdk_peer_solve_batch.argtypes = [vp, vp, vp, vp, i64, vp]
    L.sdk_peer_solve_seq.restype = i32
    L.sdk_peer_solve_seq.argtypes = [vp, vp, vp, vp, i64, vp, vp]
    L.sdk_expand_frontier.restype = i32
    L.sdk_expand_frontier.argtypes = [vp, i64, vp, vp, vp, i64, i32, vp]
    L.sdk_read_stats.restype = i32
    L.sdk_read_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), i32, vp]
    L.sdk_snapshot_stats.restype = i32
    L.sdk_snapshot_stats.argtypes = [vp, vp, vp]
    L.sdk_verify_workspace.restype = i32
    L.sdk_verify_workspace.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), vp]
    L.sdk_last_error.restype = ctypes.c_char_p
    L.sdk_last_error.argtypes = []
    L.sdk_version.restype = ctypes.c_char_p
    L.sdk_version.argtypes = []
    L.sdk_device_cu_count.restype = i32
    L.sdk_device_cu_count.argtypes = []
    L.sdk_set_solve_kernel.restype = i32
    L.sdk_set_solve_kernel.argtypes = [i32]
    L.sdk_set_plane_tuning.restype = i32
    L.sdk_set_plane_tuning.argtypes = [i32, i32, i32, i32]
    L.sdk_set_plane_search.restype = i32
    L.sdk_set_plane_search.argtypes = [i32]
    _lib = L
    return L


def active_kernel() -> int:
    """The solve kernel selection now (SDK_KERNEL_*; AUTO runs the plane kernel
    at bench-sized batches)."""
    L = load()
    cur = L.sdk_set_solve_kernel(0)
    L.sdk_set_solve_kernel(cur)
    return cur


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().sdk_last_error().decode(errors="replace")
        raise SudokuHipError(f"{what} failed ({rc}): {msg}")


def order_code(order) -> int:
    """'gen' | 'node' | SDK_ORDER_* -> SDK_ORDER_*."""
    if isinstance(order, str):
        if order not in ORDERS:
            raise ValueError(f"order must be one of {sorted(ORDERS)}")
        return ORDERS[order]
    if order not in (SDK_ORDER_GEN, SDK_ORDER_NODE):
        raise ValueError(f"bad order {order!r}")
    return int(order)
