"""C ABI: the library loads without a GPU and exports every symbol that
include/sudoku_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    with open(os.path.join(ROOT, "include", "sudoku_hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(sdk_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = _declared()
    assert "sdk_solve_batch" in names and "sdk_check_batch" in names
    from sudoku_solver_distributed_amd import _lib
    assert sorted(_lib.EXPORTS) == names


def test_library_exports_all_symbols():
    from sudoku_solver_distributed_amd import _lib, build
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    L = _lib.load()
    assert L.sdk_workspace_bytes() >= 64
    assert b"gfx950" in L.sdk_version()


def test_code_object_is_gfx950():
    from sudoku_solver_distributed_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "sudoku_solver_distributed_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith(".py"):
                with open(os.path.join(dirpath, fn)) as f:
                    src = f.read()
                assert "oracle" not in re.sub(r"#.*", "", src).replace("oracle/", ""), fn


def test_solver_raises_without_gpu():
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sudoku_solver_distributed_amd.solver import BatchSolver, SudokuHipError
    with pytest.raises(SudokuHipError):
        BatchSolver()


def test_no_wide_store_data_hazard():
    """Every >64-bit store in the product kernels has a wait state before its
    data registers are rewritten (scripts/store_hazard_check.py: hipcc does
    not pad buffer stores with a register soffset; plane_kernel.h
    PlaneStack::push pads its own)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import store_hazard_check as H
    st = "buffer_store_dwordx4 v[0:3], v64, s[0:3], s4 offen"
    assert H.scan([st, "v_bitop3_b32 v1, v28, 1, v56 bitop3:0x80"])  # the pattern that corrupted the stack
    # the window is two wait states: a write at distance 2, or behind one
    # s_nop 0, is still a hazard; s_nop 1 (two states) or two instructions clear it
    assert H.scan([st, "s_movk_i32 s0, 0x60", ";;#ASMSTART", "v_mov_b32 v3, v9"])
    assert H.scan([st, "s_nop 0", "v_mov_b32 v2, v9"])
    assert H.scan(["global_store_dwordx3 v5, v[10:12], s[2:3]", "v_add_u32 v12, v1, v2"])
    assert not H.scan([st, "s_nop 1", "v_mov_b32 v1, v2"])
    assert not H.scan([st, "s_mov_b32 s0, 1", "s_mov_b32 s1, 1", "v_mov_b32 v1, v2"])
    assert not H.scan([st, "v_mov_b32 v64, v2"])  # the address is read at issue
    assert not H.scan(["buffer_store_dwordx2 v[0:1], v64, s[0:3], s4 offen", "v_mov_b32 v1, v2"])  # 64-bit
    assert H.main() == 0  # every build variant (build.VARIANTS)


def test_plane_tuning_arguments():
    """sdk_set_plane_tuning (host-only code, no GPU needed): out-of-range
    values are refused and change nothing, negatives keep a knob, all four
    negative restore the defaults."""
    from sudoku_solver_distributed_amd import _lib, build
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.sdk_set_plane_tuning
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int] * 4
    assert f(65, -1, -1, -1) == -1      # refill > 64
    assert f(0, -1, -1, -1) == -1       # refill 0: a wave would never refill
    assert f(-1, 41, -1, -1) == -1      # tail > 40 (LDS records)
    assert f(-1, -1, 3, -1) == -1       # tail mode 1 / 2 only
    assert f(-1, -1, 0, -1) == -1
    assert f(-1, -1, 2, -1) == 0        # the per-XCD tail pool
    assert f(8, 40, 1, 32) == 0
    assert f(-1, 0, -1, -1) == 0        # tail off
    assert f(-1, -1, -1, -1) == 0       # defaults back


def test_solve_batch_grid_arguments():
    """sdk_solve_batch_grid's argument check runs before any device call: a
    negative grid is a bad argument (-2), an empty batch returns 0."""
    from sudoku_solver_distributed_amd import _lib, build
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.sdk_solve_batch_grid
    f.restype = ctypes.c_int
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    f.argtypes = [vp, vp, vp, ctypes.c_int64, vp, i32, i32, vp, i32]
    assert f(16, 16, 16, 1, 16, 0, 0, None, -1) == -2
    assert f(None, None, None, 0, None, 0, 0, None, 2) == 0
    assert f(None, None, None, 0, None, 7, 0, None, 2) == -2  # unknown order
    assert f(None, None, None, 0, None, 0, 0, None, 2 | _lib.SDK_GRID_PIPELINED) == 0  # the pipelined flag


def test_plane_tuning_rejects_oversized_chunks():
    """A claimed chunk is staged and converted in one go, so at most 64
    boards: larger chunk values are refused, nothing changed.
    Host-side only (no GPU call)."""
    from sudoku_solver_distributed_amd import _lib
    L = _lib.load()
    try:
        assert L.sdk_set_plane_tuning(-1, -1, -1, 65) == -1
        assert L.sdk_set_plane_tuning(-1, -1, -1, 255) == -1
        assert L.sdk_set_plane_tuning(-1, -1, -1, 64) == 0
        assert L.sdk_set_plane_tuning(-1, -1, -1, 0) == 0
    finally:
        L.sdk_set_plane_tuning(-1, -1, -1, -1)


def test_plane_search_knob_range():
    """sdk_set_plane_search: the setting in effect before the call back (the
    default's value, 128, when nothing overrode it), out-of-range values
    refused with -2 and nothing changed.  Host-side only."""
    from sudoku_solver_distributed_amd import _lib
    L = _lib.load()
    try:
        L.sdk_set_plane_search(-1)
        assert L.sdk_set_plane_search(48) == 128
        assert L.sdk_set_plane_search(0) == 48
        assert L.sdk_set_plane_search(1 << 24) == -2
        assert L.sdk_set_plane_search(-1) == 0
        assert L.sdk_set_plane_search(-1) == 128
    finally:
        L.sdk_set_plane_search(-1)


def test_verify_workspace_arguments():
    """sdk_verify_workspace refuses a null workspace (-2) without a GPU."""
    from sudoku_solver_distributed_amd import _lib
    L = _lib.load()
    assert L.sdk_verify_workspace(None, None, None) == -2


def test_pipelined_launch_choice():
    """solve_inflight's SDK_GRID_PIPELINED choice (host logic): all but the
    last half of the launches in flight; none back to back; pool_last
    overrides; the flag is OR-ed into the grid argument, negatives pass to
    the library's own check."""
    from sudoku_solver_distributed_amd import _lib
    from sudoku_solver_distributed_amd.solver import _grid_arg, pipelined_launches
    assert pipelined_launches(10, 6) == [True] * 7 + [False] * 3
    assert pipelined_launches(2, 6) == [False, False]
    assert pipelined_launches(5, 1) == [False] * 5
    assert pipelined_launches(4, 3, pool_last=0) == [True] * 4
    assert pipelined_launches(4, 3, pool_last=1) == [True, True, True, False]
    assert pipelined_launches(0, 6) == []
    assert _grid_arg(1, True) == 1 | _lib.SDK_GRID_PIPELINED and _grid_arg(2, False) == 2
    assert _grid_arg(-1, True) == -1
    with pytest.raises(ValueError):
        _grid_arg(1 << 16, False)
