"""CPU checks of the lane-per-board solver (csrc/lane_solver.h, selected on
the GPU with SDK_SOLVE_KERNEL=l): the same header compiled for the host
with g++ (tests/native/), compared with the oracle on the goldens, on
hard 17-clue boards, and -- for the device board loader load_dw -- against
the plain byte loader at every start offset."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import b81, load_golden
from oracle import oracle as O

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def _build(tmp, name):
    out = os.path.join(tmp, f"lib{name}.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-o", out,
                           os.path.join(NATIVE, f"{name}.cpp")])
    return ctypes.CDLL(out)


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    lib = _build(str(tmp_path_factory.mktemp("lane")), "lane_host")
    lib.lane_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    return lib


@pytest.fixture(scope="module")
def host_dw(tmp_path_factory):
    lib = _build(str(tmp_path_factory.mktemp("lanedw")), "lane_host_dw")
    lib.check_load_dw.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.check_load_dw.restype = ctypes.c_int64
    return lib


def _solve(lib, boards, node_order=0):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
    out = np.zeros_like(boards)
    st = np.zeros(len(boards), dtype=np.int32)
    g, p = ctypes.c_uint64(), ctypes.c_uint64()
    lib.lane_solve_batch(boards.ctypes.data, out.ctypes.data, st.ctypes.data, len(boards), node_order,
                         ctypes.byref(g), ctypes.byref(p))
    return out, st


def test_lane_golden_gen(host):
    cases = load_golden("golden_gen.json")
    boards = np.array([b81(c["puzzle"]) for c in cases], dtype=np.uint8)
    out, st = _solve(host, boards)
    for c, o, s in zip(cases, out, st):
        assert bool(s) == c["solved"], c["seed"]
        assert "".join(map(str, o.tolist())) == c["solution"], c["seed"]


def test_lane_golden_solve_and_node(host):
    for c in load_golden("golden_solve.json"):
        out, st = _solve(host, np.array([b81(c["puzzle"])]))
        assert bool(st[0]) == c["solved"] and "".join(map(str, out[0].tolist())) == c["solution"], c["name"]
    for c in load_golden("golden_node.json")["solve_recursive"]:
        out, st = _solve(host, np.array([b81(c["puzzle"])]), node_order=1)
        assert bool(st[0]) == c["solved"] and "".join(map(str, out[0].tolist())) == c["solution"]


@pytest.mark.parametrize("order", ["gen", "node"])
def test_lane_hard17_vs_oracle(host, order):
    from sudoku_solver_distributed_amd.gen import hard17_batch
    boards = hard17_batch(64, seed=7).numpy()
    out, st = _solve(host, boards, node_order=int(order == "node"))
    want, cnt = O.solve_unique_batch(boards)  # unique completions: every walk finds it
    assert (cnt == 1).all()
    assert st.all()
    assert (out == want).all()


def test_lane_load_dw_matches_byte_loader(host_dw):
    rng = np.random.default_rng(3)
    n = 512
    boards = rng.integers(0, 10, size=(n, 81), dtype=np.uint8)
    boards[rng.random((n, 81)) < 0.4] = 0
    boards[::7, rng.integers(0, 81)] = rng.integers(10, 256)  # some invalid bytes
    boards[1] = 0
    boards[2] = 9
    for off in range(4):
        buf = np.zeros(n * 81 + 16, dtype=np.uint8)
        buf[off:off + n * 81] = boards.reshape(-1)
        assert host_dw.check_load_dw(buf.ctypes.data + off, n) == 0, off
