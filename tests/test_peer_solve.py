"""The reference's HTTP /solve algorithm (node.py:534-557,
P2PNode.peer_sudoku_solve on a fresh single node): the oracle against the
reference's own outputs (tests/golden/golden_peer.json), the GPU loop's
header (csrc/peer_greedy.h, compiled for the host) against the oracle, and
-m gpu: sdk_peer_solve_batch against both.  The same for ONE node serving
requests in a row (its partial_solution / tried sets carry over, node.py:149,
167): tests/golden/golden_peer_seq.json, sdk_peer_solve_seq."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import b81, load_golden
from oracle import oracle as O

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
STATUS = {1: 1, 0: 0, -1: 2}  # oracle -> peer_greedy.h status


def _boards(n, seed):
    """generate_sudoku-style boards at every blank level (gen.py:31-52 on the
    CPU oracle), plus the fixture's boards."""
    from sudoku_solver_distributed_amd.gen import _draw_diagonal
    import random
    rng = random.Random(seed)
    out = []
    for k in range(n):
        g = np.asarray(_draw_diagonal(rng), dtype=np.uint8).reshape(81)
        ok, g = O.solve(g)
        g[rng.sample(range(81), [5, 20, 35, 45, 55, 64][k % 6])] = 0
        out.append(g)
    return np.array(out + [b81(c["puzzle"]) for c in load_golden("golden_peer.json")], dtype=np.uint8)


def test_oracle_matches_reference_fixture():
    cases = load_golden("golden_peer.json")
    assert len(cases) >= 80 and sum(c["returned"] == "TIMEOUT" for c in cases) >= 1
    for c in cases:
        st, g, v = O.peer_solve(b81(c["puzzle"]))
        got = "TIMEOUT" if st == -1 else "".join(map(str, g))
        assert got == c["returned"], c["name"]
        assert v == c["validations"], c["name"]


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    so = os.path.join(str(tmp_path_factory.mktemp("peer")), "libpeer_host.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-o", so,
                           os.path.join(NATIVE, "peer_host.cpp")])
    lib = ctypes.CDLL(so)
    lib.peer_host_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64]
    lib.peer_host_seq.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p]
    return lib


def test_device_loop_matches_oracle_on_host(host):
    boards = _boards(600, 11)
    out = np.empty_like(boards)
    st = np.empty(len(boards), np.int32)
    val = np.empty(len(boards), np.int32)
    host.peer_host_batch(boards.ctypes.data, out.ctypes.data, st.ctypes.data, val.ctypes.data, len(boards))
    for b, o, s, v in zip(boards, out, st, val):
        ws, wg, wv = O.peer_solve(b)
        assert s == STATUS[ws] and v == wv and np.array_equal(o, wg), "".join(map(str, b))


@pytest.mark.gpu
def test_gpu_peer_solve(solver):
    from sudoku_solver_distributed_amd.solver import SDK_NO_RETURN, SDK_SOLVED, SDK_UNSOLVABLE
    boards = _boards(3000, 12)
    out, st, val = solver.peer_solve(torch.from_numpy(boards))
    out, st, val = out.cpu().numpy(), st.cpu().numpy(), val.cpu().numpy()
    code = {1: SDK_SOLVED, 0: SDK_UNSOLVABLE, -1: SDK_NO_RETURN}
    for b, o, s, v in zip(boards, out, st, val):
        ws, wg, wv = O.peer_solve(b)
        assert s == code[ws] and v == wv and np.array_equal(o, wg), "".join(map(str, b))
    assert (st == SDK_NO_RETURN).any() and (st == SDK_UNSOLVABLE).any() and (st == SDK_SOLVED).any()


# ---------------------------------------------------- one node, many requests
def _seq_expect(fixture_seq):
    return [(r["puzzle"], r["returned"], r["validations"]) for r in fixture_seq["requests"]]


def test_oracle_node_sequence_matches_reference_fixture():
    """The reference's own answers for request sequences on one node: the
    oracle's PeerNode (state carried) reproduces every answer and the node's
    cumulative validations counter; a fresh node per request would not."""
    seqs = load_golden("golden_peer_seq.json")
    assert len(seqs) >= 20 and sum(s["state_matters"] for s in seqs) >= 10
    for k, seq in enumerate(seqs):
        node = O.PeerNode()
        for p, want, val in _seq_expect(seq):
            st, g, _ = node.solve(b81(p))
            got = "TIMEOUT" if st == -1 else "".join(map(str, g))
            assert got == want, (k, p)
            assert node.validations == val, (k, p)
        if seq["state_matters"]:
            assert any(O.peer_solve(b81(r["puzzle"]))[1].tolist() != [int(c) for c in r["returned"]]
                       for r in seq["requests"]), k


def _random_sequences(n_seq, length, seed):
    rng = np.random.default_rng(seed)
    pool = _boards(120, seed)
    return [pool[rng.integers(0, len(pool), length)] for _ in range(n_seq)]


def test_device_loop_sequence_matches_oracle_on_host(host):
    from sudoku_solver_distributed_amd._lib import SDK_PEER_STATE_BYTES
    for boards in _random_sequences(40, 12, 21):
        out = np.empty_like(boards)
        st = np.empty(len(boards), np.int32)
        val = np.empty(len(boards), np.int32)
        state = np.zeros(SDK_PEER_STATE_BYTES, np.uint8)
        host.peer_host_seq(boards.ctypes.data, out.ctypes.data, st.ctypes.data, val.ctypes.data, len(boards),
                           state.ctypes.data)
        node = O.PeerNode()
        for b, o, s_, v in zip(boards, out, st, val):
            ws, wg, wv = node.solve(b)
            assert s_ == STATUS[ws] and v == wv and np.array_equal(o, wg), "".join(map(str, b))


@pytest.mark.gpu
def test_gpu_peer_solve_seq(solver):
    """sdk_peer_solve_seq: the reference fixture's sequences, then random
    sequences against the oracle node; the state record round-trips between
    calls (two calls of half a sequence == one call of all of it)."""
    from sudoku_solver_distributed_amd.solver import SDK_NO_RETURN, SDK_SOLVED, SDK_UNSOLVABLE
    code = {1: SDK_SOLVED, 0: SDK_UNSOLVABLE, -1: SDK_NO_RETURN}
    for k, seq in enumerate(load_golden("golden_peer_seq.json")):
        boards = torch.tensor([b81(r["puzzle"]) for r in seq["requests"]], dtype=torch.uint8)
        state = solver.new_peer_state()
        out, st, val = solver.peer_solve_seq(boards, state)
        total = 0
        for r, o, s_, v in zip(seq["requests"], out.cpu().numpy(), st.cpu().numpy(), val.cpu().numpy()):
            total += int(v)
            got = "TIMEOUT" if s_ == SDK_NO_RETURN else "".join(map(str, o))
            assert got == r["returned"] and total == r["validations"], k
    for boards in _random_sequences(12, 40, 22):
        state = solver.new_peer_state()
        half = len(boards) // 2
        o1, s1, v1 = solver.peer_solve_seq(torch.from_numpy(boards[:half]), state)
        o2, s2, v2 = solver.peer_solve_seq(torch.from_numpy(boards[half:]), state)
        out = torch.cat([o1, o2]).cpu().numpy()
        st = torch.cat([s1, s2]).cpu().numpy()
        val = torch.cat([v1, v2]).cpu().numpy()
        node = O.PeerNode()
        for b, o, s_, v in zip(boards, out, st, val):
            ws, wg, wv = node.solve(b)
            assert s_ == code[ws] and v == wv and np.array_equal(o, wg), "".join(map(str, b))
