"""node.py mirror: HTTP /solve, /stats, /network and the UDP protocol on
127.0.0.1 -- two peers, and a four-peer network under concurrent /solve
load (BASELINE.json configs[4]).  CPU tests inject an oracle-backed solver
backend (test infrastructure); the -m gpu tests run the same flows on the
HIP kernels."""
import json
import threading
import time
import urllib.request
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from conftest import b81, grid9, load_golden
from oracle import oracle as O


class OracleBackend:
    """node.py's walk exactly (is_valid_move short-circuit included), like
    the HIP backend."""

    def solve(self, boards, order):
        sols, st = O.solve_batch(boards.numpy(), order="node_literal" if order == "node" else order)
        return torch.from_numpy(sols), torch.from_numpy(st), 1

    def peer_solve(self, boards):
        res = [O.peer_solve(b) for b in boards.numpy()]
        code = {1: 1, 0: 0, -1: -4}
        return (torch.from_numpy(np.array([r[1] for r in res], dtype=np.uint8)),
                torch.tensor([code[r[0]] for r in res], dtype=torch.int32),
                torch.tensor([r[2] for r in res], dtype=torch.int32))

    def new_peer_state(self):
        return O.PeerNode()

    def peer_solve_seq(self, boards, node):
        res = [node.solve(b) for b in boards.numpy()]
        code = {1: 1, 0: 0, -1: -4}
        return (torch.from_numpy(np.array([r[1] for r in res], dtype=np.uint8)),
                torch.tensor([code[r[0]] for r in res], dtype=torch.int32),
                torch.tensor([r[2] for r in res], dtype=torch.int32))

    def check(self, boards, mode):
        f = O.check if mode == 0 else O.check_sums
        return torch.tensor([int(f(b)) for b in boards.numpy()], dtype=torch.int32)

    def first_candidate(self, boards, cells):
        out = []
        for b, c in zip(boards.numpy(), cells):
            d = O.first_candidate(b, c // 9, c % 9)
            out.append(d or 0)
        return torch.tensor(out, dtype=torch.int32)


def _start(backend, anchor=None, **kw):
    from sudoku_solver_distributed_amd.node import P2PNode, make_http_server
    node = P2PNode("127.0.0.1", 0, anchor_node=anchor, handicap=0, backend=backend, **kw)
    node.bind()
    httpd = make_http_server(node, "127.0.0.1", 0)
    threading.Thread(target=httpd.serve_forever, daemon=True).start()
    threading.Thread(target=node.run, daemon=True).start()
    return node, httpd, f"http://127.0.0.1:{httpd.server_address[1]}"


def _http(url, body=None):
    req = urllib.request.Request(url, data=None if body is None else json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"},
                                 method="GET" if body is None else "POST")
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def _run_flow(backend):
    a, ha, ua = _start(backend)
    b, hb, ub = _start(backend, anchor=a.id)
    try:
        for _ in range(100):
            if a.id in b.network() or b.id in a.network():
                break
            time.sleep(0.05)
        # README.md:21 example over HTTP: node.py's walk (row-major), many solutions
        case = [c for c in load_golden("golden_solve.json") if c["name"] == "readme"][0]
        want = O.solve_batch(np.array([b81(case["puzzle"])], dtype=np.uint8), order="node")[0][0]
        code, sol = _http(ua + "/solve", {"sudoku": grid9(case["puzzle"])})
        assert code == 200 and [v for r in sol for v in r] == want.tolist()
        # node.py:62-74 goldens (reference SudokuSolver.solve_sudoku outputs)
        for c in load_golden("golden_node.json")["solve_recursive"]:
            code, sol = _http(ub + "/solve", {"sudoku": grid9(c["puzzle"])})
            assert code == 200 and "".join(str(v) for r in sol for v in r) == c["solution"]
        # unsolvable -> 400 like node.py:688 (dead at the row-major walk's first cell)
        dead = "123456780000000009" + "0" * 63
        code, body = _http(ua + "/solve", {"sudoku": grid9(dead)})
        assert code == 400 and body["error"] == "No solution found"
        code, body = _http(ua + "/solve", {"sudoku": [[10] * 9] * 9})
        assert code == 400
        code, stats = _http(ua + "/stats")
        assert code == 200 and stats["all"]["solved"] >= 1 and any(n["address"] == a.id for n in stats["nodes"])
        code, net = _http(ua + "/network")
        assert code == 200 and (b.id in net or a.id in net)
        assert _http(ua + "/nope")[0] == 404
        # UDP: a whole board handed to the peer, and the reference's cell task
        rep = a.request_solve(b.id, grid9(case["puzzle"]))
        assert rep["solved"] and _flat(rep["sudoku"]) == want.tolist()
        cell_cases = load_golden("golden_node.json")["first_candidate"][:5]
        for c in cell_cases:
            num = a.solver.solve_sudoku_destributed(grid9(c["grid"]), c["row"], c["col"])
            assert num == c["num"]
    finally:
        for n, h in ((a, ha), (b, hb)):
            n.shutdown()
            h.shutdown()


def _flat(board):
    return [v for row in board for v in row]


def test_node_flow_cpu_backend():
    _run_flow(OracleBackend())


def test_node_requires_gpu_backend_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sudoku_solver_distributed_amd.node import SudokuSolver
    from sudoku_solver_distributed_amd.solver import SudokuHipError
    with pytest.raises(SudokuHipError):
        SudokuSolver(0)


@pytest.mark.gpu
def test_node_flow_gpu():
    from sudoku_solver_distributed_amd.node import GpuSolverBackend
    _run_flow(GpuSolverBackend())


def _load_boards(n):
    """n request boards: reference-generated puzzles (golden_gen, 5-58
    blanks), the README puzzle, short-circuit boards (golden_sc), cycled."""
    pool = [c["puzzle"] for c in load_golden("golden_gen.json") if 5 <= c["empty_boxes"] <= 58]
    pool += [c["puzzle"] for c in load_golden("golden_solve.json") if c["name"] == "readme"]
    pool += [c["puzzle"] for c in load_golden("golden_sc.json")[:8]]
    return [pool[i % len(pool)] for i in range(n)]


def _network(backends, forward=None):
    """Peers 1..k-1 anchor to peer 0; wait until every peer knows every peer."""
    nodes = [_start(backends[0], forward_threshold=(forward or {}).get(0))]
    for i in range(1, len(backends)):
        nodes.append(_start(backends[i], anchor=nodes[0][0].id, forward_threshold=(forward or {}).get(i)))
    ids = {n[0].id for n in nodes}
    for _ in range(200):
        if all(set(n[0].total_peers) | {n[0].id} == ids for n in nodes):
            break
        time.sleep(0.05)
    assert all(set(n[0].total_peers) | {n[0].id} == ids for n in nodes), [n[0].total_peers for n in nodes]
    return nodes


def _load(nodes, boards, clients=32):
    """Concurrent POST /solve of every board, spread over the peers' HTTP
    ports; returns the answers in board order."""
    def one(i):
        code, sol = _http(nodes[i % len(nodes)][2] + "/solve", {"sudoku": grid9(boards[i])})
        return code, sol
    with ThreadPoolExecutor(max_workers=clients) as ex:
        return list(ex.map(one, range(len(boards))))


def _check_network_run(nodes, boards, answers):
    want, wst = O.solve_batch(np.array([b81(b) for b in boards], dtype=np.uint8), order="node_literal")
    for i, ((code, sol), w, ok) in enumerate(zip(answers, want, wst)):
        if ok:
            assert code == 200 and [v for r in sol for v in r] == w.tolist(), (i, boards[i])
        else:
            assert code == 400, (i, boards[i])
    solved = int(wst.sum())
    # gossip converges: every peer's /stats totals count every solved board once
    for _ in range(200):
        stats = [_http(n[2] + "/stats")[1] for n in nodes]
        if all(s["all"]["solved"] == solved for s in stats):
            break
        time.sleep(0.05)
    assert all(s["all"]["solved"] == solved for s in stats), [s["all"] for s in stats]
    own = {n[0].id: n[0].solver.solved_puzzles for n in nodes}
    assert sum(own.values()) == solved
    for s in stats:
        by = {e["address"]: e["solved"] for e in s["solved_by"]}
        assert all(by.get(a, 0) == v for a, v in own.items()), (by, own)
        assert s["all"]["validations"] == sum(e["validations"] for e in s["nodes"])
    return own


def _shutdown(nodes):
    for n, h, _ in nodes:
        n.shutdown()
        h.shutdown()


def test_four_peer_network_under_load():
    """configs[4] on CPU: four peers, 120 concurrent /solve requests spread
    over their HTTP ports; every answer is node.py's walk (literal oracle),
    every peer's /stats totals agree, and the batcher coalesced requests."""
    nodes = _network([OracleBackend() for _ in range(4)])
    try:
        boards = _load_boards(120)
        own = _check_network_run(nodes, boards, _load(nodes, boards))
        assert all(v > 0 for v in own.values()), own
        assert sum(n[0].solver.batcher.batches for n in nodes) < len(boards)
    finally:
        _shutdown(nodes)


def test_four_peer_forwarding():
    """A peer over its forward threshold hands whole boards to its peers over
    UDP (solve / solution with a task id): peer 0 forwards every request, the
    others solve them, and the answers and totals are unchanged."""
    nodes = _network([OracleBackend() for _ in range(4)], forward={0: 0})
    try:
        boards = _load_boards(48)
        answers = _load(nodes[:1], boards, clients=8)  # every request enters at peer 0
        own = _check_network_run(nodes, boards, answers)
        assert nodes[0][0].forwarded == len(boards) and own[nodes[0][0].id] == 0
        assert sum(n[0].served for n in nodes[1:]) == len(boards)
    finally:
        _shutdown(nodes)


@pytest.mark.gpu
def test_two_peer_gpu_network_under_load():
    """configs[4] on the HIP path: two peers (this box has one MI355X; each
    peer's GpuSolverBackend shards over the GPUs it is given), 400 concurrent
    /solve requests, answers bit-identical to node.py's walk, totals agree,
    and the requests were coalesced into far fewer GPU batches."""
    from sudoku_solver_distributed_amd.node import GpuSolverBackend
    nodes = _network([GpuSolverBackend([0]), GpuSolverBackend([0])])
    try:
        boards = _load_boards(400)
        _check_network_run(nodes, boards, _load(nodes, boards, clients=32))
        batches = sum(n[0].solver.batcher.batches for n in nodes)
        assert batches < len(boards) // 2, batches
    finally:
        _shutdown(nodes)


def _reference_mode_flow(backends):
    """solve_mode="reference": /solve answers exactly what the reference's
    P2PNode.peer_sudoku_solve returned -- on a fresh node (golden_peer.json;
    the serving node's state is reset before each request) and along request
    sequences on one node, whose partial_solution / tried sets carry over
    (golden_peer_seq.json) -- with no answer at all (HTTP 500 here) where the
    reference never returns, validations counted like node.py after every
    request, and the same through a forwarding peer (the state is that of the
    peer that serves the request)."""
    cases = load_golden("golden_peer.json")
    seqs = load_golden("golden_peer_seq.json")
    nodes = _network(backends, forward={1: 0})
    server = nodes[0][0]
    for n, _, _ in nodes:
        n.solve_mode = "reference"

    def post(entry, puzzle, want):
        code, body = _http(nodes[entry][2] + "/solve", {"sudoku": grid9(puzzle)})
        if want == "TIMEOUT":
            assert code == 500, puzzle
        else:
            assert code == 200 and "".join(str(v) for r in body for v in r) == want, puzzle

    try:
        solved = 0
        for entry in (0, 1):  # peer 1 forwards every board to peer 0
            for c in cases:
                server.reset_solve_state()
                v0 = server.solver.validations
                post(entry, c["puzzle"], c["returned"])
                assert server.solver.validations - v0 == c["validations"], c["name"]
                solved += c["returned"] != "TIMEOUT"
            for k, seq in enumerate(seqs):
                server.reset_solve_state()
                v0 = server.solver.validations
                for r in seq["requests"]:
                    post(entry, r["puzzle"], r["returned"])
                    assert server.solver.validations - v0 == r["validations"], k
                    solved += r["returned"] != "TIMEOUT"
        assert server.solver.solved_puzzles == solved
        assert nodes[1][0].forwarded == len(cases) + sum(len(q["requests"]) for q in seqs)
    finally:
        _shutdown(nodes)


def test_reference_solve_mode_cpu():
    _reference_mode_flow([OracleBackend(), OracleBackend()])


@pytest.mark.gpu
def test_reference_solve_mode_gpu():
    from sudoku_solver_distributed_amd.node import GpuSolverBackend
    _reference_mode_flow([GpuSolverBackend([0]), GpuSolverBackend([0])])


# ------------------------------------------------------------ protocol edges
def _easy_boards(n):
    return [c["puzzle"] for c in load_golden("golden_gen.json") if c["empty_boxes"] in (5, 20)][:n]


def test_udp_solve_errors_are_answered():
    """A `solve` the peer cannot serve is answered with an `error` at once
    (no requester waits for its timeout): unknown order, malformed boards,
    an oversized batch; request_solve_many splits big batches into messages
    of at most MAX_UDP_BOARDS boards."""
    from sudoku_solver_distributed_amd.node import MAX_UDP_BOARDS
    nodes = _network([OracleBackend(), OracleBackend()])
    a, b = nodes[0][0], nodes[1][0]
    try:
        t0 = time.monotonic()
        rep = a._request(b.id, {"type": "solve", "sudokus": ["0" * 81], "order": "bogus"}, 5)
        assert "unknown order" in rep["error"]
        rep = a._request(b.id, {"type": "solve", "sudokus": ["12x" + "0" * 78]}, 5)
        assert "81-digit" in rep["error"]
        rep = a._request(b.id, {"type": "solve", "sudokus": ["0" * 81] * (MAX_UDP_BOARDS + 1)}, 5)
        assert "more than" in rep["error"]
        rep = a._request(b.id, {"type": "solve", "sudoku": [[0] * 9] * 8}, 5)
        assert "9 lists" in rep["error"]
        rep = a._request(b.id, {"type": "solve", "sudoku": [[0] * 9] * 9, "row": 0}, 5)  # no col: a whole board
        assert rep["solved"]
        assert time.monotonic() - t0 < 4
        easy = _easy_boards(20)
        boards = [easy[i % len(easy)] for i in range(2 * MAX_UDP_BOARDS + 7)]
        rep = a.request_solve_many(b.id, boards, order="node")
        want, wst = O.solve_batch(np.array([b81(x) for x in boards], dtype=np.uint8), order="node_literal")
        assert rep["sudokus"] == ["".join(map(str, w)) for w in want] and rep["status"] == wst.tolist()
        assert b.served == len(boards) + 1  # + the whole board above
    finally:
        _shutdown(nodes)


def test_solve_rejects_what_is_not_a_board():
    """POST /solve takes the reference's board type only (9 lists of 9
    ints): a flat list, a string, 8 rows or a 10-wide row get HTTP 400."""
    nodes = _network([OracleBackend()])
    try:
        url = nodes[0][2] + "/solve"
        for bad in ([0] * 81, "0" * 81, [[0] * 9] * 8, [[0] * 10] + [[0] * 9] * 8, [[0.5] * 9] * 9,
                    [[True] * 9] * 9):
            code, body = _http(url, {"sudoku": bad})
            assert code == 400 and "bad request" in body["error"], bad
        code, _ = _http(url, {"sudoku": [[0] * 9] * 9})
        assert code == 200
    finally:
        _shutdown(nodes)


class _CountingBackend(OracleBackend):
    """OracleBackend whose solve reports 7 passes per board."""

    def solve(self, boards, order):
        sols, st, _ = super().solve(boards, order)
        return sols, st, 7 * boards.shape[0]


def test_validations_semantics():
    """check() / is_valid_move / the cell task add one
    each (node.py:87); a walk solve adds the backend's propagation passes;
    reference mode adds the reference's own count (test_reference_solve_mode_*)."""
    from sudoku_solver_distributed_amd.node import SudokuSolver
    s = SudokuSolver(0, backend=_CountingBackend())
    try:
        g = grid9(_easy_boards(1)[0])
        assert s.validations == 0
        s.check(g)
        s.is_valid_move(g, 0, 0, 1)
        s.solve_sudoku_destributed(g, 0, 0)
        assert s.validations == 3
        s.solve_sudoku([r[:] for r in g])
        assert s.validations == 3 + 7
        s.solve_many(torch.tensor([b81(x) for x in _easy_boards(5)], dtype=torch.uint8))
        assert s.validations == 3 + 7 + 35
    finally:
        s.close()


# ------------------------------------------------- configs[4] on the HIP path
def _four_peer_gpu(forward):
    from sudoku_solver_distributed_amd.node import GpuSolverBackend
    # each peer backed by two solvers on the box's one MI355X: the shape of
    # "2 MI355X per peer" (GpuSolverBackend splits every batch over both)
    backends = [GpuSolverBackend([0, 0]) for _ in range(4)]
    assert all(len(b.solvers) == 2 and b.solvers[0] is not b.solvers[1] for b in backends)
    nodes = _network(backends, forward=forward)
    try:
        boards = _load_boards(1200)
        t0 = time.monotonic()
        answers = _load(nodes if forward is None else nodes[:1], boards, clients=64)
        dt = time.monotonic() - t0
        own = _check_network_run(nodes, boards, answers)
        batches = sum(n[0].solver.batcher.batches for n in nodes)
        print(f"4 peers x 2 solvers, forward={forward}: {len(boards) / dt:.0f} requests/s, {batches} GPU batches")
        return nodes, own, batches
    finally:
        _shutdown(nodes)


@pytest.mark.gpu
def test_four_peer_gpu_network_under_load():
    """configs[4] on the kernels: four peers, each GpuSolverBackend([0, 0])
    (two workspaces / streams on one GPU: the multi-device branch), 1200
    concurrent /solve requests from 64 clients over all four HTTP ports;
    every answer is node.py's walk, /stats totals agree on every peer, and
    the requests were coalesced into far fewer GPU batches."""
    nodes, own, batches = _four_peer_gpu(None)
    assert all(v > 0 for v in own.values()), own
    assert batches < 1200 // 2, batches


@pytest.mark.gpu
def test_four_peer_gpu_forwarding():
    """The same with every request entering at peer 0, which forwards all of
    them (UDP solve / solution) to the other three GPU-backed peers."""
    nodes, own, _ = _four_peer_gpu({0: 0})
    assert nodes[0][0].forwarded == 1200 and own[nodes[0][0].id] == 0
    assert sum(n[0].served for n in nodes[1:]) == 1200


@pytest.mark.gpu
def test_gpu_backend_split_and_pass_count():
    """GpuSolverBackend([0, 0]) splits a batch over two solvers: same answers
    as one solver, and the pass count it reports is exactly what the two
    workspaces' counters grew by (walk-mode validations)."""
    from sudoku_solver_distributed_amd.gen import hard17_batch
    from sudoku_solver_distributed_amd.node import GpuSolverBackend, SudokuSolver
    one, two = GpuSolverBackend([0]), GpuSolverBackend([0, 0])
    boards = torch.cat([hard17_batch(3000, seed=5), torch.tensor([b81(x) for x in _load_boards(100)],
                                                                  dtype=torch.uint8)])
    s1, st1, p1 = one.solve(boards, "node")
    before = [s.stats()["sweeps"] for s in two.solvers]
    s2, st2, p2 = two.solve(boards, "node")
    after = [s.stats()["sweeps"] for s in two.solvers]
    assert torch.equal(s1, s2) and torch.equal(st1, st2)
    assert p2 == sum(a - b for a, b in zip(after, before)) and p2 > len(boards)
    node = SudokuSolver(0, backend=two)
    try:
        v0 = node.validations
        node.solve_many(boards)
        assert node.validations - v0 == p2
    finally:
        node.close()
