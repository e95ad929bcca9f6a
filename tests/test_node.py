"""node.py mirror: HTTP /solve, /stats, /network and the UDP protocol,
two peers on 127.0.0.1.  CPU tests inject an oracle-backed solver backend
(test infrastructure); test_node_gpu runs the same flow on the HIP kernels."""
import json
import threading
import time
import urllib.request

import numpy as np
import pytest
import torch

from conftest import b81, grid9, load_golden
from oracle import oracle as O


class OracleBackend:
    def solve(self, boards, order):
        sols, st = O.solve_batch(boards.numpy(), order=order)
        return torch.from_numpy(sols), torch.from_numpy(st), 1

    def check(self, boards, mode):
        f = O.check if mode == 0 else O.check_sums
        return torch.tensor([int(f(b)) for b in boards.numpy()], dtype=torch.int32)

    def first_candidate(self, boards, cells):
        out = []
        for b, c in zip(boards.numpy(), cells):
            d = O.first_candidate(b, c // 9, c % 9)
            out.append(d or 0)
        return torch.tensor(out, dtype=torch.int32)


def _start(backend, anchor=None):
    from sudoku_solver_distributed_amd.node import P2PNode, make_http_server
    node = P2PNode("127.0.0.1", 0, anchor_node=anchor, handicap=0, backend=backend)
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
