import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the GPU tests run with the hardware queues bench.py sets (read when HIP
# starts): the launches in flight then run side by side as in the timed shape
if not os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() or int(os.environ["GPU_MAX_HW_QUEUES"]) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running CPU case")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def b81(s):
    return [int(c) for c in s]


def grid9(s):
    return [[int(s[r * 9 + c]) for c in range(9)] for r in range(9)]


@pytest.fixture(scope="session")
def solver():
    from sudoku_solver_distributed_amd.solver import get_solver
    return get_solver()


@pytest.fixture(autouse=True)
def _every_board_answered(request):
    """After every test that used the session solver: every board its solve
    kernels took since the last stats reset was answered and no kernel set an
    error bit (sdk_verify_workspace), on its own workspace and on the
    solve_inflight slots' -- the no-silent-drop contract, suite-wide."""
    yield
    if "solver" not in request.fixturenames:
        return
    s = request.getfixturevalue("solver")
    s.verify()
    if s._slots:
        s.verify_inflight()
