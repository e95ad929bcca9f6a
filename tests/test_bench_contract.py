"""bench.py's roofline inputs (CPU only): the committed rocprofv3 PMC summary
of the default solve kernel must match bench.py's default workload, or the
bench line's roofline.achieved / frac would silently be null."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_default_kernel_has_matching_pmc_profile():
    from sudoku_solver_distributed_amd import _lib
    kname = _lib.KERNEL_SYMBOLS[_lib.SDK_KERNELS["auto"]]
    path = os.path.join(ROOT, "profiles", f"pmc_{kname}.json")
    assert os.path.exists(path), path
    with open(path) as f:
        pmc = json.load(f)
    # bench.py defaults at N = 1: --batch 2^20 boards per step, --seed 2024,
    # one step per launch, 6 launches in flight at 1 wave per SIMD -- the
    # counters must come from the launch shape the bench times (bench.py
    # nulls roofline.frac / traffic otherwise)
    # (bench.py sets GPU_MAX_HW_QUEUES = 8 before HIP starts)
    from unittest import mock
    from sudoku_solver_distributed_amd.solver import default_inflight
    with mock.patch.dict(os.environ, {"GPU_MAX_HW_QUEUES": "8"}):
        inflight, grid_waves = default_inflight()
    assert pmc["kernel"] == kname
    assert pmc["seed"] == 2024 and pmc.get("workload", "hard17") == "hard17"
    assert pmc["shape"] == {"boards_per_step": 1 << 20, "group": 1, "inflight": inflight, "grid_waves": grid_waves,
                            "pool_last": (inflight + 1) // 2}
    assert pmc["counters_per_launch"]["SQ_WAVES"] == 256 * 4 * grid_waves
    assert pmc["valu_insts_per_launch"] > 0
    assert pmc["hbm_bytes_per_launch"] is None or pmc["hbm_bytes_per_launch"] > 0


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


import pytest  # noqa: E402


@pytest.mark.gpu
def test_bench_two_rank_path_runs():
    """bench.py's multi-rank path (barrier, max-time all-reduce, the side
    configs' collectives, configs[3]'s split over ranks) executed once before
    the driver's 8-GPU run does: two fresh bench processes, env rendezvous on
    127.0.0.1, gloo, both ranks on cuda:0.  Rank 0 prints one JSON line."""
    import subprocess
    import sys
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
             "--device-index", "0", "--steps", "2", "--warmup", "1", "--no-cpu", "--latency-boards", "4",
             "--no-serving"],
            cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=400)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-3000:]
        outs.append(o)
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not [l for l in outs[1].splitlines() if l.startswith("{")]
    d = json.loads(lines[0])
    # strong scaling (the default): the 2^20-board step split over the two
    # ranks, each rank's launches holding 2^21 boards (four steps' shards) at
    # 2 waves per SIMD
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["dist_backend"] == "gloo"
    assert d["config"]["global_batch"] == 1 << 20 and d["config"]["boards_per_gpu_per_step"] == 1 << 19
    assert d["config"]["steps_per_launch"] == 4 and d["roofline"]["kernel"] == "plane_kernel_multi"
    assert d["config"]["grid_waves_per_simd"] == 2
    assert d["side_configs"]["pathological"]["ranks"] == 2 and d["side_configs"]["pathological"]["identical"]
    assert d["all_solved_and_checked"] and d["value"] > 0
