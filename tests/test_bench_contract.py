"""bench.py's roofline inputs (CPU only): the committed rocprofv3 PMC summary
of the default solve kernel must match bench.py's default workload, or the
bench line's roofline.achieved / frac would silently be null."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_shape(world, steps=20):
    """The launch shape bench.py's default plan gives one rank of a
    strong-scaling job of `world` ranks at the driver's --steps 20 (plan
    "run": the 20 steps' shards as one sdk_solve_batches launch on a full
    grid; bench.py sets GPU_MAX_HW_QUEUES = 8 before HIP starts)."""
    from sudoku_solver_distributed_amd._lib import SDK_MAX_BATCHES
    n_launch = -(-steps // SDK_MAX_BATCHES)
    return {"boards_per_step": (1 << 20) // world, "group": -(-steps // n_launch), "inflight": 2, "grid_waves": 0,
            "pool_last": 1, "hw_queues": 8}


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_default_shapes_have_matching_pmc_profiles(world):
    """For the driver's 1 / 2 / 4 / 8-GPU runs (--steps 20) a committed PMC
    summary of exactly that rank's launch shape exists (bench.py picks it by
    shape), so every scaling line carries roofline.frac and traffic."""
    import glob
    kname = "plane_kernel_multi"   # a multi-step launch (sdk_solve_batches)
    want = bench_shape(world)
    found = []
    for path in glob.glob(os.path.join(ROOT, "profiles", f"pmc_{kname}*.json")):
        with open(path) as f:
            pmc = json.load(f)
        if (pmc.get("kernel") == kname and pmc.get("seed") == 2024 and pmc.get("workload", "hard17") == "hard17"
                and pmc.get("shape") == want):
            found.append(pmc)
    assert found, (world, want)
    pmc = found[0]
    assert pmc["valu_insts_per_step"] > 0 and pmc["steps"] == 20
    assert pmc.get("hbm_bytes_per_step") is None or pmc["hbm_bytes_per_step"] > 0


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
    # ranks, each rank's two timed steps one launch on a full grid (plan run)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["dist_backend"] == "gloo"
    assert d["config"]["global_batch"] == 1 << 20 and d["config"]["boards_per_gpu_per_step"] == 1 << 19
    assert d["config"]["steps_per_launch"] == 2 and d["roofline"]["kernel"] == "plane_kernel_multi"
    assert d["config"]["grid_waves_per_simd"] is None
    assert d["side_configs"]["pathological"]["ranks"] == 2 and d["side_configs"]["pathological"]["identical"]
    assert d["all_solved_and_checked"] and d["value"] > 0


def test_check_steps_rotation_logic():
    """bench.check_steps on CPU tensors: step j's batch is the global batch
    rotated by 7919 j boards (this rank's [lo, hi) of it); outputs that
    agree board for board across the rotations pass, a single wrong board in
    any step, a changed given or a non-SOLVED status fails its check."""
    import torch
    import bench

    class FakeSolver:
        def check(self, grids, mode):
            return torch.ones(grids.shape[0], dtype=torch.int32)

    batch, group = 20_000, 5
    g = torch.randint(1, 10, (batch, 81), dtype=torch.uint8)      # "answers" of the global boards
    given = torch.rand(batch, 81) < 0.2
    puzzles = torch.where(given, g, torch.zeros_like(g))
    for lo, hi in ((0, batch), (5_000, 10_000)):
        inputs, bufs = [], []
        for j in range(group):
            idx = (torch.arange(lo, hi) + 7919 * j) % batch
            inputs.append(puzzles[idx])
        for i in range(2 * group):
            idx = (torch.arange(lo, hi) + 7919 * (i % group)) % batch
            bufs.append((g[idx].clone(), torch.ones(hi - lo, dtype=torch.int32)))
        fs = FakeSolver()
        assert all(bench.check_steps(fs, inputs, bufs, 2 * group, group, lo, batch).values())
        bufs[3][0][17, 4] ^= 1  # a wrong answer in one step
        ok = bench.check_steps(fs, inputs, bufs, 2 * group, group, lo, batch)
        assert not ok["rotations_agree"]
        bufs[3][0][17, 4] ^= 1
        k = int(torch.nonzero(inputs[2][0]).flatten()[0])
        bufs[2][0][0, k] = 0 if bufs[2][0][0, k] else 1  # a changed given
        assert not bench.check_steps(fs, inputs, bufs, 2 * group, group, lo, batch)["givens_kept"]
        bufs[2][0][0, k] = inputs[2][0, k]
        bufs[6][1][9] = 0
        assert not bench.check_steps(fs, inputs, bufs, 2 * group, group, lo, batch)["solved"]
