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
    # bench.py defaults: --batch 2^20, --seed 2024
    assert pmc["kernel"] == kname
    assert pmc["batch"] == 1 << 20 and pmc["seed"] == 2024
    assert pmc["valu_insts_per_launch"] > 0
    assert pmc["hbm_bytes_per_launch"] is None or pmc["hbm_bytes_per_launch"] > 0
