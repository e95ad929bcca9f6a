"""Build libsudoku_hip.so in-tree for gfx950 with hipcc (no JIT, no torch ext).

    python -m sudoku_solver_distributed_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
# translation units and their extra flags (plane_kernels.hip: see its header)
# SDK_PLANE_SCHED: machine-scheduler strategy of the plane kernel's unit
# (iterative-ilp measured +1.4 % over LLVM's default on one MI355X, same
# registers; "default" = LLVM's own, for A/B builds)
_SCHED = os.environ.get("SDK_PLANE_SCHED", "iterative-ilp")


# SDK_PLANE_LLVM: more LLVM options for the plane unit (space-separated, each
# passed through -mllvm; A/B builds of the code generator only)
_LLVM_EXTRA = os.environ.get("SDK_PLANE_LLVM", "").split()


def sources(sched: str = _SCHED):
    """Translation units and their flags for one plane-unit scheduler."""
    extra = [f for o in _LLVM_EXTRA for f in ("-mllvm", o)]
    return (("sudoku_kernels.hip", []),
            ("plane_kernels.hip", ([] if sched == "default" else ["-mllvm", f"-amdgpu-sched-strategy={sched}"]) + extra))


SRCS = sources()
# Every build this module is used for (product, diagnostic and A/B tuning
# builds): name -> (-D set, plane-unit scheduler).  scripts/store_hazard_check.py
# scans each of them for the wide-store data hazard; build() scans any other
# -D set before linking it.
VARIANTS = {
    "default": ((), _SCHED),
    "stamps": (("SDK_PLANE_STAMPS=1",), _SCHED),
    "waves5": (("SDK_PLANE_WAVES_PER_EU=5",), _SCHED),
    "waves6": (("SDK_PLANE_WAVES_PER_EU=6",), _SCHED),
    "nopinacc": (("SDK_PLANE_PIN_ACC=0",), _SCHED),
    "sched-default": ((), "default"),
    "sched-minreg": ((), "iterative-minreg"),
    "sched-maxocc": ((), "iterative-maxocc"),
    "sched-max-ilp": ((), "max-ilp"),
}
OUT = os.path.join(_HERE, "libsudoku_hip.so")
ARCH = os.environ.get("SDK_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    return "hipcc"


def build(force: bool = False, verbose: bool = False, defines=(), out: str = OUT) -> str:
    """Compile every translation unit for gfx950 and link the C-ABI library.
    `defines` / `out`: A/B builds of tuning macros into another in-tree .so
    (loaded with SDK_LIB=...)."""
    csrc = os.path.join(_HERE, "csrc")
    deps = [os.path.join(csrc, f) for f in os.listdir(csrc) if not f.endswith(".o")] + [os.path.join(ROOT, "include", "sudoku_hip.h")]
    if (not force and os.path.exists(out)
            and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps)):
        return out
    if tuple(defines) and tuple(defines) not in {v[0] for v in VARIANTS.values()}:
        # an A/B build nobody has scanned yet: the wide-store hazard check first
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import store_hazard_check
        if store_hazard_check.check_build(SRCS, defines, "+".join(defines)):
            raise RuntimeError(f"wide-store data hazard in the build with {defines} (scripts/store_hazard_check.py)")
    objs = []
    for name, extra in SRCS:
        obj = out + "." + name + ".o"
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", *extra,
               *[f"-D{d}" for d in defines],
               "-c", "-o", obj, os.path.join(csrc, name)]
        if verbose:
            cmd.append("-Rpass-analysis=kernel-resource-usage")
        subprocess.check_call(cmd)
        objs.append(obj)
    subprocess.check_call([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs])
    for obj in objs:
        os.remove(obj)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    # python -m sudoku_solver_distributed_amd.build [--force] [-v] [--tag T -DNAME=V ...]
    args = sys.argv[1:]
    defs = [a[2:] for a in args if a.startswith("-D")]
    tag = args[args.index("--tag") + 1] if "--tag" in args else None
    dst = os.path.join(_HERE, f"libsudoku_hip_{tag}.so") if tag else OUT
    print(build(force="--force" in args or bool(tag), verbose="-v" in args, defines=defs, out=dst))
