"""Static check of the gfx950 wide-store data hazard in the product kernels.

A VMEM store of more than 64 bits reads its data VGPRs after issue; a VALU
write to one of them needs TWO wait states in between on gfx940-class parts
(gfx950 included).  hipcc (ROCm 7.2) pads this only when a MUBUF store's
soffset is an inline constant, so a buffer_store_dwordx4 with a REGISTER
soffset (offset > 64 bytes) can be followed at once by a VALU write of its
data.  In the plane kernel's stack push that corrupted search levels (~0.65 %
of boards ended UNSOLVABLE); the push now keeps its data live through an
s_nop (plane_kernel.h PlaneStack::push).

The scan looks at every instruction issued inside the hazard window: an
instruction is one wait state, `s_nop N` is N + 1; a VALU write of a data
VGPR before two wait states have passed is a hit.

Every build variant build.py can produce is scanned (build.VARIANTS: the
default, the diagnostic stamps build, the tuning builds and every machine
scheduler strategy), and build.build() scans any other -D set it is asked to
compile before linking it.

    python scripts/store_hazard_check.py            # all variants, exit 1 on a hit
    python scripts/store_hazard_check.py stamps      # one variant
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sudoku_solver_distributed_amd", "csrc")
STORE = re.compile(r"(buffer|global|flat|scratch)_store_(dwordx[34]|b96|b128)\s")
WAIT_STATES = 2  # gfx940 / gfx950: VALU write of a >64-bit VMEM store's data


def _regs(spec):
    m = re.match(r"v\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", spec)
    return {int(m.group(1))} if m else set()


def _nop_states(t):
    m = re.match(r"s_nop\s+(0x[0-9a-fA-F]+|\d+)", t)
    return int(m.group(1), 0) + 1 if m else None


def scan(lines):
    """(line number, store, offending instruction) for every wide store whose
    data VGPR is written by a VALU instruction fewer than WAIT_STATES wait
    states after it."""
    lines = [l.strip() for l in lines]
    hits = []
    for i, l in enumerate(lines):
        m = STORE.match(l)
        if not m:
            continue
        ops = [x.strip() for x in l.split(None, 1)[1].split(",")]
        data = _regs(ops[0] if m.group(1) == "buffer" else ops[1])
        waited = 0
        for t in lines[i + 1:]:
            if waited >= WAIT_STATES:
                break
            if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
                continue  # comments, directives, labels, asm markers
            nop = _nop_states(t)
            if nop is not None:
                waited += nop
                continue
            if t.startswith("v_") and " " in t and _regs(t.split(None, 1)[1].split(",")[0].strip()) & data:
                hits.append((i + 1, l, t))
                break
            if t.startswith("s_branch") or t.startswith("s_cbranch") or t.startswith("s_setpc") or t.startswith("s_endpgm"):
                break  # the window continues at the target: hipcc pads control flow itself
            waited += 1
    return hits


def compile_asm(src, extra, out, defines=()):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *extra,
                           *[f"-D{d}" for d in defines], "--cuda-device-only", "-S", "-o", out,
                           os.path.join(CSRC, src)], stderr=subprocess.DEVNULL)


def check_build(srcs, defines=(), label="default", tmp=None, verbose=True):
    """Scan one build (translation units + their flags, -D set); returns hits."""
    tmp = tmp or tempfile.mkdtemp()
    bad = 0
    for src, extra in srcs:
        out = os.path.join(tmp, f"{label}.{src}.s")
        compile_asm(src, extra, out, defines)
        with open(out) as f:
            hits = scan(f)
        for h in hits:
            if verbose:
                print("[%s] %s:%d %s -> %s" % (label, src, *h))
        bad += len(hits)
    return bad


def main(names=None, jobs=None):
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd import build as B  # the product build's flags
    tmp = tempfile.mkdtemp()
    todo = [(n, v) for n, v in B.VARIANTS.items() if not names or n in names]
    jobs = jobs or max(1, min(8, os.cpu_count() or 1, len(todo)))
    with ThreadPoolExecutor(jobs) as ex:  # each job is a hipcc child process
        counts = list(ex.map(lambda nv: check_build(B.sources(nv[1][1]), nv[1][0], nv[0], tmp), todo))
    for (name, _), n in zip(todo, counts):
        print(f"{name}: wide-store data hazards: {n}")
    return 1 if sum(counts) else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or None))
