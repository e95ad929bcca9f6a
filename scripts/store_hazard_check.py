"""Static check of the gfx950 wide-store data hazard in the product kernels.

A buffer/global store of more than 64 bits reads its data VGPRs after
issue; a VALU write to one of them needs a wait state in between.  hipcc
(ROCm 7.2) pads this only when a MUBUF store's soffset is an inline constant,
so a buffer_store_dwordx4 with a REGISTER soffset (offset > 64 bytes) can be
followed at once by a VALU write of its data.  In the plane kernel's stack
push that corrupted search levels (~0.65 % of boards ended UNSOLVABLE); the
push now keeps its data live through an s_nop (plane_kernel.h PlaneStack::push).

    python scripts/store_hazard_check.py   # compiles both .hip files to asm, exit 1 on a hit
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sudoku_solver_distributed_amd", "csrc")
STORE = re.compile(r"(buffer|global|flat)_store_dwordx([34])\s")


def _regs(spec):
    m = re.match(r"v\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", spec)
    return {int(m.group(1))} if m else set()


def scan(lines):
    """(line number, store, offending instruction) for every wide store whose
    data VGPR is written by the next instruction without a wait state."""
    lines = [l.strip() for l in lines]
    hits = []
    for i, l in enumerate(lines):
        m = STORE.match(l)
        if not m:
            continue
        ops = [x.strip() for x in l.split(None, 1)[1].split(",")]
        data = _regs(ops[0] if m.group(1) == "buffer" else ops[1])
        for t in lines[i + 1:]:
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue  # comments, directives, labels, asm markers
            if t.startswith("v_") and " " in t and _regs(t.split(None, 1)[1].split(",")[0].strip()) & data:
                hits.append((i + 1, l, t))
            break
    return hits


def compile_asm(src, extra, out):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *extra,
                           "--cuda-device-only", "-S", "-o", out, os.path.join(CSRC, src)],
                          stderr=subprocess.DEVNULL)


def main():
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd import build as B  # the product build's flags
    tmp = tempfile.mkdtemp()
    bad = 0
    for src, extra in B.SRCS:
        out = os.path.join(tmp, src + ".s")
        compile_asm(src, extra, out)
        with open(out) as f:
            hits = scan(f)
        for h in hits:
            print("%s:%d %s -> %s" % (src, *h))
        bad += len(hits)
    print("wide-store data hazards:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
