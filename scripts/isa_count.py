"""Static VALU count of one plane pass, for bench.py's useful_lane_frac:
the loop body of scripts/microbench/pass_rate.hip (plane::pass alone on a
register-resident board, same flags as the product build), minus its
accumulate; and, for reference, the plane kernel's largest basic block
(the pass inlined, with whatever the scheduler moved in or out of it).

    python scripts/isa_count.py   -> profiles/isa_plane_pass.json
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "sudoku_solver_distributed_amd", "csrc", "plane_kernels.hip")
MICRO = os.path.join(ROOT, "scripts", "microbench", "pass_rate.hip")
ACC_VALU = 4  # pass_rate's `acc += r + und[0] + und[1] + und[2]`


def largest_block(src, extra, symbol):
    asm = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *extra,
                           "--cuda-device-only", "-S", "-o", asm, src], stderr=subprocess.DEVNULL)
    lines = open(asm).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(symbol))
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    blocks, cur = [], []
    for l in lines[st:en]:
        if re.match(r"^\S+:", l):
            blocks.append(cur)
            cur = []
        else:
            t = l.strip()
            if t and not t.startswith((";", ".")):
                cur.append(t.split()[0])
    blocks.append(cur)
    body = max(blocks, key=len)
    return collections.Counter(body), len(body)


def main():
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd import build as B  # same flags as the product build
    extra = dict(B.SRCS)["plane_kernels.hip"]
    c, n = largest_block(MICRO, extra, "_Z9pass_loop")
    valu = sum(v for k, v in c.items() if k.startswith("v_")) - ACC_VALU
    ck, nk = largest_block(SRC, extra, "_Z12plane_kernel")
    out = {"kernel": "plane_kernel", "source": "plane::pass alone (scripts/microbench/pass_rate.hip loop body, "
                                               "hipcc -O3 gfx950 %s)" % " ".join(extra),
           "pass_block_instructions": n, "valu_per_pass": valu,
           "salu_per_pass": sum(v for k, v in c.items() if k.startswith("s_")),
           "top": c.most_common(8),
           "kernel_largest_block_valu": sum(v for k, v in ck.items() if k.startswith("v_"))}
    path = os.path.join(ROOT, "profiles", "isa_plane_pass.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    sys.exit(main())
