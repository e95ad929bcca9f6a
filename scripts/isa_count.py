"""Static VALU count of one plane pass (the plane kernel's largest basic
block is plane::pass inlined), for bench.py's useful_lane_frac.

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


def main():
    asm = os.path.join(tempfile.mkdtemp(), "plane.s")
    sys.path.insert(0, ROOT)
    from sudoku_solver_distributed_amd import build as B  # same flags as the product build
    extra = dict(B.SRCS)["plane_kernels.hip"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *extra,
                           "--cuda-device-only", "-S", "-o", asm, SRC], stderr=subprocess.DEVNULL)
    lines = open(asm).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith("_Z12plane_kernel"))
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
    c = collections.Counter(body)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    out = {"kernel": "plane_kernel", "source": "plane_kernels.hip (hipcc -O3 gfx950 %s)" % " ".join(extra),
           "pass_block_instructions": len(body), "valu_per_pass": valu,
           "salu_per_pass": sum(v for k, v in c.items() if k.startswith("s_")),
           "top": c.most_common(8)}
    path = os.path.join(ROOT, "profiles", "isa_plane_pass.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    sys.exit(main())
