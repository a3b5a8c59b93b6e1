#!/usr/bin/env python
"""VGPR / AGPR / LDS usage of the compiled kernels of one .hip source (occupancy check):

    python tools/vgprs.py csrc/kernels/gemm_glds.hip [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-I" + os.path.join(ROOT, "csrc", "kernels"), "--cuda-device-only", "-S", src, "-o", out],
                       check=True, stderr=subprocess.DEVNULL)
        s = open(out).read()
    for b in s.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        if filt not in name:
            continue
        agpr = re.match(r":\s+(\d+)", b).group(1)
        v = re.search(r"\.vgpr_count:\s+(\d+)", b).group(1)
        lds = re.search(r"\.group_segment_fixed_size:\s+(\d+)", b).group(1)
        scr = re.search(r"\.private_segment_fixed_size:\s+(\d+)", b)
        scr = scr.group(1) if scr else "?"
        print(f"{name[:70]:70s} vgpr {v:>4s} agpr {agpr:>4s} lds {lds:>6s} scratch {scr:>5s}")


if __name__ == "__main__":
    main()
