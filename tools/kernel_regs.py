#!/usr/bin/env python3
"""VGPR / SGPR / scratch (spill) bytes / LDS of every kernel in HIP code
objects (the .co files of the hiprtc cache or an extracted offload bundle),
from the AMDGPU metadata note (llvm-readelf --notes).
usage: tools/kernel_regs.py FILE.co [...]"""
import re
import subprocess
import sys

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
KEYS = (".name", ".vgpr_count", ".agpr_count", ".sgpr_count", ".private_segment_fixed_size",
        ".group_segment_fixed_size", ".vgpr_spill_count", ".sgpr_spill_count")


def kernels(path):
    out = subprocess.run([READELF, "--notes", path], capture_output=True, text=True, check=True).stdout
    cur, res = {}, []
    for ln in out.splitlines():
        m = re.match(r"\s*-?\s*(\.[a-z_]+):\s+(\S+)", ln)
        if not m or m.group(1) not in KEYS:
            continue
        k, v = m.group(1), m.group(2)
        if k == ".agpr_count" and cur:  # a kernel's map starts with it (keys sorted)
            res.append(cur)
            cur = {}
        if k == ".name":
            if not v.endswith(".kd"):
                cur["name"] = v
        else:
            cur[k[1:]] = v
    if cur:
        res.append(cur)
    return [k for k in res if "name" in k]


if __name__ == "__main__":
    print("%-28s %6s %6s %6s %8s %6s %6s  %s" % ("kernel", "vgpr", "agpr", "sgpr", "scratch", "vspill", "lds", "file"))
    for f in sys.argv[1:]:
        for k in kernels(f):
            print("%-28s %6s %6s %6s %8s %6s %6s  %s" % (k["name"], k.get("vgpr_count", ""), k.get("agpr_count", ""),
                                                       k.get("sgpr_count", ""), k.get("private_segment_fixed_size", ""),
                                                       k.get("vgpr_spill_count", ""), k.get("group_segment_fixed_size", ""),
                                                       f.rsplit("/", 1)[-1]))
