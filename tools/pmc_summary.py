"""Summarise tools/pmc.sh output: per kernel, the mean of each counter per
dispatch (FETCH_SIZE doubled: gfx950 reports half of wide streaming reads,
MI355X_MICROARCH.md "HBM")."""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "p_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in out[k]:
            out[k]["HBM_READ_BYTES"] = out[k]["FETCH_SIZE"] * 1024 * 2  # KB, x2 (gfx950)
        if "WRITE_SIZE" in out[k]:
            out[k]["HBM_WRITE_BYTES"] = out[k]["WRITE_SIZE"] * 1024
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    for k, cs in res.items():
        if not k.startswith("nt") and "nt_" not in k:
            continue
        print(k[:90])
        for c in sorted(cs):
            print(f"   {c:28s} {cs[c]:.6g}")
