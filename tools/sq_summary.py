"""Per-kernel means of rocprofv3 --pmc counter CSVs (one dir per pass):
python3 tools/sq_summary.py DIR [DIR...]; derived ratios for the bundle scan."""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "nt_" not in k:
                continue
            k = k.split("(")[0].split(" ")[-1][:40]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k, "launches", len(next(iter(d.values()))))
    for c in sorted(m):
        print("   %-22s %.4g" % (c, m[c]))
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
            if c in m:
                print("   %-22s %.3f of wave cycles" % (c, m[c] / wc))
    if "SQ_INSTS_LDS" in m and "SQ_LDS_BANK_CONFLICT" in m and m["SQ_INSTS_LDS"]:
        print("   bank-conflict cycles per LDS instruction %.3f" % (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]))
