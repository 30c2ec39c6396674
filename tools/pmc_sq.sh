#!/bin/bash
# SQ issue/stall breakdown of the scan and call kernels for a bench config
# (one PMC pass, 8 SQ counters + GRBM_GUI_ACTIVE; PMC="..." overrides the set).
# usage: [PMC=..] tools/pmc_sq.sh OUTDIR [bench args]
set -u
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
PMC=${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE}
timeout -s KILL 120 rocprofv3 --pmc $PMC \
  --kernel-trace --output-format csv -d "$out/sq" -o p -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" \
  > "$out/sq.log" 2>&1
st=$?
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/sq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "nt_" not in k: continue
        k = k.split("(")[0].split(" ")[-1][:40]  # the kernel's name (a split calling kernel per pass)
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: sum(v) / len(v) for c, v in sorted(d.items())})
PY
exit $st
