#!/bin/bash
# Same-box A/B of _ab/old (see tools/ab_run.sh) against the working tree on
# c5 (the metric's configuration), c50k and c10k, twice, alternating.
# tools/ab3.sh TAG
set -o pipefail
tag=${1:-ab}
mkdir -p gpurun_out/$tag
for i in 1 2; do
 for v in old new; do
  for c in c5 c50k c10k; do
   if [ $v = old ]; then b=_ab/old/bench.py; else b=bench.py; fi
   timeout -k 10 150 python -u $b --config $c --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/$tag/${v}_${c}_$i.log 2>&1 || exit 1
  done
 done
done
python3 - "$tag" <<'PY'
import json, glob, sys, re
tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}/*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d["value"], d["roofline"]["kernel_avg_ms"], d["roofline"]["call_exposed_ms"])
PY
