#!/bin/bash
# Same-box A/B of _ab/old against the working tree on c4 (2 M reads) and c3 (2 M), twice, alternating.
set -o pipefail
tag=${1:-abc4}
mkdir -p gpurun_out/$tag
for i in 1 2; do
 for v in old new; do
  for c in c4 c3; do
   if [ $v = old ]; then b=_ab/old/bench.py; else b=bench.py; fi
   timeout -k 10 200 python -u $b --config $c --reads 2000000 --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/$tag/${v}_${c}_$i.log 2>&1 || exit 1
  done
 done
done
python3 - "$tag" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d["value"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"], d["roofline"]["call_exposed_ms"])
PY
