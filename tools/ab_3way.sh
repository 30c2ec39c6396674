#!/bin/bash
# Same-box A/B/C: _ab/old, _ab/exp and the working tree on c4 (2 M reads) and
# c5, twice, alternating.  tools/ab_3way.sh TAG
set -o pipefail
tag=${1:-ab3w}
mkdir -p gpurun_out/$tag
for i in 1 2; do
 for v in old exp new; do
  for c in ${AB_CONFIGS:-c4 c5}; do
   case $v in old) b=_ab/old/bench.py;; exp) b=_ab/exp/bench.py;; *) b=bench.py;; esac
   extra=""; case $c in c4|c3) extra="--reads 2000000";; esac
   timeout -k 10 200 python -u $b --config $c $extra --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/$tag/${v}_${c}_$i.log 2>&1 || exit 1
  done
 done
done
python3 - "$tag" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], d["value"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])
PY
