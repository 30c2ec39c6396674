#!/bin/bash
# Timing experiments (results wrong): _ab/exp is a tuning build (make
# EXTRA=-DNT_TUNING_BUILD) whose bench copy accepts NT_JIT_OPTS; each variant
# is a -D switch of the experiment copy's nt_tscan.h.  tools/exp_run.sh TAG "opts1" "opts2" ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
for i in 1 2; do
  k=0
  for o in "" "$@"; do
    for c in c5 c50k; do
      NT_JIT_OPTS="$o" timeout -k 10 150 python -u _ab/exp/bench.py --config $c --steps 10 --warmup 5 --no-cpu-baseline \
        > gpurun_out/$tag/v${k}_${c}_$i.log 2>&1 || exit 1
    done
    k=$((k+1))
  done
done
python3 - "$tag" "" "$@" <<'PY'
import json, glob, sys
tag, opts = sys.argv[1], sys.argv[2:]
for f in sorted(glob.glob(f"gpurun_out/{tag}/*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            v = int(f.split("/")[-1][1:].split("_")[0])
            print(f.split("/")[-1], repr(opts[v]), d["value"], d["roofline"]["kernel_avg_ms"])
PY
