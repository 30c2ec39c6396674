set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6f
for pt in 0.0 0.5 1.0; do
  for pl in "" "--no-pipeline"; do
    timeout -k 10 150 python -u bench.py --config c10k --steps 10 --warmup 5 --no-cpu-baseline --p-tract $pt $pl > gpurun_out/r6f/c10k_${pt}${pl}.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6f/*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); r = d["roofline"]
            print(f.split("/")[-1], d["value"], "step", d["ms_per_step"], "scan", r["kernel_avg_ms"], "call", r["call_kernel_avg_ms"], "exposed", r["call_exposed_ms"], "telo", d["config"]["telomeric_reads_rank0"])
PY
