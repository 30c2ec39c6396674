set -o pipefail
mkdir -p gpurun_out/g28
run() {
  n=$(echo "x$1$2$3$4" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=$1 NT_TRATIO=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/g28/$n.log 2>&1 || { tail -5 gpurun_out/g28/$n.log; exit 1; }
  echo "tsub=$1 ratio=$2: $(tail -1 gpurun_out/g28/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["kernel_launches_per_step"], r["call_kernel_avg_ms"])')"
}
for i in 1 2; do
run 3 0.25 $i
run 1 1 $i
run 2 1 $i
run 3 0.3 $i
done
