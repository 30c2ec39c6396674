set -o pipefail
mkdir -p gpurun_out/g27
run() {
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=$1 NT_TRATIO=$2 timeout -k 10 200 python bench.py --no-cpu-baseline $3 > gpurun_out/g27/$n.log 2>&1 || { tail -5 gpurun_out/g27/$n.log; exit 1; }
  echo "tsub=$1 ratio=$2 $3: $(tail -1 gpurun_out/g27/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["kernel_launches_per_step"], r["call_kernel_avg_ms"])')"
}
run 1 1
run 2 1
run 2 0.25
run 3 0.25
run 3 0.35
run 4 0.3
run 3 0.2
