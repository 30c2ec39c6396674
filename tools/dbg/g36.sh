set -o pipefail
mkdir -p gpurun_out/g36
run() {
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup $2 > gpurun_out/g36/$n.log 2>&1 || { tail -5 gpurun_out/g36/$n.log; exit 1; }
  echo "tsub=$1 warm=$2: $(tail -1 gpurun_out/g36/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for i in a b c; do run 2 3 $i; run 2 30 $i; run 1 30 $i; done
