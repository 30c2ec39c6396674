set -o pipefail
mkdir -p gpurun_out/g37
R=$(pwd)
run() {  # dir tsub tag
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  (cd $1 && NT_TSUB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10) > gpurun_out/g37/$n.log 2>&1 || { tail -5 gpurun_out/g37/$n.log; exit 1; }
  echo "$1 tsub=$2: $(tail -1 gpurun_out/g37/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for i in a b; do run $R 2 $i; run $R/.abtest/u16 2 $i; run $R 1 $i; run $R/.abtest/u16 1 $i; done
