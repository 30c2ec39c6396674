set -o pipefail
mkdir -p gpurun_out/g45
R=$(pwd)
run() {  # variant config reads
  n=$(echo "x$1$2" | tr -c 'a-zA-Z0-9' '_')
  (cd $R/.abtest/$1 && NT_TSUB=1 timeout -k 10 200 python bench.py --no-cpu-baseline --config $2 --reads $3 --steps 10 --warmup 5) > gpurun_out/g45/$n.log 2>&1 || { tail -5 gpurun_out/g45/$n.log; exit 1; }
  echo "$1 $2: $(tail -1 gpurun_out/g45/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for v in base NO_ACC NO_EXT NO_FINAL NO_WRAP; do run $v c4 1000000; run $v c10k 1000000; run $v c50k 1000000; done
