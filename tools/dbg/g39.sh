set -o pipefail
mkdir -p gpurun_out/g41
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "bundle or example or offsets or subbatch or random" > gpurun_out/g41/tests.log 2>&1 || { tail -30 gpurun_out/g41/tests.log; exit 1; }
tail -1 gpurun_out/g41/tests.log
run() {  # dir tsub tag
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  (cd $1 && NT_TSUB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10) > gpurun_out/g41/$n.log 2>&1 || { tail -5 gpurun_out/g41/$n.log; exit 1; }
  echo "$1 tsub=$2: $(tail -1 gpurun_out/g41/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for i in a b; do run $R 2 $i; run $R/.abtest/u16 2 $i; run $R 1 $i; run $R/.abtest/u16 1 $i; done
