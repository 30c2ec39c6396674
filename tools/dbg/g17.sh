set -o pipefail
mkdir -p gpurun_out/g17
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g17/tests.log 2>&1 || { tail -40 gpurun_out/g17/tests.log; exit 1; }
tail -1 gpurun_out/g17/tests.log
run() {
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=$2 NT_JIT_OPTS="$1" timeout -k 10 200 python bench.py --no-cpu-baseline $3 > gpurun_out/g17/$n.log 2>&1 || { tail -5 gpurun_out/g17/$n.log; exit 1; }
  echo "$1 tsub=$2 $3: $(tail -1 gpurun_out/g17/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
run "" 1
run "" 2
run "" 4
run "" 8
run "" 16
