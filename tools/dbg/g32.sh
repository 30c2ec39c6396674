set -o pipefail
mkdir -p gpurun_out/g34
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g34/tests.log 2>&1 || { tail -40 gpurun_out/g34/tests.log; exit 1; }
tail -1 gpurun_out/g34/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g34/smoke.log 2>&1 || { tail -20 gpurun_out/g34/smoke.log; exit 1; }
tail -1 gpurun_out/g34/smoke.log
run() {
  n=$(echo "x$1$2" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 $3 > gpurun_out/g34/$n.log 2>&1 || { tail -5 gpurun_out/g34/$n.log; exit 1; }
  echo "tsub=$1 $3: $(tail -1 gpurun_out/g34/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"], r["frac"])')"
}
run 1 a
run 2 a
run 2 b
run 1 c --per-read
