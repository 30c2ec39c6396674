set -o pipefail
mkdir -p gpurun_out/g43
NT_JIT_OPTS="-DNT_TS_RING=12 -DNT_TSCAN_WAVES_EU=1 -DNT_TS_XPRIME=1" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "bundle or example" > gpurun_out/g43/tests.log 2>&1 || { tail -30 gpurun_out/g43/tests.log; exit 1; }
tail -1 gpurun_out/g43/tests.log
run() {
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=$2 NT_JIT_OPTS="$1" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/g43/$n.log 2>&1 || { tail -5 gpurun_out/g43/$n.log; exit 1; }
  echo "$1 tsub=$2: $(tail -1 gpurun_out/g43/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for i in a b; do
run "" 2 $i
run "-DNT_TS_RING=12 -DNT_TSCAN_WAVES_EU=1 -DNT_TS_XPRIME=1" 2 $i
run "-DNT_TS_RING=12 -DNT_TSCAN_WAVES_EU=1" 2 $i
run "-DNT_TS_RING=16 -DNT_TSCAN_WAVES_EU=1 -DNT_TS_XPRIME=1" 1 $i
done
