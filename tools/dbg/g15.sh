set -o pipefail
mkdir -p gpurun_out/g15
run() {
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  NT_TSCAN_BPC=$2 NT_JIT_OPTS="$1" timeout -k 10 200 python bench.py --no-cpu-baseline $3 > gpurun_out/g15/$n.log 2>&1 || { tail -5 gpurun_out/g15/$n.log; exit 1; }
  echo "$1 bpc=$2 $3: $(tail -1 gpurun_out/g15/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
run "" 1
run "-DNT_TSCAN_WAVES_EU=1" 1
run "-DNT_TSCAN_WAVES_EU=1 -DNT_TS_XPRIME=1" 1
run "-DNT_TS_XPRIME=1" 1
run "" 8
