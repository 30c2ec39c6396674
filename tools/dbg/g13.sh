set -o pipefail
mkdir -p gpurun_out/g13
run() {
  n=$(echo "x$1$2$3" | tr -c 'a-zA-Z0-9' '_')
  NT_TSCAN_BPC=$2 NT_JIT_OPTS="$1" timeout -k 10 200 python bench.py --no-cpu-baseline $3 > gpurun_out/g13/$n.log 2>&1 || { tail -5 gpurun_out/g13/$n.log; exit 1; }
  echo "$1 bpc=$2 $3: $(tail -1 gpurun_out/g13/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
run "" 8
run "-DNT_TS_DBG_NOCNT=1" 8
run "-DNT_TS_DBG_NOAUX=1" 8
run "-DNT_TS_DBG_NOAUX=1 -DNT_TS_DBG_NOCNT=1" 8
run "-DNT_TS_DBG_NOOUT=1" 8
run "" 1
