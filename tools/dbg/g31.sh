set -o pipefail
mkdir -p gpurun_out/g31
run() {
  n=$(echo "x$1$2" | tr -c 'a-zA-Z0-9' '_')
  NT_TSUB=1 NT_JIT_OPTS="$1" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/g31/$n.log 2>&1 || { tail -5 gpurun_out/g31/$n.log; exit 1; }
  echo "$1: $(tail -1 gpurun_out/g31/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for i in 1 2; do run "" $i; run "-DNT_TS_DBG_HALFCNT=1" $i; run "-DNT_TS_DBG_NOCNT=1" $i; done
