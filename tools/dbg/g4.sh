set -o pipefail
mkdir -p gpurun_out/g4
for v in "-DNT_TS_DBG_NOOUT=1" "-DNT_TS_DBG_NOOUT=1 -DNT_TSCAN_WAVES_EU=4" "-DNT_TS_XPRIME=1" "-DNT_TS_PIN=0"; do
  n=$(echo "x$v" | tr -c 'a-zA-Z0-9' '_')
  NT_JIT_OPTS="$v" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/g4/$n.log 2>&1 || { tail -5 gpurun_out/g4/$n.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/g4/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
done
