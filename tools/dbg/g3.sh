set -o pipefail
mkdir -p gpurun_out/g3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/g3/tests.log 2>&1 || { tail -30 gpurun_out/g3/tests.log; exit 1; }
tail -2 gpurun_out/g3/tests.log
for v in "" "-DNT_TS_DBG_NOWALK=1" "-DNT_TSCAN_WAVES_EU=4"; do
  n=$(echo "x$v" | tr -c 'a-zA-Z0-9' '_')
  NT_JIT_OPTS="$v" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/g3/$n.log 2>&1 || { tail -5 gpurun_out/g3/$n.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/g3/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
done
