set -o pipefail
mkdir -p gpurun_out/g30
python -c "import ctypes; h=ctypes.CDLL('libamdhip64.so'); lo=ctypes.c_int(); hi=ctypes.c_int(); h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)); print('prio range', lo.value, hi.value)"
run() {
  n=$(echo "x$1$2" | tr -c 'a-zA-Z0-9' '_')
  NT_CALL_PRIO=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/g30/$n.log 2>&1 || { tail -5 gpurun_out/g30/$n.log; exit 1; }
  echo "prio=$1: $(tail -1 gpurun_out/g30/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"])')"
}
for i in 1 2; do run 0 $i; run -1 $i; run 1 $i; done
