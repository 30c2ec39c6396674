set -o pipefail
mkdir -p gpurun_out/g18
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g18/tests.log 2>&1 || { tail -40 gpurun_out/g18/tests.log; exit 1; }
tail -1 gpurun_out/g18/tests.log
timeout -k 10 300 python bench.py > gpurun_out/g18/bench.log 2>&1 || { tail -5 gpurun_out/g18/bench.log; exit 1; }
tail -1 gpurun_out/g18/bench.log
for c in c10k c4 c3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --reads 2000000 > gpurun_out/g18/$c.log 2>&1 || { tail -5 gpurun_out/g18/$c.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/g18/$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["call_kernel_avg_ms"], d["config"]["scan_path"])')"
done
bash tools/profile_round.sh gpurun_out/g18/prof
