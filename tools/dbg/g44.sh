set -o pipefail
mkdir -p gpurun_out/g44
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g44/tests.log 2>&1 || { tail -40 gpurun_out/g44/tests.log; exit 1; }
tail -1 gpurun_out/g44/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g44/smoke.log 2>&1 || { tail -20 gpurun_out/g44/smoke.log; exit 1; }
tail -1 gpurun_out/g44/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/g44/bench.log 2>&1 || { tail -5 gpurun_out/g44/bench.log; exit 1; }
tail -1 gpurun_out/g44/bench.log | cut -c1-300
for c in c10k c4 c3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --reads 2000000 > gpurun_out/g44/$c.log 2>&1 || { tail -5 gpurun_out/g44/$c.log; exit 1; }
  echo "$c: $(tail -1 gpurun_out/g44/$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["kernel_launches_per_step"], r["call_kernel_avg_ms"], d["config"]["scan_path"])')"
done
bash tools/profile_round.sh gpurun_out/g44/prof
