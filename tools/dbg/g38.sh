set -o pipefail
mkdir -p gpurun_out/g38
timeout -k 10 300 python bench.py > gpurun_out/g38/bench.log 2>&1 || { tail -5 gpurun_out/g38/bench.log; exit 1; }
tail -1 gpurun_out/g38/bench.log | cut -c1-600
bash tools/profile_round.sh gpurun_out/g38/prof
grep -E "tscan|call|bundle" gpurun_out/g38/prof/stats/run_kernel_stats.csv | cut -c1-140
