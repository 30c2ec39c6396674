set -o pipefail
mkdir -p gpurun_out/g26
timeout -k 10 120 python tools/dbg/tlayout_check.py 13001 > gpurun_out/g26/tl1.log 2>&1 || { tail -20 gpurun_out/g26/tl1.log; exit 1; }
tail -1 gpurun_out/g26/tl1.log
timeout -k 10 120 python tools/dbg/tlayout_check.py 6451 > gpurun_out/g26/tl2.log 2>&1 || { tail -20 gpurun_out/g26/tl2.log; exit 1; }
tail -1 gpurun_out/g26/tl2.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g26/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --no-cpu-baseline > gpurun_out/g26/bench.log 2>&1 || { tail -5 gpurun_out/g26/bench.log; exit 1; }
grep -E "bundle" gpurun_out/g26/prof/run_kernel_stats.csv | cut -c1-150
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bundle or example or random" > gpurun_out/g26/tests.log 2>&1 || { tail -30 gpurun_out/g26/tests.log; exit 1; }
tail -1 gpurun_out/g26/tests.log
grep -E "tscan" gpurun_out/g26/prof/run_kernel_stats.csv | cut -c1-150
