set -o pipefail
mkdir -p gpurun_out/g19
timeout -k 10 120 python tools/dbg/tlayout_check.py 13001 > gpurun_out/g19/tl1.log 2>&1 || { tail -20 gpurun_out/g19/tl1.log; exit 1; }
tail -2 gpurun_out/g19/tl1.log
timeout -k 10 120 python tools/dbg/tlayout_check.py 3001 > gpurun_out/g19/tl2.log 2>&1 || { tail -20 gpurun_out/g19/tl2.log; exit 1; }
tail -1 gpurun_out/g19/tl2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/g19/tests.log 2>&1 || { tail -30 gpurun_out/g19/tests.log; exit 1; }
tail -1 gpurun_out/g19/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g19/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/g19/bench.log 2>&1 || { tail -5 gpurun_out/g19/bench.log; exit 1; }
grep -E "bundle|tscan|call" gpurun_out/g19/prof/run_kernel_stats.csv | cut -c1-150
