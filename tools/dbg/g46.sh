set -o pipefail
mkdir -p gpurun_out/g46
timeout -k 10 120 python tools/dbg/tlayout_check.py 13001 > gpurun_out/g46/tl1.log 2>&1 || { tail -20 gpurun_out/g46/tl1.log; exit 1; }
tail -1 gpurun_out/g46/tl1.log
timeout -k 10 120 python tools/dbg/tlayout_check.py 6451 > gpurun_out/g46/tl2.log 2>&1 || { tail -20 gpurun_out/g46/tl2.log; exit 1; }
tail -1 gpurun_out/g46/tl2.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g46/prof -o run -- python3 tools/dbg/tlayout_big.py > gpurun_out/g46/big.log 2>&1 || { tail -5 gpurun_out/g46/big.log; exit 1; }
grep -E "bundle" gpurun_out/g46/prof/run_kernel_stats.csv | cut -c1-150
