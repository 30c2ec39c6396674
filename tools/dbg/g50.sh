set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 400000 0.05 1000000 > gpurun_out/g50a.log 2>&1 && cat gpurun_out/g50a.log &&
timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 0.05 20000 > gpurun_out/g50b.log 2>&1 && cat gpurun_out/g50b.log
