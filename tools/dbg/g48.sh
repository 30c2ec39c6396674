set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 400000 > gpurun_out/g48a.log 2>&1 && cat gpurun_out/g48a.log &&
timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 > gpurun_out/g48b.log 2>&1 && cat gpurun_out/g48b.log &&
timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 400000 0 > gpurun_out/g48c.log 2>&1 && cat gpurun_out/g48c.log
