set -o pipefail
mkdir -p gpurun_out
NT_DBG_POISON_AUX=165 timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 > gpurun_out/g49a.log 2>&1 && cat gpurun_out/g49a.log &&
NT_DBG_POISON_AUX=0 timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 > gpurun_out/g49b.log 2>&1 && cat gpurun_out/g49b.log
