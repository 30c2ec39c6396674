set -o pipefail
mkdir -p gpurun_out
CFG=c50k NT_DBG_POISON_AUX=165 timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 0 > gpurun_out/g52a.log 2>&1 && head -c 3000 gpurun_out/g52a.log &&
CFG=c50k POISON_TP=1 timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 0 > gpurun_out/g52b.log 2>&1 && head -c 3000 gpurun_out/g52b.log &&
CFG=c4 POISON_TP=1 timeout -k 10 300 python -u tools/dbg/fullsize_diff.py 20000 0.05 > gpurun_out/g52c.log 2>&1 && head -c 3000 gpurun_out/g52c.log
