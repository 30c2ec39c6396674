set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6g
tools/gpu_steps.sh \
 "r6g/tests|500|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 'p3 or tvr or random_reads or baseline_config or bundle or merged or mixed or exceptions or c4'" \
 "r6g/ab|600|bash tools/ab_c4.sh r6g/ab"
