set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6m
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6m/tests|600|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'bundle or ragged or example or short or spanning or windows or tvr or offsets or full_size_config_sampled_vs_oracle'" \
 "r6m/ab|700|AB_CONFIGS='c5 c50k c10k' bash tools/ab_3way.sh r6m/ab"
