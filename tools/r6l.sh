set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6l
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6l/tests|600|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'bundle or ragged or example or short or spanning or windows or tvr or offsets or full_size_config_sampled_vs_oracle'" \
 "r6l/ab|700|bash tools/ab3.sh r6l/ab" \
 "r6l/abc4|700|bash tools/ab_c4.sh r6l/abc4"
