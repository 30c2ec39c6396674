set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6k
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6k/tests|600|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'bundle or ragged or example or short or spanning or windows or tvr or offsets or full_size_config_sampled_vs_oracle'" \
 "r6k/ab|700|bash tools/ab3.sh r6k/ab" \
 "r6k/abc4|700|bash tools/ab_c4.sh r6k/abc4"
tools/gpu_steps.sh \
 "r6k/vib1|60|tools/vib -1 1" \
 "r6k/vib2|60|tools/vib -1 2"
