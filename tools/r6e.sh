set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6e
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6e/tests|400|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'bundle or ragged or example or short or mixed or merged or pipelined or spanning or windows or full_size_config_sampled_vs_oracle and c10k'" \
 "r6e/ab|400|bash tools/ab3.sh r6e/ab"
