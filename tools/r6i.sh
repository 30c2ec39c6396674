set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6i
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6i/tail|300|python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'short_last_half_stripe or ragged or full_size_config_sampled_vs_oracle and c10k'" \
 "r6i/ab|700|bash tools/ab3.sh r6i/ab" \
 "r6i/abc4|700|bash tools/ab_c4.sh r6i/abc4"
