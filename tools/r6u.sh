set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6u
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6u/smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "r6u/gpu_tests|1000|python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread" \
 "r6u/bench|300|python -u bench.py"
