set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6j/smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "r6j/gpu_tests|1000|python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread" \
 "r6j/bench|300|python -u bench.py"
