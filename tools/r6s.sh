set -u
cd "$GRAFT_REPO_ROOT"
tag=${1:-r6s}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "$tag/bench_c5|200|python -u bench.py --no-cpu-baseline > gpurun_out/$tag/bench_c5.json" \
 "$tag/bench_c4|200|python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/$tag/bench_c4.json" \
 "$tag/bench_c10k|200|python -u bench.py --config c10k --no-cpu-baseline > gpurun_out/$tag/bench_c10k.json"
