set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6c
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6c/tests|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread -k 'bundle or ragged or example or short or e2e or cli or driver or filter'" \
 "r6c/ab|400|bash tools/ab3.sh r6c/ab" \
 "r6c/host4k|200|python -u tools/host_path_bench.py --reads 4000 > gpurun_out/r6c/host_path_4000.json" \
 "r6c/host16k|200|python -u tools/host_path_bench.py --reads 16000 > gpurun_out/r6c/host_path_16000.json" \
 "r6c/e2e|600|python -u tools/e2e_bench.py --reads 80000 --plots --gzip-levels 6,1 --cleanup > gpurun_out/r6c/e2e_plain_80000x50kb.json"
