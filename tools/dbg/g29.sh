set -o pipefail
mkdir -p gpurun_out/g29
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "bundle_ranges" > gpurun_out/g29/tests.log 2>&1 || { tail -40 gpurun_out/g29/tests.log; exit 1; }
tail -4 gpurun_out/g29/tests.log
