set -o pipefail
mkdir -p gpurun_out/g47
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "full_size" > gpurun_out/g47/tests.log 2>&1 || { tail -30 gpurun_out/g47/tests.log; exit 1; }
tail -4 gpurun_out/g47/tests.log
