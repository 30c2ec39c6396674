set -o pipefail
mkdir -p gpurun_out/g51
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g51/tests.log 2>&1 || { tail -40 gpurun_out/g51/tests.log; exit 1; }
tail -5 gpurun_out/g51/tests.log
