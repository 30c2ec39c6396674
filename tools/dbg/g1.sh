set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/g1/tests.log 2>&1 || { tail -30 gpurun_out/g1/tests.log; exit 1; }
tail -3 gpurun_out/g1/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/g1/b3.log 2>&1 && tail -1 gpurun_out/g1/b3.log | cut -c1-400
NT_JIT_OPTS="-DNT_TSCAN_WAVES_EU=4" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/g1/b4.log 2>&1 && tail -1 gpurun_out/g1/b4.log | cut -c1-400
NT_JIT_OPTS="-DNT_TS_XPRIME=1" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/g1/bx.log 2>&1 && tail -1 gpurun_out/g1/bx.log | cut -c1-400
