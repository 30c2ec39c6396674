#!/bin/bash
# One GPU round trip of the bundle-scan inner loop: the bundle-scan parity
# tests and a c50k bench line (tag: output suffix).
set -o pipefail
tag=${1:-q}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "example or bundle or ragged or mixed or short or plan" > gpurun_out/t_$tag.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config c50k --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/b_$tag.log 2>&1
