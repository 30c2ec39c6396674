#!/bin/bash
# Bench sweep over environment knobs: [BENCH_ARGS=..] tools/sweep.sh "ENV=.. ENV=.." ...
set -u
for spec in "$@"; do
  echo "=== $spec"
  env $spec timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/sweep.log 2>&1
  st=$?
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'scan', r['kernel_avg_ms'], 'call', r['call_kernel_avg_ms'])" || tail -3 gpurun_out/sweep.log
  if [ $st -eq 124 ] || [ $st -gt 128 ]; then break; fi
done
