#!/bin/bash
# Bench alternative builds of libnanotel.so shipped under variants/ (tuning):
# each is swapped in, benched, and the original restored.
set -u
lib=telomere-analyzer_amd/nanotel_amd/libnanotel.so
cp $lib /tmp/libnanotel.orig.so
for v in "$@"; do
  cp "variants/$v" $lib
  echo "=== $v"
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "gpurun_out/bench_$v.log" 2>&1
  st=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'scan', r['kernel_avg_ms'], 'call', r.get('call_exposed_ms'), 'callk', r['call_kernel_avg_ms'])" || tail -3 "gpurun_out/bench_$v.log"
  if [ $st -eq 124 ] || [ $st -gt 128 ]; then break; fi
done
cp /tmp/libnanotel.orig.so $lib
