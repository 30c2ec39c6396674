#!/bin/bash
# Bench sweep over hiprtc compile options of the scan (NT_JIT_OPTS), one
# option set per argument: [BENCH_ARGS=..] tools/jit_sweep.sh "" "-DX=1 -DY=1" ...
set -u
i=0
for opts in "$@"; do
  i=$((i+1))
  echo "=== NT_JIT_OPTS='$opts'"
  NT_JIT_OPTS="$opts" timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/jsweep_$i.log 2>&1
  st=$?
  python3 -c "import json; d=json.loads(open('gpurun_out/jsweep_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'scan', r['kernel_avg_ms'], 'call', r.get('call_exposed_ms'), 'callk', r['call_kernel_avg_ms'], 'frac', r['frac'])" || tail -3 gpurun_out/jsweep_$i.log
  if [ $st -eq 124 ] || [ $st -gt 128 ]; then break; fi
done
