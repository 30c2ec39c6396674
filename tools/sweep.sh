#!/bin/bash
# Bench sweep over environment knobs: [BENCH_ARGS=..] tools/sweep.sh "ENV=.. ENV=.." ...
# (a '+' inside a value is a space: "NT_JIT_OPTS=-DA=1+-DB=2")
# one log per spec (gpurun_out/sw_<i>.log), a summary line per spec on stdout
set -u
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i + 1))
  log=gpurun_out/sw_$i.log
  echo "=== [$i] $spec"
  # "K=V K2=V2": exported for the run; a '+' in a value stands for a space
  # (NT_JIT_OPTS=-DA=1+-DB=2)
  ( for kv in $spec; do k=${kv%%=*}; v=${kv#*=}; export "$k=${v//+/ }"; done
    timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} ) > $log 2>&1
  st=$?
  python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'scan', r['kernel_avg_ms'], 'call', r.get('call_exposed_ms'), 'callk', r['call_kernel_avg_ms'])" || tail -3 $log
  if [ $st -eq 124 ] || [ $st -gt 128 ]; then echo "status $st: stopping"; break; fi
done
