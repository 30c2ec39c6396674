#!/bin/bash
# Run GPU steps one after another; stop at the first crash-like exit status
# (timeout 124/137, abort 134, segfault 139, or a negative signal), continue
# past ordinary failures (status 1) so the rest of the evidence is collected.
# usage: tools/gpu_steps.sh "name|timeout_s|command" ...
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (timeout ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
  st=$?
  echo "=== [$name] exit=$st in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/${name}.log"
  case $st in
    124|134|137|139) echo "crash-like status $st: stopping"; exit $st;;
  esac
  if [ $st -gt 128 ]; then echo "signal status $st: stopping"; exit $st; fi
done
exit 0
