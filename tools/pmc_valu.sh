#!/bin/bash
# VALU/SALU instruction counts of the scan and call kernels for a bench config.
# usage: tools/pmc_valu.sh OUTDIR [bench args]
set -u
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
  --kernel-trace --output-format csv -d "$out/p1" -o p -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" \
  > "$out/p1.log" 2>&1
