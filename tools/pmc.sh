#!/bin/bash
# PMC passes for the bench kernels (rocprofv3 --pmc, kernel trace only; one
# counter group per pass).  usage: tools/pmc.sh OUTDIR [bench args...]
# Writes OUTDIR/p<i>/p_counter_collection.csv; summarise with tools/pmc_summary.py.
set -u
out=$1; shift
args="$*"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
passes=(
  "FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM"
  "WRITE_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT SQ_INSTS_BRANCH"
  "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SCRATCH_LOAD SQ_INSTS_SCRATCH_STORE"
)
mkdir -p "$out"
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p --kernel-trace --output-format csv -d "$out/p$i" -o p -- \
    python3 bench.py --no-cpu-baseline $args > "$out/p$i.log" 2>&1
  st=$?
  echo "pass $i ($p): exit $st"
  if [ $st -ne 0 ]; then tail -5 "$out/p$i.log"; fi
  if [ $st -eq 124 ] || [ $st -gt 128 ]; then exit $st; fi
done
