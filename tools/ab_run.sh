#!/bin/bash
# A/B of two builds on one box: _ab/old (a copy of the package built from an
# earlier tree) against the working tree, c50k and c10k, twice, alternating.
# tools/ab_run.sh [extra bench args] [tag]; AB_ORDER="new old" reverses the order.
# Make _ab/old from a clean tree: git stash; python -c 'import __graft_entry__ as g;
# g.build()'; mkdir -p _ab/old; cp -r telomere-analyzer_amd bench.py tests _ab/old/;
# git stash pop; rebuild.  (_ab/ is git-ignored; delete it when done.)
set -o pipefail
extra=${1:-}; tag=${2:-ab}
mkdir -p gpurun_out
for i in 1 2; do
 for v in ${AB_ORDER:-old new}; do
  for c in c50k c10k; do
   if [ $v = old ]; then b=_ab/old/bench.py; else b=bench.py; fi
   timeout -k 10 150 python -u $b --config $c --steps 20 --warmup 10 --no-cpu-baseline $extra > gpurun_out/${tag}_${v}_${c}_$i.log 2>&1 || exit 1
  done
 done
done
