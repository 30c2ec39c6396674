#!/bin/bash
# Round profile evidence for bench.py's default workload:
#  1. rocprofv3 --kernel-trace --stats of the bench command itself,
#  2. two PMC passes (FETCH_SIZE, WRITE_SIZE: separate, they do not fit one pass)
# then tools/traffic_json.py turns them into profiles/pmc_traffic.json.
# usage: tools/profile_round.sh OUTDIR [extra bench args]
set -u
out=$1; shift
args="$*"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- \
  python3 bench.py --no-cpu-baseline $args > "$out/stats.log" 2>&1 || { echo "stats pass failed"; tail -5 "$out/stats.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/$c" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $args > "$out/$c.log" 2>&1 || { echo "$c pass failed"; tail -5 "$out/$c.log"; exit 1; }
done
echo "profile passes done"
