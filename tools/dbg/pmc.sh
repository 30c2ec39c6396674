# PMC passes on bench.py (2 steps) for a JIT option variant: tools/dbg/pmc.sh OUT "opts" "counters..." ...
set -o pipefail
out=$1; shift; opts=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for c in "$@"; do
  i=$((i+1))
  NT_JIT_OPTS="$opts" timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/p$i" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
done
echo done
