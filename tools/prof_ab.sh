set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in old new; do
  if [ $v = old ]; then b=_ab/old/bench.py; else b=bench.py; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run -- python3 $b --config c50k --steps 10 --warmup 5 --no-cpu-baseline --no-pipeline > gpurun_out/prof_$v.log 2>&1 || exit 1
done
