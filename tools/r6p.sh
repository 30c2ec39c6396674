set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6p
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6p/profile_c5|600|bash tools/profile_round.sh gpurun_out/r6p/c5" \
 "r6p/traffic|60|python3 tools/traffic_json.py gpurun_out/r6p/c5 c5 12500000 1 gpurun_out/r6p/pmc_traffic_c5.json" \
 "r6p/sqA|150|cd /tmp && rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6p/sqA -o p -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1" \
 "r6p/sqB|150|cd /tmp && rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6p/sqB -o p -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1" \
 "r6p/bench_c4|200|python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/r6p/bench_c4.json" \
 "r6p/bench_c3|200|python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/r6p/bench_c3.json" \
 "r6p/bench_c10k|200|python -u bench.py --config c10k --no-cpu-baseline > gpurun_out/r6p/bench_c10k.json" \
 "r6p/bench_c50k|200|python -u bench.py --config c50k --no-cpu-baseline > gpurun_out/r6p/bench_c50k.json" \
 "r6p/bench_c5|200|python -u bench.py > gpurun_out/r6p/bench_c5.json"
