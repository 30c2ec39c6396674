set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "r6a/probe|60|./tools/fused_probe_bin 64000 50000" \
 "r6a/tests|400|python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'spanning or without_windows or short_last_read or ragged or bundle_plan or example'" \
 "r6a/bench|200|python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline" \
 "r6a/sqA|150|cd /tmp && rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6a/sqA -o p -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1" \
 "r6a/sqB|150|cd /tmp && rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6a/sqB -o p -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1"
