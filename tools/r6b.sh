set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_steps.sh \
 "r6b/tests|500|python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'spanning or without_windows or short_last_read or ragged or bundle or example or random_reads or mixed or merged or short or exceptions or pipelined'" \
 "r6b/bench_c5|200|python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline" \
 "r6b/bench_c50k|200|python -u bench.py --config c50k --steps 10 --warmup 3 --no-cpu-baseline" \
 "r6b/sqB|150|cd /tmp && rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $R/gpurun_out/r6b/sqB -o p -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1" \
 "r6b/sqA|150|cd /tmp && rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/r6b/sqA -o p -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1" \
 "r6b/pcs|120|cd /tmp && timeout -s KILL 100 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d $R/gpurun_out/r6b/pcs -o p -- python3 $R/bench.py --config c50k --no-cpu-baseline --steps 3 --warmup 1"
