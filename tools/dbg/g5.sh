set -o pipefail
mkdir -p gpurun_out/g5
rocprofv3 -L > gpurun_out/g5/counters.txt 2>&1 || true
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
bash tools/dbg/pmc.sh gpurun_out/g5/def "" "$A" FETCH_SIZE WRITE_SIZE && \
bash tools/dbg/pmc.sh gpurun_out/g5/noout "-DNT_TS_DBG_NOOUT=1" "$A" FETCH_SIZE WRITE_SIZE
