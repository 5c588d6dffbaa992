#!/bin/bash
# Memory-pipeline PMC passes (TA/TD/TCP/TCC occupancy and stalls) over the C2 bench.
set -e
TAG=${1:-pmcd}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--profile --steps 2 --warmup 1"
pass() {
    local name=$1; shift
    echo "[pmc] $name: $*"
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 bench.py $ARGS \
        > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
}
pass ta1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
pass ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_WAVEFRONTS_sum
pass td TD_TD_BUSY_sum TD_TC_STALL_sum
pass tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
pass tcc1 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum
pass tcc2 TCC_TAG_STALL_sum TCC_BUSY_sum TCC_LATENCY_FIFO_FULL_sum GRBM_GUI_ACTIVE
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS
pass sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_INST_LDS
echo PMC_DONE
