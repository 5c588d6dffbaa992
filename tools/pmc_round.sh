#!/bin/bash
# rocprofv3 PMC passes over the C2 bench (one counter group per run; no trace
# domains combined with --pmc).  Run on the GPU box from the repo root:
#   tools/pmc_round.sh TAG
# then `python tools/pmc_summary.py gpurun_out/TAG` folds them into per-kernel
# averages.
set -e
TAG=${1:-pmc}
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
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS
pass sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_INST_LDS
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
echo PMC_DONE
