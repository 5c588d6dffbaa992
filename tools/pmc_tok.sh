#!/bin/bash
# dev tool: SQ / TCP / TCC counters of the tokeniser kernels (tools/tok_bench.py), one pass each
OUT=${1:-gpurun_out/pmc_tok}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" -- python3 tools/tok_bench.py 10000000 1; }
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/sq -o p > $OUT/sq.out 2>&1 || { echo sq failed; exit 1; }
run SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d $OUT/sq2 -o p > $OUT/sq2.out 2>&1 || { echo sq2 failed; exit 1; }
run TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum -d $OUT/tcp -o p > $OUT/tcp.out 2>&1 || { echo tcp failed; exit 1; }
run TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $OUT/tcc -o p > $OUT/tcc.out 2>&1 || { echo tcc failed; exit 1; }
echo PMC_DONE
