#!/bin/bash
# dev tool: kernel trace, HBM traffic, L1 translation + L2 latency of the
# C4-regime walk (tools/c4_bench.py)
OUT=${1:-gpurun_out/c4}; NF=${2:-20000000}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o run -- python3 tools/c4_bench.py $NF 10000000 3 > $OUT/kt.out 2>&1 || { echo kt failed; tail -5 $OUT/kt.out; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $OUT/tcc -o p -- python3 tools/c4_bench.py $NF 10000000 1 > $OUT/tcc.out 2>&1 || { echo tcc failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum -d $OUT/tcp -o p -- python3 tools/c4_bench.py $NF 10000000 1 > $OUT/tcp.out 2>&1 || { echo tcp failed; exit 1; }
echo C4_DONE
