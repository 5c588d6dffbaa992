#!/bin/bash
# A/B: 64 vs 128 probes per frontier iteration (TM_WALK_NH variant build)
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O; export TMPDIR=/tmp
EMQX_TM_LIB=emqx_amd/variants/libemqx_tm_nh2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "c1_full or deep or c2_parity or walk_rows or forced" > $O/parity_nh2.log 2>&1 || { tail -20 $O/parity_nh2.log; exit 1; }
tail -1 $O/parity_nh2.log
run() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-c5 --no-cpu --profile > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }; }
for rep in 1 2; do
run base_$rep
EMQX_TM_LIB=emqx_amd/variants/libemqx_tm_nh2.so run nh2_$rep
EMQX_TM_LIB=emqx_amd/variants/libemqx_tm_nh2.so TM_QCAP=512 run nh2q512_$rep
done
