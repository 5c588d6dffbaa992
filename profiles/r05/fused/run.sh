#!/bin/bash
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O; export TMPDIR=/tmp
run() { timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-c5 --no-cpu --profile > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }; }
for rep in 1 2; do
TM_FRESH_FUSED=0 run unfused_$rep
run fused1_$rep
EMQX_TM_LIB=emqx_amd/variants/libemqx_tm_w2.so run fused2_$rep
EMQX_TM_LIB=emqx_amd/variants/libemqx_tm_w3.so run fused3_$rep
done
for f in $O/*.json; do echo $f; cat $f; done
