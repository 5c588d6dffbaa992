#!/bin/bash
# C5 legs (K = 10 / 100 / 1000) only.  usage: tools/gpu_c5.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/c5}
mkdir -p $OUT
for k in 10 100 1000; do
    timeout -k 10 400 python -u bench.py --workload c5 --c5-k $k --steps 5 --warmup 1 > $OUT/bench_c5_k$k.json 2> $OUT/bench_c5_k$k.err || { tail -20 $OUT/bench_c5_k$k.err; exit 1; }
    cat $OUT/bench_c5_k$k.json
done
