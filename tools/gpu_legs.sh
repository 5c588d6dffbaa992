#!/bin/bash
# Bench legs beside the C2 headline: C5 at K = 10 / 100 / 1000, C4 at 100M filters.
set -e
OUT=gpurun_out/${1:-legs}
mkdir -p $OUT
for k in 10 100 1000; do
    timeout -k 10 400 python -u bench.py --workload c5 --c5-k $k --steps 5 --warmup 1 > $OUT/bench_c5_k$k.json 2> $OUT/bench_c5_k$k.err || { tail -20 $OUT/bench_c5_k$k.err; exit 1; }
    cat $OUT/bench_c5_k$k.json
done
timeout -k 10 900 python -u bench.py --workload c4 --steps 10 --warmup 2 > $OUT/bench_c4_100m.json 2> $OUT/bench_c4_100m.err || { tail -20 $OUT/bench_c4_100m.err; exit 1; }
cat $OUT/bench_c4_100m.json
