#!/bin/bash
# Round-2 legs: C5 at K = 10 / 100 / 1000, the dispatch (fan-out) leg, the
# coalesced per-publish leg.  usage: tools/gpu_legs_r2.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/legs_r2}
mkdir -p $OUT
for k in 10 100 1000; do
    timeout -k 10 400 python -u bench.py --workload c5 --c5-k $k --steps 5 --warmup 1 > $OUT/bench_c5_k$k.json 2> $OUT/bench_c5_k$k.err || { tail -20 $OUT/bench_c5_k$k.err; exit 1; }
    tail -c 400 $OUT/bench_c5_k$k.json
done
timeout -k 10 400 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $OUT/bench_dispatch.json 2> $OUT/bench_dispatch.err || { tail -20 $OUT/bench_dispatch.err; exit 1; }
tail -c 600 $OUT/bench_dispatch.json
timeout -k 10 300 python -u bench.py --workload coalesce > $OUT/bench_coalesce.json 2> $OUT/bench_coalesce.err || { tail -20 $OUT/bench_coalesce.err; exit 1; }
tail -c 600 $OUT/bench_coalesce.json
