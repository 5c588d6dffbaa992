#!/bin/bash
# C4 leg (100M IoT filters, one GPU = one shard).  usage: tools/gpu_c4_r2.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/c4_r2}
mkdir -p $OUT
timeout -k 10 1000 python -u bench.py --workload c4 --steps 10 --warmup 2 > $OUT/bench_c4_100m.json 2> $OUT/bench_c4_100m.err || { tail -20 $OUT/bench_c4_100m.err; exit 1; }
tail -c 1500 $OUT/bench_c4_100m.json
