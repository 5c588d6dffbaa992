#!/bin/bash
# kernel-trace stats of the dispatch leg.  usage: tools/prof_dispatch.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/prof_dispatch}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --workload dispatch --steps 5 --warmup 1 > $OUT/bench_dispatch_kt.json 2> $OUT/bench_dispatch_kt.err || { tail -20 $OUT/bench_dispatch_kt.err; exit 1; }
cut -d, -f1-5 $OUT/kt/kt_kernel_stats.csv | head -20
