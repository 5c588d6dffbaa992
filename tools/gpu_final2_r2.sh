#!/bin/bash
# Round-2 measurement, part 2: dispatch PMC (fill traffic) and the legs.
set -o pipefail
OUT=${1:-gpurun_out/final2}
mkdir -p $OUT
bash tools/pmc_dispatch.sh $(basename $OUT)/pmcd > $OUT/pmcd.log 2>&1 || { echo "pmc dispatch failed"; tail -20 $OUT/pmcd.log; exit 1; }
tail -5 $OUT/pmcd.log
cp $OUT/pmcd/pmc_dispatch.json profiles/pmc_dispatch.json
export TMPDIR=/tmp
# headline kernel stats with --profile: the 10M-topic steps only (no latency
# sweep, no two-in-flight pass), so the walk's rocprof average is the headline's
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { tail -20 $OUT/bench_kt.err; exit 1; }
grep tm_match_tiles $OUT/kt/kt_kernel_stats.csv
bash tools/gpu_legs_r2.sh $OUT/legs || exit 1
