#!/bin/bash
# Round-2 measurement, part 1: PMC traffic of the C2 walk, rocprof kernel
# stats of the C2 bench, the default bench line (with traffic from part 1).
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_traffic.sh $(basename $OUT)/pmct > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
tail -12 $OUT/pmc.log
cp $OUT/pmct/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { tail -20 $OUT/bench_kt.err; exit 1; }
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
