#!/bin/bash
# Round-2 measurement, part 3: C4 PMC traffic, then the C4 leg with it.
set -o pipefail
OUT=${1:-gpurun_out/final5}
mkdir -p $OUT
bash tools/pmc_traffic_c4.sh $(basename $OUT)/pmc4 > $OUT/pmc4.log 2>&1 || { echo "pmc c4 failed"; tail -20 $OUT/pmc4.log; exit 1; }
tail -6 $OUT/pmc4.log
cp $OUT/pmc4/pmc_c4.json profiles/pmc_c4.json
bash tools/gpu_c4_r2.sh $OUT/c4 || exit 1
