#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / L2 passes of the C2 bench -> roofline.traffic (profiles/pmc_latest.json).
set -e
TAG=${1:-pmct}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--profile --steps 2 --warmup 1"
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "l2 TCC_HIT_sum TCC_MISS_sum"; do
    set -- $pass
    name=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 bench.py $ARGS \
        > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT --write $OUT/pmc_latest.json | tail -12
