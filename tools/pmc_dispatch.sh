#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the fan-out leg -> gpurun_out/TAG/pmc_dispatch.json (tm_fan_fill)
set -e
TAG=${1:-pmc_dispatch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--workload dispatch --steps 2 --warmup 1"
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
    set -- $pass
    name=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 bench.py $ARGS \
        > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT --workload dispatch --kernel tm_fan_fill --write $OUT/pmc_dispatch.json | tail -30
