#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the C4 leg (100M IoT filters) -> profiles/pmc_c4.json
set -e
TAG=${1:-pmc_c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--workload c4 --profile --steps 2 --warmup 1"
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
    set -- $pass
    name=$1; shift
    timeout -s KILL 500 rocprofv3 --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 bench.py $ARGS \
        > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT --workload C4 --filters 100000000 --write $OUT/pmc_c4.json | tail -12
