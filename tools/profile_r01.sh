#!/bin/bash
# rocprofv3 passes for the judged profile (run on the GPU box from the repo root).
# Kernel trace + stats, then one PMC pass per counter group (no trace domains
# combined with --pmc).
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--profile --steps 5 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/bench_kt.json 2> $OUT/bench_kt.err
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p --output-format csv -- python3 bench.py --profile --steps 2 --warmup 1 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o p --output-format csv -- python3 bench.py --profile --steps 2 --warmup 1 > $OUT/pmc_write.json 2> $OUT/pmc_write.err
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_l2 -o p --output-format csv -- python3 bench.py --profile --steps 2 --warmup 1 > $OUT/pmc_l2.json 2> $OUT/pmc_l2.err
echo PROFILE_DONE
