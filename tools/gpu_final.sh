#!/bin/bash
# Round-end session: full GPU suite + C2 bench + kernel trace (tools/gpu_round.sh),
# the dispatch leg with its kernel trace, then FETCH_SIZE / WRITE_SIZE passes of
# the dispatch leg (one counter group per pass).  Run from the repo root.
set -e
TAG=${1:-final}
bash tools/gpu_round.sh $TAG
bash tools/gpu_dispatch.sh ${TAG}_dispatch
OUT=gpurun_out/${TAG}_dpmc
mkdir -p $OUT
export TMPDIR=/tmp
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
    set -- $pass
    name=$1; shift
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d $OUT/$name -o p --output-format csv -- python3 bench.py --workload dispatch --steps 2 --warmup 1 \
        > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
grep -A3 "tm_fan_fill\|tm_fan_scan_local" $OUT/summary.txt | head -30 || true
echo FINAL_DONE
