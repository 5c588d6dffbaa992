#!/bin/bash
# async per-publish pipeline knobs: completer threads and batches in flight.
set -o pipefail
OUT=${1:-gpurun_out/ab_async}
mkdir -p $OUT
CFGS=${CFGS:-"2:3 4:3 4:4 6:4"}
for cfg in $CFGS; do
    cfg=${cfg/:/ }
    set -- $cfg
    TM_ASYNC_COMPLETERS=$1 TM_ASYNC_DEPTH=$2 timeout -k 10 300 python -u bench.py --workload coalesce --no-cpu > $OUT/c$1_d$2.json 2> $OUT/c$1_d$2.err || { tail -20 $OUT/c$1_d$2.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['legs']['async']; print('completers', sys.argv[2], 'depth', sys.argv[3], round(a['calls_per_s']/1e6,2), 'M calls/s p99', round(a['p99_us']), 'us deliver/batch', round(a['host_us_per_batch']['us_deliver']), 'mean batch', round(a['mean_batch']))" $OUT/c$1_d$2.json $1 $2
done
