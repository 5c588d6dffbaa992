#!/bin/bash
# C5 legs (K = 10 / 100 / 1000) with the HEAD library and this tree.
set -o pipefail
OUT=${1:-gpurun_out/ab_c5}
mkdir -p $OUT
for k in 10 100 1000; do
for lib in variants/libemqx_tm_HEAD.so libemqx_tm.so; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 400 python -u bench.py --workload c5 --c5-k $k --steps 5 --warmup 1 > $OUT/c5_k${k}_$n.json 2> $OUT/c5_k${k}_$n.err || { tail -20 $OUT/c5_k${k}_$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'K', sys.argv[3], round(d['value']/1e6,1), 'M/s churn', round(d['churn_apply_ms'],2), 'device', round(d['device_pipeline_ms'],2))" $OUT/c5_k${k}_$n.json $n $k
done
done
