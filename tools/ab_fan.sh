#!/bin/bash
# fan-out change: dispatch parity tests, then the dispatch leg with HEAD vs this tree.
set -o pipefail
OUT=${1:-gpurun_out/ab_fan}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dispatch.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in variants/libemqx_tm_HEAD.so libemqx_tm.so; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 400 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['deliveries_per_s']/1e9,2), 'G deliveries/s, fill', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'dispatch_ms', round(d['dispatch_ms'],3))" $OUT/$n.json $n
done
for lib in variants/libemqx_tm_HEAD.so libemqx_tm.so; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 400 python -u bench.py --workload c5 --c5-k 100 --steps 5 --warmup 1 > $OUT/c5_$n.json 2> $OUT/c5_$n.err || { tail -20 $OUT/c5_$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'C5 K=100', round(d['value']/1e6,1), 'M/s churn', round(d['churn_apply_ms'],2), 'device', round(d['device_pipeline_ms'],2))" $OUT/c5_$n.json $n
done
