#!/bin/bash
# dispatch leg: HEAD library vs listed variants (emqx_amd/variants/*.so).
set -o pipefail
OUT=${1:-gpurun_out/ab_fan2}; shift
mkdir -p $OUT
for lib in variants/libemqx_tm_HEAD.so "$@"; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 400 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['deliveries_per_s']/1e9,2), 'G deliveries/s, fill', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'dispatch_ms', round(d['dispatch_ms'],3))" $OUT/$n.json $n
done
