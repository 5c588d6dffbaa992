#!/bin/bash
# A/B of the walk kernel: HEAD library (emqx_amd/variants/libemqx_tm_HEAD.so) vs this tree, C2.
# usage: tools/ab_walk.sh OUTDIR [extra variant names...]
set -o pipefail
OUT=${1:-gpurun_out/ab_walk}; shift
mkdir -p $OUT
for lib in variants/libemqx_tm_HEAD.so libemqx_tm.so "$@"; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s kernel', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'reads/pub', r['per_publish'].get('bucket_reads'), 'pipeline_ms', round(d['pipeline_ms'],3))" $OUT/$n.json $n
done
echo AB_DONE
