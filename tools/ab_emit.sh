#!/bin/bash
# What does the walk's emission cost: store instructions or row footprint?
# HEAD, timing-only variants (no stores; same stores into 4 slots per topic),
# and smaller row strides (TM_ROWCAP: rows longer than K take the slow path).
set -o pipefail
OUT=${1:-gpurun_out/ab_emit}
mkdir -p $OUT
run() {   # name lib [env...]
    n=$1; lib=$2; shift 2
    env "$@" EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --profile --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s kernel', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'reads/pub', r['per_publish'].get('bucket_reads'), 'slow', d.get('slow_path_topics'), 'pipe', round(d['pipeline_ms'],3))" $OUT/$n.json $n
}
# the log variant must be bit-exact before its time counts
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_EMIT_LOG.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/parity_emit_log.log 2>&1 || { tail -30 $OUT/parity_emit_log.log; exit 1; }
tail -2 $OUT/parity_emit_log.log
run head libemqx_tm.so
run emit_log variants/libemqx_tm_EMIT_LOG.so
run no_emit variants/libemqx_tm_NO_EMIT.so
run emit_hot variants/libemqx_tm_EMIT_HOT.so
run rowcap64 libemqx_tm.so TM_ROWCAP=64
run rowcap32 libemqx_tm.so TM_ROWCAP=32
run head2 libemqx_tm.so
run emit_log2 variants/libemqx_tm_EMIT_LOG.so
echo AB_DONE
