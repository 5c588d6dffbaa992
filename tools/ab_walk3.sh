#!/bin/bash
# round 3: where the walk's emission time goes (timing-only variants):
# no log stores in the frontier loop; no epilogue (sort + staging); both.
set -o pipefail
OUT=${1:-gpurun_out/ab_walk3}
mkdir -p $OUT
run() {   # name lib [env...]
    n=$1; lib=$2; shift 2
    env "$@" EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --profile --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s kernel', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'pipe', round(d['pipeline_ms'],3))" $OUT/$n.json $n
}
run head libemqx_tm.so
run no_log variants/libemqx_tm_NO_LOG.so
run no_epi variants/libemqx_tm_NO_EPI.so
run no_both variants/libemqx_tm_NO_BOTH.so
run head2 libemqx_tm.so
echo AB_DONE
