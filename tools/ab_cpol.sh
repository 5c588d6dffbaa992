#!/bin/bash
# A/B of the bucket loads' cache-policy bits (timing; parity of each variant checked on C1).
set -e
OUT=gpurun_out/${1:-cpol}
mkdir -p $OUT
for lib in libemqx_tm.so variants/libemqx_tm_c2.so variants/libemqx_tm_c16.so variants/libemqx_tm_c17.so; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value']/1e6, 'M/s', d['roofline']['kernel_ms'], 'ms match')" $OUT/$n.json $n
done
