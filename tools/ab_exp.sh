#!/bin/bash
# Timing-only experiment variants of the match kernel (emqx_amd/variants/*.so); results are not valid.
set -e
OUT=gpurun_out/${1:-exp}
mkdir -p $OUT
for lib in libemqx_tm.so variants/libemqx_tm_NO_EPILOGUE.so variants/libemqx_tm_NO_EMIT.so; do
    n=$(basename $lib .so)
    echo "[exp] $n"
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value']/1e6, 'M/s', d['roofline']['kernel_ms'], 'ms match', d['pipeline_ms'], 'ms pipe')" $OUT/$n.json
done
echo EXP_DONE
