#!/bin/bash
# dev tool: A/B of walk variants (emqx_amd/variants/libemqx_tm_*.so) on the C4-regime bench
OUT=${1:-gpurun_out/ab_c4}; NF=${2:-2000000}
mkdir -p $OUT
for lib in emqx_amd/variants/libemqx_tm_*.so; do
  name=$(basename $lib .so)
  EMQX_TM_LIB=$PWD/$lib timeout -k 10 300 python3 tools/c4_bench.py $NF 10000000 4 > $OUT/$name.out 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.out; exit 1; }
  echo "$name $(tail -2 $OUT/$name.out | head -1)"
done
echo AB_DONE
