#!/bin/bash
# A/B of tokeniser variants (emqx_amd/variants/libemqx_tm_*.so): kernel trace of tools/tok_bench.py each
OUT=${1:-gpurun_out/ab_tok}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in emqx_amd/variants/libemqx_tm_*.so; do
  name=$(basename $lib .so)
  EMQX_TM_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$name -o run -- python3 tools/tok_bench.py 10000000 3 > $OUT/$name.out 2>&1 || { echo "$name failed"; exit 1; }
done
echo AB_DONE
