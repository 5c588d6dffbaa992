#!/bin/bash
# round 4 / af: tokeniser fill A/B -- next tile's offsets + byte window prefetched (pf*), WPE 4 (…4), against base
set -o pipefail
O=gpurun_out/r4af
mkdir -p $O
export TMPDIR=/tmp
for lib in emqx_amd/variants/libemqx_tm_*.so; do
  name=$(basename $lib .so)
  EMQX_TM_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python3 tools/tok_bench.py 10000000 6 > $O/$name.out 2>&1 || { echo "$name failed"; tail -20 $O/$name.out; exit 1; }
  echo "$name"; find $O/$name -name '*kernel_stats.csv' -exec grep -h "tok_fill\|tok_count" {} \;
done
echo AB_DONE
