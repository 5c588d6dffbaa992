#!/bin/bash
# round 4 / ai: churn A/B -- n_lext prefetched with the node records (pf) against base; apply mode, K = 100 / 10, interleaved
set -o pipefail
O=gpurun_out/r4ai
mkdir -p $O
export TMPDIR=/tmp
for k in 100 10; do
for v in base pf base pf base pf; do
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 300 python -u tools/churn_prof.py $k 12 0 apply > $O/k${k}_$v.txt 2>&1 || { tail -20 $O/k${k}_$v.txt; exit 1; }
echo "$v $(tail -6 $O/k${k}_$v.txt | awk '{print $NF}' | tr '\n' ' ')"
done
done
echo DONE
