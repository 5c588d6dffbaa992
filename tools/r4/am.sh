#!/bin/bash
# round 4 / am: the big host tables preferring the GPU's NUMA node (mbind MPOL_PREFERRED, mb) against base; churn profile and C5 K = 100, interleaved
set -o pipefail
O=gpurun_out/r4am
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
for v in base mb; do
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 apply > $O/k100_${v}_$r.txt 2>&1 || { tail -20 $O/k100_${v}_$r.txt; exit 1; }
echo "$v $(tail -5 $O/k100_${v}_$r.txt | awk '{print $NF}' | tr '\n' ' ')"
done
done
for r in 1 2; do
for v in base mb; do
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -20 $O/c5_${v}_$r.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_${v}_$r.json').read().strip().splitlines()[-1]); print('$v c5 k=100', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3))"
done
done
echo DONE
