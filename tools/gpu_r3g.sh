#!/bin/bash
# round 3: small-batch walk anatomy (phases build) + host churn profile on the box
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_phases.so timeout -k 10 300 python3 -u tools/lat_phases.py > $O/phases.jsonl 2> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
cat $O/phases.jsonl
TM_PAR_TRACE=1 timeout -k 10 300 python3 -u tools/churn_prof.py 100 6 > $O/churn100.log 2>&1 || { tail -20 $O/churn100.log; exit 1; }
tail -30 $O/churn100.log
