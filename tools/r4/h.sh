#!/bin/bash
# round 4 / h: C5 churn breakdown on the box's host (TM_PAR_TRACE phases), K = 100 and 10
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_plain.txt 2>&1 || { tail -20 $O/k100_plain.txt; exit 1; }
tail -6 $O/k100_plain.txt
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_trace.txt 2>&1 || { tail -20 $O/k100_trace.txt; exit 1; }
tail -24 $O/k100_trace.txt
timeout -k 10 300 python -u tools/churn_prof.py 10 10 0 > $O/k10_plain.txt 2>&1 || { tail -20 $O/k10_plain.txt; exit 1; }
tail -4 $O/k10_plain.txt
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 10 6 0 > $O/k10_trace.txt 2>&1 || { tail -20 $O/k10_trace.txt; exit 1; }
tail -12 $O/k10_trace.txt
echo DONE
