#!/bin/bash
# round 3 (session 2): churn phases on the box after the worker-state reuse
# and edge-phase prefetch (TM_PAR_TRACE), host-only and with a device engine.
set -o pipefail
O=gpurun_out/r3z
mkdir -p $O
export TMPDIR=/tmp
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 8 -1 > $O/host.txt 2>&1 || { tail -20 $O/host.txt; exit 1; }
grep "^K=" $O/host.txt
TM_PAR_TRACE=1 TM_POOL_PIN=0 timeout -k 10 300 python -u tools/churn_prof.py 100 8 0 > $O/dev_pin0.txt 2>&1 || { tail -20 $O/dev_pin0.txt; exit 1; }
grep "^K=" $O/dev_pin0.txt
TM_PAR_TRACE=1 TM_POOL_PIN=1 timeout -k 10 300 python -u tools/churn_prof.py 100 8 0 > $O/dev_pin1.txt 2>&1 || { tail -20 $O/dev_pin1.txt; exit 1; }
grep "^K=" $O/dev_pin1.txt
tail -8 $O/host.txt
echo DONE
