#!/bin/bash
# round 3 (session 2): churn with hot insert parts split by the third word --
# churn phases host-only, the whole GPU suite (delta gather on the workers),
# C5 K=100 three times.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 8 -1 > $O/host.txt 2>&1 || { tail -20 $O/host.txt; exit 1; }
grep "^K=" $O/host.txt | tail -4
grep "par ins" $O/host.txt | tail -2 | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_$i.json 2> $O/c5_$i.err || { tail -20 $O/c5_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_$i.json').read().strip().splitlines()[-1]); print('C5', round(d['value']/1e9,3), 'churn', round(d['churn_apply_ms'],3), 'dev', round(d['device_pipeline_ms'],3))"
done
echo DONE
