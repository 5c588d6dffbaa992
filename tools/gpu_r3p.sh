#!/bin/bash
# round 3 (session 2): C5 after the churn plan's false-sharing fix and the
# pinned delta tails: K = 100 / 1000 legs and the device-engine churn profile.
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
export TMPDIR=/tmp
TM_PAR_TRACE=1 timeout -k 10 300 python3 -u tools/churn_prof.py 100 6 0 > $O/churn100_dev.log 2>&1 || { tail -20 $O/churn100_dev.log; exit 1; }
grep "^K=\|_many\|plan " $O/churn100_dev.log | tail -12
for k in 100 1000; do
  timeout -k 10 400 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k$k.json 2> $O/c5_k$k.err || { tail -20 $O/c5_k$k.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_k$k.json').read().strip().splitlines()[-1]); print('K=$k', round(d['value']/1e9,3), 'G/s step', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3), 'device', round(d['device_pipeline_ms'],3))"
done
echo DONE
