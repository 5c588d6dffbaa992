#!/bin/bash
# round 4 / j: batch wait on its end event (not the stream), churn setup/plan/range/summary changes:
# full GPU suite, C5 legs K = 100 / 10, churn host profile
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for k in 100 10; do
timeout -k 10 300 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k$k.json 2> $O/c5_k$k.err || { tail -20 $O/c5_k$k.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k$k.json').read().strip().splitlines()[-1]); print('c5 k=$k', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'churn', round(d['churn_apply_ms'],3), d['host_ms'])"
done
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_trace.txt 2>&1 || { tail -20 $O/k100_trace.txt; exit 1; }
tail -13 $O/k100_trace.txt
echo DONE
