#!/bin/bash
# round 4 / t: parent summaries rewritten only when their slot changes: churn profile + C5 legs
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_plain.txt 2>&1 || { tail -20 $O/k100_plain.txt; exit 1; }
tail -4 $O/k100_plain.txt
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 6 0 > $O/k100_trace.txt 2>&1 || { tail -20 $O/k100_trace.txt; exit 1; }
tail -13 $O/k100_trace.txt
for k in 100 10; do
timeout -k 10 300 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k$k.json 2> $O/c5_k$k.err || { tail -20 $O/c5_k$k.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k$k.json').read().strip().splitlines()[-1]); print('c5 k=$k', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()})"
done
echo DONE
