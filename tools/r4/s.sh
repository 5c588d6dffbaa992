#!/bin/bash
# round 4 / s: where the C5 step's batch wait goes
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
export TMPDIR=/tmp
TM_WAIT_TRACE=1 timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_wt.json 2> $O/c5_wt.err || { tail -20 $O/c5_wt.err; exit 1; }
grep "^\[wait\]\|^\[tm_batch_wait\]" $O/c5_wt.err | tail -16
python -c "import json; d=json.loads(open('$O/c5_wt.json').read().strip().splitlines()[-1]); print('c5', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'queue', round(d['device_queue_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()})"
echo DONE
