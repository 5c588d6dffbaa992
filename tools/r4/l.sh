#!/bin/bash
# round 4 / l: C5 legs with the device queueing time (launch call -> pipeline start)
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
for k in 100 10; do
timeout -k 10 300 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k$k.json 2> $O/c5_k$k.err || { tail -20 $O/c5_k$k.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k$k.json').read().strip().splitlines()[-1]); print('c5 k=$k', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'queue', round(d['device_queue_ms'],3), 'churn', round(d['churn_apply_ms'],3), d['host_ms'])"
done
echo DONE
