#!/bin/bash
# round 3 (session 2): C5 K=100 host churn vs worker-thread count on the
# box's 16-CPU lease (TM_HOST_THREADS), interleaved to see box noise.
set -o pipefail
O=gpurun_out/r3x
mkdir -p $O
export TMPDIR=/tmp
for t in 16 12 8 16 12 8 10; do
  TM_HOST_THREADS=$t timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_t$t.json 2> $O/c5_t$t.err || { tail -20 $O/c5_t$t.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_t$t.json').read().strip().splitlines()[-1]); print('T=$t', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3), 'dev', round(d['device_pipeline_ms'],3))"
done
echo DONE
