#!/bin/bash
# round 3 (session 2): C5 K=1000 twice on the final tree.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --c5-k 1000 --steps 10 --warmup 2 > $O/c5k1000_$i.json 2> $O/c5k1000_$i.err || { tail -20 $O/c5k1000_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5k1000_$i.json').read().strip().splitlines()[-1]); print('C5 K=1000', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3), 'dev', round(d['device_pipeline_ms'],3))"
done
echo DONE
