#!/bin/bash
# round 3 (session 2): C5 K=100 host churn with the worker pool pinned to the
# GPU's NUMA node (default) vs unpinned (TM_POOL_PIN=0), interleaved.
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
export TMPDIR=/tmp
lscpu | grep -i "numa\|socket\|model name" || true
for d in /sys/class/drm/card*/device; do echo "$d node $(cat $d/numa_node 2>/dev/null)"; done
python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
i=0
for p in 1 0 1 0 1 0 1 0; do
  i=$((i+1))
  TM_POOL_PIN=$p timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_p${p}_$i.json 2> $O/c5_p${p}_$i.err || { tail -20 $O/c5_p${p}_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_p${p}_$i.json').read().strip().splitlines()[-1]); print('pin=$p', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3), 'dev', round(d['device_pipeline_ms'],3))"
done
TM_POOL_PIN=1 timeout -k 10 300 python -u bench.py --workload c5 --c5-k 1000 --steps 10 --warmup 2 > $O/c5_k1000.json 2> $O/c5_k1000.err || { tail -20 $O/c5_k1000.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k1000.json').read().strip().splitlines()[-1]); print('K=1000 pin', round(d['value']/1e9,3), 'churn', round(d['churn_apply_ms'],3), 'dev', round(d['device_pipeline_ms'],3))"
echo DONE
