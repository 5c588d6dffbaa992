#!/bin/bash
# round 4 / al: C5 legs, churn workers pinned (default) vs TM_POOL_PIN=0, interleaved on one box
set -o pipefail
O=gpurun_out/r4al
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for k in 100 10; do
for p in 1 0; do
TM_POOL_PIN=$p timeout -k 10 300 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k${k}_p${p}_$r.json 2> $O/c5_k${k}_p${p}_$r.err || { tail -20 $O/c5_k${k}_p${p}_$r.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k${k}_p${p}_$r.json').read().strip().splitlines()[-1]); print('pin=$p c5 k=$k', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3), [round(x,2) for x in d.get('churn_ms_steps', [])])"
done
done
done
echo DONE
