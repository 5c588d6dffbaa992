#!/bin/bash
# round 4 / u: C5 K = 100 with and without graph replay, interleaved (does a graph launch slow the host churn?)
set -o pipefail
O=gpurun_out/r4u
mkdir -p $O
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_$tag.json 2> $O/c5_$tag.err || { tail -20 $O/c5_$tag.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'queue', round(d['device_queue_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()})"
}
run g1 TM_X=0
run n1 TM_NO_GRAPH=1
run g2 TM_X=0
run n2 TM_NO_GRAPH=1
run g3 TM_X=0
run n3 TM_NO_GRAPH=1
echo DONE
