#!/bin/bash
# round 4 / aa: smoke() and the default bench line (200 timed steps) as the driver runs them
set -o pipefail
O=gpurun_out/r4aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
t0=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall: $(( $(date +%s) - t0 )) s"
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4aa/bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('C2', round(d['value']/1e9,3), 'steps', d['steps'], 'ms', round(d['ms_per_step'],3), 'frac', round(r['frac'],3), 'k_ms', round(r['kernel_ms'],3), 'fresh', round(d['fresh_publishes_per_s']/1e9,3), 'e2e', round(d['e2e']['publishes_per_s']/1e6,1), 'two', round(d['two_in_flight']['publishes_per_s']/1e9,3), 'dense', round(d['dense_csr']['publishes_per_s']/1e9,3))
for k,v in d['c5'].items(): print(k, round(v['publishes_per_s']/1e9,3), 'churn', round(v['churn_ms'],3))
PY
echo DONE
