#!/bin/bash
# round 4 / m: anchored + edges (home of the edge into the parent), PLUS_CHAIN 3
# full GPU suite, default bench line (C2 + C5 legs), C2 kernel trace (finalize prefetch), churn host profile
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4m/bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('C2', round(d['value']/1e9,3), 'frac', round(r['frac'],3), 'k_ms', round(r['kernel_ms'],3), 'reads', round(r['per_publish']['bucket_reads'],2), 'tok', round(d['tokenize_ms'],3), 'fresh', round(d['fresh_publishes_per_s']/1e9,3))
for k,v in d['c5'].items(): print(k, {x: (round(y,3) if isinstance(y,float) else y) for x,y in v.items()})
print('dense', d['dense_csr'], 'two', d['two_in_flight'], 'lat', d['latency_sweep']['65536'])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err || { tail -20 $O/c2_prof.err; exit 1; }
find $O/kt_c2 -name '*kernel_stats.csv' -exec head -8 {} \;
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_trace.txt 2>&1 || { tail -20 $O/k100_trace.txt; exit 1; }
tail -13 $O/k100_trace.txt
echo DONE
