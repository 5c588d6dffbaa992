#!/bin/bash
# round 4 / an: final tree after the churn prefetch and worker pinning -- full GPU suite, default bench line, C2 kernel trace; apply_many vs two calls (churn profile, C5 legs)
set -o pipefail
O=gpurun_out/r4an
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4an/bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('C2', round(d['value']/1e9,3), 'frac', round(r['frac'],3), 'k_ms', round(r['kernel_ms'],3), 'traffic', r['traffic'], 'fresh', round(d['fresh_publishes_per_s']/1e9,3), 'e2e', round(d['e2e']['publishes_per_s']/1e6,1))
print('lat', {k: (round(v['p50_ms'],3), round(v['p99_ms'],3)) for k,v in d['latency_sweep'].items()}, 'fresh lat', {k: (round(v['p50_ms'],3), round(v['p99_ms'],3)) for k,v in d['fresh_latency_sweep'].items()})
for k,v in d['c5'].items(): print(k, round(v['publishes_per_s']/1e9,3), 'ms', round(v['ms_per_step'],3), 'dev', round(v['device_ms'],3), 'churn', round(v['churn_ms'],3), {a: round(b,3) for a,b in v['host_ms'].items()})
print('cpu', d['cpu_baseline']['value'], 'c1', round(d['c1']['gpu_publishes_per_s']/1e6,1))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err || { tail -20 $O/c2_prof.err; exit 1; }
find $O/kt_c2 -name '*kernel_stats.csv' -exec head -4 {} \;
echo DONE
