#!/bin/bash
# round 4 / c: full GPU suite, default bench line (C5 legs, fresh latency), C4 20M [0,0] with direct scatter
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload c4 --devices 0,0 --c4-filters 20000000 --steps 10 --warmup 2 > $O/c4_20m_00.json 2> $O/c4_20m_00.err || { tail -20 $O/c4_20m_00.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_20m_00.json').read().strip().splitlines()[-1]); print('c4 20M [0,0]', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), d['phase_ms'], 'waits', d['host_waits_per_step'], 'walk', round(d['device_match_ms'],3), d['parity_sample_ok'])"
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4c/bench.json').read().strip().splitlines()[-1])
print('C2', round(d['value']/1e9,3), 'frac', round(d['roofline']['frac'],3), 'k_ms', round(d['roofline']['kernel_ms'],3), 'tok', round(d['tokenize_ms'],3), 'fresh', round(d['fresh_publishes_per_s']/1e9,3))
print('fresh lat', d['fresh_latency_sweep'])
print('lat', d['latency_sweep'])
for k,v in d['c5'].items(): print(k, {x: (round(y,3) if isinstance(y,float) else y) for x,y in v.items()})
PY
echo DONE
