#!/bin/bash
# round 4 / b: C4 in-process step v2 (per-device partition, one host wait)
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  tests/test_gpu_sharded_group.py tests/test_gpu_sharded.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|SKIP|passed|failed" $O/pytest.log | tail -15
timeout -k 10 400 python -u bench.py --workload c4 --devices 0,0 --c4-filters 20000000 --steps 10 --warmup 2 > $O/c4_20m_00.json 2> $O/c4_20m_00.err || { tail -20 $O/c4_20m_00.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_20m_00.json').read().strip().splitlines()[-1]); print('c4 20M [0,0]', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), d['phase_ms'], 'waits', d['host_waits_per_step'], 'walk', round(d['device_match_ms'],3), 'csr', d['publish_order_csr'], 'fresh', round(d['fresh_ms'],2), d['parity_sample_ok'], d['part_topics'][:2])"
timeout -k 10 600 python -u bench.py --workload c4 --steps 10 --warmup 2 > $O/c4_100m.json 2> $O/c4_100m.err || { tail -20 $O/c4_100m.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_100m.json').read().strip().splitlines()[-1]); print('c4 100M [0]', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'waits', d['host_waits_per_step'], 'walk', round(d['device_match_ms'],3), 'frac', round(d['roofline']['frac'],3), 'fresh', round(d['fresh_ms'],2), d['parity_sample_ok'])"
echo DONE
