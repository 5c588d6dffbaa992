#!/bin/bash
# round 4 / ab: sharded group after the copy-in path's removal (tests + C4 20M over 2 shards)
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_sharded_group.py tests/test_gpu_coalesce.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py --workload c4 --devices 0,0 --c4-filters 20000000 --steps 10 --warmup 2 > $O/c4_20m_00.json 2> $O/c4_20m_00.err || { tail -20 $O/c4_20m_00.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_20m_00.json').read().strip().splitlines()[-1]); print('c4 20M [0,0]', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'waits', d['host_waits_per_step'], d['parity_sample_ok'])"
echo DONE
