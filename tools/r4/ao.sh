#!/bin/bash
# round 4 / ao: last host-side change (apply's exception path) -- smoke, churn GPU tests, C5 K = 100 leg
set -o pipefail
O=gpurun_out/r4ao
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_skew.py tests/test_gpu_skew_full.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_k100.json 2> $O/c5_k100.err || { tail -20 $O/c5_k100.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k100.json').read().strip().splitlines()[-1]); print('c5 k=100', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3))"
echo DONE
