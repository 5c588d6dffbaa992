#!/bin/bash
# round 3 (session 2): the final tree after the churn changes -- GPU suite,
# smoke, default bench line, C5 K=100 twice.
set -o pipefail
O=gpurun_out/r3zz
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('C2', d['value'], d['roofline']['frac'], d['p99_batch_ms'])"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_$i.json 2> $O/c5_$i.err || { tail -20 $O/c5_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_$i.json').read().strip().splitlines()[-1]); print('C5', round(d['value']/1e9,3), 'churn', round(d['churn_apply_ms'],3), 'dev', round(d['device_pipeline_ms'],3))"
done
echo DONE
