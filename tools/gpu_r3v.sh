#!/bin/bash
# round 3 (session 2) final tree: GPU suite, smoke, kernel stats of the
# default bench, PMC traffic of the walk, the default bench line, C5 K=100
# with the async delta upload, the per-publish legs.
set -o pipefail
O=gpurun_out/r3v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
head -6 $O/kt/kt_kernel_stats.csv
bash tools/pmc_traffic.sh r3v/pmct > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -12 $O/pmc.log
cp $O/pmct/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_k100.json 2> $O/c5_k100.err || { tail -20 $O/c5_k100.err; exit 1; }
cat $O/c5_k100.json
timeout -k 10 400 python -u bench.py --workload coalesce > $O/coalesce.json 2> $O/coalesce.err || { tail -20 $O/coalesce.err; exit 1; }
python -c "import json; d=json.loads(open('$O/coalesce.json').read().strip().splitlines()[-1]); print('async', d['value'], 'sync', d['legs']['sync']['calls_per_s'], 'cpu', d.get('cpu_baseline',{}).get('value'))"

timeout -k 10 400 python -u bench.py --workload c5 --c5-k 1000 --steps 10 --warmup 2 > $O/c5_k1000.json 2> $O/c5_k1000.err || { tail -20 $O/c5_k1000.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k1000.json').read().strip().splitlines()[-1]); print('C5 K=1000', d['value'], d['device_pipeline_ms'], d['churn_apply_ms'])"
timeout -k 10 400 python -u bench.py --workload dispatch > $O/dispatch.json 2> $O/dispatch.err || { tail -20 $O/dispatch.err; exit 1; }
python -c "import json; d=json.loads(open('$O/dispatch.json').read().strip().splitlines()[-1]); print('dispatch', d['value'], d['deliveries_per_s'], d['roofline']['frac'])"
echo DONE
