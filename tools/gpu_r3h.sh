#!/bin/bash
# round 3 (session 2): GPU suite, smoke, kernel stats of the default bench,
# default bench line, host churn profile and the C5 K=100 leg.
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
TM_PAR_TRACE=1 timeout -k 10 300 python3 -u tools/churn_prof.py 100 6 > $O/churn100.log 2>&1 || { tail -20 $O/churn100.log; exit 1; }
grep -v "par edges" $O/churn100.log | tail -12
timeout -k 10 400 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_k100.json 2> $O/c5_k100.err || { tail -20 $O/c5_k100.err; exit 1; }
cat $O/c5_k100.json
bash tools/ab_walk3.sh gpurun_out/r3h/ab_walk3 || exit 1
