#!/bin/bash
# round 4 / ag: tm_trie_apply_many (one plan, one edge phase per delta) against the two calls; C5 GPU parity tests
set -o pipefail
O=gpurun_out/r4ag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_skew.py tests/test_gpu_skew_full.py > $O/pytest_skew.log 2>&1 || { tail -40 $O/pytest_skew.log; exit 1; }
tail -2 $O/pytest_skew.log
for k in 100 10; do
for m in two apply two apply; do
timeout -k 10 300 python -u tools/churn_prof.py $k 10 0 $m > $O/k${k}_$m.txt 2>&1 || { tail -20 $O/k${k}_$m.txt; exit 1; }
tail -4 $O/k${k}_$m.txt
done
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py $k 6 0 apply > $O/k${k}_trace.txt 2>&1 || { tail -20 $O/k${k}_trace.txt; exit 1; }
grep -E "^\[(plan|par|apply)|^K=" $O/k${k}_trace.txt | tail -9
done
for k in 100 10; do
timeout -k 10 300 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k$k.json 2> $O/c5_k$k.err || { tail -20 $O/c5_k$k.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k$k.json').read().strip().splitlines()[-1]); print('c5 k=$k', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()}, 'parity', d.get('parity_sample_ok'))"
done
echo DONE
