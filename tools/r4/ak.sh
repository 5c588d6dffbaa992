#!/bin/bash
# round 4 / ak: churn workers pinned to the GPU's NUMA node by default -- C5 legs (twice each) and the churn GPU tests
set -o pipefail
O=gpurun_out/r4ak
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_skew.py tests/test_gpu_skew_full.py tests/test_gpu_replicated.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
for k in 100 10; do
timeout -k 10 300 python -u bench.py --workload c5 --c5-k $k --steps 10 --warmup 2 > $O/c5_k${k}_$r.json 2> $O/c5_k${k}_$r.err || { tail -20 $O/c5_k${k}_$r.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_k${k}_$r.json').read().strip().splitlines()[-1]); print('c5 k=$k', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()})"
done
done
echo DONE
