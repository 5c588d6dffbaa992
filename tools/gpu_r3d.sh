#!/bin/bash
# round 3: new GPU tests + C5 / C4-group benches + emission A/B (one box acquisition)
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_replicated.py tests/test_gpu_sharded_group.py tests/test_gpu_skew.py tests/test_gpu_skew_full.py tests/test_gpu_group.py -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
# assertion failures (1) leave the GPU healthy: go on; anything else ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in 100 1000; do
  timeout -k 10 400 python -u bench.py --workload c5 --c5-k $k --steps 5 --warmup 1 > $O/c5_k$k.json 2> $O/c5_k$k.err || { tail -20 $O/c5_k$k.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,1), 'M/s churn', round(d['churn_apply_ms'],2), 'device', round(d['device_pipeline_ms'],2))" $O/c5_k$k.json
done
timeout -k 10 600 python -u bench.py --workload c4 --c4-filters 20000000 --devices 0,0 --steps 5 --warmup 1 > $O/c4_group_20m.json 2> $O/c4_group_20m.err || { tail -20 $O/c4_group_20m.err; exit 1; }
tail -1 $O/c4_group_20m.json
tools/ab_emit.sh $O/ab_emit
