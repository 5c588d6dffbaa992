#!/bin/bash
# round 3: replicated engine + in-process sharded group tests, C4 group bench, emission A/B
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_replicated.py tests/test_gpu_sharded_group.py tests/test_gpu_skew_full.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -12 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload c4 --c4-filters 20000000 --devices 0,0 --steps 5 --warmup 1 > $O/c4_group_20m.json 2> $O/c4_group_20m.err || { tail -20 $O/c4_group_20m.err; exit 1; }
tail -1 $O/c4_group_20m.json
tools/ab_emit.sh $O/ab_emit
