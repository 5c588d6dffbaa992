#!/bin/bash
# round 3 (session 2): async completion polled on a pinned flag written by the
# stream after the export (TM_ASYNC_SPIN_US) -- per-publish tests with it on,
# then the sync / async probe at 0 / 300 / 1000 us of polling.
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
export TMPDIR=/tmp
TM_ASYNC_SPIN_US=300 timeout -k 10 600 python -u -m pytest tests/test_gpu_coalesce.py tests/test_gpu_nif.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sp in 0 300 1000 0 300; do
  TM_ASYNC_SPIN_US=$sp timeout -k 10 300 python -u tools/sync_probe.py 200000 64 > $O/sync_$sp.jsonl 2> $O/sync_$sp.err || { tail -20 $O/sync_$sp.err; exit 1; }
  echo "spin $sp"; cat $O/sync_$sp.jsonl
done
echo DONE
