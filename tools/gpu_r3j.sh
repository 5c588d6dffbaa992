#!/bin/bash
# round 3 (session 2): GPU suite on the tree with U=12 read-back, pinned delta
# tails, batched futex wakes, small-batch tokeniser tiles; sync/async probe;
# latency with fewer small-batch tiles; C5 K=100; default bench line.
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/sync_probe.py 200000 64 > $O/sync_probe.jsonl 2> $O/sync_probe.err || { tail -20 $O/sync_probe.err; exit 1; }
cat $O/sync_probe.jsonl
for v in TILES1024 TILES512; do
  EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_$v.json 2> $O/lat_$v.err || { tail -20 $O/lat_$v.err; exit 1; }
  echo $v; cat $O/lat_$v.json
done
timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_head.json 2> $O/lat_head.err || { tail -20 $O/lat_head.err; exit 1; }
echo head; cat $O/lat_head.json
timeout -k 10 400 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_k100.json 2> $O/c5_k100.err || { tail -20 $O/c5_k100.err; exit 1; }
cat $O/c5_k100.json
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo DONE
