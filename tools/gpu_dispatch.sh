#!/bin/bash
# Fan-out (tm_batch_dispatch) session on the GPU box: parity tests, the
# dispatch bench leg, and its kernel-trace summary.  Run from the repo root.
set -e
OUT=gpurun_out/${1:-dispatch}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dispatch.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_dispatch.log 2>&1 || { tail -40 $OUT/pytest_dispatch.log; exit 1; }
tail -3 $OUT/pytest_dispatch.log
timeout -k 10 400 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $OUT/bench_dispatch.json 2> $OUT/bench_dispatch.err || { tail -20 $OUT/bench_dispatch.err; exit 1; }
cat $OUT/bench_dispatch.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --workload dispatch --steps 5 --warmup 1 > $OUT/bench_dispatch_kt.json 2> $OUT/bench_dispatch_kt.err || { tail -20 $OUT/bench_dispatch_kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cat {} \;
echo DISPATCH_DONE
