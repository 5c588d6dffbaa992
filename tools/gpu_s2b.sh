#!/bin/bash
# GPU session: filter-sharded parity tests, then the C4 bench (1 GPU).
set -e
OUT=gpurun_out/${1:-s2b}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_sharded.log 2>&1 || { tail -40 $OUT/pytest_sharded.log; exit 1; }
tail -3 $OUT/pytest_sharded.log
timeout -k 10 1000 python -u bench.py --workload c4 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
tail -3 $OUT/bench_c4.err
