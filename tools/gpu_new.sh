#!/bin/bash
# GPU session for the newer device paths: sharded, routes, skew/dedup, rules; C4 and C5 bench legs.
set -e
OUT=gpurun_out/${1:-new}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_routes.py tests/test_gpu_skew.py tests/test_gpu_rules.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 600 python -u bench.py --workload c4 --c4-filters ${C4F:-20000000} --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
timeout -k 10 600 python -u bench.py --workload c5 --c5-k ${C5K:-100} --steps 5 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
