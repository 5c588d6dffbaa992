#!/bin/bash
# GPU tests, then the co-location A/B, then the C5 K=1000 leg.
set -o pipefail
OUT=${1:-gpurun_out/s3c}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_coloc.sh $OUT/ab || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --c5-k 1000 --steps 5 --warmup 1 > $OUT/bench_c5_k1000.json 2> $OUT/bench_c5_k1000.err || { tail -20 $OUT/bench_c5_k1000.err; exit 1; }
tail -c 600 $OUT/bench_c5_k1000.json
