#!/bin/bash
# One GPU-box session: parity tests, bench, kernel-trace profile (run from the repo root).
#   tools/gpu_round.sh TAG [pytest-args...]
# Every GPU step has its own time limit and the steps are chained: the first
# failure ends the script.
set -e
TAG=${1:-run}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[gpu_round] pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "[gpu_round] bench"
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "[gpu_round] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --profile --steps 5 --warmup 2 > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { tail -20 $OUT/bench_kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cat {} \;
echo GPU_ROUND_DONE
