#!/bin/bash
# GPU tests, C2 bench line, rocprof kernel stats of C2 and of the C5 K=1000 leg.
# usage: tools/gpu_s3.sh OUTDIR [tests...]
set -o pipefail
OUT=${1:-gpurun_out/s3}; shift
mkdir -p $OUT
T=${@:-tests}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run -- python bench.py --no-cpu --steps 5 --warmup 1 > $OUT/prof_c2.log 2>&1 || { echo "prof c2 failed"; tail -20 $OUT/prof_c2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run -- python bench.py --workload c5 --c5-k 1000 --steps 3 --warmup 1 > $OUT/prof_c5.log 2>&1 || { echo "prof c5 failed"; tail -20 $OUT/prof_c5.log; exit 1; }
tail -1 $OUT/prof_c5.log
echo done
