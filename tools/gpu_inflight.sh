#!/bin/bash
# TM_BATCH_STREAM: parity tests, then the C2 bench with 1 and 2 batches in flight.
set -o pipefail
OUT=${1:-gpurun_out/inflight}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for k in 1 2 3; do
    timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --inflight $k > $OUT/bench_if$k.json 2> $OUT/bench_if$k.err || { tail -20 $OUT/bench_if$k.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('inflight', sys.argv[2], round(d['value']/1e9,3), 'G/s ms_per_step', round(d['ms_per_step'],3), 'walk', round(r['kernel_ms'],3), 'pipeline', round(d['pipeline_ms'],3))" $OUT/bench_if$k.json $k
done
