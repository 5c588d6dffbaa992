#!/bin/bash
# generic-path grid: C5 K=1000 and C2 under TM_SLOW_WAVES values (this tree).
set -o pipefail
OUT=${1:-gpurun_out/ab_slow}
mkdir -p $OUT
for w in 512 1024 2048 4096; do
    TM_SLOW_WAVES=$w timeout -k 10 400 python -u bench.py --workload c5 --c5-k 1000 --steps 5 --warmup 1 > $OUT/c5_w$w.json 2> $OUT/c5_w$w.err || { tail -20 $OUT/c5_w$w.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('slow waves', sys.argv[2], 'C5 K=1000', round(d['value']/1e6,1), 'M/s device', round(d['device_pipeline_ms'],2), 'walk', round(d['device_walk_ms'],2), 'churn', round(d['churn_apply_ms'],2))" $OUT/c5_w$w.json $w
done
timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C2 default slow grid', round(d['value']/1e9,3), 'G/s pipeline', round(d['pipeline_ms'],3))" $OUT/c2.json
