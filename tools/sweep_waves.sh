#!/bin/bash
# Occupancy sweep of the match kernel (resident waves per CU) on C2.
set -e
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
for w in 4 8 12 16; do
    TM_WAVES_PER_CU=$w timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/w$w.json 2> $OUT/w$w.err || { tail -20 $OUT/w$w.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('waves/CU', sys.argv[2], d['value']/1e6, 'M/s', d['roofline']['kernel_ms'], 'ms match')" $OUT/w$w.json $w
done
