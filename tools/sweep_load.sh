#!/bin/bash
# Edge-hash load factor and occupancy sweeps of the match kernel on C2.
set -e
OUT=gpurun_out/${1:-sweepl}
mkdir -p $OUT
for ld in 0.25 0.35 0.5; do
    TM_LOAD=$ld timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/l$ld.json 2> $OUT/l$ld.err || { tail -20 $OUT/l$ld.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('load', sys.argv[2], d['value']/1e6, 'M/s', d['roofline']['kernel_ms'], 'ms match')" $OUT/l$ld.json $ld
done
for w in 8 12; do
    TM_WAVES_PER_CU=$w timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/w$w.json 2> $OUT/w$w.err || { tail -20 $OUT/w$w.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('waves/CU', sys.argv[2], d['value']/1e6, 'M/s', d['roofline']['kernel_ms'], 'ms match')" $OUT/w$w.json $w
done
