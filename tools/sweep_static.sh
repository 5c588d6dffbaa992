#!/bin/bash
# dev tool: walk time vs TM_STATIC_FRAC on C2 (tools/tok_bench.py) and the C4 regime
OUT=${1:-gpurun_out/sweep_static}; NF=${2:-20000000}
mkdir -p $OUT
for f in ${FRACS:-0 0.5 0.75 0.9 1.0}; do
  TM_STATIC_FRAC=$f timeout -k 10 200 python3 tools/tok_bench.py 10000000 4 > $OUT/c2_$f.out 2>&1 || { echo "c2 $f failed"; exit 1; }
  echo "c2 frac $f: $(grep -o "'ms_match': [0-9.]*" $OUT/c2_$f.out | tail -2 | tr '\n' ' ')"
done
for f in ${FRACS:-0 0.5 0.75 0.9 1.0}; do
  TM_STATIC_FRAC=$f timeout -k 10 300 python3 tools/c4_bench.py $NF 10000000 3 > $OUT/c4_$f.out 2>&1 || { echo "c4 $f failed"; exit 1; }
  echo "c4 frac $f: $(grep -o "'ms_match': [0-9.]*" $OUT/c4_$f.out | tail -2 | tr '\n' ' ')"
done
echo SWEEP_DONE
