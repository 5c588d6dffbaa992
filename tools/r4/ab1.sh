#!/bin/bash
# round 4 / ab1: tokeniser words-per-lane / waves-per-EU A/B (variants built by tools/build_variant.sh)
set -o pipefail
O=gpurun_out/r4ab1
bash tools/ab_tok.sh $O || exit 1
for d in $O/libemqx_tm_*; do
  [ -d "$d" ] || continue
  echo "== $(basename $d)"
  db=$(find $d -name '*.db' | head -1)
  python3 tools/kstats.py "$db" 6 | grep -E "tok_|kernel " || true
done
echo DONE
