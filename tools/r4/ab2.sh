#!/bin/bash
# round 4 / ab2: non-temporal tokeniser streams (TM_TOK_NT) -- does the walk after a fresh tokenise keep its caches?
set -o pipefail
O=gpurun_out/r4ab2
bash tools/ab_tok.sh $O || exit 1
for d in $O/libemqx_tm_*; do
  [ -d "$d" ] || continue
  echo "== $(basename $d)"
  db=$(find $d -name '*.db' | head -1)
  python3 tools/kstats.py "$db" 6 | grep -E "tok_|match_tiles|kernel " || true
done
echo DONE
