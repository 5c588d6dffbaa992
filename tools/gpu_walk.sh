#!/bin/bash
# walk-kernel change: parity tests first, then the A/B against HEAD.
set -o pipefail
OUT=${1:-gpurun_out/walk}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_walk.sh $OUT/ab
