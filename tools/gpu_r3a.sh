#!/bin/bash
# round 3: GPU tests (replicated engine refactor) then the emission A/B
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r3a/pytest.log
[ $rc -eq 0 ] || exit $rc
tools/ab_emit.sh gpurun_out/r3a/ab_emit
