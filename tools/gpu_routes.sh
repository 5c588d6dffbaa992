#!/bin/bash
# route resolution parity tests + timing (HEAD vs this tree) under rocprof.
set -o pipefail
OUT=${1:-gpurun_out/routes}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_route_feed.py tests/test_gpu_rules.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in variants/libemqx_tm_HEAD.so libemqx_tm.so; do
    n=$(basename $lib .so)
    EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof_$n -o run -- python3 tools/routes_rules_bench.py 100 5 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    cat $OUT/$n.json
done
