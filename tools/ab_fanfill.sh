#!/bin/bash
# A/B of the fan-out fill tile (16 vs 8 deliveries per thread): dispatch tests
# on the variant, then the dispatch bench leg for both builds.
set -e
OUT=gpurun_out/ab_fanfill
mkdir -p $OUT
export TMPDIR=/tmp
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_fp8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dispatch.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_fp8.log 2>&1 || { tail -30 $OUT/pytest_fp8.log; exit 1; }
tail -2 $OUT/pytest_fp8.log
timeout -k 10 300 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $OUT/fp16.json 2> $OUT/fp16.err || { tail -20 $OUT/fp16.err; exit 1; }
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_fp8.so timeout -k 10 300 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $OUT/fp8.json 2> $OUT/fp8.err || { tail -20 $OUT/fp8.err; exit 1; }
python - <<'PY'
import json
for k in ("fp16", "fp8"):
    d = json.load(open(f"gpurun_out/ab_fanfill/{k}.json"))
    print(k, round(d["value"] / 1e6, 1), "M/s", "fill", round(d["roofline"]["kernel_ms"], 3), "ms", "dispatch", round(d["dispatch_ms"], 3))
PY
echo AB_DONE
