#!/bin/bash
# A/B of the tile kernel's LDS stack size / register budget (run from the repo root on the GPU box).
set -e
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
TM_QCAP=384 EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_w4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "c1_full or c2_parity or forced_slow or deep" > $OUT/pytest_q384.log 2>&1 || { tail -40 $OUT/pytest_q384.log; exit 1; }
tail -3 $OUT/pytest_q384.log
for cfg in "512 libemqx_tm.so" "384 variants/libemqx_tm_w4.so" "384 variants/libemqx_tm_w5.so"; do
    set -- $cfg
    echo "[ab] qcap=$1 lib=$2"
    TM_QCAP=$1 EMQX_TM_LIB=$PWD/emqx_amd/$2 timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/bench_q$1_$(basename $2 .so).json 2> $OUT/bench_q$1_$(basename $2 .so).err || { tail -20 $OUT/bench_q$1_$(basename $2 .so).err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value']/1e6, 'M/s', d['roofline']['kernel_ms'], 'ms match', d['pipeline_ms'], 'ms pipe', d['slow_path_topics'], 'slow')" $OUT/bench_q$1_$(basename $2 .so).json
done
echo AB_DONE
