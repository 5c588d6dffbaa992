#!/bin/bash
# round 3 (session 2): generic-path LDS sort of 1,024 instead of 2,048 entries
# (12 -> 24 KB per wave bounds its occupancy): C5 K = 1000 parity and timing.
set -o pipefail
O=gpurun_out/r3r
mkdir -p $O
export TMPDIR=/tmp
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_SORT1024.so timeout -k 10 600 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_skew_full.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "skew or slow or deep or c5" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in head SORT1024 head SORT1024; do
  lib=$PWD/emqx_amd/libemqx_tm.so
  [ $v = head ] || lib=$PWD/emqx_amd/variants/libemqx_tm_$v.so
  EMQX_TM_LIB=$lib timeout -k 10 400 python -u bench.py --workload c5 --c5-k 1000 --steps 10 --warmup 2 > $O/c5_$v.json 2> $O/c5_$v.err || { tail -20 $O/c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,3), 'G/s step', round(d['ms_per_step'],3), 'churn', round(d['churn_apply_ms'],3), 'device', round(d['device_pipeline_ms'],3), 'walk', round(d['device_walk_ms'],3))"
done
echo DONE
