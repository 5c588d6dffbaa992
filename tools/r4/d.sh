#!/bin/bash
# round 4 / d: fan-out rows mode + async pipeline (busy-wait launch, inline launch)
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dispatch.py tests/test_gpu_coalesce.py tests/test_gpu_nif.py tests/test_gpu_replicated.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload dispatch --steps 10 --warmup 2 > $O/dispatch.json 2> $O/dispatch.err || { tail -20 $O/dispatch.err; exit 1; }
python -c "import json; d=json.loads(open('$O/dispatch.json').read().strip().splitlines()[-1]); print('dispatch', round(d['value']/1e9,3), 'disp_ms', round(d['dispatch_ms'],3), 'fill', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],3), 'csr form', d['dispatch_csr'])"
for cfg in "0 0" "40 1" "20 1" "80 1"; do
  set -- $cfg
  TM_ASYNC_BUSY_WAIT_US=$1 TM_ASYNC_INLINE=$2 timeout -k 10 300 python -u bench.py --workload coalesce --topics 2000000 > $O/coalesce_$1_$2.json 2> $O/coalesce_$1_$2.err || { tail -20 $O/coalesce_$1_$2.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/coalesce_$1_$2.json').read().strip().splitlines()[-1])
for k,v in d['legs'].items(): print('busy_wait $1 inline $2', k, round(v['calls_per_s']/1e6,3), 'M/s p50', round(v['p50_us']), 'p99', round(v['p99_us']), 'batch', round(v['mean_batch'],1), 'inline', v.get('inline_launches'), v['rows_equal_batch_path'])
print('cpu', round(d['cpu_baseline']['value']/1e6,3))"
done
echo DONE
