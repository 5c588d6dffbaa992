#!/bin/bash
# round 4 / y: blocked coalesced callers launch on any free slot (urgent calls): tests + coalesce legs
set -o pipefail
O=gpurun_out/r4y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_coalesce.py tests/test_gpu_concurrency.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
timeout -k 10 400 python -u bench.py --workload coalesce > $O/coalesce_$i.json 2> $O/coalesce_$i.err || { tail -20 $O/coalesce_$i.err; exit 1; }
python -c "import json; d=json.loads(open('$O/coalesce_$i.json').read().strip().splitlines()[-1]); print('coalesce', {k: (round(v['calls_per_s']/1e6,3), round(v['p50_us']), round(v['p99_us']), round(v['mean_batch'],1), v['inline_launches']) for k,v in d['legs'].items()}, 'cpu', round(d['cpu_baseline']['value']/1e6,3))"
done
echo DONE
