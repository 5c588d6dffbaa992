#!/bin/bash
# round 4 / ac: the walk with two probe batches in flight per wave (TM_WALK_P2=1) -- parity, then A/B on C2
set -o pipefail
O=gpurun_out/r4ac
mkdir -p $O
export TMPDIR=/tmp
TM_WALK_P2=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_p2.log 2>&1 || { tail -40 $O/pytest_p2.log; exit 1; }
tail -2 $O/pytest_p2.log
for v in base p2 base p2; do
  if [ $v = p2 ]; then export TM_WALK_P2=1; else unset TM_WALK_P2; fi
  timeout -k 10 300 python -u bench.py --no-c5 --no-cpu --steps 50 > $O/c2_$v.json 2> $O/c2_$v.err || { tail -20 $O/c2_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c2_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']/1e9,3), 'k_ms', round(r['kernel_ms'],3), 'iters', round(r['iterations_per_tile'],1), 'reads', round(r['per_publish']['bucket_reads'],2), 'slow', d['slow_path_topics'])"
done
echo DONE
