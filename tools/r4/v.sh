#!/bin/bash
# round 4 / v: churn per step in the C5 leg (step 0 has no walk beside it) vs the host-only profile
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_plain.txt 2>&1 || { tail -20 $O/k100_plain.txt; exit 1; }
tail -4 $O/k100_plain.txt
timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('c5', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', d['churn_ms_steps'])"
TM_HOST_THREADS=15 timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_t15.json 2> $O/c5_t15.err || { tail -20 $O/c5_t15.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_t15.json').read().strip().splitlines()[-1]); print('c5 t15', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'churn', d['churn_ms_steps'])"
echo DONE
