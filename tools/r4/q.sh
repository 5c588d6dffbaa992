#!/bin/bash
# round 4 / q: PMC traffic of C2 and C4 on the signature kernels (roofline.traffic), dispatch line
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_traffic.sh r4q/pmc_c2 || exit 1
bash tools/pmc_traffic_c4.sh r4q/pmc_c4 || exit 1
timeout -k 10 300 python -u bench.py --workload dispatch --steps 5 --warmup 2 > $O/dispatch.json 2> $O/dispatch.err || { tail -20 $O/dispatch.err; exit 1; }
python -c "import json; d=json.loads(open('$O/dispatch.json').read().strip().splitlines()[-1]); print('dispatch', round(d['value']/1e9,3), 'disp_ms', round(d['dispatch_ms'],3), 'fill', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],3))"
echo DONE
