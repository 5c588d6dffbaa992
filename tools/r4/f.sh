#!/bin/bash
# round 4 / f: fan-out without scratch; kernel trace of dispatch; PMC traffic of C2 and C4 (round 4 kernels)
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dispatch.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_disp -o kt --output-format csv -- python3 bench.py --workload dispatch --steps 5 --warmup 2 > $O/dispatch.json 2> $O/dispatch.err || { tail -20 $O/dispatch.err; exit 1; }
find $O/kt_disp -name '*kernel_stats.csv' -exec head -14 {} \;
python -c "import json; d=json.loads(open('$O/dispatch.json').read().strip().splitlines()[-1]); print('dispatch', round(d['value']/1e9,3), 'disp_ms', round(d['dispatch_ms'],3), 'fill', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],3), 'csr form', d['dispatch_csr'])"
bash tools/pmc_traffic.sh r4f/pmc_c2 || exit 1
bash tools/pmc_traffic_c4.sh r4f/pmc_c4 || exit 1
echo DONE
