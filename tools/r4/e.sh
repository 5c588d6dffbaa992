#!/bin/bash
# round 4 / e: tokeniser (one-pass hashes), fan-out fill fast path; kernel traces of C2 and dispatch
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tokenize.py tests/test_gpu_dispatch.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err || { tail -20 $O/c2_prof.err; exit 1; }
find $O/kt_c2 -name '*kernel_stats.csv' -exec head -12 {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_disp -o kt --output-format csv -- python3 bench.py --workload dispatch --steps 5 --warmup 2 > $O/dispatch.json 2> $O/dispatch.err || { tail -20 $O/dispatch.err; exit 1; }
find $O/kt_disp -name '*kernel_stats.csv' -exec head -25 {} \;
python -c "import json; d=json.loads(open('$O/dispatch.json').read().strip().splitlines()[-1]); print('dispatch', round(d['value']/1e9,3), 'disp_ms', round(d['dispatch_ms'],3), 'fill', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],3), 'csr form', d['dispatch_csr'])"
echo DONE
