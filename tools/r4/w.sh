#!/bin/bash
# round 4 / w: pipelined tm_match_batch (chunks over two streams): parity tests + e2e line
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u bench.py --no-c5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('C2', round(d['value']/1e9,3), 'e2e', d['e2e'], 'fresh lat', {k: (round(v['p50_ms'],3), round(v['p99_ms'],3)) for k,v in d['fresh_latency_sweep'].items()})"
echo DONE
