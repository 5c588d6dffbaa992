#!/bin/bash
# round 4 / z: parity file (pipelined growth test), multi-rank rehearsals on device 0 (in-process group, torchrun x2)
set -o pipefail
O=gpurun_out/r4z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --gpus 2 --devices 0,0 --steps 5 --warmup 2 --topics 5000000 > $O/group.json 2> $O/group.err || { tail -20 $O/group.err; exit 1; }
python -c "import json; d=json.loads(open('$O/group.json').read().strip().splitlines()[-1]); print('group', round(d['value']/1e9,3), d.get('parity_sample_ok'), d.get('devices'))"
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --devices 0,0 --steps 5 --warmup 2 --topics 5000000 --no-cpu --latency-batches 20 --e2e-topics 100000 > $O/tr2.json 2> $O/tr2.err || { tail -30 $O/tr2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/tr2.json').read().strip().splitlines()[-1]); print('torchrun x2', round(d['value']/1e9,3), d.get('parity_sample_ok'), d['n_gpus'])"
echo DONE
