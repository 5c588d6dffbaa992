#!/bin/bash
# round 4 / r: one-shot tm_match_batch (GPU suite + default line's fresh latency); C5 wait trace;
# C4 20M [0,0] and 100M on the signature kernels; coalesce legs
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u bench.py --no-c5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('C2', round(d['value']/1e9,3), 'k_ms', round(d['roofline']['kernel_ms'],3), 'traffic', d['roofline']['traffic'], 'fresh lat', d['fresh_latency_sweep'], 'e2e', round(d['e2e']['publishes_per_s']/1e6,1))"
TM_WAIT_TRACE=1 timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_wt.json 2> $O/c5_wt.err || { tail -20 $O/c5_wt.err; exit 1; }
grep "^\[wait\]" $O/c5_wt.err | tail -12
python -c "import json; d=json.loads(open('$O/c5_wt.json').read().strip().splitlines()[-1]); print('c5', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'queue', round(d['device_queue_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()})"
timeout -k 10 400 python -u bench.py --workload c4 --devices 0,0 --c4-filters 20000000 --steps 10 --warmup 2 > $O/c4_20m_00.json 2> $O/c4_20m_00.err || { tail -20 $O/c4_20m_00.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_20m_00.json').read().strip().splitlines()[-1]); print('c4 20M [0,0]', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), d['phase_ms'], 'waits', d['host_waits_per_step'], 'walk', round(d['device_match_ms'],3), d['parity_sample_ok'])"
timeout -k 10 600 python -u bench.py --workload c4 --steps 10 --warmup 2 > $O/c4_100m.json 2> $O/c4_100m.err || { tail -20 $O/c4_100m.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_100m.json').read().strip().splitlines()[-1]); print('c4 100M [0]', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'walk', round(d['device_match_ms'],3), 'frac', round(d['roofline']['frac'],3), d['roofline']['traffic'], d['parity_sample_ok'])"
timeout -k 10 400 python -u bench.py --workload coalesce > $O/coalesce.json 2> $O/coalesce.err || { tail -20 $O/coalesce.err; exit 1; }
python -c "import json; d=json.loads(open('$O/coalesce.json').read().strip().splitlines()[-1]); print('coalesce', {k: (round(v['calls_per_s']/1e6,3), round(v['p50_us']), round(v['p99_us'])) for k,v in d['legs'].items()}, 'cpu', round(d['cpu_baseline']['value']/1e6,3))"
echo DONE
