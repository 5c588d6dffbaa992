#!/bin/bash
# round 4 / o: 30-bit literal signature in the '#'-id field of '#'-less children:
# full GPU suite, default bench line, C2 kernel trace, C5 K = 100 timeline probes
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/r4o/bench.json').read().strip().splitlines()[-1])
r=d['roofline']
print('C2', round(d['value']/1e9,3), 'frac', round(r['frac'],3), 'k_ms', round(r['kernel_ms'],3), 'reads', round(r['per_publish']['bucket_reads'],2), 'iters/tile', round(r['iterations_per_tile'],1), 'probes/iter', round(r['probes_per_iteration'],1), 'tok', round(d['tokenize_ms'],3), 'fresh', round(d['fresh_publishes_per_s']/1e9,3))
for k,v in d['c5'].items(): print(k, {x: (round(y,3) if isinstance(y,float) else y) for x,y in v.items()})
print('dense', d['dense_csr'], 'two', d['two_in_flight'], 'lat', d['latency_sweep']['65536'], 'fresh lat', d['fresh_latency_sweep']['65536'])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/c2_prof.json 2> $O/c2_prof.err || { tail -20 $O/c2_prof.err; exit 1; }
find $O/kt_c2 -name '*kernel_stats.csv' -exec head -4 {} \;
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload c5 --c5-k 100 --steps 10 --warmup 2 > $O/c5_$tag.json 2> $O/c5_$tag.err || { tail -20 $O/c5_$tag.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c5_$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), 'dev', round(d['device_pipeline_ms'],3), 'queue', round(d['device_queue_ms'],3), 'churn', round(d['churn_apply_ms'],3), {k: round(v,3) for k,v in d['host_ms'].items()})"
}
run default TM_X=0
run nograph TM_NO_GRAPH=1
run thr14 TM_HOST_THREADS=14
echo DONE
