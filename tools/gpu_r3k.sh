#!/bin/bash
# round 3 (session 2): packed k5 path codes (lane inside the log entry): GPU
# suite, A/B against the pre-packing build, small-batch tile sizing, the
# per-publish legs (coalesce bench).
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
run() {   # name lib
    n=$1; lib=$2; shift 2
    env "$@" EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --profile --steps 10 --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s kernel', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'pipe', round(d['pipeline_ms'],3))" $O/$n.json $n
}
run head libemqx_tm.so
run prepack variants/libemqx_tm_PREPACK.so
run head2 libemqx_tm.so
run prepack2 variants/libemqx_tm_PREPACK.so
for v in TILES256 TILES128; do
  EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_$v.json 2> $O/lat_$v.err || { tail -20 $O/lat_$v.err; exit 1; }
  echo $v; cat $O/lat_$v.json
done
timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_head.json 2> $O/lat_head.err || { tail -20 $O/lat_head.err; exit 1; }
echo head; cat $O/lat_head.json
timeout -k 10 400 python -u bench.py --workload coalesce > $O/coalesce.json 2> $O/coalesce.err || { tail -20 $O/coalesce.err; exit 1; }
python -c "import json; d=json.loads(open('$O/coalesce.json').read().strip().splitlines()[-1]); print('async', d['value'], 'sync', d['legs']['sync']['calls_per_s'], 'cpu', d.get('cpu_baseline',{}).get('value'))"
echo DONE
