#!/bin/bash
# round 3 (session 2): walk epilogue read-back unroll A/B; the per-publish
# path's small batches (sync / async legs) with a kernel trace.
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
export TMPDIR=/tmp
run() {   # name lib
    n=$1; lib=$2; shift 2
    env "$@" EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --profile --steps 10 --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s kernel', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'pipe', round(d['pipeline_ms'],3))" $O/$n.json $n
}
for v in LOGU8 LOGU16; do
  EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "c1_full or walk_rows or c2_parity" > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; exit 1; }
  tail -1 $O/parity_$v.log
done
run head libemqx_tm.so
run u8 variants/libemqx_tm_LOGU8.so
run u12 variants/libemqx_tm_LOGU12.so
run u16 variants/libemqx_tm_LOGU16.so
run head2 libemqx_tm.so
run u16b variants/libemqx_tm_LOGU16.so
timeout -k 10 300 python -u tools/sync_probe.py 200000 64 > $O/sync_probe.jsonl 2> $O/sync_probe.err || { tail -20 $O/sync_probe.err; exit 1; }
cat $O/sync_probe.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt_sync -o kt --output-format csv -- python3 tools/sync_probe.py 20000 64 > $O/sync_probe_kt.jsonl 2> $O/sync_probe_kt.err || { tail -20 $O/sync_probe_kt.err; exit 1; }
for v in TILES4096 TILES8192; do
  EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_$v.so timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_$v.json 2> $O/lat_$v.err || { tail -20 $O/lat_$v.err; exit 1; }
  echo $v; cat $O/lat_$v.json
done
timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_head.json 2> $O/lat_head.err || { tail -20 $O/lat_head.err; exit 1; }
echo head; cat $O/lat_head.json
TM_PAR_TRACE=1 timeout -k 10 300 python3 -u tools/churn_prof.py 100 6 0 > $O/churn100_dev.log 2>&1 || { tail -20 $O/churn100_dev.log; exit 1; }
grep "^K=" $O/churn100_dev.log
echo DONE
