#!/bin/bash
# round 3 (session 2): walk counters by ballots (SALU) instead of per-lane
# VALU adds -- parity incl. the V/H counters vs the oracle, then A/B.
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
run() {   # name lib
    n=$1; lib=$2; shift 2
    env "$@" EMQX_TM_LIB=$PWD/emqx_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu --profile --steps 10 --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,1), 'M/s kernel', round(r['kernel_ms'],3), 'ms frac', round(r['frac'],3), 'V', r['per_publish']['V'], 'H', r['per_publish']['H'], 'reads', r['per_publish']['bucket_reads'])" $O/$n.json $n
}
run head libemqx_tm.so
run vstats variants/libemqx_tm_VSTATS.so
run head2 libemqx_tm.so
run vstats2 variants/libemqx_tm_VSTATS.so
run head3 libemqx_tm.so
run vstats3 variants/libemqx_tm_VSTATS.so
echo DONE
