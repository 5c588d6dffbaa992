#!/bin/bash
# C2 walk under runtime knobs: "VAR=value" arguments, one bench run each (plus the default).
set -o pipefail
OUT=${OUT:-gpurun_out/ab_env}
mkdir -p $OUT
for kv in "DEFAULT=1" "$@"; do
    n=${kv//=/_}
    env $kv timeout -k 10 300 python -u bench.py --profile --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['value']/1e9,3), 'G/s walk', round(r['kernel_ms'],3), 'frac', round(r['frac'],3), 'pipeline', round(d['pipeline_ms'],3))" $OUT/$n.json $kv
done
