#!/bin/bash
# round 3 (session 2): PMC traffic of the packed-key walk (C2), the dispatch
# leg, and C4 at 100M IoT filters on one GPU (one shard).
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
bash tools/pmc_traffic.sh r3l/pmct > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -12 $O/pmc.log
timeout -k 10 400 python -u bench.py --workload dispatch > $O/dispatch.json 2> $O/dispatch.err || { tail -20 $O/dispatch.err; exit 1; }
tail -c 1500 $O/dispatch.json
timeout -k 10 700 python -u bench.py --workload c4 > $O/c4_100m.json 2> $O/c4_100m.err || { tail -20 $O/c4_100m.err; exit 1; }
tail -c 2000 $O/c4_100m.json
echo DONE
