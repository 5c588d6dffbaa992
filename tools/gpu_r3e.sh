#!/bin/bash
# round 3: full GPU suite with the emission log as the default walk, graph
# latency A/B, PMC traffic + kernel stats + the default bench line.
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_graph.json 2> $O/lat_graph.err || { tail -20 $O/lat_graph.err; exit 1; }
TM_NO_GRAPH=1 timeout -k 10 200 python -u tools/lat_probe.py > $O/lat_nograph.json 2> $O/lat_nograph.err || { tail -20 $O/lat_nograph.err; exit 1; }
cat $O/lat_graph.json $O/lat_nograph.json
bash tools/pmc_traffic.sh r3e/pmct > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
tail -12 $O/pmc.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --profile --steps 10 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
