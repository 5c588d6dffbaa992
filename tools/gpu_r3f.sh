#!/bin/bash
# round 3: single-pass tokeniser (tickets + look-back): full GPU suite, A/B of
# lookup widths, kernel trace of the small-batch latency probe, bench line.
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cp emqx_amd/libemqx_tm.so emqx_amd/variants/libemqx_tm_wpl2.so
tools/ab_tok.sh $O/ab_tok > $O/ab_tok.log 2>&1 || { tail -20 $O/ab_tok.log; exit 1; }
for d in $O/ab_tok/*/; do echo "== $d"; python3 tools/kstats.py $d/run_results.db 6; done > $O/ab_tok_summary.txt
cat $O/ab_tok_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lat -o lat --output-format csv -- python3 tools/lat_probe.py > $O/lat.json 2> $O/lat.err || { tail -20 $O/lat.err; exit 1; }
cat $O/lat.json
timeout -k 10 500 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','pipeline_ms','pipeline_fresh_ms','tokenize_ms','p99_batch_ms')}, d['roofline']['kernel_ms'], d['roofline']['frac'])"
