#!/bin/bash
# round 3 (session 2): flat tokeniser (split in tiles, one thread per word
# for the lookups) -- token equality vs the host, parity, then timing A/B.
set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py tests/test_gpu_parity.py tests/test_gpu_sharded_group.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in flat noflat flat noflat; do
  if [ $v = noflat ]; then export TM_TOK_NO_FLAT=1; else unset TM_TOK_NO_FLAT; fi
  timeout -k 10 300 python -u tools/tok_probe.py > $O/tok_$v.json 2> $O/tok_$v.err || { tail -20 $O/tok_$v.err; exit 1; }
  echo $v; cat $O/tok_$v.json
done
unset TM_TOK_NO_FLAT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/tok_probe.py > $O/tok_kt.json 2> $O/tok_kt.err || { tail -20 $O/tok_kt.err; exit 1; }
grep -i "tok_" $O/kt/kt_kernel_stats.csv
echo DONE
