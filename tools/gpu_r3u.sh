#!/bin/bash
# round 3 (session 2): flat tokeniser with 4 (2) words per thread per round:
# token equality, then timing vs the tile-lookup tokeniser.
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tokenize.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in flat noflat lu2 flat noflat lu2; do
  lib=$PWD/emqx_amd/libemqx_tm.so
  unset TM_TOK_NO_FLAT
  [ $v = noflat ] && export TM_TOK_NO_FLAT=1
  [ $v = lu2 ] && lib=$PWD/emqx_amd/variants/libemqx_tm_TOKLU2.so
  EMQX_TM_LIB=$lib timeout -k 10 300 python -u tools/tok_probe.py > $O/tok_$v.json 2> $O/tok_$v.err || { tail -20 $O/tok_$v.err; exit 1; }
  echo $v; python -c "import json; print(json.load(open('$O/tok_$v.json'))['tokenize_ms_median'])"
done
unset TM_TOK_NO_FLAT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/tok_probe.py > $O/tok_kt.json 2> $O/tok_kt.err || { tail -20 $O/tok_kt.err; exit 1; }
grep -i "tok_" $O/kt/kt_kernel_stats.csv
echo DONE
