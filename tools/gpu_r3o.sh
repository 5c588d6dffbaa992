#!/bin/bash
# round 3 (session 2): where the tokeniser's fill time goes (timing-only
# variants: no tail compare for 9+-byte words; no lookups at all).
set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
export TMPDIR=/tmp
for v in head TOKNOTAIL TOKNOLOOKUP head; do
  lib=$PWD/emqx_amd/libemqx_tm.so
  [ $v = head ] || lib=$PWD/emqx_amd/variants/libemqx_tm_$v.so
  EMQX_TM_LIB=$lib timeout -k 10 300 python -u tools/tok_probe.py > $O/tok_$v.json 2> $O/tok_$v.err || { tail -20 $O/tok_$v.err; exit 1; }
  echo $v; cat $O/tok_$v.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/tok_probe.py > $O/tok_kt.json 2> $O/tok_kt.err || { tail -20 $O/tok_kt.err; exit 1; }
grep -i "tok_" $O/kt/kt_kernel_stats.csv
echo DONE
