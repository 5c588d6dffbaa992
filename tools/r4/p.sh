#!/bin/bash
# round 4 / p: host cost of HIP event calls on completed events
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 120 python -u tools/r4/evt_probe.py > $O/evt.txt 2>&1 || { tail -20 $O/evt.txt; exit 1; }
cat $O/evt.txt
echo DONE
