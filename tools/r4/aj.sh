#!/bin/bash
# round 4 / aj: C5 churn's process-to-process spread vs CPU placement -- unpinned, TM_POOL_PIN=1, whole process on node 0 / node 1 (taskset)
set -o pipefail
O=gpurun_out/r4aj
mkdir -p $O
export TMPDIR=/tmp
ls /sys/devices/system/node/ | grep node; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done
for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d numa $(cat $d/numa_node)"; done 2>/dev/null | head -3
which taskset || exit 0
N0=$(cat /sys/devices/system/node/node0/cpulist); N1=$(cat /sys/devices/system/node/node1/cpulist 2>/dev/null || echo $N0)
run() { local tag=$1; shift; timeout -k 10 300 "$@" python -u tools/churn_prof.py 100 10 0 apply > $O/$tag.txt 2>&1 || { tail -5 $O/$tag.txt; return 1; }; echo "$tag $(tail -5 $O/$tag.txt | awk '{print $NF}' | tr '\n' ' ')"; }
for i in 1 2 3; do
run free$i env && run pin$i env TM_POOL_PIN=1 && run n0_$i taskset -c $N0 && run n1_$i taskset -c $N1 || exit 1
done
echo DONE
