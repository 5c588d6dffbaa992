#!/bin/bash
# round 4 / ae: the box's CPU quota and throttling around the churn apply; plan parts; thread-count sweep
set -o pipefail
O=gpurun_out/r4ae
mkdir -p $O
export TMPDIR=/tmp
{ cat /sys/fs/cgroup/cpu.max; cat /sys/fs/cgroup/cpu.stat; nproc; cat /proc/self/status | grep -i cpus_allowed_list; } > $O/cgroup_before.txt 2>&1 || true
cat $O/cgroup_before.txt
TM_PAR_TRACE=1 timeout -k 10 300 python -u tools/churn_prof.py 100 6 0 > $O/k100_trace.txt 2>&1 || { tail -20 $O/k100_trace.txt; exit 1; }
grep -A40 "plan part" $O/k100_trace.txt | tail -30
{ cat /sys/fs/cgroup/cpu.stat; } > $O/cgroup_after_trace.txt 2>&1 || true
cat $O/cgroup_after_trace.txt
for t in 16 12 8; do
TM_HOST_THREADS=$t timeout -k 10 300 python -u tools/churn_prof.py 100 10 0 > $O/k100_t$t.txt 2>&1 || { tail -20 $O/k100_t$t.txt; exit 1; }
echo "threads $t"; tail -3 $O/k100_t$t.txt
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | grep -i throttl || true
done
echo DONE
