# A/B of the C5 churn apply (dev tool): ab_prev/ holds a build of an earlier tree
# (git worktree + build, copied in, git-ignored); both run tools/churn_prof.py
# alternately on the same box.
set -e
mkdir -p gpurun_out/ab2
for r in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then d=ab_prev; else d=.; fi
    (cd $d && TM_PAR_TRACE=1 timeout -k 10 120 python tools/churn_prof.py 100 8 0 > /root/repo/gpurun_out/ab2/${v}_k100_$r.txt 2>&1)
    (cd $d && TM_PAR_TRACE=1 timeout -k 10 120 python tools/churn_prof.py 10 8 0 > /root/repo/gpurun_out/ab2/${v}_k10_$r.txt 2>&1)
    echo "$v r$r k100: $(grep 'apply sync' gpurun_out/ab2/${v}_k100_$r.txt | tail -6 | awk "{print \$13}" | tr '\n' ' ')"
    echo "$v r$r k10:  $(grep 'apply sync' gpurun_out/ab2/${v}_k10_$r.txt | tail -6 | awk "{print \$13}" | tr '\n' ' ')"
  done
done
