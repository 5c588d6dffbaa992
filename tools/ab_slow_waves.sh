# A/B of the generic-path grid (dev tool): ab_prev/ holds a copy of an earlier
# build (emqx_amd/ with its .so files, bench.py, oracle/), git-ignored; both run
# the C5 K = 1000 leg alternately on the same box.
set -e
mkdir -p gpurun_out/abs2
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then d=ab_prev; else d=.; fi
    (cd $d && timeout -k 10 200 python -u bench.py --workload c5 --c5-k 1000 --steps 30 --warmup 2 > /root/repo/gpurun_out/abs2/${v}_$r.json 2> /root/repo/gpurun_out/abs2/${v}_$r.err)
    echo "$v $r $(python tools/summarize.py gpurun_out/abs2/${v}_$r.json | grep device_pipeline_ms)"
  done
done
