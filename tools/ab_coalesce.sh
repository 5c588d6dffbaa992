# A/B of the per-publish legs (dev tool): ab_prev/ holds a copy of an earlier
# build (emqx_amd/ with its .so files, bench.py, oracle/), git-ignored; both
# run `bench.py --workload coalesce` alternately on the same box.
set -e
mkdir -p gpurun_out/abc
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then d=ab_prev; else d=.; fi
    (cd $d && timeout -k 10 200 python -u bench.py --workload coalesce > /root/repo/gpurun_out/abc/${v}_$r.json 2> /root/repo/gpurun_out/abc/${v}_$r.err)
    python - "$v" "$r" <<'PY'
import json, sys
v, r = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"gpurun_out/abc/{v}_{r}.json") if l.startswith("{")][-1])
print(v, r, {k: (round(x["calls_per_s"] / 1e6, 3), round(x["p99_us"]), round(x["max_us"])) for k, x in d["legs"].items()})
PY
  done
done
