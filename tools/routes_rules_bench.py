"""Timing of device route resolution (tm_batch_routes) under C5 skew and of
the batched emqx_topic:match/2 kernel (tm_rules_match).  Dev/measurement tool:
run under rocprofv3 --kernel-trace for per-kernel times.

    python tools/routes_rules_bench.py [K] [reps]
"""
import json
import os
from dataclasses import replace
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402
from emqx_amd.skew import workload  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
allf, derived, hot, pubs = workload(gen.SkewParams(k_per_hot=K), 100_000, 10_000_000, seed=5)
eng = Engine(device=0)
t0 = time.time()
fl = allf.tolist()
# every filter routed to 1..3 destinations (nodes / share groups, aggre ids)
ev = [(1, f, 1 + (i % 3)) for i, f in enumerate(fl)] + [(1, f, 7) for f in fl[::5]]
eng.route_apply(ev)
eng.sync()
print(f"routes: {len(ev)} in {time.time() - t0:.1f}s", file=sys.stderr)
b = eng.prepare(pubs, dedup=True)
b.launch().wait()
st = b.stats()
ms = []
for _ in range(reps):
    t = time.perf_counter()
    ro, fid, dest = b.routes()
    ms.append(1e3 * (time.perf_counter() - t))
out = {"workload": f"C5 K={K}: {len(fl)} filters, {b.n} distinct topics of {len(pubs)} publishes",
       "matches": int(st["matches"]), "routes": int(len(dest)),
       "routes_ms_host_incl_d2h": {"min": min(ms), "mean": float(np.mean(ms))}}
# rules: 100k names x 64 ACL-like rules
names = gen.gen_topics(gen.C2, gen.gen_filters(gen.C2), 9, 100_000).tolist()
rules = gen.gen_filters(replace(gen.C2, n_filters=64, seed=3)).tolist()
ms = []
for _ in range(reps):
    t = time.perf_counter()
    m = eng.rules_match(names, rules)
    ms.append(1e3 * (time.perf_counter() - t))
out["rules"] = {"names": len(names), "rules": len(rules), "true": int(m.sum()),
                "ms_host_incl_copies": {"min": min(ms), "mean": float(np.mean(ms))}}
print(json.dumps(out))
