"""p50 / p99 batch latency (device-resident batches, launch -> results in HBM)
on the C2 trie, as bench.py measures it, for quick A/B (e.g. TM_NO_GRAPH=1)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

p = gen.C2
F = gen.gen_filters(p)
T = gen.gen_topics(p, F, 1000, 1 << 20)
eng = Engine(device=0)
eng.insert_many(F)
eng.sync()
out = {"graphs": os.environ.get("TM_NO_GRAPH", "0") != "1"}
for bsz in (4096, 65536, 1 << 20):
    b = eng.prepare(T.slice(0, bsz))
    for _ in range(5):
        b.launch().wait()
    lat = []
    for _ in range(300):
        t = time.perf_counter()
        b.launch().wait()
        lat.append(1e3 * (time.perf_counter() - t))
    out[str(bsz)] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99))}
    b.free()
print(json.dumps(out), flush=True)
