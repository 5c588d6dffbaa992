"""Per-publish path probe (dev tool): the C2 trie, then 64 threads blocking in
tm_match_coalesced (the sync leg) and 16 x 256 async calls; prints calls/s,
latency percentiles and the pipeline's host time per batch (launch / wait /
deliver).  Run under rocprofv3 --kernel-trace to see one small batch's
kernels and the gaps between them.

    python tools/sync_probe.py [calls] [threads]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import gen  # noqa: E402
from emqx_amd import load as LD  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 64
filters = gen.gen_filters(gen.C2)
topics = gen.gen_topics(gen.C2, filters, 1000, calls)
eng = Engine(device=0)
eng.insert_many(filters)
eng.sync()
LD.run(eng, topics.slice(0, 20_000), LD.ASYNC, 4, 64, hashes=False)
for name, mode, th, win in (("sync", LD.SYNC, threads, 1), ("async", LD.ASYNC, 16, 256)):
    b0 = eng.async_stats()
    st, _, _ = LD.run(eng, topics, mode, th, win, hashes=False)
    b1 = eng.async_stats()
    nb = max(b1["batches"] - b0["batches"], 1)
    out = {"leg": name, "calls_per_s": calls / st["seconds"], "p50_us": st["p50_us"], "p99_us": st["p99_us"],
           "batches": nb, "mean_batch": (b1["requests"] - b0["requests"]) / nb,
           "host_us_per_batch": {k: (b1[k] - b0[k]) / nb for k in ("us_launch", "us_wait", "us_deliver")}}
    print(json.dumps(out), flush=True)
