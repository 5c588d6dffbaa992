"""Per-publish path sweep (dev tool): C2 trie, the native load generator over a
few caller shapes; prints calls/s, latency, mean batch, host time per batch.

    python tools/coalesce_sweep.py [n_topics]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from emqx_amd import gen  # noqa: E402
from emqx_amd import load as LD  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    F = gen.gen_filters(gen.C2)
    T = gen.gen_topics(gen.C2, F, 1000, n)
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.sync()
    offs, ids = eng.match_batch(T)
    exp_h = LD.row_hashes(offs, ids)
    LD.run(eng, T.slice(0, 20000), LD.ASYNC, 4, 64, hashes=False)
    shapes = [("sync", LD.SYNC, 16, 1), ("sync", LD.SYNC, 64, 1), ("async", LD.ASYNC, 16, 32),
              ("async", LD.ASYNC, 16, 64), ("async", LD.ASYNC, 16, 128), ("async", LD.ASYNC, 16, 256),
              ("async", LD.ASYNC, 8, 128), ("async", LD.ASYNC, 8, 256)]
    for name, mode, th, win in shapes:
        cnt = n if mode == LD.ASYNC else min(n, 300_000)
        sub = T if cnt == n else T.slice(0, cnt)
        b0 = eng.async_stats()
        t0 = time.time()
        st, counts, hs = LD.run(eng, sub, mode, th, win)
        b1 = eng.async_stats()
        nb = max(b1["batches"] - b0["batches"], 1)
        print(json.dumps({"mode": name, "threads": th, "window": win, "calls_per_s": cnt / st["seconds"],
                          "p50_us": st["p50_us"], "p99_us": st["p99_us"], "mean_us": st["mean_us"], "max_us": st["max_us"], "ok": bool(np.array_equal(hs, exp_h[:cnt])),
                          "mean_batch": (b1["requests"] - b0["requests"]) / nb,
                          "us_per_batch": {k: (b1[k] - b0[k]) / nb for k in ("us_launch", "us_wait", "us_deliver")},
                          "wall": time.time() - t0}), flush=True)


if __name__ == "__main__":
    main()
