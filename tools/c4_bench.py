"""C4-regime walk timing (dev tool): an IoT trie far larger than the Infinity
Cache, device-resident tokens, the tile walk launched repeatedly.  Run under
rocprofv3 --kernel-trace or --pmc.

    python tools/c4_bench.py [n_filters (default 20M)] [n_topics (10M)] [reps (5)]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

nf = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
p = gen.IotParams(n_filters=nf)
t0 = time.time()
eng = Engine(device=0, frozen_dict=True)
eng.dict_load(gen.gen_iot_vocab(p))
for lo in range(0, nf, 5_000_000):
    eng.insert_many(gen.gen_iot_filters(p, lo, min(nf, lo + 5_000_000)))
eng.sync()
print(f"trie {eng.stats()} in {time.time() - t0:.0f}s", flush=True)
topics = gen.gen_iot_topics(p, 4000, nt)
b = eng.prepare(topics)
for i in range(reps):
    b.launch().wait()
    st = b.stats()
    print({k: st[k] for k in ("topics", "visits", "hash_hits", "words", "matches", "probes", "ms_match", "ms_total")},
          flush=True)
n = st["topics"]
print(f"per publish: V {st['visits'] / n:.2f} H {st['hash_hits'] / n:.2f} probes {st['probes'] / n:.2f} "
      f"probe GB {st['probes'] * 64 / 1e9:.2f} -> {st['probes'] * 64 / st['ms_match'] / 1e6:.0f} GB/s bucket reads")
