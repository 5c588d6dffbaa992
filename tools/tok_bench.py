"""Device tokeniser timing on fresh C2 batches (dev tool, run under rocprofv3
--kernel-trace): every launch after a re-prepare tokenises the resident bytes.

    python tools/tok_bench.py [n_topics] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
F = gen.gen_filters(gen.C2)
T = gen.gen_topics(gen.C2, F, 1000, n)
eng = Engine(device=0)
eng.insert_many(F)
eng.sync()
for _ in range(reps):
    b = eng.prepare(T)
    b.launch().wait()
    print(b.stats(), flush=True)
    b.free()
