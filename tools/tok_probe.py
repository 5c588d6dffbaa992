"""Device tokeniser time on the C2 batch (dev tool): 10M topics resident in
HBM, re-tokenised every launch; prints the median of ms_tokenize (count +
scan + fill, HIP events) -- for A/B of tokeniser builds via EMQX_TM_LIB."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
F = gen.gen_filters(gen.C2)
T = gen.gen_topics(gen.C2, F, 1000, n)
eng = Engine(device=0)
eng.insert_many(F)
eng.sync()
b = eng.prepare(T)
b.launch().wait()
tok = []
for _ in range(9):
    b.retokenize().launch().wait()
    tok.append(b.stats()["ms_tokenize"])
print(json.dumps({"topics": n, "tokenize_ms_median": float(np.median(tok)), "all": tok}), flush=True)
