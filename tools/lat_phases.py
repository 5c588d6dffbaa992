"""Small-batch walk anatomy (dev tool, with a TM_EXPERIMENT_PHASES build via
EMQX_TM_LIB): per tile, frontier iterations, frontier-loop and prologue
cycles (s_memtime), probes; and the walk's event time, at several batch sizes
on the C2 trie."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

p = gen.C2
F = gen.gen_filters(p)
T = gen.gen_topics(p, F, 1000, 1 << 16)
eng = Engine(device=0)
eng.insert_many(F)
eng.sync()


def tile_topics(n):
    tt = 64
    while tt > 1 and (n + tt - 1) // tt < 2048:
        tt >>= 1
    return tt


for bsz in (64, 4096, 65536):
    b = eng.prepare(T.slice(0, bsz))
    for _ in range(3):
        b.launch().wait()
    ms = []
    for _ in range(20):
        b.launch().wait()
        ms.append(b.stats()["ms_match"])
    st = b.stats()
    tt = tile_topics(bsz)
    nt = (bsz + tt - 1) // tt
    print(json.dumps({"batch": bsz, "tile_topics": tt, "tiles": nt, "walk_ms_p50": float(np.median(ms)),
                      "iters_per_tile": st["visits"] / nt, "loop_cycles_per_tile": st["hash_hits"] / nt,
                      "prologue_cycles_per_wave": st["words"] / min(nt, 2048),
                      "probes_per_tile": st["probes"] / nt}), flush=True)
    b.free()
