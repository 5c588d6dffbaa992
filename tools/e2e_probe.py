"""Stage timing of the host-inclusive path (diagnostic): split API on one batch
re-prepared in place vs tm_match_batch on the engine's scratch batch."""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from emqx_amd import _native as N  # noqa: E402
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
p = gen.C2
filters = gen.gen_filters(p)
topics = gen.gen_topics(p, filters, 1000, n)
eng = Engine(device=0)
for f in filters.tolist():
    eng.insert(f)
eng.sync()
buf = np.ascontiguousarray(topics.buf)
offs = np.ascontiguousarray(topics.offs.astype(np.uint64))
r = N.Result()
h = C.c_void_p()
for it in range(4):
    t0 = time.perf_counter()
    N.check(eng.L.tm_batch_prepare(eng.h, buf.ctypes.data, offs.ctypes.data, n, C.byref(h)), "prepare")
    t1 = time.perf_counter()
    N.check(eng.L.tm_batch_launch(eng.h, h), "launch")
    t2 = time.perf_counter()
    N.check(eng.L.tm_batch_wait(eng.h, h), "wait")
    t3 = time.perf_counter()
    N.check(eng.L.tm_batch_result(eng.h, h, C.byref(r)), "result")
    t4 = time.perf_counter()
    N.check(eng.L.tm_batch_result(eng.h, h, C.byref(r)), "result")
    t5 = time.perf_counter()
    print(f"split it{it}: prepare {1e3*(t1-t0):.1f} launch {1e3*(t2-t1):.1f} wait {1e3*(t3-t2):.1f} "
          f"result {1e3*(t4-t3):.1f} result-again {1e3*(t5-t4):.1f} ms", flush=True)
for it in range(3):
    t0 = time.perf_counter()
    N.check(eng.L.tm_match_batch(eng.h, buf.ctypes.data, offs.ctypes.data, n, C.byref(r)), "match")
    print(f"match_batch it{it}: {1e3*(time.perf_counter()-t0):.1f} ms", flush=True)
