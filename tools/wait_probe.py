import time, sys
sys.path.insert(0, '/root/repo')
import numpy as np
from emqx_amd import gen
from emqx_amd.engine import Engine
F = gen.gen_filters(gen.C1)
T = gen.gen_topics(gen.C1, F, 7, 65536)
eng = Engine(device=0)
eng.insert_many(F); eng.sync()
for dedup in (False, True):
    b = eng.prepare(T, dedup=dedup)
    b.launch().wait()
    ts = []
    for _ in range(50):
        t = time.perf_counter(); b.wait(); ts.append(1e6 * (time.perf_counter() - t))
    ts2 = []
    for _ in range(50):
        t = time.perf_counter(); b.stats(); ts2.append(1e6 * (time.perf_counter() - t))
    ts3 = []
    for _ in range(20):
        b.launch(); time.sleep(0.01)
        t = time.perf_counter(); b.wait(); ts3.append(1e6 * (time.perf_counter() - t))
    print(f"dedup={dedup}: wait on a done batch {np.median(ts):.1f} us, stats {np.median(ts2):.1f} us, wait after the batch finished {np.median(ts3):.1f} us")
    b.free()
