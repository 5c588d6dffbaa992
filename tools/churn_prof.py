"""C5 churn apply on the host mirror alone (dev tool; TM_PAR_TRACE=1 prints
the parallel phases): 10k deltas per step, K filters per hot topic.

    python tools/churn_prof.py [K] [steps] [device] [apply|two]   (device -1: host-only engine;
    apply: one tm_trie_apply_many per step, two: delete_many + insert_many)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402
from emqx_amd.skew import Churn, workload  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
device = int(sys.argv[3]) if len(sys.argv) > 3 else -1
mode = sys.argv[4] if len(sys.argv) > 4 else "apply"
p = gen.SkewParams(k_per_hot=K)
allf, derived, hot, pubs = workload(p, 100_000, 100_000, seed=5)
eng = Engine(device=device)
eng.insert_many(allf)
churn = Churn(hot, derived.tolist(), seed=11)
deltas = []
for _ in range(steps):
    dels, adds = churn.step(10_000)
    deltas.append((gen.Strings.from_list(dels), gen.Strings.from_list(adds)))
def throttled():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f)}
    except OSError:
        return {}


th0 = throttled()
for d, a in deltas:
    t = time.perf_counter()
    if mode == "apply":
        eng.apply_many(d, a)
        t1 = t
    else:
        eng.delete_many(d)
        t1 = time.perf_counter()
        eng.insert_many(a)
    t2 = time.perf_counter()
    if device >= 0:
        eng.sync()   # the delta upload, as the next launch would do it
    t3 = time.perf_counter()
    print(f"K={K} {mode} sync {1e3 * (t3 - t2):.2f} ms del {1e3 * (t1 - t):.2f} ms  ins {1e3 * (t2 - t1):.2f} ms  total {1e3 * (t2 - t):.2f}", flush=True)
th1 = throttled()
print("cgroup cpu.stat deltas:", {k: th1[k] - th0.get(k, 0) for k in th1}, flush=True)
