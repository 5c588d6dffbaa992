"""The engine's concurrent host code under a sanitizer (run by
tests/test_sanitize.py in a child process with the clang runtime preloaded,
EMQX_TM_LIB / EMQX_NIF_MOCK_LIB pointing at a sanitized build: ASan + UBSan,
or TSan; emqx_amd/build.py build_sanitized).  Host-only engines (device -1):

1. bulk insert + four 10k-delta tm_trie_apply_many steps on 8 workers (the
   parallel mutation: plan, phase 1 over first-two-word subtrees, the edge
   phase by bucket ranges, the merge), checked against a 1-worker engine;
2. the lingering workers: back-to-back parallel deltas with gaps shorter and
   longer than the spin deadline between them (workers spinning, sleeping on
   the futex and woken mid-spin);
3. concurrent tm_match_coalesced callers on a host engine (every call
   returns its error: the queue shards, no device);
4. the erl_nif shim with 4 concurrent writer processes on one engine
   (insert / delete / lookup / empty) and engines dropped while others work
   (the resource destructor), the final trie compared with the oracle.

The reference's threading contract: trie writes are serialised by a mnesia
transaction, reads are dirty (src/emqx_trie.erl:55-56, 81-116;
src/emqx_router.erl:185-186).  Prints "SANITIZE OK" at the end."""

from __future__ import annotations

import os
import random
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from emqx_amd import _native as N  # noqa: E402
from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402
from emqx_amd.skew import Churn, workload  # noqa: E402


def same(A, B):
    a, b = A.stats(), B.stats()
    assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
    B.debug_check()


def parallel_churn():
    p = gen.SkewParams(seed=31, n_hot=1200, k_per_hot=60)
    allf, derived, hot, _ = workload(p, 20_000, 100, seed=31, background_pool=500)
    A = Engine(device=-1, host_threads=1)
    B = Engine(device=-1, host_threads=8)
    for e in (A, B):
        e.insert_many(allf)
    same(A, B)
    churn = Churn(hot, derived.tolist(), seed=7)
    for _ in range(4):
        dels, adds = churn.step(10_000)
        d, a = gen.Strings.from_list(dels), gen.Strings.from_list(adds)
        for e in (A, B):
            Churn.apply(e, d, a)
        same(A, B)
    # 2. lingering workers: deltas back to back, then with gaps around the
    # spin deadline (0.3 ms inside a call, 0.15 ms grace after it)
    for gap in (0.0, 0.0, 0.0002, 0.001, 0.02, 0.0, 0.005):
        dels, adds = churn.step(6_000)
        d, a = gen.Strings.from_list(dels), gen.Strings.from_list(adds)
        for e in (A, B):
            Churn.apply(e, d, a)
        time.sleep(gap)
    same(A, B)
    B.delete_many(gen.Strings.from_list(sorted(churn.live_set)[::3]))
    A.delete_many(gen.Strings.from_list(sorted(churn.live_set)[::3]))
    same(A, B)
    A.close()
    B.close()
    print("parallel churn ok", flush=True)


def coalesced_callers():
    eng = Engine(device=-1)
    eng.insert(b"a/+")
    eng.coalesce_config(max_batch=8, linger_us=100)
    errs = []

    def worker(k):
        for i in range(40):
            t = b"x" * (N.TM_MAX_TOPIC_LEN + 1) if (k + i) % 11 == 0 else b"a/%d" % i
            try:
                eng.match_coalesced(t)
                errs.append("matched on a host engine")
            except N.TmError as e:
                if e.rc != (N.TM_EINVAL if len(t) > N.TM_MAX_TOPIC_LEN else N.TM_ENODEV):
                    errs.append(e.rc)
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errs and all(not t.is_alive() for t in ths), errs[:3]
    eng.close()
    print("coalesced callers ok", flush=True)


def nif_writers():
    from oracle import oracle as O

    from nif_harness import Nif
    nif = Nif()
    e = nif.new(-1)
    words = [b"a", b"b", b"c", b"+", b"#", b"$SYS", b"", b"dd"]
    pools = []
    for k in range(4):          # disjoint filter pools per writer: the final set is known
        rng = random.Random(k)
        pool = set()
        while len(pool) < 150:
            ws = [b"w%d" % k] + [rng.choice(words) for _ in range(rng.randint(0, 4))]
            if b"#" in ws[:-1]:
                continue
            pool.add(b"/".join(ws))
        pools.append(sorted(pool))
    live = [set() for _ in range(4)]
    errs = []

    def writer(k):
        rng = random.Random(100 + k)
        pid = k + 1
        try:
            for step in range(600):
                f = rng.choice(pools[k])
                if f in live[k] and rng.random() < 0.5:
                    assert nif.call("delete", e, f, pid=pid) == "ok"
                    live[k].discard(f)
                else:
                    assert nif.call("insert", e, f, pid=pid) == "ok"
                    live[k].add(f)
                if step % 40 == 0:
                    nif.call("lookup", e, rng.choice(pools[k]), pid=pid)
                    nif.call("empty", e, pid=pid)
                if step % 150 == 0:      # a short-lived engine of its own, dropped while the others work
                    x = nif.new(-1)
                    nif.call("insert", x, f, pid=pid)
                    nif.drop(x)
        except Exception as ex:   # noqa: BLE001 (reported by the main thread)
            errs.append(repr(ex))
    ths = [threading.Thread(target=writer, args=(k,)) for k in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not errs and all(not t.is_alive() for t in ths), errs[:3]
    t = O.Trie()
    for s in live:
        for f in sorted(s):
            t.insert(f)
    for pool in pools:
        for f in pool:
            exp = t.lookup(f)
            got = nif.call("lookup", e, f)
            if not exp:
                assert got == [], f
            else:
                (_, ec, topic), = exp
                assert got == [("trie_node", f, ec, topic if topic is not None else "undefined", "undefined")], f
    nif.drop(e)
    print("nif writers ok", flush=True)


def check_instrumented():
    """The sanitized builds are what this process runs: the runtime is in,
    and the engine and shim mapped are the ones the environment names."""
    import ctypes
    sym = {"asan": "__asan_report_load8", "tsan": "__tsan_init"}[os.environ["EMQX_SANITIZER"]]
    assert hasattr(ctypes.CDLL(None), sym), f"{sym} missing: sanitizer runtime not loaded"
    N.lib()
    from nif_harness import Nif
    Nif()
    with open("/proc/self/maps") as f:
        maps = f.read()
    for var in ("EMQX_TM_LIB", "EMQX_NIF_MOCK_LIB"):
        assert os.path.realpath(os.environ[var]) in maps, f"{var} not mapped"
    print("instrumented:", os.environ["EMQX_SANITIZER"], flush=True)


if __name__ == "__main__":
    check_instrumented()
    which = sys.argv[1:] or ["churn", "coalesced", "nif"]
    if "churn" in which:
        parallel_churn()
    if "coalesced" in which:
        coalesced_callers()
    if "nif" in which:
        nif_writers()
    print("SANITIZE OK", flush=True)
