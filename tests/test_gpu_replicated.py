"""One engine over several devices (tm_create_replicated, the NIF's
new([Device]) and tm_group_*): one host trie, an HBM replica per device, a
mutation made once and uploaded to every replica -- needs an MI355X.

A one-GPU box runs two replicas on device 0: each has its own stream, HBM
tables and async pipeline, so the dealing of per-publish calls, the split of
whole batches and the delta upload to every replica are exactly the
multi-GPU ones.  Expected rows come from the oracle (src/emqx_trie.erl
restated) or from a single-replica engine that the oracle already pins."""

import ctypes as C
import random
import threading
from dataclasses import replace

import numpy as np
import pytest
from test_gpu_parity import assert_same, engine_rows, oracle_rows

from emqx_amd import _native as N
from emqx_amd import gen
from emqx_amd.engine import Engine, Group
from nif_harness import Nif
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nif():
    return Nif()


def _recv_all(nif, pid, refs, timeout_s=60):
    import time
    got = {}
    deadline = time.time() + timeout_s
    while len(got) < len(refs):
        msg = nif.recv(pid, int(max(1, (deadline - time.time()) * 1000)))
        assert msg is not None, f"pid {pid}: {len(refs) - len(got)} replies missing"
        assert msg[0] == "emqx_tm_match"
        got[msg[1][1]] = msg[2]
    return got


def test_nif_engine_over_two_replicas_async_under_concurrent_subscribes(nif, device_pair):
    """new([0, 0]) (and new([0, 1]) on a box with two GPUs): match_async calls from 16 processes are dealt over both
    replicas while a writer keeps subscribing; every reply equals the oracle's
    set, and a match issued after an insert returned sees the filter whichever
    replica serves it (read-your-writes through the shared host trie)."""
    rng = random.Random(21)
    words = [b"a", b"b", b"c", b"d", b"+", b"#", b"$SYS"]
    filters = set()
    while len(filters) < 1500:
        ws = [rng.choice(words) for _ in range(rng.randint(1, 5))]
        if b"#" not in ws[:-1]:
            filters.add(b"/".join(ws))
    e, t = nif.new(device_pair), O.Trie()
    for f in sorted(filters):
        assert nif.call("insert", e, f) == "ok"
        t.insert(f)
    names = [b"a", b"b", b"c", b"d", b"e", b""]
    topics = [b"/".join(rng.choice(names) for _ in range(rng.randint(1, 6))) for _ in range(4000)]
    exp = {tp: sorted(set(t.match(tp))) for tp in topics}
    stop = threading.Event()
    errors = []

    def writer():
        # subscribes under rw/, which no query topic reaches (t, the oracle of
        # the base filters, does not see them); each one is checked at once
        # through match_async (read-your-writes)
        try:
            k = 0
            while not stop.is_set() and k < 400:
                f = b"rw/%d/+" % k
                assert nif.call("insert", e, f, pid=900) == "ok"
                for _ in range(2):   # two calls: consecutive calls go to different replicas
                    r = nif.ref()
                    assert nif.call("match_async", e, b"rw/%d/x" % k, r, pid=900) == "ok"
                    got = _recv_all(nif, 900, [(r.ident, None)])
                    assert got[r.ident] == sorted(set(t.match(b"rw/%d/x" % k)) | {f}), (k, got)
                k += 1
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    def process(pid):
        try:
            mine = topics[pid % 16::16]
            for i in range(0, len(mine), 32):
                refs = []
                for tp in mine[i:i + 32]:
                    r = nif.ref()
                    assert nif.call("match_async", e, tp, r, pid=pid) == "ok"
                    refs.append((r.ident, tp))
                got = _recv_all(nif, pid, refs)
                for ident, tp in refs:
                    assert got[ident] == exp[tp], tp
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    wt = threading.Thread(target=writer)
    wt.start()
    th = [threading.Thread(target=process, args=(p,)) for p in range(100, 116)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    stop.set()
    wt.join()
    assert not errors, errors[0]
    # batch NIFs on the replicated engine (fresh batches go round-robin over the replicas)
    for _ in range(4):
        assert nif.call("match_batch", e, topics[:300]) == [exp[tp] for tp in topics[:300]]
    nif.drop(e)


def _c2_small(n_filters=100_000, n_topics=100_000, seed=2201):
    p = replace(gen.C2, n_filters=n_filters)
    F = gen.gen_filters(p)
    T = gen.gen_topics(p, F, seed, n_topics)
    return F, T


def test_replicated_engine_splits_large_batches_like_one_engine(device_pair):
    F, T = _c2_small()
    one = Engine(device=0)
    one.insert_many(F)
    rep = Engine(devices=device_pair)
    assert rep.replicas == 2
    assert rep.insert_many(F) == len(F)
    o1, i1 = one.match_batch(T)
    o2, i2 = rep.match_batch(T)          # >= 65,536 publishes: one slice per replica
    assert np.array_equal(o1, o2) and np.array_equal(i1, i2)
    # the same ids name the same filters (one host trie)
    for i in np.unique(i2)[:3000]:
        assert rep.filter_bytes(int(i)) == one.filter_bytes(int(i))
    # an oracle sample of the rows
    Tl = T.tolist()
    idx = list(range(0, len(Tl), 33))
    sub = [Tl[i] for i in idx]
    exp, _ = oracle_rows(F.tolist(), sub, nthreads=16)
    got = [[rep.filter_bytes(int(x)) for x in i2[o2[i]:o2[i + 1]]] for i in idx]
    assert_same(sub, got, exp)
    # small batches run on one replica, round-robin: both give the oracle's rows
    for k in range(4):
        s = Tl[k * 500:(k + 1) * 500]
        e2, _ = oracle_rows(F.tolist(), s)
        assert_same(s, engine_rows(rep, s), e2)


def test_c3_full_trie_split_over_device_pair_sampled_per_slice(device_pair):
    """BASELINE config C3 at its own size: C2's 1M-filter trie replicated on
    both devices of device_pair (tm_group), 1M C2 publishes split into one
    slice per replica; every slice's 3,000-row sample -- gathered on its own
    device (tm_group_sample) -- equals the oracle's rows (src/emqx_trie.erl
    restated), and the merged CSR equals one single-replica engine's."""
    from emqx_amd import selfcheck as SC
    F = gen.gen_filters(gen.C2)
    T = gen.gen_topics(gen.C2, F, 1000, 1_000_000)
    grp = Group(device_pair)
    assert grp.insert_many(F) == len(F)
    grp.sync()
    b = grp.prepare(T)
    b.launch().wait()
    n = len(T)
    assert b.stats()["topics"] == n
    rep = grp.engine()
    Fl, Tl = F.tolist(), T.tolist()
    lo = [0, n // 2, n]
    for k in range(2):
        idx = lo[k] + SC.sample_index(lo[k + 1] - lo[k])
        assert len(idx) >= 3000
        so, si = b.sample(idx)
        sub = [Tl[int(i)] for i in idx]
        exp, _ = oracle_rows(Fl, sub, nthreads=16)
        got = [[rep.filter_bytes(int(x)) for x in si[so[j]:so[j + 1]]] for j in range(len(idx))]
        assert_same(sub, got, exp)
    # the whole split result = one engine's on device 0
    offs, ids = b.result()
    b.free()
    grp.close()
    one = Engine(device=0)
    one.insert_many(F)
    o1, i1 = one.match_batch(T)
    assert np.array_equal(o1, offs) and np.array_equal(i1, ids)
    one.close()


def test_replicated_routes_rules_and_dispatch_equal_one_engine():
    p = replace(gen.C1, n_filters=4000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 77, 70_000).tolist()
    rng = np.random.default_rng(5)
    one, grp = Engine(device=0), Group([0, 0])
    rep = grp.engine()
    events = []
    for j, f in enumerate(F):
        for d in rng.choice(16, int(rng.integers(1, 4)), replace=False):
            events.append((N.TM_ROUTE_WRITE, f, int(d)))
    assert one.route_apply(events) == grp.route_apply(events)
    for j, f in enumerate(F[:1500]):
        for s in rng.choice(5000, int(rng.integers(1, 3)), replace=False):
            one.subscribe(f, int(s), 0)
            rep.subscribe(f, int(s), 0)
    # match_routes_batch: 70k publishes are split over the replicas
    a = one.match_routes_batch(T)
    b = rep.match_routes_batch(T)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    # rules: names split over the replicas
    rules = F[:200]
    ra = one.rules_match(T[:20_000], rules)
    rb = rep.rules_match(T[:20_000], rules)
    assert np.array_equal(ra, rb)
    for i in range(0, 20_000, 997):
        for j in range(0, 200, 7):
            assert bool(rb[i, j]) == O.match(T[i], rules[j])
    # fan-out of a split group batch = one engine's
    gb = grp.prepare(T)
    gb.launch().wait()
    go, gs = gb.dispatch()
    b1 = one.prepare(T)
    b1.launch().wait()
    oo, _, os_ = b1.dispatch()
    assert np.array_equal(go, oo) and np.array_equal(gs, os_)
    gb.free()
    b1.free()
    grp.close()


def test_group_ids_stay_consistent_with_deletes_during_a_launch():
    """with one engine per replica, a capacity re-launch on
    one slice could free a deleted id early there and the replicas' ids
    diverge.  One host trie cannot diverge: launch a group batch, delete
    filters it matches, wait (topics matching ~200 filters each overflow the
    first staging and re-launch), insert new filters, and every id of the
    result still names a filter that matches its topic; new ids never collide
    with ids the live result holds."""
    import itertools
    lit = [b"a", b"b", b"c", b"d", b"e", b"f"]
    F = []   # every filter matching a/b/c/d/e/f: each level literal or '+', optionally cut by '#'
    for k in range(len(lit) + 1):
        for pick in itertools.product((0, 1), repeat=k):
            ws = [lit[i] if pick[i] == 0 else b"+" for i in range(k)]
            F.append(b"/".join(ws + ([b"#"] if k < len(lit) else [])))
    F = sorted(set(F))
    assert len(F) == 127
    T = [b"a/b/c/d/e/f"] * 2000 + [b"a/b/c/d/e/g"] * 1000 + [b"a/x/c/d/e/f"] * 1000
    grp = Group([0, 0])
    for f in F:
        grp.insert(f)
    rep = grp.engine()
    b = grp.prepare(T)
    b.launch()
    deleted = [f for f in F if f.split(b"/")[1:2] == [b"+"]][::2]
    for f in deleted:
        grp.delete(f)
    b.wait()
    offs, ids = b.result()
    held = set(int(x) for x in ids)
    before = {i: rep.filter_bytes(i) for i in held}
    new = [b"n/%d/+" % k for k in range(500)]
    for f in new:
        grp.insert(f)
    new_ids = {rep.filter_id(f) for f in new}
    assert not (new_ids & held)
    for i in held:
        assert rep.filter_bytes(i) == before[i]
    for k, tp in enumerate(T):
        for x in ids[offs[k]:offs[k + 1]]:
            assert O.match(tp, before[int(x)]), (tp, before[int(x)])
    # and a fresh launch after the deletes matches the oracle exactly
    live = sorted(set(F) - set(deleted)) + new
    b.launch().wait()
    o2, i2 = b.result()
    exp, _ = oracle_rows(live, T)
    assert_same(T, [[rep.filter_bytes(int(x)) for x in i2[o2[k]:o2[k + 1]]] for k in range(len(T))], exp)
    b.free()
    grp.close()


def test_group_coalesced_calls_from_threads():
    p = replace(gen.C1, n_filters=3000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 78, 6000).tolist()
    grp = Group([0, 0])
    for f in F:
        grp.insert(f)
    exp, _ = oracle_rows(F, T)
    L = N.lib()
    errors = []

    def worker(w):
        try:
            buf = (C.c_uint32 * 4096)()
            n = C.c_uint32()
            for i in range(w, len(T), 8):
                N.check(L.tm_group_match_coalesced(grp.h, T[i], len(T[i]), buf, 4096, C.byref(n)), "coalesced")
                got = [grp.filter_bytes(int(buf[k])) for k in range(n.value)]
                assert got == exp[i], T[i]
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    th = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]
    st = grp.engine().async_stats()
    assert st["depth"] == 2 * 4 and st["requests"] == len(T)   # both replicas' pipelines served calls
    grp.close()
