"""C5 workload tooling and TM_BATCH_DEDUP on the host (no device)."""

import pytest

from emqx_amd import gen
from emqx_amd.engine import Engine
from emqx_amd.skew import Churn, workload
from oracle import oracle as O


def test_derived_filters_match_their_hot_topic():
    p = gen.SkewParams(seed=2, n_hot=40, k_per_hot=30)
    hot, derived = gen.gen_skew(p)
    H = hot.tolist()
    assert len(set(H)) == 40
    per = {h: 0 for h in H}
    for f in derived.tolist():
        hits = [h for h in H if O.match(h, f)]
        assert hits
        for h in hits:
            per[h] += 1
    assert min(per.values()) >= 25


def test_workload_skew_and_dedup_rows():
    p = gen.SkewParams(seed=3, n_hot=100, k_per_hot=5)
    allf, derived, hot, pubs = workload(p, 500, 20_000, seed=3, background_pool=3000)
    T = pubs.tolist()
    hot_set = set(hot.tolist())
    frac = sum(t in hot_set for t in T) / len(T)
    assert 0.85 < frac < 0.95
    e = Engine(device=-1)
    b = e.prepare(pubs, dedup=True)
    row_of, n_rows = b.row_map()
    assert n_rows == len(set(T))
    first = {}
    for i, r in enumerate(row_of.tolist()):
        assert first.setdefault(r, T[i]) == T[i]
    assert sorted(first) == list(range(n_rows))


def test_churn_keeps_live_set_consistent():
    p = gen.SkewParams(seed=4, n_hot=20, k_per_hot=10)
    hot, derived = gen.gen_skew(p)
    c = Churn(hot, derived.tolist(), seed=1)
    n0 = len(c.live)
    dels, adds = c.step(50)
    assert len(dels) == 25 and len(adds) == 25
    assert len(c.live) == n0 and len(c.live_set) == n0
    assert not (set(dels) & c.live_set) and set(adds) <= c.live_set


def test_c5_checker_equals_the_trie_oracle_under_churn():
    """oracle/c5_checker.py (the full-scale C5 test's expected rows) against the
    trie oracle over the whole snapshot, on a small C5 workload with churn."""
    import random

    from oracle.c5_checker import FinalSnapshot, SnapshotOracle
    from oracle import pyoracle as P

    p = gen.SkewParams(seed=12, n_hot=60, k_per_hot=80, vocab=8)   # small vocab: many cross-family matches
    allf, derived, hot, pubs = workload(p, 2000, 5000, seed=12, background_pool=800)
    background = allf.tolist()[len(derived):]
    chk = SnapshotOracle(derived, background)
    live = set(derived.tolist())
    churn = Churn(hot, derived.tolist(), seed=5)
    T = sorted(set(pubs.tolist()))[:400] + hot.tolist()
    added = []
    for rnd in range(3):
        if rnd:
            dels, adds = churn.step(400)
            # a base filter deleted and subscribed again: listed once by FinalSnapshot
            adds += [f for f in dels[:5] if f not in churn.live_set]
            churn.live_set.update(adds)
            added += adds
            for f in dels:
                chk.delete(f)
                live.discard(f)
            for f in adds:
                chk.insert(f)
                live.add(f)
        fin = FinalSnapshot(derived, background, churn.live_set, added)
        assert fin.rows(T) == chk.rows(T), rnd
        fin.close()
        orc = P.Oracle()
        F = sorted(live) + background
        for f in F:
            orc.register(f)
            orc.insert(f)
        buf, offs = P.pack(T)
        counts, idx, _ = orc.match_batch(buf, offs)
        orc.close()
        cut = [0]
        for c in counts.tolist():
            cut.append(cut[-1] + c)
        exp = [[F[int(j)] for j in idx[cut[i]:cut[i + 1]]] for i in range(len(T))]
        assert chk.rows(T) == exp, rnd
    chk.close()


def test_parallel_churn_builds_the_same_trie_as_the_serial_pass():
    """tm_trie_insert_many / delete_many of 2,048+ filters on a big trie run
    their mutation pass on the engine's workers (first-two-word subtrees, then
    the edge hash by bucket ranges).  The result must be the serial pass's
    trie: same nodes, edges and filters, the same edge_count of every node on
    the churned paths, and a consistent edge hash (tm_debug_check)."""
    import random

    p = gen.SkewParams(seed=21, n_hot=2500, k_per_hot=100)
    allf, derived, hot, _ = workload(p, 60_000, 100, seed=21, background_pool=500)
    A = Engine(device=-1, host_threads=1)      # one thread: the serial pass
    B = Engine(device=-1, host_threads=8)
    for e in (A, B):
        e.insert_many(allf)

    def same():
        a, b = A.stats(), B.stats()
        assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
        B.debug_check()

    same()
    churn = Churn(hot, derived.tolist(), seed=3)
    touched = []
    for _ in range(4):
        dels, adds = churn.step(10_000)
        for e in (A, B):
            Churn.apply(e, gen.Strings.from_list(dels), gen.Strings.from_list(adds))
        touched += dels[:300] + adds[:300]
        same()
    rng = random.Random(4)
    for f in touched + rng.sample(sorted(churn.live_set), 1000):
        ws = f.split(b"/")
        for k in range(1, len(ws) + 1):
            pre = b"/".join(ws[:k])
            assert A.lookup(pre) == B.lookup(pre), pre


@pytest.mark.parametrize("threads", [1, 8])
def test_apply_many_equals_delete_many_then_insert_many(threads):
    """tm_trie_apply_many plans the deletes and the inserts of a delta
    together, before any delete runs.  Its result must be the two calls'
    (delete_many, then insert_many): same nodes, edges, filters and lookups,
    including inserts whose planned deepest node a delete of the same call
    removes (a sibling leaf deleted: its node dies and the insert walks again)
    and filters deleted and re-added in one delta."""
    import random

    p = gen.SkewParams(seed=23, n_hot=2500, k_per_hot=100)
    allf, derived, hot, _ = workload(p, 60_000, 100, seed=23, background_pool=500)
    A = Engine(device=-1, host_threads=threads)   # the two calls
    B = Engine(device=-1, host_threads=threads)   # one apply
    for e in (A, B):
        e.insert_many(allf)
    churn = Churn(hot, derived.tolist(), seed=5)
    rng = random.Random(6)
    touched = []
    for step in range(3):
        dels, adds = churn.step(10_000)
        # deep leaves deleted while an insert extends the same path one level
        # further (its planned node is the deleted leaf), and re-adds
        extra_del = rng.sample([f for f in sorted(churn.live_set) if not f.endswith(b"#")], 300)
        extra_add = [f + b"/zz%d" % step for f in extra_del[:150]] + extra_del[150:]
        dels = dels + extra_del
        adds = adds + extra_add
        A.delete_many(gen.Strings.from_list(dels))
        A.insert_many(gen.Strings.from_list(adds))
        nd, ni = B.apply_many(gen.Strings.from_list(dels), gen.Strings.from_list(adds))
        assert (nd, ni) == (len(dels), len(adds))
        a, b = A.stats(), B.stats()
        assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
        B.debug_check()
        touched += dels[:200] + adds[:200] + extra_add
    for f in touched:
        ws = f.split(b"/")
        for k in range(1, len(ws) + 1):
            pre = b"/".join(ws[:k])
            assert A.lookup(pre) == B.lookup(pre), pre
    # small deltas (the serial passes) and empty lists
    assert B.apply_many([], []) == (0, 0)
    A.delete_many([b"a/b/c"]); A.insert_many([b"a/b/c/d", b"a/b/c"])
    assert B.apply_many([b"a/b/c"], [b"a/b/c/d", b"a/b/c"]) == (1, 2)
    assert B.lookup(b"a/b/c/d") == A.lookup(b"a/b/c/d") and B.lookup(b"a/b/c") == A.lookup(b"a/b/c")
    B.debug_check()


def test_parallel_insert_creates_a_shared_first_level_edge_once():
    """A bulk insert whose filters share a NEW first word but differ in the
    second word is dealt to different workers (first-two-word subtrees): the
    level-0 edge they all need must be created once, not once per worker."""
    p = gen.SkewParams(seed=22, n_hot=500, k_per_hot=40)
    allf, _, _, _ = workload(p, 20_000, 100, seed=22, background_pool=500)
    A = Engine(device=-1, host_threads=1)
    B = Engine(device=-1, host_threads=8)
    adds = [b"nw%d/%d/x" % (i % 5, i) for i in range(3000)] + [b"nw%d" % (i % 3) for i in range(6)]
    adds += [b"+/nz%d/%d" % (i % 4, i) for i in range(2500)]
    for e in (A, B):
        e.insert_many(allf)
        e.insert_many(gen.Strings.from_list(adds))
    a, b = A.stats(), B.stats()
    assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
    B.debug_check()
    for f in adds[::7] + [b"nw0", b"nw1", b"+/nz1"]:
        assert A.lookup(f) == B.lookup(f), f
    # and the deletes of the same filters leave both tries equal again
    for e in (A, B):
        e.delete_many(gen.Strings.from_list(adds))
    a, b = A.stats(), B.stats()
    assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
    B.debug_check()


def test_parallel_insert_splits_a_hot_two_word_prefix():
    """A bulk insert with most of its filters under one first-two-words prefix
    (C5's "+/+" share) splits that part by the third word: the prefix's
    depth-2 node is then shared by workers, so its new children, its own
    filter and the new nodes above it must each come out once."""
    p = gen.SkewParams(seed=23, n_hot=500, k_per_hot=40)
    allf, _, _, _ = workload(p, 20_000, 100, seed=23, background_pool=500)
    A = Engine(device=-1, host_threads=1)
    B = Engine(device=-1, host_threads=8)
    adds = [b"hp/hq/%d/%d" % (i % 50, i) for i in range(3000)] + [b"hp/hq", b"hp/hq/#", b"hp/hq/+"]
    adds += [b"+/+/w%d/%d/#" % (i % 7, i) for i in range(1500)] + [b"other%d/x" % i for i in range(500)]
    for e in (A, B):
        e.insert_many(allf)
        e.insert_many(gen.Strings.from_list(adds))
    a, b = A.stats(), B.stats()
    assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
    B.debug_check()
    for f in adds[::5] + [b"hp/hq", b"hp/hq/7", b"+/+/w3"]:
        assert A.lookup(f) == B.lookup(f), f
    # the deletes split the same way (depth-2 records shared under the
    # stripe locks): half, then the rest, which empties the hot prefix's
    # depth-2 node from several workers at once
    for part in (adds[::2], adds[1::2]):
        for e in (A, B):
            e.delete_many(gen.Strings.from_list(part))
        a, b = A.stats(), B.stats()
        assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
        B.debug_check()
    for f in [b"hp/hq", b"hp/hq/7", b"+/+/w3"] + adds[1::97]:
        assert A.lookup(f) == B.lookup(f) is None, f


def test_parallel_inserts_that_grow_the_edge_hash():
    """Parallel insert batches of ~20% of the trie each: the edge phase finds
    the table too full for a batch's inserts, re-packs it after the deletes
    and buckets the inserts for the new table.  Each batch must leave the
    serial pass's trie (same counts, consistent hash, same lookups)."""
    p = gen.SkewParams(seed=24, n_hot=600, k_per_hot=40)
    allf, _, _, _ = workload(p, 12_000, 100, seed=24, background_pool=500)
    A = Engine(device=-1, host_threads=1)
    B = Engine(device=-1, host_threads=8)
    for e in (A, B):
        e.insert_many(allf)
    grew = 0
    for step in range(8):
        n = max(2048, B.stats()["filters"] // 5)
        adds = [b"g%d/%d/x%d/+/y" % (step, i % 97, i) for i in range(n)]
        s0 = B.stats()["slots"]
        for e in (A, B):
            e.insert_many(gen.Strings.from_list(adds))
        grew += B.stats()["slots"] > s0
        a, b = A.stats(), B.stats()
        assert all(a[k] == b[k] for k in ("nodes", "edges", "filters", "words")), (a, b)
        B.debug_check()
        for f in adds[::41]:
            assert A.lookup(f) == B.lookup(f) is not None, f
    assert grew >= 1
