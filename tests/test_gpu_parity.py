"""Parity of the HIP path (through the C ABI) with the oracle -- needs an MI355X.

Bit-exact per-topic sorted, deduplicated match sets on: the reference's KATs,
the committed golden vectors, seeded C1/C2 workloads, deep/irregular/adversarial
topics, the forced slow path, churn with delta uploads, and size-independent
properties of a full 10M-publish C2 batch."""

import os
import random
from dataclasses import replace

import numpy as np
import pytest
from conftest import lb, load_golden

from emqx_amd import emqx_router as R
from emqx_amd import emqx_trie as TR
from emqx_amd import gen
from emqx_amd.emqx_batch import PublishBatcher
from emqx_amd.engine import Engine
from oracle import oracle as O
from oracle import pyoracle as P

pytestmark = pytest.mark.gpu


def rows_of(offs, ids):
    return [ids[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


def oracle_rows(filters, topics, nthreads=8):
    """Oracle restatement: per-topic lists of filter bytes, sorted, dedup'd."""
    orc = P.Oracle()
    for f in filters:
        orc.register(f)
        orc.insert(f)
    buf, offs = P.pack(topics)
    counts, idx, st = orc.match_batch(buf, offs, nthreads=nthreads)
    cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    orc.close()
    return [[filters[int(j)] for j in idx[cut[i]:cut[i + 1]]] for i in range(len(topics))], st


def engine_rows(eng, topics):
    offs, ids = eng.match_batch(topics)
    cache = {}

    def fb(i):
        i = int(i)
        if i not in cache:
            cache[i] = eng.filter_bytes(i)
        return cache[i]
    return [[fb(i) for i in r] for r in rows_of(offs, ids)]


def assert_same(topics, got, exp):
    bad = [i for i in range(len(topics)) if got[i] != exp[i]]
    assert not bad, [(topics[i], got[i], exp[i]) for i in bad[:3]]


def test_kat_trie_on_device():
    kat = load_golden("kat_trie.json")
    for case in kat["cases"]:
        TR.clear_tables()
        for op, arg, *rest in case["ops"]:
            if op == "insert":
                TR.insert(arg.encode())
            elif op == "delete":
                TR.delete(arg.encode())
            elif op == "empty":
                assert TR.empty() is arg
        for topic, exp in case.get("match", []):
            assert TR.match(topic.encode()) == sorted(e.encode() for e in exp), case["name"]
        for topic, n in case.get("match_len", []):
            assert len(TR.match(topic.encode())) == n


def test_kat_router_on_device():
    kat = load_golden("kat_router.json")
    for case in kat["cases"]:
        R.clear_tables()
        for t in case["add"]:
            R.add_route(t.encode())
        if "topics" in case:
            assert sorted(R.topics()) == [t.encode() for t in case["topics"]]
        if "match" in case:
            topic, exp = case["match"]
            assert sorted(r.topic for r in R.match_routes(topic.encode())) == [e.encode() for e in exp]
            assert [sorted(r.topic for r in rr) for rr in R.match_routes_batch([topic.encode()])] == \
                [[e.encode() for e in exp]]
        if "has" in case:
            assert R.has_routes(case["has"][0].encode()) is case["has"][1]
        for t in case.get("delete", []):
            R.delete_route(t.encode())
        if "topics_after" in case:
            assert R.topics() == []
        if "match_after" in case:
            assert R.match_routes(case["match_after"][0].encode()) == []


@pytest.mark.parametrize("fixture", ["synth_c1_small.json", "synth_c2_small.json", "synth_adversarial.json"])
def test_golden_vectors_on_device(fixture):
    g = load_golden(fixture)
    F = [lb(f) for f in g["filters"]]
    T = [lb(t) for t in g["topics"]]
    eng = Engine(device=0)
    for f in F:
        eng.insert(f)
    got = engine_rows(eng, T)
    exp = [[F[j] for j in row] for row in g["expected"]]
    assert_same(T, got, exp)


def test_c1_full_parity_and_walk_counters():
    F = gen.gen_filters(gen.C1).tolist()
    Ts = gen.gen_topics(gen.C1, gen.Strings.from_list(F), 1001, gen.C1_TOPICS)
    T = Ts.tolist()
    eng = Engine(device=0)
    for f in F:
        eng.insert(f)
    exp, st = oracle_rows(F, T)
    b = eng.prepare(Ts)
    b.launch().wait()
    offs, ids = b.result()
    bst = b.stats()
    cache = {}
    got = [[cache.setdefault(int(i), eng.filter_bytes(int(i))) for i in r] for r in rows_of(offs, ids)]
    assert_same(T, got, exp)
    # V and H counted on the device equal the oracle walk's (layout-independent)
    assert bst["visits"] == st["visits"] and bst["hash_hits"] == st["hash_hits"]
    assert bst["words"] == st["words"] and bst["matches"] == st["matches"]
    b.free()


@pytest.mark.parametrize("rowcap", [None, "4"])
def test_walk_rows_are_the_result_without_a_csr_pass(rowcap):
    """wait() leaves the result where the walk wrote it (tm_batch_rows: row i =
    ids[start[i] .. + count[i]), rows of different tiles in any order); the
    dense CSR is built only on request.  Both equal the oracle's rows; with a
    4-entry row cap most rows come from the generic path's runs instead."""
    if rowcap:
        os.environ["TM_ROWCAP"] = rowcap
    try:
        eng = Engine(device=0)
    finally:
        os.environ.pop("TM_ROWCAP", None)
    p = replace(gen.C1, n_filters=4000)
    F = gen.gen_filters(p).tolist()
    Ts = gen.gen_topics(p, gen.Strings.from_list(F), 77, 30000)
    T = Ts.tolist()
    for f in F:
        eng.insert(f)
    exp, _ = oracle_rows(F, T)
    b = eng.prepare(Ts)
    b.launch().wait()
    st = b.stats()
    assert st["ms_csr"] == 0.0   # no CSR pass in launch + wait
    cnt, start, stg = b.rows(len(T))
    assert int(cnt.sum()) == st["matches"]
    cache = {}
    got = [[cache.setdefault(int(i), eng.filter_bytes(int(i))) for i in stg[int(start[k]):int(start[k]) + int(cnt[k])]]
           for k in range(len(T))]
    assert_same(T, got, exp)
    if rowcap:
        assert st["slow_topics"] > 1000
    # tm_batch_sample: any rows, any order, gathered on the device (no CSR pass)
    pick = np.array([len(T) - 1, 0, 5, 5] + list(range(3, len(T), 211)), dtype=np.uint32)
    so, si = b.sample(pick)
    assert b.stats()["ms_csr"] == 0.0
    for j, k in enumerate(pick.tolist()):
        assert np.array_equal(si[so[j]:so[j + 1]], stg[int(start[k]):int(start[k]) + int(cnt[k])])
    so, si = b.sample([])
    assert len(so) == 1 and len(si) == 0
    with pytest.raises(RuntimeError):
        b.sample([len(T)])          # past the last row: TM_EINVAL
    # the dense CSR, built on request, holds the same rows in topic order
    offs, ids = b.result()
    assert b.stats()["ms_csr"] > 0.0
    assert np.array_equal(np.diff(offs.astype(np.int64)), cnt.astype(np.int64))
    for k in range(0, len(T), 97):
        assert np.array_equal(ids[offs[k]:offs[k + 1]], stg[int(start[k]):int(start[k]) + int(cnt[k])])
    # a relaunch drops the dense CSR; asking again rebuilds it
    b.launch().wait()
    assert b.stats()["ms_csr"] == 0.0
    offs2, ids2 = b.result()
    assert np.array_equal(offs, offs2) and np.array_equal(ids, ids2)
    b.free()


def test_fresh_batch_edge_topics_parity():
    """A fresh batch (device tokeniser + walk) of C1 in full with the walk
    counters, plus deep / irregular / empty topics and a 3,000-byte word (the
    tokeniser's HBM fallback and the generic path), equal the oracle."""
    eng = Engine(device=0)
    # (C1 already holds b"" and b"+/+": oracle ids are positions in a duplicate-free list)
    F = list(dict.fromkeys(gen.gen_filters(gen.C1).tolist() + [b"", b"+/+", b"a/#", b"+x/#"]))
    Ts = gen.gen_topics(gen.C1, gen.Strings.from_list(F), 1001, gen.C1_TOPICS)
    T = Ts.tolist() + [b"", b"", b"/", b"+x/y", b"a/" + b"/".join([b"q"] * 14), b"a" * 3000 + b"/b", b"a/b"]
    for f in F:
        eng.insert(f)
    exp, st = oracle_rows(F, T)
    b = eng.prepare(T)
    b.launch().wait()
    bst = b.stats()
    offs, ids = b.result()
    cache = {}
    got = [[cache.setdefault(int(i), eng.filter_bytes(int(i))) for i in r] for r in rows_of(offs, ids)]
    assert_same(T, got, exp)
    assert bst["matches"] == st["matches"] and bst["slow_topics"] >= 3
    b.free()


def test_c2_parity_sample():
    F = gen.gen_filters(gen.C2).tolist()
    T = gen.gen_topics(gen.C2, gen.Strings.from_list(F), 2002, 200_000).tolist()
    eng = Engine(device=0)
    for f in F:
        eng.insert(f)
    exp, _ = oracle_rows(F, T, nthreads=16)
    assert_same(T, engine_rows(eng, T), exp)


def test_forced_slow_path_parity():
    os.environ["TM_ROWCAP"] = "4"
    try:
        eng = Engine(device=0)
    finally:
        del os.environ["TM_ROWCAP"]
    p = replace(gen.C1, n_filters=3000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 5, 20000).tolist()
    for f in F:
        eng.insert(f)
    b = eng.prepare(T)
    b.launch().wait()
    assert b.stats()["slow_topics"] > 1000
    b.free()
    exp, _ = oracle_rows(F, T)
    assert_same(T, engine_rows(eng, T), exp)


@pytest.mark.parametrize("slow_lds", [None, "2"])
def test_long_rows_every_generic_sort(slow_lds):
    """Rows far past the fast path's K go to the generic path, whose probe
    stack lives in LDS (TM_SLOW_LDS=2: every topic outgrows it and walks again
    in global scratch) and whose sort runs in LDS up to 1,024 path-coded
    matches (as two LDS runs merged on the way out up to 2,048) or 2,048
    byte-ordered ones, in global scratch beyond: topics with ~1,000, ~1,300,
    ~2,600 (depth 10), ~2,000 (depth 11, ordered by bytes) and ~10,000
    matches, beside ordinary ones."""
    import itertools
    F = set()
    topics = []
    for depth, hashes in ((10, False), (9, True), (10, True), (11, False), (12, True)):
        ws = [b"l%d%s_%d" % (depth, b"h" if hashes else b"", i) for i in range(depth)]
        topics.append(b"/".join(ws))
        for mask in itertools.product((0, 1), repeat=depth):
            lv = [b"+" if m else w for m, w in zip(mask, ws)]
            F.add(b"/".join(lv))
            if hashes:
                F.add(b"/".join(lv + [b"#"]))
                F.add(b"/".join(lv[:-1] + [b"#"]))
    F = sorted(F | {b"#", b"+/#", b"zz/top"})
    T = topics + [b"zz/top", b"l10_0/x", b"nothing/here"] + topics
    env = {"TM_SLOW_LDS": slow_lds} if slow_lds else {}
    os.environ.update(env)
    try:
        eng = Engine(device=0)
    finally:
        for k in env:
            os.environ.pop(k, None)
    eng.insert_many(F)
    eng.sync()
    exp, _ = oracle_rows(F, T)
    # path-coded rows sorted as two LDS runs (1,029 and 1,282 entries) and
    # in global scratch (2,563); by bytes (deeper than 10 levels) in global
    # scratch (2,054 and 10,245)
    assert [len(r) for r in exp[:5]] == [1029, 1282, 2563, 2054, 10245]
    assert_same(T, engine_rows(eng, T), exp)


def test_deep_irregular_and_edge_topics():
    rng = random.Random(9)
    W = [b"a", b"b", b"", b"!", b"%", b"$q", b"#x", b"~", b"\xc3\xa9"]
    F = set()
    for _ in range(3000):
        d = rng.randint(1, 26)
        ws = [rng.choice(W + [b"+"]) for _ in range(d)]
        if rng.random() < 0.4:
            ws[-1] = b"#"
        F.add(b"/".join(ws))
    F = sorted(F)
    T = []
    for _ in range(4000):
        d = rng.randint(1, 30)
        T.append(b"/".join(rng.choice(W + [b"+x", b"c"]) for _ in range(d)))
    T += [b"", b"/", b"$", b"$q", b"a/" * 40 + b"a", b"+x/a", b"a/+x/#x"]
    eng = Engine(device=0)
    for f in F:
        eng.insert(f)
    exp, _ = oracle_rows(F, T)
    assert_same(T, engine_rows(eng, T), exp)


def test_literal_wildcard_words_in_names_follow_the_trie():
    # invalid publish names containing '+'/'#' words: the hot path is emqx_trie:match/1,
    # whose set (deduplicated) the engine must reproduce
    F = [b"#", b"+/#", b"a/#", b"a/+", b"a/#/b", b"a/#/#", b"+/+", b"a/+/#", b"#/#"]
    T = [b"a/#", b"a/+", b"a/#/b", b"#", b"+", b"+/+", b"a/+/c", b"#/#"]
    eng = Engine(device=0)
    tr = O.Trie()
    for f in F:
        eng.insert(f)
        tr.insert(f)
    assert engine_rows(eng, T) == [sorted(set(tr.match(t))) for t in T]


def test_empty_trie_empty_batch_and_readyourwrites():
    eng = Engine(device=0)
    offs, ids = eng.match_batch([b"a/b", b"c"])
    assert list(offs) == [0, 0, 0] and len(ids) == 0
    offs, ids = eng.match_batch([])
    assert list(offs) == [0] and len(ids) == 0
    eng.insert(b"a/+")
    assert eng.match(b"a/b") == [b"a/+"]          # a match issued after insert sees it
    eng.delete(b"a/+")
    assert eng.match(b"a/b") == []
    eng.insert(b"a/#")
    assert eng.match(b"a") == [b"a/#"]


def test_churn_with_delta_uploads():
    rng = random.Random(4)
    p = replace(gen.C2, n_filters=40_000)
    F = gen.gen_filters(p).tolist()
    live = set(F[:20_000])
    eng = Engine(device=0)
    tr = O.Trie()
    for f in live:
        eng.insert(f)
        tr.insert(f)
    T = gen.gen_topics(p, gen.Strings.from_list(F), 77, 4000).tolist()
    for rnd in range(6):
        for _ in range(2000):             # interleaved subscribe / unsubscribe deltas
            f = rng.choice(F)
            if f in live and rng.random() < 0.5:
                live.discard(f); eng.delete(f); tr.delete(f)
            else:
                live.add(f); eng.insert(f); tr.insert(f)
        got = engine_rows(eng, T)
        assert got == [sorted(set(tr.match(t))) for t in T], rnd
    st = eng.stats()
    assert st["uploads_delta"] >= 1 and st["delta_slots"] > 0


def test_full_c2_batch_properties():
    """10M publishes against 1M filters: CSR consistency, every row strictly
    increasing in filter bytes, every listed filter matches its topic, and a
    random sample of rows equals the oracle."""
    F = gen.gen_filters(gen.C2)
    Ts = gen.gen_topics(gen.C2, F, 3003, 10_000_000)
    fl = F.tolist()
    eng = Engine(device=0)
    for f in fl:
        eng.insert(f)
    b = eng.prepare(Ts)
    b.launch().wait()
    offs, ids = b.result()
    st = b.stats()
    assert offs[0] == 0 and np.all(np.diff(offs.astype(np.int64)) >= 0)
    assert int(offs[-1]) == len(ids) == st["matches"]
    rng = np.random.default_rng(0)
    sample = rng.choice(len(Ts), 3000, replace=False)
    from emqx_amd import emqx_topic as T
    cache = {}
    got, topics = [], []
    for i in sample:
        t = Ts[int(i)]
        row = [cache.setdefault(int(x), eng.filter_bytes(int(x))) for x in ids[offs[i]:offs[i + 1]]]
        assert all(row[k] < row[k + 1] for k in range(len(row) - 1)), t
        assert all(T.match(t, f) for f in row), t
        got.append(row)
        topics.append(t)
    exp, _ = oracle_rows(fl, topics, nthreads=16)
    assert_same(topics, got, exp)
    b.free()


def test_publish_batcher_emqx_batch_semantics():
    p = replace(gen.C1, n_filters=2000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 3, 5000).tolist()
    eng = Engine(device=0)
    for f in F:
        eng.insert(f)
    out = {}

    def on_result(topics, offs, ids):
        for i, t in enumerate(topics):
            out.setdefault(t, [eng.filter_bytes(int(x)) for x in ids[offs[i]:offs[i + 1]]])

    pb = PublishBatcher(eng, on_result, batch_size=999, linger_ms=5)
    for t in T:
        pb.publish(t)
    pb.close()
    exp, _ = oracle_rows(F, T)
    for t, e in zip(T, exp):
        assert out[t] == e


def test_stream_batches_overlap_and_read_your_writes():
    """TM_BATCH_STREAM: two batches on streams of their own, launched back to
    back (the second launched before the first is waited for), with trie
    inserts and deletes between rounds: every row equals the oracle's on the
    trie as it stood at that batch's launch."""
    p = replace(gen.C1, n_filters=4000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 21, 20000).tolist()
    eng = Engine(device=0)
    live = set(F[:3000])
    eng.insert_many(sorted(live))
    a, b = eng.prepare(T[:10000], stream=True), eng.prepare(T[10000:], stream=True)
    rng = random.Random(4)
    for rnd in range(4):
        snap = sorted(live)
        a.launch()
        b.launch()
        a.wait()
        b.wait()
        orc = P.Oracle()
        for f in snap:
            orc.register(f)
            orc.insert(f)
        for batch, part in ((a, T[:10000]), (b, T[10000:])):
            offs, ids = batch.result()
            buf, o = P.pack(part)
            counts, idx, _ = orc.match_batch(buf, o)
            cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
            for t in range(0, len(part), 7):
                exp = [snap[int(j)] for j in idx[cut[t]:cut[t + 1]]]
                got = [eng.filter_bytes(int(x)) for x in ids[offs[t]:offs[t + 1]]]
                assert got == exp, (rnd, part[t])
        # churn between rounds: reaches the next launches (read-your-writes)
        add = rng.sample([f for f in F if f not in live], 200)
        rem = rng.sample(sorted(live), 200)
        eng.insert_many(add)
        eng.delete_many(rem)
        live |= set(add)
        live -= set(rem)
    a.free()
    b.free()


def test_sync_async_queues_the_upload_behind_a_walk_in_flight():
    """tm_sync_async: deltas applied while a batch walks are uploaded behind it
    on the engine stream -- the walk in flight keeps its snapshot, the next
    launch sees the new filters."""
    p = replace(gen.C1, n_filters=3000)
    F = gen.gen_filters(p).tolist()
    Ts = gen.gen_topics(p, gen.Strings.from_list(F), 31, 50_000)
    T = Ts.tolist()
    eng = Engine(device=0)
    eng.insert_many(F[:2000])
    eng.sync()
    b = eng.prepare(Ts)
    b.launch()
    eng.insert_many(F[2000:])       # while the walk is in flight
    eng.delete_many(F[:100])
    eng.sync_async()
    b.wait()
    cache = {}

    def rows():
        offs, ids = b.result()
        return [[cache.setdefault(int(i), eng.filter_bytes(int(i))) for i in r] for r in rows_of(offs, ids)]
    exp_old, _ = oracle_rows(F[:2000], T)
    assert_same(T, rows(), exp_old)
    b.launch().wait()
    exp_new, _ = oracle_rows(F[100:], T)
    assert_same(T, rows(), exp_new)
    b.free()


def test_match_batch_one_shot_result_and_its_fallbacks():
    """tm_match_batch builds the CSR and copies it into mapped host memory
    behind the walk (one host wait).  Rows far above the initial id capacity
    (32 per topic) make the first call take the result() path (the copy could
    not hold them) and grow it; the next call fits and is one-shot.  Both,
    and a batch beyond the one-shot size, equal the oracle."""
    rng = random.Random(71)
    words = [b"a%d" % i for i in range(3)]
    F = set()
    for _ in range(8000):
        F.add(b"/".join(rng.choice(words + [b"+"]) for _ in range(6)))
    F = sorted(F | {b"#", b"+/#", b"+/+/#"})
    T = [b"/".join(rng.choice(words) for _ in range(6)) for _ in range(2000)]
    eng = Engine(device=0)
    for f in F:
        eng.insert(f)
    exp, _ = oracle_rows(F, T)
    assert sum(len(r) for r in exp) > 40 * len(T)   # above the initial id capacity (32 per topic)
    for _ in range(2):
        assert_same(T, engine_rows(eng, T), exp)
    st = eng.stats()
    assert st["filters"] == len(F)


def test_match_batch_pipelined_equals_one_batch():
    """tm_match_batch above one chunk (2.5M publishes: chunks of 2^20 on two
    streams, each chunk's ids copied to their place in the merged CSR while the
    next one walks) returns exactly the CSR of the same publishes run as one
    batch (prepare / launch / wait / result), whose parity the other tests hold."""
    F = gen.gen_filters(gen.C2)
    T = gen.gen_topics(gen.C2, F, 2501, 2_500_000)
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.sync()
    b = eng.prepare(T)
    b.launch().wait()
    exp_offs, exp_ids = b.result()
    b.free()
    for _ in range(2):   # the second call reuses the pipeline's buffers
        offs, ids = eng.match_batch(T)
        assert np.array_equal(offs, exp_offs)
        assert np.array_equal(ids, exp_ids)


def test_match_batch_pipelined_grows_its_result_buffer():
    """The pipelined tm_match_batch sizes the merged ids from the first chunk's
    rate; a first chunk of publishes that match (almost) nothing, then dense ones,
    makes it grow the buffer mid-batch (the earlier chunks' copies kept).
    Equal to the one-batch result, empty rows and all."""
    F = gen.gen_filters(gen.C2)
    T = gen.gen_topics(gen.C2, F, 2701, 1_200_000)
    none = gen.Strings.from_list([b"zz/%d/unknown" % i for i in range(1_100_000)])
    A = gen.Strings.concat([none, T])
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.sync()
    b = eng.prepare(A)
    b.launch().wait()
    exp_offs, exp_ids = b.result()
    b.free()
    # the first chunk's rate is far below the rest's (root wildcards still match it)
    assert exp_offs[1 << 20] * 4 < exp_offs[-1] - exp_offs[1_100_000]
    offs, ids = eng.match_batch(A)
    assert np.array_equal(offs, exp_offs)
    assert np.array_equal(ids, exp_ids)


def _widen(ids8, ib):
    raw = np.asarray(ids8, np.uint8).reshape(-1, ib).astype(np.uint32)
    out = np.zeros(len(raw), np.uint32)
    for b in range(ib):
        out |= raw[:, b] << np.uint32(8 * b)
    return out


def test_match_batch_packed_equals_u32_ids():
    """tm_match_batch_packed: the ids of tm_match_batch, 3 bytes each (little
    endian) while the trie holds < 2^24 nodes, packed on the device before the
    copy.  Same row offsets and, widened, the same ids: for a one-chunk batch,
    a pipelined 2.5M-publish batch, one whose buffer grows mid-batch and an
    empty one; tm_filters_copy_packed names the same filters as tm_filters_copy."""
    F = gen.gen_filters(gen.C2)
    T = gen.gen_topics(gen.C2, F, 2501, 2_500_000)
    none = gen.Strings.from_list([b"zz/%d/unknown" % i for i in range(1_100_000)])
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.sync()
    for batch in (T.slice(0, 70_000), T, gen.Strings.concat([none, T.slice(0, 1_200_000)]),
                  gen.Strings.from_list([])):
        offs, ids = eng.match_batch(batch)
        offs, ids = offs.copy(), ids.copy()
        po, pids, ib = eng.match_batch_packed(batch)
        assert ib == 3
        assert np.array_equal(po, offs)
        assert len(pids) == 3 * len(ids)
        assert np.array_equal(_widen(pids, ib), ids)
    b = eng.prepare(T.slice(0, 300_000))   # the batch-owned form (the NIF's match_batch)
    b.launch().wait()
    offs, ids = b.result()
    offs, ids = offs.copy(), ids.copy()
    po, pids, ib = b.result_packed()
    b.free()
    assert ib == 3 and np.array_equal(po, offs) and np.array_equal(_widen(pids, ib), ids)
    offs, ids = eng.match_batch(T.slice(0, 5000))
    ids = ids.copy()
    _, pids, ib = eng.match_batch_packed(T.slice(0, 5000))
    assert eng.filters_copy_packed(pids, ib) == eng.filters_copy(ids)
    # a removed filter drops out of both copies alike
    gone = eng.filters_copy(ids[:1])[0][1]
    eng.delete(gone)
    eng.sync()
    assert eng.filters_copy_packed(pids, ib) == eng.filters_copy(ids)
