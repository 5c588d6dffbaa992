"""tm_match_coalesced: many threads calling emqx_trie:match/1 one topic at a
time (the NIF's dirty schedulers) are served by shared device batches, each
caller getting exactly tm_trie_match's row (checked against the oracle)."""

import threading
from dataclasses import replace

import numpy as np
import pytest

from emqx_amd import _native as N
from emqx_amd import gen
from emqx_amd.engine import Engine
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_concurrent_callers_share_batches_and_match_oracle():
    p = replace(gen.C1, n_filters=2000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 31, 3200).tolist()
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.coalesce_config(max_batch=64, linger_us=200)
    got = [None] * len(T)
    errors = []

    def worker(k):
        try:
            for i in range(k, len(T), 16):
                got[i] = eng.match_coalesced(T[i])
        except Exception as e:  # surfaced below
            errors.append(e)
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors and all(not t.is_alive() for t in ths)
    batches, requests = eng.coalesce_config()
    assert requests == len(T) and batches < requests      # callers did share batches
    trie = O.Trie()
    for f in F:
        trie.insert(f)
    for i in range(0, len(T), 7):
        assert [eng.filter_bytes(x) for x in got[i]] == sorted(trie.match(T[i])), T[i]
    for i in range(len(T)):
        assert got[i] == eng.match_ids(T[i])


def test_bad_topic_fails_alone():
    eng = Engine(device=0)
    eng.insert(b"a/#")
    with pytest.raises(N.TmError):
        eng.match_coalesced(b"x" * (N.TM_MAX_TOPIC_LEN + 1))
    assert [eng.filter_bytes(x) for x in eng.match_coalesced(b"a/b")] == [b"a/#"]


# ---------------------------------------------------------------- async pipeline
from emqx_amd import load as LD  # noqa: E402


def _c2_engine(n_filters=200_000):
    p = replace(gen.C2, n_filters=n_filters)
    F = gen.gen_filters(p)
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.sync()
    return p, F, eng


@pytest.mark.parametrize("mode,threads,window", [(LD.SYNC, 64, 1), (LD.ASYNC, 8, 512), (LD.ASYNC, 1, 1)])
def test_load_generator_rows_equal_batch_rows(mode, threads, window):
    """Every per-publish call (blocking or async) gets exactly the row the
    whole-batch path gives (row length + FNV hash of the sorted ids)."""
    p, F, eng = _c2_engine()
    n = 20_000 if window > 1 or threads > 1 else 2_000
    T = gen.gen_topics(p, F, 41, n)
    offs, ids = eng.match_batch(T)
    exp_c = np.diff(offs.astype(np.int64))
    exp_h = LD.row_hashes(offs, ids)
    st, counts, hashes = LD.run(eng, T, mode, threads, window)
    assert st["errors"] == 0 and st["calls"] == n
    assert np.array_equal(counts.astype(np.int64), exp_c)
    assert np.array_equal(hashes, exp_h)
    ast = eng.async_stats()
    assert ast["requests"] == n and ast["batches"] <= n
    if mode == LD.ASYNC and window > 1:
        assert ast["max_batch"] > 64          # outstanding calls were coalesced


def _all_filters_of(words):
    """Every filter matching the topic words: each level literal or '+', and
    every prefix closed by '#'."""
    import itertools
    out = []
    for k in range(len(words) + 1):
        for choice in itertools.product((0, 1), repeat=k):
            lv = [w if c == 0 else b"+" for w, c in zip(words, choice)]
            out.append(b"/".join(lv + [b"#"]))
            if k == len(words):
                out.append(b"/".join(lv))
    return out


def test_async_rows_past_the_readback_hint():
    """600 calls with 95 matches each: more staging entries than the up-front
    read-back (48 per call), fewer than the staging area (65536)."""
    eng = Engine(device=0)
    ws = [b"p", b"q", b"r", b"s", b"t"]
    F = _all_filters_of(ws)
    eng.insert_many(F)
    T = [b"/".join(ws)] * 600
    eng.coalesce_config(max_batch=600, linger_us=200_000)      # one batch of all 600
    offs, ids = eng.match_batch(T)
    assert int(offs[1]) == len(F) == 95
    st, counts, hashes = LD.run(eng, T, LD.ASYNC, 1, 600)
    assert st["errors"] == 0 and set(counts.tolist()) == {len(F)}
    assert np.array_equal(hashes, LD.row_hashes(offs, ids))


def test_async_staging_miss_recovers_through_the_csr_path():
    """Rows longer than the fast path's K (generic kernel) and a batch whose
    staging area overflows: the capacity miss re-runs the batch the CSR way."""
    eng = Engine(device=0)
    ws = [b"a", b"b", b"c", b"d", b"e", b"f", b"g", b"h"]
    F = _all_filters_of(ws)
    eng.insert_many(F)
    T = [b"/".join(ws)] * 200 + [b"a/b/x", b"zz"]
    eng.coalesce_config(max_batch=len(T), linger_us=200_000)
    offs, ids = eng.match_batch(T)
    assert int(offs[1]) == len(F) and int(offs[-1]) > 65536
    st, counts, hashes = LD.run(eng, T, LD.ASYNC, 1, len(T))
    assert st["errors"] == 0
    assert np.array_equal(counts.astype(np.int64), np.diff(offs.astype(np.int64)))
    assert np.array_equal(hashes, LD.row_hashes(offs, ids))
    assert eng.async_stats()["recoveries"] >= 1


def test_async_read_your_writes_and_errors_per_batch():
    eng = Engine(device=0)
    done = threading.Event()
    out = {}

    def cb(rc, ids):
        out["rc"], out["ids"] = rc, ids
        done.set()
    eng.insert(b"x/+")
    eng.match_async(b"x/y", cb)
    assert done.wait(30) and out["rc"] == 0 and [eng.filter_bytes(i) for i in out["ids"]] == [b"x/+"]
    eng.insert(b"x/#")                                          # visible to the next call
    done.clear()
    eng.match_async(b"x/y", cb)
    assert done.wait(30) and sorted(eng.filter_bytes(i) for i in out["ids"]) == [b"x/#", b"x/+"]
    eng.delete(b"x/+")
    done.clear()
    eng.match_async(b"x/y", cb)
    assert done.wait(30) and [eng.filter_bytes(i) for i in out["ids"]] == [b"x/#"]


def test_async_overflow_is_delivered_to_the_batch_and_engine_recovers():
    import os
    os.environ["TM_RESULT_LIMIT"] = "500"
    try:
        eng = Engine(device=0)
    finally:
        del os.environ["TM_RESULT_LIMIT"]
    eng.insert_many([b"#", b"+/#", b"a/#", b"a/+"])
    T = [b"a/%d" % i for i in range(400)]                       # 1600 matches in one batch > 500
    eng.coalesce_config(max_batch=400, linger_us=200_000)
    st, counts, _ = LD.run(eng, T, LD.ASYNC, 1, 400, hashes=False)
    assert st["errors"] > 0 and all(c in (4, 0xFFFFFFFF) for c in counts.tolist())
    eng.coalesce_config(max_batch=1, linger_us=0)
    st, counts, _ = LD.run(eng, T[:50], LD.ASYNC, 1, 1, hashes=False)   # one call per batch: fits
    assert st["errors"] == 0 and set(counts.tolist()) == {4}


def test_mixed_batch_and_async_callers_under_churn():
    """match_batch callers, async callers and trie writers on one engine at
    once: async rows equal a batch match on the same final trie for topics
    whose filters did not change, and nothing fails or hangs."""
    p, F, eng = _c2_engine(50_000)
    T = gen.gen_topics(p, F, 43, 30_000)
    stop = threading.Event()
    errors = []

    def batcher():
        try:
            while not stop.is_set():
                o, _ = eng.match_batch(T.slice(0, 4096))
                assert int(o[-1]) >= 0
        except Exception as e:
            errors.append(e)

    def writer():
        try:
            k = 0
            while not stop.is_set():
                eng.insert(b"zz/churn/%d/#" % k)           # no C2 topic starts with zz
                eng.delete(b"zz/churn/%d/#" % (k - 5))
                k += 1
        except Exception as e:
            errors.append(e)
    ths = [threading.Thread(target=batcher), threading.Thread(target=writer)]
    for t in ths:
        t.start()
    try:
        st, counts, hashes = LD.run(eng, T, LD.ASYNC, 4, 256)
    finally:
        stop.set()
        for t in ths:
            t.join(60)
    assert not errors and st["errors"] == 0
    offs, ids = eng.match_batch(T)
    assert np.array_equal(counts.astype(np.int64), np.diff(offs.astype(np.int64)))
    assert np.array_equal(hashes, LD.row_hashes(offs, ids))
