"""TM_BATCH_DEDUP on the device (tm_dedup_*): identical publishes (equal
bytes) of a batch are tokenised and walked once -- the rows are the batch's
distinct topics in first-occurrence order, as in the host's dedup.  Every
publish's result, read through row_of or through its expanded (count,
start) in HBM, must equal the oracle's row for its own bytes
(src/emqx_trie.erl restated) -- needs an MI355X."""

import numpy as np
import pytest
from test_gpu_parity import assert_same, oracle_rows

from emqx_amd import gen
from emqx_amd.engine import Engine, _d2h

pytestmark = pytest.mark.gpu

FILTERS = [b"a/+", b"a/#", b"+/b", b"#", b"$SYS/#", b"+/+/c", b"a//b", b"a/+/+/+/+/+/+/+/+/+/+/+/#",
           b"x/y", b"%y/+", b"", b"/", b"+", b"a/b/c/d/e/f/g/h/i/j/k/l/m"]


def _check(eng, b, T):
    row_of, n_rows = b.row_map()
    offs, ids = b.result()
    st = b.stats()
    assert len(offs) == n_rows + 1 and st["publishes"] == len(T) and st["topics"] == n_rows
    # rows in first-occurrence order
    seen = {}
    for i, r in enumerate(row_of.tolist()):
        seen.setdefault(r, i)
    assert sorted(seen) == list(range(n_rows))
    assert all(seen[r] < seen[r + 1] for r in range(n_rows - 1))
    names = {}

    def fb(x):
        x = int(x)
        if x not in names:
            names[x] = eng.filter_bytes(x)
        return names[x]
    exp, _ = oracle_rows(sorted(set(FILTERS) | set(extra_filters)), T)
    got = [[fb(x) for x in ids[offs[r]:offs[r + 1]]] for r in row_of.tolist()]
    assert_same(T, got, exp)
    # every publish's expanded row in HBM: the same ids; delivered = their sum
    cnt_p, start_p, ids_p, delivered = b.publish_rows_device()
    pc = np.zeros(len(T), np.uint32)
    ps = np.zeros(len(T), np.uint64)
    _d2h(pc, cnt_p)
    _d2h(ps, start_p)
    cnt_r, start_r, stg = b.rows(n_rows)
    assert np.array_equal(pc, cnt_r[row_of]) and np.array_equal(ps, start_r[row_of])
    assert delivered == st["delivered"] == int(pc.sum()) == sum(len(e) for e in exp)
    return row_of, n_rows


extra_filters = []


def test_device_dedup_edge_topics_match_the_oracle_per_publish():
    eng = Engine(device=0)
    for f in FILTERS:
        eng.insert(f)
    base = [b"a/b", b"a/b", b"$x/a", b"%x/a", b"$x/a", b"", b"", b"/", b"a//b", b"a//b", b"+x/y", b"+x/y",
            b"a/zz1", b"a/zz2", b"x/y", b"x/y/", b"a/b/c/d/e/f/g/h/i/j/k/l/m", b"a/b/c/d/e/f/g/h/i/j/k/l/m",
            b"$SYS/x", b"$SYS/x", b"a/1/2/3/4/5/6/7/8/9/10/11/12", b"q",
            # long topics (over the 64 bytes the dedup keeps in registers): equal
            # heads, different tails at bytes 65, 130 and 4,000
            b"L/" + b"x" * 62 + b"/1", b"L/" + b"x" * 62 + b"/2", b"L/" + b"y" * 126 + b"/1",
            b"L/" + b"y" * 126 + b"/2", b"L/" + b"z" * 3996 + b"/1", b"L/" + b"z" * 3996 + b"/2"]
    T = [base[(i * 11) % len(base)] for i in range(3000)]   # (11: coprime with len(base), every topic occurs)
    b = eng.prepare(T, dedup=True)
    b.launch().wait()
    row_of, n_rows = _check(eng, b, T)
    # equal bytes share a row, different bytes never do (even when their
    # tokens are equal: "a/zz1" / "a/zz2", unknown words)
    assert row_of[T.index(b"a/zz1")] != row_of[T.index(b"a/zz2")]
    assert n_rows == len(set(base))
    for i in range(len(T)):
        assert row_of[i] == row_of[T.index(T[i])]
    assert b.stats()["slow_topics"] > 0            # deep topics: the generic path over compacted rows
    # a replay walks the same rows; a fresh pass (retokenize) deduplicates again
    b.launch().wait()
    _check(eng, b, T)
    b.retokenize().launch().wait()
    assert b.stats()["ms_dedup"] > 0
    _check(eng, b, T)
    # a new filter with a new word: the rows are tokenised again (not deduplicated again)
    extra_filters.append(b"a/zz1")
    eng.insert(b"a/zz1")
    b.launch().wait()
    assert b.stats()["ms_tokenize"] > 0 and b.stats()["ms_dedup"] == 0
    _check(eng, b, T)
    extra_filters.clear()
    b.free()


def test_device_dedup_hash_collisions_stay_exact():
    """TM_DEDUP_WEAK_HASH: the dedup's hash is the topic's length, so every
    two topics of one length collide -- in the workgroup's election and in the
    global table.  The claim compares bytes before joining a slot (a follower
    whose bytes differ from its leader's runs in the next election, a claim
    probes past an occupant with other bytes), so rows never mix two topics
    and collisions cost no extra rows: one row per distinct topic, in
    first-occurrence order, and every publish's result equals the oracle's."""
    import os
    os.environ["TM_DEDUP_WEAK_HASH"] = "1"
    try:
        eng = Engine(device=0)
    finally:
        del os.environ["TM_DEDUP_WEAK_HASH"]
    for f in FILTERS:
        eng.insert(f)
    base = [b"a/b", b"a/c", b"x/y", b"a/b", b"q/r", b"a/c", b"$x/a", b"%x/a", b"a//b", b"a/zz1", b"a/zz2", b"a/zz1"]
    T = [base[(i * 5) % len(base)] for i in range(2000)]
    b = eng.prepare(T, dedup=True)
    b.launch().wait()
    row_of, n_rows = _check(eng, b, T)
    # every row's publishes have equal bytes
    first = {}
    for i, r in enumerate(row_of.tolist()):
        assert first.setdefault(r, T[i]) == T[i]
    assert n_rows == len(set(base))           # collisions resolved by the bytes, not by extra rows
    b.free()


def test_device_dedup_large_skewed_batch_and_empty_batch():
    p = gen.SkewParams(seed=3, n_hot=300, k_per_hot=20)
    from emqx_amd.skew import workload
    allf, derived, hot, pubs = workload(p, 5000, 400_000, seed=3, background_pool=20_000)
    eng = Engine(device=0)
    eng.insert_many(allf)
    b = eng.prepare(pubs, dedup=True)
    b.launch().wait()
    row_of, n_rows = b.row_map()
    T = pubs.tolist()
    assert n_rows == len(set(T))
    first = {}
    for i, r in enumerate(row_of.tolist()):
        assert first.setdefault(r, T[i]) == T[i]
    # every 13th publish, through its row, equals the oracle's row for its own bytes
    pick = list(range(0, len(T), 13))
    Ts = [T[i] for i in pick]
    exp, _ = oracle_rows(allf.tolist(), Ts, nthreads=16)
    so, si = b.sample(row_of[pick])
    names = {}
    got = [[names.setdefault(int(x), eng.filter_bytes(int(x))) for x in si[so[j]:so[j + 1]]] for j in range(len(pick))]
    assert_same(Ts, got, exp)
    st = b.stats()
    offs, _ = b.result()
    assert st["delivered"] == int(np.diff(offs.astype(np.int64))[row_of].sum())
    b.free()
    e0 = eng.prepare([], dedup=True)
    e0.launch().wait()
    assert e0.row_map()[1] == 0 and e0.stats()["delivered"] == 0
    e0.free()
