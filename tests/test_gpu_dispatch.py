"""Device fan-out (tm_batch_dispatch): emqx_broker's publish -> route ->
dispatch over a whole batch, checked against the oracle's Broker restatement
(oracle/oracle.py, pinned by tests/golden/kat_broker.json) on the same inputs."""

import random
from dataclasses import replace

import numpy as np
import pytest
from conftest import load_golden
from test_broker import run_kat_ops

from emqx_amd import emqx_broker as B
from emqx_amd import emqx_router as R
from emqx_amd import gen
from emqx_amd.engine import Engine
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def assert_rows_mode_equal(b, offs, out):
    """TM_DISPATCH_ROWS (the fan-out over the walk's rows where they lie, no
    dense CSR first) gives every publish the same deliveries, in the same
    order, as the CSR form."""
    first, cnt, subs = b.dispatch_rows()
    assert len(subs) == int(offs[-1])
    assert np.array_equal(cnt.astype(np.uint64), np.diff(offs))
    for i in range(len(cnt)):
        assert np.array_equal(subs[int(first[i]):int(first[i]) + int(cnt[i])], out[offs[i]:offs[i + 1]]), i


def test_kat_broker_on_device():
    kat = load_golden("kat_broker.json")
    for case in kat["cases"]:
        B.clear_tables()
        run_kat_ops(case["ops"], B.subscribe, B.unsubscribe, B.subscriber_down,
                    lambda t: B.publish_batch([t])[0], B.subscribers, B.topics)


def test_dispatch_random_churn_vs_oracle():
    rng = random.Random(5)
    p = replace(gen.C1, n_filters=2500)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 17, 5000).tolist()
    B.clear_tables()
    orc = O.Broker()
    for rnd in range(3):
        for _ in range(6000):
            f, pid = rng.choice(F), rng.randrange(300)
            r = rng.random()
            if r < 0.3:
                B.unsubscribe(f, pid)
                orc.unsubscribe(f, pid)
            elif r < 0.31:
                assert B.subscriber_down(pid) == orc.subscriber_down(pid)
            else:
                B.subscribe(f, pid)
                orc.subscribe(f, pid)
        got = B.publish_batch(T)
        for t, row in zip(T, got):
            assert row == orc.publish(t), (rnd, t)
        assert sorted(B.topics()) == sorted(orc.routes)


@pytest.mark.parametrize("big", [None, "100000", "0"])
def test_dispatch_skewed_fanout_and_modes(big, monkeypatch):
    """One '#' filter with 150k subscribers next to thousands of 1-subscriber
    filters: the fill kernel's workgroups straddle both kinds of runs.  `big`
    lowers the per-scan-block delivery count above which match offsets are
    kept as u64 instead of u32 (TM_FAN_BIG, normally 2^32 - 1): some blocks,
    and then every block, take the u64 path."""
    if big is not None:
        monkeypatch.setenv("TM_FAN_BIG", big)
    p = replace(gen.C1, n_filters=4000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 23, 3000).tolist()
    eng = Engine(device=0)
    subs = {}
    for i, f in enumerate(F):
        eng.subscribe(f, 1_000_000 + i)
        subs[f] = [1_000_000 + i]
    hot = list(range(150_000))
    for s in hot:
        eng.subscribe(b"#", s)
    subs[b"#"] = subs.get(b"#", []) + hot
    b = eng.prepare(T)
    b.launch()
    b.wait()
    roff, ids = b.result()
    offs, moff, out = b.dispatch(match_offsets=True)
    c_offs, _, none = b.dispatch(counts_only=True)
    assert none is None and np.array_equal(c_offs, offs)
    total, fill_ms, d_row, d_moff, d_subs = b.dispatch_device()
    assert total == int(offs[-1]) and fill_ms > 0 and d_subs and d_moff is None
    total, _, _, d_moff, _ = b.dispatch_device(match_offsets=True)
    assert total == int(offs[-1]) and d_moff
    offs2, moff2, out2 = b.dispatch(match_offsets=True)        # re-dispatch: offsets made global once
    assert np.array_equal(moff2, moff) and np.array_equal(offs2, offs) and np.array_equal(out2, out)
    assert_rows_mode_equal(b, offs, out)
    names = [eng.filter_bytes(int(i)) for i in ids]
    for i, t in enumerate(T):
        exp = []
        for j in range(int(roff[i]), int(roff[i + 1])):
            assert int(moff[j]) == offs[i] + len(exp)
            exp.extend(subs.get(names[j], []))
        got = out[offs[i]:offs[i + 1]]
        assert len(got) == len(exp) and np.array_equal(got, np.asarray(exp, np.uint32)), t
        # every publish matches '#' unless it is a '$' topic
        assert (len(got) >= len(hot)) == (not t.startswith(b"$"))
    b.free()


def test_dispatch_dedup_rows_and_unsubscribe_all():
    eng = Engine(device=0)
    for s in range(5):
        eng.subscribe(b"a/+", s)
        eng.subscribe(b"a/b", 10 + s)
    T = [b"a/b", b"a/c", b"a/b", b"x", b"a/b"]
    b = eng.prepare(T, dedup=True)
    b.launch()
    b.wait()
    rows, _ = b.row_map()
    offs, _, out = b.dispatch()
    per = {T[i]: out[offs[rows[i]]:offs[rows[i] + 1]].tolist() for i in range(len(T))}
    assert per[b"a/b"] == [0, 1, 2, 3, 4, 10, 11, 12, 13, 14]
    assert per[b"a/c"] == [0, 1, 2, 3, 4] and per[b"x"] == []
    for s in range(5):
        assert eng.subscriber_down(s) == 1
        assert eng.unsubscribe(b"a/b", 10 + s)
    assert not eng.unsubscribe(b"a/b", 10)
    assert eng.empty()
    b2 = eng.prepare(T)
    b2.launch()
    b2.wait()
    offs, _, out = b2.dispatch()
    assert int(offs[-1]) == 0


def test_dispatch_sparse_subscribers_take_the_search_path():
    """Most matched filters have no local subscriber: fill tiles then cover far
    more match entries than they can stage in LDS (the per-delivery search
    path).  A '#' subscriber set then makes every tile dense (the staged path)."""
    p = replace(gen.C1, n_filters=4000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 29, 40000).tolist()
    eng = Engine(device=0)
    eng.insert_many(F)
    subs = {}
    rng = np.random.default_rng(8)
    for i, f in enumerate(F):
        if rng.random() < 0.01:
            subs[f] = [7 * i + q for q in range(int(rng.integers(1, 4)))]
            for s in subs[f]:
                eng.subscribe(f, s)

    def check():
        b = eng.prepare(T)
        b.launch()
        b.wait()
        roff, ids = b.result()
        offs, moff, out = b.dispatch(match_offsets=True)
        names = [eng.filter_bytes(int(i)) for i in ids]
        for i in range(len(T)):
            exp = []
            for j in range(int(roff[i]), int(roff[i + 1])):
                assert int(moff[j]) == offs[i] + len(exp)
                exp.extend(subs.get(names[j], []))
            assert np.array_equal(out[offs[i]:offs[i + 1]], np.asarray(exp, np.uint32)), T[i]
        assert_rows_mode_equal(b, offs, out)
        b.free()
        return int(offs[-1]), len(ids)
    nd, nm = check()
    assert nm > 4 * 3072 and nd < nm // 4           # sparse: tiles span > FAN_LDS_ENTRIES entries
    subs[b"#"] = [5_000_000 + s for s in range(64)]
    for s in subs[b"#"]:
        eng.subscribe(b"#", s)
    nd, nm = check()
    assert nd > nm                                   # dense: staged path


def test_dispatch_rows_mode_with_generic_path_rows():
    """Rows mode over staging that also holds the generic path's rows: topics
    deeper than the fast path and rows longer than K (a topic matching every
    literal/'+'/'#' combination of 8 levels: 511 filters)."""
    import itertools
    lit = [b"a", b"b", b"c", b"d", b"e", b"f", b"g", b"h"]
    F = []
    for k in range(len(lit) + 1):
        for pick in itertools.product((0, 1), repeat=k):
            ws = [lit[i] if pick[i] == 0 else b"+" for i in range(k)]
            F.append(b"/".join(ws + ([b"#"] if k < len(lit) else [])))
    F = sorted(set(F))
    eng = Engine(device=0)
    for j, f in enumerate(F):
        for q in range(j % 3):
            eng.subscribe(f, 100 * j + q)
    deep = b"/".join(lit + [b"x"] * 6)
    T = [b"a/b/c/d/e/f/g/h", deep, b"a/b", b"zz", b"a/b/c/d/e/f/g/h/i/j/k/l"] * 300
    b = eng.prepare(T)
    b.launch().wait()
    assert b.stats()["slow_topics"] > 0
    offs, _, out = b.dispatch()
    assert_rows_mode_equal(b, offs, out)
    b.free()
