"""Device route resolution (tm_batch_routes): aggre(match_routes(T)) per publish,
checked against the oracle's match sets and a host restatement of the route bag."""

import random
from dataclasses import replace

import numpy as np
import pytest
from conftest import load_golden

from emqx_amd import emqx_router as R
from emqx_amd import gen
from emqx_amd.engine import Engine
from oracle import pyoracle as P

pytestmark = pytest.mark.gpu


def test_kat_match_routes_aggre():
    kat = load_golden("kat_router.json")
    case = [c for c in kat["cases"] if c["name"] == "t_match_routes"][0]
    R.clear_tables()
    for t in case["add"]:
        R.add_route(t.encode())
    topic, exp = case["match"]
    assert R.aggre_batch([topic.encode()]) == [[(e.encode(), R.NODE) for e in exp]]
    for t in case["delete"]:
        R.delete_route(t.encode())
    assert R.aggre_batch([topic.encode()]) == [[]]


def test_routes_random_with_groups_and_churn():
    rng = random.Random(3)
    p = replace(gen.C1, n_filters=3000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 9, 6000).tolist()
    nodes = ["n%d" % i for i in range(4)]
    groups = ["g%d" % i for i in range(3)]
    eng = Engine(device=0)
    bag = {}                                  # topic -> {aggregated dest: count}, first-added order

    def agg(d):
        return d[0] if isinstance(d, tuple) else d
    ids = {}

    def did(a):
        return ids.setdefault(a, len(ids))
    for rnd in range(3):
        for _ in range(4000):
            f = rng.choice(F)
            d = rng.choice(nodes) if rng.random() < 0.6 else (rng.choice(groups), rng.choice(nodes))
            a = agg(d)
            if f in bag and a in bag[f] and rng.random() < 0.4:
                assert eng.route_delete(f, did(a))
                bag[f][a] -= 1
                if bag[f][a] == 0:
                    del bag[f][a]
                if not bag[f]:
                    del bag[f]
            else:
                eng.route_add(f, did(a))
                bag.setdefault(f, {})
                bag[f][a] = bag[f].get(a, 0) + 1
        offs, fids, dests = eng.match_routes_batch(T)
        live = sorted(bag)
        orc = P.Oracle()
        for f in live:
            orc.register(f)
            orc.insert(f)
        buf, o = P.pack(T)
        counts, idx, _ = orc.match_batch(buf, o)
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        inv = {v: k for k, v in ids.items()}
        for t in range(len(T)):
            exp = [(live[int(j)], a) for j in idx[cut[t]:cut[t + 1]] for a in bag[live[int(j)]]]
            got = [(eng.filter_bytes(int(fids[k])), inv[int(dests[k])]) for k in range(offs[t], offs[t + 1])]
            assert got == exp, (rnd, T[t])


def test_routes_skewed_rows_entry_parallel():
    """C5-style skew: hot topics matched by hundreds of filters (rows past the
    fast path's K, generic kernel) next to cold ones, every filter routed to
    1-3 destinations: the entry-parallel route kernels (per-entry counts, a
    multi-block scan over the entries, per-entry fill) against the oracle."""
    hot, derived = gen.gen_skew(gen.SkewParams(n_hot=40, k_per_hot=400, seed=13))
    F = sorted(set(derived.tolist()))
    T = hot.tolist() + gen.gen_topics(replace(gen.C1, n_filters=2000), gen.Strings.from_list(F), 4, 2000).tolist()
    eng = Engine(device=0)
    ndest = {}
    for i, f in enumerate(F):
        ndest[f] = 1 + i % 3
        for d in range(ndest[f]):
            eng.route_add(f, d)
    offs, fids, dests = eng.match_routes_batch(T)
    orc = P.Oracle()
    for f in F:
        orc.register(f)
        orc.insert(f)
    buf, o = P.pack(T)
    counts, idx, _ = orc.match_batch(buf, o)
    assert int(counts[:len(hot)].max()) > 128          # rows past K took the generic path
    assert int(counts.sum()) > 4 * 4096                # the entry scan spans several blocks
    cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    for t in range(len(T)):
        exp = [(F[int(j)], d) for j in idx[cut[t]:cut[t + 1]] for d in range(ndest[F[int(j)]])]
        got = [(eng.filter_bytes(int(fids[k])), int(dests[k])) for k in range(offs[t], offs[t + 1])]
        assert got == exp, T[t]
