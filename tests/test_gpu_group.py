"""Replicated multi-device group (tm_group_*, BASELINE config C3) -- needs an MI355X.

A single GPU box runs the group with several replicas on device 0: every
replica is a full engine with its own stream and HBM trie, so the split /
concurrent launch / concatenation logic is exactly the multi-GPU one."""

from dataclasses import replace

import numpy as np
import pytest
from test_gpu_parity import assert_same, oracle_rows

from emqx_amd import _native as N
from emqx_amd import gen
from emqx_amd.engine import Engine, Group

pytestmark = pytest.mark.gpu


def group_rows(grp, offs, ids):
    cache = {}

    def fb(i):
        i = int(i)
        if i not in cache:
            cache[i] = grp.filter_bytes(i)
        return cache[i]
    return [[fb(x) for x in ids[offs[i]:offs[i + 1]]] for i in range(len(offs) - 1)]


def test_two_replicas_on_one_device_split_a_c2_sample():
    F = gen.gen_filters(gen.C2)
    T = gen.gen_topics(gen.C2, F, 2102, 200_000).tolist()
    fl = F.tolist()
    grp = Group([0, 0])
    assert len(grp) == 2
    assert grp.insert_many(F) == len(fl)
    grp.sync()
    offs, ids = grp.match_batch(T)
    assert int(offs[-1]) == len(ids)
    # both replicas give every filter the same id
    for i in np.unique(ids)[:2000]:
        assert grp.filter_bytes(int(i), 0) == grp.filter_bytes(int(i), 1)
    exp, _ = oracle_rows(fl, T, nthreads=16)
    assert_same(T, group_rows(grp, offs, ids), exp)
    # the same CSR as one engine over the whole batch
    eng = Engine(device=0)
    eng.insert_many(F)
    o1, i1 = eng.match_batch(T)
    assert np.array_equal(o1, offs) and np.array_equal(i1, ids)


@pytest.mark.parametrize("k,n", [(3, 10_007), (2, 1), (3, 2), (2, 0)])
def test_split_form_ragged_slices(k, n):
    p = replace(gen.C1, n_filters=3000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 9, max(n, 1)).tolist()[:n]
    grp = Group([0] * k)
    for f in F:
        grp.insert(f)
    b = grp.prepare(T)
    b.launch().wait()
    offs, ids = b.result()
    st = b.stats()
    assert len(offs) == n + 1 and st["topics"] == n and st["matches"] == len(ids)
    exp, _ = oracle_rows(F, T) if n else ([], None)
    assert_same(T, group_rows(grp, offs, ids), exp)
    # re-launch of the same prepared batch gives the same CSR
    b.launch().wait()
    o2, i2 = b.result()
    assert np.array_equal(o2, offs) and np.array_equal(i2, ids)
    b.free()


def test_group_mutations_reach_every_replica():
    p = replace(gen.C2, n_filters=20_000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 31, 6000).tolist()
    grp = Group([0, 0])
    live = set(F[:10_000])
    grp.insert_many(sorted(live))
    rng = np.random.default_rng(3)
    for rnd in range(3):
        for j in rng.choice(len(F), 1500, replace=False):   # subscribe / unsubscribe deltas
            f = F[int(j)]
            if f in live:
                live.discard(f)
                grp.delete(f)
            else:
                live.add(f)
                grp.insert(f)
        offs, ids = grp.match_batch(T)
        exp, _ = oracle_rows(sorted(live), T)
        assert_same(T, group_rows(grp, offs, ids), exp)


def test_group_route_feed():
    grp = Group([0, 0])
    W, D = N.TM_ROUTE_WRITE, N.TM_ROUTE_DELETE
    assert grp.route_apply([(W, b"a/+", 1), (W, b"a/b", 2), (W, b"a/+", 3), (D, b"x/y", 1)]) == 3
    offs, ids = grp.match_batch([b"a/b", b"a/c"])
    assert group_rows(grp, offs, ids) == [[b"a/+", b"a/b"], [b"a/+"]]
    assert grp.route_apply([(D, b"a/+", 1), (D, b"a/+", 3), (D, b"a/b", 2)]) == 3
    offs, ids = grp.match_batch([b"a/b", b"a/c"])
    assert list(offs) == [0, 0, 0]
