"""Filter-sharded group in ONE process (tm_sharded_*, BASELINE config C4
without torch or a collective) -- needs an MI355X.

A one-GPU box runs the shards on device 0: each shard is an engine with its
own trie, stream and HBM tables, so the owner partition, the per-shard token
batches and the reassembly in publish order are exactly the multi-GPU ones
(only the part copies are same-device).  Expected rows come from the oracle
(src/emqx_trie.erl restated) over the full filter set."""

import random
from dataclasses import replace

import numpy as np
import pytest
from sharded_worker import workload
from test_gpu_parity import assert_same, oracle_rows

from emqx_amd import gen
from emqx_amd.engine import Engine, ShardedGroup
from oracle import pyoracle as P

pytestmark = pytest.mark.gpu
# this module never imports torch: the in-process sharded group is torch-free


def _iot_candidates(p, topics):
    """The IoT filters that can match any of `topics`: those whose second level
    d<X> is a topic's (every IoT filter's and topic's second level is literal,
    so no other filter can match them)."""
    want = np.unique(gen.iot_device_ids(gen.Strings.from_list(topics)))
    cand = []
    for lo in range(0, p.n_filters, 5_000_000):
        fl = gen.gen_iot_filters(p, lo, min(p.n_filters, lo + 5_000_000))
        cand.extend(fl[int(i)] for i in np.flatnonzero(np.isin(gen.iot_device_ids(fl), want)))
    return cand


def rows_of(grp, offs, ids):
    cache = {}

    def fb(g):
        g = int(g)
        if g not in cache:
            cache[g] = grp.filter_bytes(g)
        return cache[g]
    return [[fb(x) for x in ids[offs[i]:offs[i + 1]]] for i in range(len(offs) - 1)]


@pytest.mark.parametrize("G", [1, 2, 3])
def test_shards_on_one_device_with_online_dictionary_deltas(G):
    """The IoT workload plus irregular filters and topics ('$', '' levels,
    deep, root wildcards); the dictionary starts EMPTY and grows only by the
    deltas of insert_many (new words, first-appearance order, every shard)."""
    F, T, _vocab = workload(41)
    grp = ShardedGroup([0] * G)
    assert len(grp) == G
    for lo in range(0, len(F), 700):           # several subscribe batches, each bringing new words
        grp.insert_many(F[lo:lo + 700])
    # the word ids agree on every shard
    tok = [grp.engine(g).tokenize(T) for g in range(G)]
    assert all(np.array_equal(tok[0].words, x.words) for x in tok[1:])
    b = grp.prepare(T)
    b.run()
    st = b.stats()
    assert st["host_waits"] == 1                 # the whole step behind one host wait
    offs, ids = b.result()
    assert sum(st["part_topics"]) == len(T) and st["matches"] == len(ids)
    assert min(st["part_topics"]) > 0            # every shard owned publishes
    exp, _ = oracle_rows(F, T)
    assert_same(T, rows_of(grp, offs, ids), exp)
    # unsubscribe every 7th filter, subscribe filters with words never seen
    # before, and re-run the SAME prepared batch: it is re-tokenised (the
    # dictionary grew) and matches the new snapshot
    gone = F[::7]
    grp.delete_many(gone)
    fresh = [b"device/dnew%d/sensor/s3/#" % k for k in range(50)] + [b"newroot%d/+/x" % k for k in range(20)] + \
            [b"device/d1/newword/#", b"+/dnew3/#"]
    grp.insert_many(fresh)
    T2 = T + [b"device/dnew%d/sensor/s3/m1" % k for k in range(50)] + [b"newroot%d/q/x" % k for k in range(20)] + \
         [b"device/d1/newword/z"]
    b.run()
    o2, i2 = b.result()
    live = sorted(set(F) - set(gone)) + fresh
    exp2, _ = oracle_rows(live, T)
    assert_same(T, rows_of(grp, o2, i2), exp2)
    b.free()
    o3, i3 = grp.match_batch(T2)
    exp3, _ = oracle_rows(live, T2)
    assert_same(T2, rows_of(grp, o3, i3), exp3)
    # empty and one-publish batches
    o4, i4 = grp.match_batch([])
    assert list(o4) == [0] and len(i4) == 0
    o5, i5 = grp.match_batch([T2[-1]])
    assert rows_of(grp, o5, i5) == [exp3[-1]]
    grp.close()


def test_sharded_rows_equal_one_engine(device_pair):
    F, T, vocab = workload(42)
    one = Engine(device=0, frozen_dict=True)
    one.dict_load(vocab)
    one.insert_many(F)
    grp = ShardedGroup(device_pair)
    grp.dict_load(vocab)
    grp.insert_many(F)
    o1, i1 = one.match_batch(T)
    og, ig = grp.match_batch(T)
    assert np.array_equal(o1, og)
    rows1 = [[one.filter_bytes(int(x)) for x in i1[o1[i]:o1[i + 1]]] for i in range(len(T))]
    assert rows_of(grp, og, ig) == rows1
    grp.close()


def test_c4_20m_iot_filters_two_shards_properties_and_oracle_sample():
    """C4 at 20M IoT filters over two shards on one device: CSR properties on
    every row, and 3,000 rows checked against the oracle.  A topic
    device/d<X>/sensor/s<Y>/m<Z> can only be matched by filters whose second
    level is d<X> (every IoT filter's second level is literal), so the oracle
    over the filters with a sampled second level gives those rows exactly."""
    p = replace(gen.C4, n_filters=20_000_000)
    grp = ShardedGroup([0, 0])
    grp.dict_load(gen.gen_iot_vocab(p))
    inserted = 0
    for lo in range(0, p.n_filters, 5_000_000):
        inserted += grp.insert_many(gen.gen_iot_filters(p, lo, lo + 5_000_000))
    assert inserted >= p.n_filters                # replicated filters count once per shard
    n = 2_000_000
    Ts = gen.gen_iot_topics(p, 4242, n)
    b = grp.prepare(Ts)
    b.run()
    st = b.stats()
    assert st["host_waits"] == 1
    offs, ids = b.result()
    lens = np.diff(offs.astype(np.int64))
    # every row: offsets consistent, at most one filter of each IoT kind
    assert offs[0] == 0 and int(offs[-1]) == len(ids) == st["matches"] and (lens >= 0).all() and (lens <= 3).all()
    assert sum(st["part_topics"]) == n and min(st["part_topics"]) > 0
    # global ids: shard = gid % 2 holds them (a row's ids are distinct)
    for i in range(0, n, 997):
        r = ids[offs[i]:offs[i + 1]]
        assert len(set(r.tolist())) == len(r)
    # the oracle over the filters that can match the sampled topics
    T = Ts.tolist()
    sample = list(range(0, n, n // 3000))[:3000]
    ts = [T[i] for i in sample]
    cand = _iot_candidates(p, ts)
    exp, _ = oracle_rows(cand, ts)
    got = [[grp.filter_bytes(int(x)) for x in ids[offs[i]:offs[i + 1]]] for i in sample]
    assert_same(ts, got, exp)
    assert sum(len(r) for r in exp) > 300        # the sample exercises real matches
    b.free()
    grp.close()


def test_link_kinds_and_three_shards(monkeypatch):
    """Every link kind's code on one device, three shards: parts copied
    through pinned host memory (the path taken when two devices cannot reach
    each other's memory, TM_SHARD_LINK=staged), the peer path (peer stores
    and hipMemcpyPeer, TM_SHARD_LINK=peer: here into the same HBM), and the
    runtime's peer probe run for a device paired with itself
    (TM_SHARD_LINK=probe), where peer access is refused: the denied branch
    must fall back to a working link.  Every row equals the oracle's, one host
    wait per step, the result identical to the same-device links'."""
    F, T, vocab = workload(43)
    exp, _ = oracle_rows(F, T)
    res = {}
    for mode in ("same", "staged", "peer", "probe"):
        if mode != "same":
            monkeypatch.setenv("TM_SHARD_LINK", mode)
        grp = ShardedGroup([0, 0, 0])
        monkeypatch.delenv("TM_SHARD_LINK", raising=False)
        links = {grp.link(i, j) for i in range(3) for j in range(3)}
        if mode == "probe":     # refused peer access to itself -> staged (or peer, should the runtime grant it)
            assert len(links) == 1 and links <= {"staged", "peer"}, links
        else:
            assert links == {mode}, links
        grp.dict_load(vocab)
        grp.insert_many(F)
        b = grp.prepare(T)
        for _ in range(2):                      # a second step over the same plan
            b.run()
            assert b.stats()["host_waits"] == 1
        offs, ids = b.result()
        got = rows_of(grp, offs, ids)
        assert_same(T, got, exp)
        res[mode] = got
        b.free()
        grp.close()
    assert res["same"] == res["staged"] == res["peer"] == res["probe"]


def test_c4_100m_iot_filters_one_shard_properties_and_oracle_sample():
    """BASELINE config C4's full filter count (100M IoT filters) on one shard:
    CSR properties on every row and 3,000 rows against the oracle over the
    filters that can match them."""
    p = gen.C4
    grp = ShardedGroup([0])
    grp.dict_load(gen.gen_iot_vocab(p))
    inserted = 0
    for lo in range(0, p.n_filters, 5_000_000):
        inserted += grp.insert_many(gen.gen_iot_filters(p, lo, lo + 5_000_000))
    assert inserted == p.n_filters
    n = 2_000_000
    Ts = gen.gen_iot_topics(p, 4343, n)
    b = grp.prepare(Ts)
    b.run()
    st = b.stats()
    assert st["host_waits"] == 1
    offs, ids = b.result()
    lens = np.diff(offs.astype(np.int64))
    assert offs[0] == 0 and int(offs[-1]) == len(ids) == st["matches"] and (lens >= 0).all() and (lens <= 3).all()
    assert st["matches"] > n // 2                 # 100M filters over 10M ids: most topics match something
    T = Ts.tolist()
    sample = list(range(0, n, n // 3000))[:3000]
    ts = [T[i] for i in sample]
    exp, _ = oracle_rows(_iot_candidates(p, ts), ts)
    got = [[grp.filter_bytes(int(x)) for x in ids[offs[i]:offs[i + 1]]] for i in sample]
    assert_same(ts, got, exp)
    assert sum(len(r) for r in exp) > 1000
    b.free()
    grp.close()
