"""Config C5 on the device: hot-topic skew with rows longer than the fast
path's K (generic path), TM_BATCH_DEDUP batches and churn deltas between
launches; every batch is checked against the oracle on that batch's snapshot."""

import numpy as np
import pytest

from emqx_amd import gen
from emqx_amd.engine import Engine
from emqx_amd.skew import Churn, workload
from oracle import pyoracle as P

pytestmark = pytest.mark.gpu


def test_skew_dedup_churn_parity():
    p = gen.SkewParams(seed=7, n_hot=150, k_per_hot=150)
    allf, derived, hot, pubs = workload(p, 3000, 30_000, seed=7, background_pool=5000)
    background = allf.tolist()[len(derived):]
    eng = Engine(device=0)
    eng.insert_many(allf)
    churn = Churn(hot, derived.tolist(), seed=3)
    b = eng.prepare(pubs, dedup=True)
    T = pubs.tolist()
    for rnd in range(3):
        if rnd:
            dels, adds = churn.step(600)
            Churn.apply(eng, dels, adds)
        b.launch().wait()
        row_of, n_rows = b.row_map()                    # (the device dedup's, after the wait)
        assert n_rows < len(pubs) // 3                  # the skew collapses most publishes
        # one row per distinct topic (bytes), in first-occurrence order
        row_of_bytes = {}
        for i, r in enumerate(row_of.tolist()):
            assert row_of_bytes.setdefault(T[i], r) == r
        assert len(row_of_bytes) == n_rows and sorted(row_of_bytes.values()) == list(range(n_rows))
        offs, ids = b.result()
        assert len(offs) == n_rows + 1
        st = b.stats()
        assert st["slow_topics"] > 0                    # hot rows exceed K = 128
        F = sorted(churn.live_set) + background
        orc = P.Oracle()
        for f in F:
            orc.register(f)
            orc.insert(f)
        U = sorted(row_of_bytes)                        # every distinct publish, by its own bytes
        buf, o = P.pack(U)
        counts, idx, _ = orc.match_batch(buf, o, nthreads=8)
        orc.close()
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        cache = {}
        for j, tp in enumerate(U):
            r = row_of_bytes[tp]
            got = [cache.setdefault(int(x), eng.filter_bytes(int(x))) for x in ids[offs[r]:offs[r + 1]]]
            exp = [F[int(k)] for k in idx[cut[j]:cut[j + 1]]]
            assert got == exp, (rnd, tp[:60])
    assert eng.stats()["uploads_delta"] >= 1


def test_churn_applied_while_the_device_walks():
    """The C5 bench's pipeline: deltas i + 1 are applied on the host while
    batch i runs.  Batch i must equal the oracle on snapshot i (deltas <= i),
    and its ids must still name their filters after deltas i + 1 deleted some
    of them (freed ids are not reused while a result may hold them)."""
    p = gen.SkewParams(seed=9, n_hot=120, k_per_hot=60)
    allf, derived, hot, pubs = workload(p, 2000, 20_000, seed=9, background_pool=4000)
    background = allf.tolist()[len(derived):]
    eng = Engine(device=0)
    eng.insert_many(allf)
    churn = Churn(hot, derived.tolist(), seed=4)
    b = eng.prepare(pubs, dedup=True)
    b.launch().wait()          # sizes the staging area: no capacity re-run inside the pipelined rounds
    row_of, n_rows = b.row_map()
    T = pubs.tolist()
    distinct = {}
    for i, r in enumerate(row_of.tolist()):
        distinct.setdefault(r, T[i])
    Td = [distinct[r] for r in range(n_rows)]
    snapshot = sorted(churn.live_set) + background
    b.launch()
    for rnd in range(3):
        dels, adds = churn.step(800)                      # deltas of the NEXT step
        Churn.apply(eng, gen.Strings.from_list(dels), gen.Strings.from_list(adds))
        b.wait()
        offs, ids = b.result()
        got = [[eng.filter_bytes(int(x)) for x in ids[offs[r]:offs[r + 1]]] for r in range(n_rows)]
        orc = P.Oracle()
        for f in snapshot:
            orc.register(f)
            orc.insert(f)
        buf, o = P.pack(Td)
        counts, idx, _ = orc.match_batch(buf, o, nthreads=8)
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        for r in range(n_rows):
            assert got[r] == [snapshot[int(j)] for j in idx[cut[r]:cut[r + 1]]], (rnd, Td[r][:60])
        snapshot = sorted(churn.live_set) + background
        b.launch()                                         # sees the deltas applied above
    b.wait()
    b.free()


def test_fresh_dedup_batches_replay_through_churn():
    """A fresh deduplicated batch every step (the C5 leg: retokenize().launch()):
    from the third launch on, the launch replays a captured graph (dedup,
    tokeniser, walk, expand).  The trie changes between launches, and every
    launch must equal the oracle on its own snapshot -- the replay must not keep
    stale trie arguments."""
    p = gen.SkewParams(seed=11, n_hot=100, k_per_hot=40)
    allf, derived, hot, pubs = workload(p, 2000, 30_000, seed=11, background_pool=4000)
    background = allf.tolist()[len(derived):]
    eng = Engine(device=0)
    eng.insert_many(allf)
    churn = Churn(hot, derived.tolist(), seed=5)
    b = eng.prepare(pubs, dedup=True)
    T = pubs.tolist()
    for rnd in range(6):
        dels, adds = churn.step(500)
        Churn.apply(eng, gen.Strings.from_list(dels), gen.Strings.from_list(adds))
        snapshot = sorted(churn.live_set) + background
        b.retokenize().launch().wait()
        st = b.stats()
        assert st["publishes"] == len(T) and st["ms_dedup"] > 0.0
        row_of, n_rows = b.row_map()
        distinct = {}
        for i, r in enumerate(row_of.tolist()):
            distinct.setdefault(r, T[i])
        Td = [distinct[r] for r in range(n_rows)]
        offs, ids = b.result()
        got = [[eng.filter_bytes(int(x)) for x in ids[offs[r]:offs[r + 1]]] for r in range(n_rows)]
        orc = P.Oracle()
        for f in snapshot:
            orc.register(f)
            orc.insert(f)
        buf, o = P.pack(Td)
        counts, idx, _ = orc.match_batch(buf, o, nthreads=8)
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        for r in range(n_rows):
            assert got[r] == [snapshot[int(j)] for j in idx[cut[r]:cut[r + 1]]], (rnd, Td[r][:60])
        orc.close()
    assert eng.stats()["graph_launches"] >= 3   # (launches 3..6 replayed the graph captured at launch 2)
    b.free()
