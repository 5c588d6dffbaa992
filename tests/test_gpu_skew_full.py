"""BASELINE config C5 at full scale on the device: 10k hot topics x K = 1000
derived filters (10M) + 100k background filters, a 10M-publish batch with
TM_BATCH_DEDUP, 10,000 subscribe/unsubscribe deltas between two launches.
Every row of both batches is checked for CSR consistency and duplicate-free
ids; 3,000 rows per batch (300 hot, 2,700 background) are checked exactly
against the oracle on that batch's snapshot (oracle/c5_checker.py: inverted
index for the derived filters, trie oracle for the background ones, brute
force for the churned-in ones)."""

import numpy as np
import pytest
from oracle.c5_checker import SnapshotOracle

from emqx_amd import gen
from emqx_amd.engine import Engine
from emqx_amd.skew import Churn, workload

pytestmark = pytest.mark.gpu


def _check_all_rows(offs, ids, st):
    n = len(offs) - 1
    lens = np.diff(offs.astype(np.int64))
    assert offs[0] == 0 and (lens >= 0).all() and int(offs[-1]) == len(ids) == st["matches"]
    # no filter twice in a row: sort (row, id) pairs and compare neighbours
    row = np.repeat(np.arange(n, dtype=np.int64), lens)
    key = row << 32 | ids.astype(np.int64)
    key.sort()
    assert not (key[1:] == key[:-1]).any()


def test_c5_k1000_dedup_batches_around_10k_deltas():
    p = gen.SkewParams(k_per_hot=1000)
    allf, derived, hot, pubs = workload(p, 100_000, 10_000_000, seed=5)
    background = allf.tolist()[len(derived):]
    chk = SnapshotOracle(derived, background)
    eng = Engine(device=0)
    eng.insert_many(allf)
    churn = Churn(hot, derived.tolist(), seed=11)
    b = eng.prepare(pubs, dedup=True)
    hot_l = hot.tolist()
    hot_set = set(hot_l)
    rng = np.random.default_rng(7)
    T = pubs
    for rnd in range(2):
        if rnd:
            dels, adds = churn.step(10_000)            # between the two launches
            Churn.apply(eng, gen.Strings.from_list(dels), gen.Strings.from_list(adds))
            for f in dels:
                chk.delete(f)
            for f in adds:
                chk.insert(f)
        b.launch().wait()
        # the device dedup's map (rows exist once the batch was waited; a grown
        # dictionary may split rows, so it is read after every launch)
        row_of, n_rows = b.row_map()
        offs, ids = b.result()
        st = b.stats()
        assert len(offs) == n_rows + 1 and st["slow_topics"] > 0 and st["publishes"] == len(T)
        _check_all_rows(offs, ids, st)
        # every publish's row, expanded on the device: delivered = sum of its rows' lengths
        assert st["delivered"] == int(np.diff(offs.astype(np.int64))[row_of].sum())
        if rnd == 0:
            # rows are in first-occurrence order: row r's first publish
            first = np.full(n_rows, -1, np.int64)
            order = np.arange(len(row_of) - 1, -1, -1)
            first[row_of[order]] = order
            assert (np.diff(first) > 0).all()
            rows = rng.permutation(n_rows)
            hot_pub, bg_pub = [], []
            for r in rows.tolist():
                i = int(first[r])
                tp = bytes(T.buf[int(T.offs[i]):int(T.offs[i + 1])])
                (hot_pub if tp in hot_set else bg_pub).append((i, tp))
                if len(hot_pub) >= 300 and len(bg_pub) >= 2700:
                    break
            pick = hot_pub[:300] + bg_pub[:2700]
            ts = [tp for _, tp in pick]
        sample = [int(row_of[i]) for i, _ in pick]
        exp = chk.rows(ts)
        cache = {}
        got = [[cache.setdefault(int(x), eng.filter_bytes(int(x))) for x in ids[offs[r]:offs[r + 1]]]
               for r in sample]
        bad = [i for i in range(len(sample)) if got[i] != exp[i]]
        assert not bad, (rnd, ts[bad[0]], len(got[bad[0]]), len(exp[bad[0]]))
        assert sum(len(exp[i]) for i in range(300)) > 300 * 500   # the hot rows are long (K = 1000)
    b.free()
    chk.close()
