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
    row_of, n_rows = b.row_map()
    assert n_rows < len(pubs) // 3                      # the skew collapses most publishes
    T = pubs.tolist()
    distinct = {}
    for i, r in enumerate(row_of.tolist()):
        distinct.setdefault(r, T[i])
        assert distinct[r] == T[i]
    for rnd in range(3):
        if rnd:
            dels, adds = churn.step(600)
            Churn.apply(eng, dels, adds)
        b.launch().wait()
        offs, ids = b.result()
        assert len(offs) == n_rows + 1
        st = b.stats()
        assert st["slow_topics"] > 0                    # hot rows exceed K = 128
        F = sorted(churn.live_set) + background
        orc = P.Oracle()
        for f in F:
            orc.register(f)
            orc.insert(f)
        Td = [distinct[r] for r in range(n_rows)]
        buf, o = P.pack(Td)
        counts, idx, _ = orc.match_batch(buf, o, nthreads=8)
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        cache = {}
        for r in range(n_rows):
            got = [cache.setdefault(int(x), eng.filter_bytes(int(x))) for x in ids[offs[r]:offs[r + 1]]]
            exp = [F[int(j)] for j in idx[cut[r]:cut[r + 1]]]
            assert got == exp, (rnd, Td[r][:60])
    assert eng.stats()["uploads_delta"] >= 1
