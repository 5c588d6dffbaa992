"""The host barrier / max-reduce the replicated multi-rank bench uses
(emqx_amd/hostsync.py), exercised with real processes at world 2 and 3, and the
split + concatenate rule of the replicated group (tm_group) restated on the
oracle: slices matched independently concatenate to the whole batch's CSR."""

import multiprocessing as mp
import os
import time
from dataclasses import replace

import numpy as np
import pytest

from emqx_amd import gen
from emqx_amd.hostsync import FileGroup


def _worker(rank, world, key, q):
    g = FileGroup(rank, world, key=key)
    time.sleep(0.05 * rank)                 # ranks arrive at different times
    g.barrier()
    t_after = time.monotonic()
    m = g.allmax(10.0 + rank)
    g.barrier()
    g.close()
    q.put((rank, t_after, m))


@pytest.mark.parametrize("world", [2, 3])
def test_barrier_and_allmax(world, tmp_path):
    key = f"test_{os.getpid()}_{world}"
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, key, q)) for r in range(world)]
    t0 = time.monotonic()
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    # nobody left the first barrier before the last rank arrived (rank world-1 sleeps longest)
    assert all(t - t0 >= 0.05 * (world - 1) - 0.01 for _, t, _ in res)
    assert all(m == 10.0 + world - 1 for _, _, m in res)
    assert not os.path.exists(f"/tmp/emqx_tm_sync_{key}")


def test_barrier_times_out_without_peers():
    g = FileGroup(0, 2, key=f"lonely_{os.getpid()}")
    with pytest.raises(TimeoutError):
        g.barrier(timeout=0.2)


def test_replicated_split_concatenates_to_the_whole_batch():
    """tm_group's contract on the oracle: contiguous slices matched separately,
    row offsets shifted by the previous slices' totals, equal the whole CSR."""
    from oracle import pyoracle as P
    p = replace(gen.C1, n_filters=2000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 7, 5001).tolist()
    orc = P.Oracle()
    for f in F:
        orc.register(f)
        orc.insert(f)
    buf, offs = P.pack(T)
    whole_c, whole_i, _ = orc.match_batch(buf, offs)
    for k in (2, 3, 8):
        lo = [len(T) * i // k for i in range(k + 1)]
        cs, ids = [], []
        for i in range(k):
            b, o = P.pack(T[lo[i]:lo[i + 1]])
            c, x, _ = orc.match_batch(b, o)
            cs.append(c)
            ids.append(x)
        assert np.array_equal(np.concatenate(cs), whole_c)
        assert np.array_equal(np.concatenate(ids), whole_i)
    orc.close()
