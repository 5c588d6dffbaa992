"""The multi-device self-check of bench.py (emqx_amd/selfcheck.py) on the CPU:
two ranks (real processes, the host file group) post sampled rows; rank 0
re-matches every rank's publishes and compares digests.  The oracle stands in
for the device replicas; a rank whose rows differ in one filter is caught."""

import multiprocessing as mp
import os
from dataclasses import replace

import numpy as np

from emqx_amd import gen
from emqx_amd import selfcheck as SC
from emqx_amd.hostsync import FileGroup


def _oracle(F):
    from oracle import pyoracle as P
    orc = P.Oracle()
    for f in F:
        orc.register(f)
        orc.insert(f)
    return orc


def _rows(orc, F, T):
    from oracle import pyoracle as P
    buf, offs = P.pack(T)
    c, idx, _ = orc.match_batch(buf, offs)
    o = np.concatenate([[0], np.cumsum(c.astype(np.int64))])
    return [[F[int(x)] for x in idx[o[i]:o[i + 1]]] for i in range(len(T))]


def _rank(rank, world, key, corrupt, q):
    p = replace(gen.C1, n_filters=1500)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 900 + rank, 8000).tolist()
    orc = _oracle(F)
    g = FileGroup(rank, world, key=key)
    idx = SC.sample_index(len(T))
    rows = _rows(orc, F, [T[i] for i in idx])
    if corrupt and rank == 1:            # one filter dropped from one row
        j = next(k for k, r in enumerate(rows) if r)
        rows[j] = rows[j][1:]
    payloads = g.allgather(SC.payload([T[i] for i in idx], rows, f"rank {rank}"))
    verdict = None
    if rank == 0:
        verdict = SC.check(payloads, lambda ts: _rows(orc, F, ts))
    g.barrier()
    g.close()
    orc.close()
    q.put((rank, verdict))


def _run(world, corrupt):
    key = f"sc_{os.getpid()}_{world}_{int(corrupt)}"
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, key, corrupt, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    return res[0]


def test_sample_index_covers_the_ends():
    assert list(SC.sample_index(5)) == [0, 1, 2, 3, 4]
    i = SC.sample_index(10_000_000)
    assert i[0] == 0 and i[-1] == 9_999_999 and 2900 <= len(i) <= 3000
    assert (np.diff(i) > 0).all()


def test_digest_depends_on_order_and_bytes():
    assert SC.digest([b"a/#", b"a/+"]) != SC.digest([b"a/+", b"a/#"])
    assert SC.digest([b"ab", b"c"]) != SC.digest([b"a", b"bc"])
    assert SC.digest([]) == SC.digest([])


def test_two_ranks_agree():
    v = _run(2, corrupt=False)
    assert v["parity_sample_ok"] and v["sampled_rows"] == 2 * 3000
    assert [s["mismatches"] for s in v["slices"]] == [0, 0]


def test_a_wrong_row_on_one_rank_is_caught():
    v = _run(2, corrupt=True)
    assert not v["parity_sample_ok"]
    assert v["slices"][0]["mismatches"] == 0 and v["slices"][1]["mismatches"] == 1
    assert v["mismatches"][0][0] == "rank 1"


def test_iot_device_ids_vectorised():
    """gen.iot_device_ids (the bench's and tests' candidate filter selection
    for C4 samples) equals splitting every string in Python."""
    p = replace(gen.C4, n_filters=50_000, n_ids=100_000)
    for s in (gen.gen_iot_filters(p), gen.gen_iot_topics(p, 4001, 20_000)):
        ids = gen.iot_device_ids(s)
        assert ids.tolist() == [int(x.split(b"/")[1][1:]) for x in s.tolist()]
    assert len(gen.iot_device_ids(gen.Strings.from_list([]))) == 0
