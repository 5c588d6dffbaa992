"""Concurrency and lifetime contracts of the engine's Python/C surface --
needs an MI355X.

* Two threads launching and waiting batches on ONE replica's shared stream
  while small repeated batches are captured into HIP graphs: a wait never
  lands on a capturing stream (round-3 advisor finding), every row stays the
  oracle's.
* Graph replays re-record the timing events: ms_match is fresh per launch.
* A borrowed engine view (Group.engine(), ShardedGroup.engine()) keeps its
  owner alive and is invalidated when the owner is closed.
Expected rows come from the oracle (src/emqx_trie.erl restated)."""

import threading
from dataclasses import replace

import pytest
from test_gpu_parity import assert_same, engine_rows, oracle_rows

from emqx_amd import gen
from emqx_amd.engine import Engine, Group, ShardedGroup

pytestmark = pytest.mark.gpu


def _c1(n_filters=3000, n_topics=6000, seed=311):
    p = replace(gen.C1, n_filters=n_filters)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), seed, n_topics).tolist()
    return F, T


def _rows(eng, b, T):
    offs, ids = b.result()
    return [[eng.filter_bytes(int(x)) for x in ids[offs[i]:offs[i + 1]]] for i in range(len(T))]


def test_two_threads_launch_and_wait_on_one_replica_while_graphs_are_captured():
    F, T = _c1()
    eng = Engine(device=0)
    eng.insert_many(F)
    halves = [T[:3000], T[3000:]]
    exp = [oracle_rows(F, h)[0] for h in halves]
    errors = []
    ms = [[], []]

    def worker(k):
        try:
            b = eng.prepare(halves[k])          # shared replica stream (no TM_BATCH_STREAM)
            for it in range(60):                # repeated launches: captured, then replayed
                b.launch().wait()
                ms[k].append(b.stats()["ms_match"])
                if it % 20 == 19:
                    assert_same(halves[k], _rows(eng, b, halves[k]), exp[k])
            b.free()
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]
    assert all(v > 0 for m in ms for v in m)
    eng.close()


def test_graph_replays_report_fresh_kernel_times():
    """A batch under the graph limit is captured on its second identical
    launch and replayed after; the walk's HIP events are external nodes of the
    graph, so every replay re-records them (a plain record in a capture would
    leave the first launch's times in place)."""
    F, T = _c1(n_topics=20_000)
    eng = Engine(device=0)
    eng.insert_many(F)
    b = eng.prepare(T)
    ms = []
    for _ in range(8):
        b.launch().wait()
        st = b.stats()
        ms.append((st["ms_match"], st["ms_total"]))
    assert all(m > 0 and t >= m for m, t in ms)
    assert len({m for m, _ in ms[2:]}) > 1, ms        # replays: times change launch to launch
    exp, _ = oracle_rows(F, T[:2000])
    assert_same(T[:2000], _rows(eng, b, T)[:2000], exp)
    b.free()
    eng.close()


def test_borrowed_engine_views_outlive_nothing():
    F, T = _c1(n_filters=500, n_topics=200)
    e = Group([0]).engine()                 # the Group is only referenced by its view
    for f in F:
        e.insert(f)
    exp, _ = oracle_rows(F, T)
    assert_same(T, engine_rows(e, T), exp)
    grp = Group([0, 0])
    v = grp.engine()
    v.insert(b"a/+")
    grp.close()
    with pytest.raises(RuntimeError):
        v.insert(b"a/b")
    with pytest.raises(RuntimeError):
        v.stats()
    sg = ShardedGroup([0, 0])
    sv = sg.engine(1)
    assert sv.stats()["filters"] == 0
    sg.close()
    with pytest.raises(RuntimeError):
        sv.stats()
