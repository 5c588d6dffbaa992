"""The erl_nif shim on the device, through the test stand-in for the Erlang
runtime (tests/nif_mock): match_async replies sent from the engine's
completion threads to many processes, batch calls racing async calls and trie
writers (no reply may alias another caller's buffers or a moved filter), the
route / fan-out batch shapes, and an engine dropped with replies in flight.
Expected sets come from the oracle trie (src/emqx_trie.erl restated)."""

import random
import threading
import time

import pytest

from oracle import oracle as O

from nif_harness import Nif

pytestmark = pytest.mark.gpu

WORDS = [b"a", b"b", b"c", b"d", b"e", b"+", b"#", b"$SYS"]


def _filters(rng, n):
    out = set()
    while len(out) < n:
        ws = [rng.choice(WORDS) for _ in range(rng.randint(1, 5))]
        if b"#" in ws[:-1]:
            continue
        out.add(b"/".join(ws))
    return sorted(out)


def _topics(rng, n):
    names = [w for w in WORDS if w not in (b"+", b"#")] + [b"f", b""]
    return [b"/".join(rng.choice(names) for _ in range(rng.randint(1, 6))) for _ in range(n)]


def _expected(trie, topic):
    return sorted(set(trie.match(topic)))


@pytest.fixture(scope="module")
def nif():
    return Nif()


def _recv_all(nif, pid, refs, timeout_s=60):
    """Replies for `refs` (any order): {ref ident: result}."""
    got = {}
    deadline = time.time() + timeout_s
    while len(got) < len(refs):
        msg = nif.recv(pid, int(max(1, (deadline - time.time()) * 1000)))
        assert msg is not None, f"pid {pid}: {len(refs) - len(got)} replies missing"
        assert msg[0] == "emqx_tm_match"
        got[msg[1][1]] = msg[2]
    return got


def test_match_async_from_many_processes(nif):
    rng = random.Random(11)
    e, t = nif.new(0), O.Trie()
    for f in _filters(rng, 1500):
        assert nif.call("insert", e, f) == "ok"
        t.insert(f)
    topics = _topics(rng, 4000)
    errors = []

    def process(pid):
        try:
            mine = topics[pid::16]
            for i in range(0, len(mine), 32):              # a burst of publishes, then their replies
                chunk = mine[i:i + 32]
                refs = []
                for tp in chunk:
                    r = nif.ref()
                    assert nif.call("match_async", e, tp, r, pid=pid) == "ok"
                    refs.append((r.ident, tp))
                got = _recv_all(nif, pid, refs)
                for ident, tp in refs:
                    assert got[ident] == _expected(t, tp), tp
        except BaseException as ex:   # noqa: BLE001 -- reported below
            errors.append(ex)

    th = [threading.Thread(target=process, args=(p,)) for p in range(100, 116)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[0]
    nif.drop(e)


def test_batches_race_async_calls_and_writers(nif):
    """ADVICE r1 (high/medium): batch replies came from the engine's shared
    scratch and filter bytes were read after the lock was dropped.  Batch,
    async and writer threads on one engine; churned filters live under `zz/`,
    which no query topic reaches, so the expected sets are fixed."""
    rng = random.Random(12)
    e, t = nif.new(0), O.Trie()
    for f in _filters(rng, 800):
        nif.call("insert", e, f)
        t.insert(f)
    topics = _topics(rng, 600)
    exp = {tp: _expected(t, tp) for tp in topics}
    stop = threading.Event()
    errors = []

    def writer():
        try:
            w = random.Random(5)
            live = []
            while not stop.is_set():
                if live and w.random() < 0.5:
                    assert nif.call("delete", e, live.pop(w.randrange(len(live))), pid=900) == "ok"
                else:
                    ws = [b"w%d" % w.randrange(50) for _ in range(w.randint(1, 4))] + [b"x" * w.randrange(200)]
                    f = b"zz/" + b"/".join(ws)
                    assert nif.call("insert", e, f, pid=900) == "ok"
                    live.append(f)
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    def batcher(pid):
        try:
            r = random.Random(pid)
            for _ in range(25):
                k = r.randint(1, 200)
                s = r.randrange(len(topics))
                batch = [topics[(s + j) % len(topics)] for j in range(k)]
                rows = nif.call("match_batch", e, batch, pid=pid)
                assert rows == [exp[tp] for tp in batch]
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    def asyncer(pid):
        try:
            for i in range(0, len(topics), 40):
                refs = []
                for tp in topics[i:i + 40]:
                    r = nif.ref()
                    assert nif.call("match_async", e, tp, r, pid=pid) == "ok"
                    refs.append((r.ident, tp))
                got = _recv_all(nif, pid, refs)
                for ident, tp in refs:
                    assert got[ident] == exp[tp], tp
        except BaseException as ex:   # noqa: BLE001
            errors.append(ex)

    wt = threading.Thread(target=writer)
    wt.start()
    th = [threading.Thread(target=batcher, args=(p,)) for p in (200, 201)]
    th += [threading.Thread(target=asyncer, args=(p,)) for p in (300, 301, 302, 303)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    stop.set()
    wt.join()
    assert not errors, errors[0]
    nif.drop(e)


def test_routes_and_dispatch_batches(nif):
    rng = random.Random(13)
    e, t = nif.new(0), O.Trie()
    filters = _filters(rng, 300)
    dests, subs = {}, {}
    for f in filters:
        for d in rng.sample(range(8), rng.randint(1, 3)):
            assert nif.call("route_add", e, f, d) == "ok"
            dests.setdefault(f, []).append(d)
        t.insert(f)
    topics = _topics(rng, 300)
    rows = nif.call("match_routes_batch", e, topics)
    for tp, row in zip(topics, rows):
        assert row == [(f, d) for f in _expected(t, tp) for d in dests[f]], tp
    for f in filters[:120]:                       # (a first subscriber also routes the filter to node 0)
        for s in rng.sample(range(1000), rng.randint(1, 4)):
            assert nif.call("subscribe", e, f, s, 0) == "ok"
            subs.setdefault(f, []).append(s)
    rows = nif.call("dispatch_batch", e, topics)
    for tp, row in zip(topics, rows):
        assert row == [s for f in _expected(t, tp) for s in subs.get(f, [])], tp
    nif.drop(e)


def test_engine_dropped_with_replies_in_flight(nif):
    """The last reference to the engine can go away while matches are queued:
    every queued call is still answered, and the engine is destroyed after."""
    rng = random.Random(14)
    before = nif.live_resources()
    e, t = nif.new(0), O.Trie()
    for f in _filters(rng, 400):
        nif.call("insert", e, f)
        t.insert(f)
    topics = _topics(rng, 3000)
    refs = []
    for tp in topics:
        r = nif.ref()
        assert nif.call("match_async", e, tp, r, pid=500) == "ok"
        refs.append((r.ident, tp))
    nif.drop(e)                                   # the calls in flight hold the engine
    got = _recv_all(nif, 500, refs)
    for ident, tp in refs:
        assert got[ident] == _expected(t, tp), tp
    deadline = time.time() + 30
    while nif.live_resources() != before and time.time() < deadline:
        time.sleep(0.05)
    assert nif.live_resources() == before
