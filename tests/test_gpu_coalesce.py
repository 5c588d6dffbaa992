"""tm_match_coalesced: many threads calling emqx_trie:match/1 one topic at a
time (the NIF's dirty schedulers) are served by shared device batches, each
caller getting exactly tm_trie_match's row (checked against the oracle)."""

import threading
from dataclasses import replace

import pytest

from emqx_amd import _native as N
from emqx_amd import gen
from emqx_amd.engine import Engine
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_concurrent_callers_share_batches_and_match_oracle():
    p = replace(gen.C1, n_filters=2000)
    F = gen.gen_filters(p).tolist()
    T = gen.gen_topics(p, gen.Strings.from_list(F), 31, 3200).tolist()
    eng = Engine(device=0)
    eng.insert_many(F)
    eng.coalesce_config(max_batch=64, linger_us=200)
    got = [None] * len(T)
    errors = []

    def worker(k):
        try:
            for i in range(k, len(T), 16):
                got[i] = eng.match_coalesced(T[i])
        except Exception as e:  # surfaced below
            errors.append(e)
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not errors and all(not t.is_alive() for t in ths)
    batches, requests = eng.coalesce_config()
    assert requests == len(T) and batches < requests      # callers did share batches
    trie = O.Trie()
    for f in F:
        trie.insert(f)
    for i in range(0, len(T), 7):
        assert [eng.filter_bytes(x) for x in got[i]] == sorted(trie.match(T[i])), T[i]
    for i in range(len(T)):
        assert got[i] == eng.match_ids(T[i])


def test_bad_topic_fails_alone():
    eng = Engine(device=0)
    eng.insert(b"a/#")
    with pytest.raises(N.TmError):
        eng.match_coalesced(b"x" * (N.TM_MAX_TOPIC_LEN + 1))
    assert [eng.filter_bytes(x) for x in eng.match_coalesced(b"a/b")] == [b"a/#"]
