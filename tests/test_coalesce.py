"""tm_match_coalesced on a host-only engine: the leader/follower hand-off
completes for many concurrent callers and every caller gets its own error
(no device -> TM_ENODEV, too long -> TM_EINVAL), none hangs."""

import threading

import pytest

from emqx_amd import _native as N
from emqx_amd.engine import Engine


def test_concurrent_callers_all_return_their_error():
    eng = Engine(device=-1)
    eng.insert(b"a/+")
    eng.coalesce_config(max_batch=8, linger_us=100)
    rcs = []
    lock = threading.Lock()

    def worker(k):
        for i in range(50):
            t = b"x" * (N.TM_MAX_TOPIC_LEN + 1) if (k + i) % 13 == 0 else b"a/%d" % i
            try:
                eng.match_coalesced(t)
                rc = 0
            except N.TmError as e:
                rc = e.rc
            with lock:
                rcs.append((len(t) > N.TM_MAX_TOPIC_LEN, rc))
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(12)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=60)
    assert all(not t.is_alive() for t in ths)
    assert len(rcs) == 600
    assert all(rc == (N.TM_EINVAL if bad else N.TM_ENODEV) for bad, rc in rcs)
    batches, requests = eng.coalesce_config()
    assert requests == sum(1 for bad, _ in rcs if not bad) and 0 < batches <= requests
