"""The per-publish ABI on a host-only engine: every call returns at once with
its own error (no device -> TM_ENODEV, longer than ?MAX_TOPIC_LEN -> TM_EINVAL),
none hangs, and no device batch is formed."""

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
    assert eng.coalesce_config() == (0, 0)


def test_async_refused_without_device():
    eng = Engine(device=-1)
    with pytest.raises(N.TmError) as ei:
        eng.match_async(b"a/b", lambda rc, ids: None)
    assert ei.value.rc == N.TM_ENODEV
    with pytest.raises(N.TmError) as ei:
        eng.match_async(b"x" * (N.TM_MAX_TOPIC_LEN + 1), lambda rc, ids: None)
    assert ei.value.rc == N.TM_EINVAL
    st = eng.async_stats()
    assert st["batches"] == 0 and st["requests"] == 0


def test_filter_copy_and_id_reuse_host_engine():
    """A deleted filter's id keeps its bytes until the id is reused; with no
    batch holding results (host-only engine), the next new node reuses it."""
    eng = Engine(device=-1)
    eng.insert(b"a/+/#")
    fid = eng.filter_id(b"a/+/#")
    assert eng.filter_copy(fid) == eng.filter_bytes(fid) == b"a/+/#"
    eng.delete(b"a/+/#")
    assert eng.filter_copy(fid) == b"a/+/#"        # still names the filter a result may hold
    with pytest.raises(KeyError):
        eng.filter_id(b"a/+/#")
    eng.insert(b"x/y/z")                            # reuses the freed ids
    assert eng.filter_copy(eng.filter_id(b"x/y/z")) == b"x/y/z"
    with pytest.raises(KeyError):
        eng.filter_copy(10_000)


def test_filters_copy_packs_live_filters_and_skips_dead_ids():
    eng = Engine(device=-1)
    fs = [b"a/+/#", b"sensor/1/temp", b"#", b"x/" + b"y" * 300]
    for f in fs:
        eng.insert(f)
    ids = [eng.filter_id(f) for f in fs]
    assert eng.filters_copy(ids) == list(enumerate(fs))   # grows past the first guess (300-B filter)
    got = eng.filters_copy([ids[2], 99_999, ids[0]])      # never a filter: skipped, not <<>>
    assert got == [(0, b"#"), (2, b"a/+/#")]
    assert eng.filters_copy([]) == []
