"""Error contract of the batch path -- needs an MI355X.

* a batch whose match count does not fit the u32 CSR fails with TM_EOVERFLOW
  (never a wrapped, silently wrong CSR); the limit is lowered through the
  test-only TM_RESULT_LIMIT knob so the case runs at a small size;
* a topic longer than ?MAX_TOPIC_LEN (src/emqx_topic.erl:45) is TM_EINVAL."""

import os

import pytest
from test_gpu_parity import assert_same, engine_rows, oracle_rows

from emqx_amd import _native as N
from emqx_amd.engine import Engine

pytestmark = pytest.mark.gpu


def limited_engine(limit):
    os.environ["TM_RESULT_LIMIT"] = str(limit)
    try:
        return Engine(device=0)
    finally:
        del os.environ["TM_RESULT_LIMIT"]


def test_result_past_the_limit_is_eoverflow_not_wrapped():
    eng = limited_engine(1000)
    F = [b"#", b"+/#", b"a/#", b"a/+"]
    for f in F:
        eng.insert(f)
    big = [b"a/%d" % i for i in range(300)]           # 4 matches each: 1200 > 1000
    with pytest.raises(N.TmError) as ei:
        eng.match_batch(big)
    assert ei.value.rc == N.TM_EOVERFLOW
    # the engine stays usable, and a batch under the limit is exact
    small = big[:250]                                   # 1000 matches == limit
    exp, _ = oracle_rows(F, small)
    assert_same(small, engine_rows(eng, small), exp)
    # the split API fails the same way at wait()
    b = eng.prepare(big)
    with pytest.raises(N.TmError) as ei:
        b.launch().wait()
    assert ei.value.rc == N.TM_EOVERFLOW
    b.free()


def test_slow_path_rows_count_against_the_limit():
    eng = limited_engine(50)
    deep = b"/".join([b"a"] * 20)                       # > 10 levels: generic kernel
    for k in range(1, 21):
        eng.insert(b"/".join([b"a"] * k) + b"/#")
    with pytest.raises(N.TmError) as ei:
        eng.match_batch([deep] * 3)                      # 3 x 20 = 60 > 50
    assert ei.value.rc == N.TM_EOVERFLOW
    offs, ids = eng.match_batch([deep, deep])            # 40
    assert int(offs[-1]) == 40


def test_topic_longer_than_max_topic_len_is_einval():
    eng = Engine(device=0)
    eng.insert(b"+/#")
    ok = b"a/" + b"x" * (N.TM_MAX_TOPIC_LEN - 2)
    assert len(ok) == N.TM_MAX_TOPIC_LEN
    assert eng.match(ok) == [b"+/#"]
    for topics in ([ok + b"y"], [b"a/b", ok + b"y", b"c/d"]):
        with pytest.raises(N.TmError) as ei:
            eng.match_batch(topics)
        assert ei.value.rc == N.TM_EINVAL
        with pytest.raises(N.TmError) as ei:
            eng.prepare(topics)
        assert ei.value.rc == N.TM_EINVAL
    assert eng.match(b"a/b") == [b"+/#"]               # still usable


def test_sharded_prepare_refuses_long_topics_and_recovers():
    """tm_sharded_prepare checks every topic while it stages the batch
    (offsets, ?MAX_TOPIC_LEN): TM_EINVAL, and the batch handle re-prepared
    with valid publishes matches them."""
    from emqx_amd.engine import ShardedGroup
    grp = ShardedGroup([0])
    grp.insert_many([b"+/#", b"a/b"])
    ok = b"a/" + b"x" * (N.TM_MAX_TOPIC_LEN - 2)
    b = grp.prepare([b"a/b", ok])
    b.run()
    offs, ids = b.result()
    assert len(offs) == 3 and int(offs[-1]) == 3
    for topics in ([ok + b"y"], [b"a/b", ok + b"y", b"c/d"]):
        with pytest.raises(N.TmError) as ei:
            b.reprepare(topics)
        assert ei.value.rc == N.TM_EINVAL
    b.reprepare([b"a/b", b"c/d"]).run()
    offs, ids = b.result()
    assert [grp.filter_bytes(int(x)) for x in ids[offs[0]:offs[1]]] == [b"+/#", b"a/b"]
    assert [grp.filter_bytes(int(x)) for x in ids[offs[1]:offs[2]]] == [b"+/#"]
    b.free()
    grp.close()


def test_staging_skew_in_one_walk_group_falls_back_to_one_region():
    """Every match of a batch reserved by waves of one walk group (1-topic
    tiles: topic t -> wave t -> group t % 8; only topics t % 8 == 0 match):
    that group's region overflows while the batch fits the limit.  The engine
    must not retry per-group regions sized 8x the group (they exceed the
    limit) but stage the batch as one region, and return exact rows."""
    import itertools
    os.environ["TM_RESULT_LIMIT"] = "2000"
    os.environ["TM_STAGING_MIN"] = "64"
    try:
        eng = Engine(device=0)
    finally:
        del os.environ["TM_RESULT_LIMIT"]
        del os.environ["TM_STAGING_MIN"]
    words = [b"a", b"b", b"c", b"d", b"e", b"f"]
    F = [b"/".join(c) for c in itertools.product(*[(w, b"+") for w in words])]     # 64 filters
    F += [b"/".join(words[:k] + [b"#"]) for k in range(len(words) + 1)]          # 7 more
    for f in F:
        eng.insert(f)
    # 64 topics, one per tile; the 8 of group 0 match 71 filters each: 568
    # entries in a 256-entry region, 8 x 568 > the 2,000 limit, 568 < it
    T = [b"a/b/c/d/e/f" if t % 8 == 0 else b"q%d" % t for t in range(64)]
    exp, _ = oracle_rows(F, T)
    assert len(exp[0]) == 71
    for _ in range(2):   # and again on the grown batch
        assert_same(T, engine_rows(eng, T), exp)
