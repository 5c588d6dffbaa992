"""emqx_batch mirror pinned by the reference's own suite (test/emqx_batch_SUITE.erl:
26-56, transcribed as data into tests/golden/kat_batch.json)."""

import queue

import pytest
from conftest import load_golden

from emqx_amd import emqx_batch as B

KAT = load_golden("kat_batch.json")


@pytest.mark.parametrize("case", KAT["cases"], ids=[c["name"] for c in KAT["cases"]])
def test_kat_batch(case):
    commits = []
    mailbox = queue.Queue()
    b = B.init({**case["opts"], "commit_fun": lambda q: commits.append(list(q)), "mailbox": mailbox})
    for st in case["steps"]:
        if "push" in st:
            b = B.push(st["push"], b)
        if "size" in st:
            assert B.size(b) == st["size"]
            assert B.items(b) == st["items"]
        if "await_linger_within_ms" in st:
            msg = mailbox.get(timeout=st["await_linger_within_ms"] / 1000.0)   # linger_timer_not_triggered
            assert msg == B.LINGER_EXPIRED
        if st.get("commit"):
            b = B.commit(b)
    assert commits == case["commits"]
    B.reset(b)


def test_commit_rearms_linger():
    """After a size commit the next push arms a new timer (push/2's first clause,
    src/emqx_batch.erl:56-62, applies again once reset/1 cleared it)."""
    mailbox = queue.Queue()
    commits = []
    b = B.init({"batch_size": 1, "linger_ms": 50, "commit_fun": commits.append, "mailbox": mailbox})
    b = B.push("x", b)
    b = B.push("y", b)                      # 2 = batch_size + 1 -> commit
    assert commits == [["x", "y"]] and B.size(b) == 0 and b.linger_timer is None
    b = B.push("z", b)
    assert b.linger_timer is not None
    assert mailbox.get(timeout=2.0) == B.LINGER_EXPIRED
    B.reset(b)
