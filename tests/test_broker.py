"""Oracle restatement of emqx_broker's subscriber bag + dispatch, pinned by the
reference's own known-answer tests (tests/golden/kat_broker.json, transcribed
from test/emqx_broker_SUITE.erl and test/emqx_client_SUITE.erl) and by a
brute-force restatement over emqx_topic:match/2."""

import random

from conftest import load_golden

from oracle import oracle as O


def run_kat_ops(ops, sub, unsub, down, pub, subscribers, topics):
    for op in ops:
        if op[0] == "sub":
            sub(op[1].encode(), op[2])
        elif op[0] == "unsub":
            unsub(op[1].encode(), op[2])
        elif op[0] == "down":
            down(op[1])
        elif op[0] == "pub":
            exp = [(f.encode(), p) for f, p in op[2]]
            assert pub(op[1].encode()) == exp, op
        elif op[0] == "subscribers":
            assert subscribers(op[1].encode()) == op[2], op
        elif op[0] == "topics":
            assert sorted(topics()) == sorted(t.encode() for t in op[1]), op
        else:
            raise AssertionError(op)


def test_oracle_broker_kats():
    kat = load_golden("kat_broker.json")
    assert len(kat["cases"]) >= 7
    for case in kat["cases"]:
        b = O.Broker()
        run_kat_ops(case["ops"], b.subscribe, b.unsubscribe, b.subscriber_down, b.publish, b.subscribers,
                    lambda: list(b.routes))


def test_oracle_broker_vs_brute_force_with_churn():
    rng = random.Random(7)
    words = [b"a", b"b", b"", b"$SYS", b"c"]
    filters = set()
    while len(filters) < 60:
        d = rng.randint(1, 4)
        ws = [rng.choice(words + [b"+"]) for _ in range(d)]
        if rng.random() < 0.3:
            ws[-1] = b"#"
        filters.add(b"/".join(ws))
    filters = sorted(filters)
    names = sorted({b"/".join(rng.choice(words) for _ in range(rng.randint(1, 4))) for _ in range(80)})
    b = O.Broker()
    bag = {}
    for _ in range(600):
        f, pid = rng.choice(filters), rng.randrange(12)
        if rng.random() < 0.35 and pid in bag.get(f, []):
            assert b.unsubscribe(f, pid)
            bag[f].remove(pid)
        elif rng.random() < 0.03:
            n = b.subscriber_down(pid)
            assert n == sum(pid in v for v in bag.values())
            for v in bag.values():
                if pid in v:
                    v.remove(pid)
        else:
            b.subscribe(f, pid)
            if pid not in bag.setdefault(f, []):
                bag[f].append(pid)
    for t in names:
        exp = [(f, p) for f in sorted(bag) if O.match(t, f) for p in bag[f]]
        assert b.publish(t) == exp, t
