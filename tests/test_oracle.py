"""The oracle (C restatement + Python restatement) pinned against the reference's
known-answer tests, and cross-checked against brute-force emqx_topic:match/2.
CPU only."""

import random

import numpy as np
import pytest
from conftest import lb, load_golden

from emqx_amd import gen
from oracle import oracle as O
from oracle import pyoracle as P

ATOMS = {"''": O.EMPTY, "'+'": O.PLUS, "'#'": O.HASH}


def test_kat_topic_match_both_oracles():
    kat = load_golden("kat_topic.json")
    for name, flt, exp in kat["match"]:
        assert O.match(name.encode(), flt.encode()) is exp, (name, flt)
        assert P.topic_match(name.encode(), flt.encode()) is exp, (name, flt)


def test_kat_words_wildcard_join():
    kat = load_golden("kat_topic.json")
    for t, ws in kat["words"]:
        assert O.words(t.encode()) == [ATOMS.get(w, w.encode()) for w in ws]
    for t, exp in kat["wildcard"]:
        assert O.wildcard(t.encode()) is exp
        assert bool(P.lib().tmo_wildcard(t.encode(), len(t))) is exp
    for ws, exp in kat["join"]:
        assert O.join([ATOMS.get(w, w.encode()) for w in ws]) == exp.encode()
    for t, exp in kat["join_words"]:
        assert O.join(O.words(t.encode())) == exp.encode()


def _apply_trie_case(case, tr):
    for op, arg, *rest in case["ops"]:
        if op == "insert":
            tr.insert(arg.encode())
        elif op == "delete":
            tr.delete(arg.encode())
        elif op == "empty":
            assert tr.empty() is arg


@pytest.mark.parametrize("impl", ["py", "c"])
def test_kat_trie(impl):
    kat = load_golden("kat_trie.json")
    for case in kat["cases"]:
        tr = O.Trie() if impl == "py" else P.Oracle()
        _apply_trie_case(case, tr)
        for topic, exp in case.get("match", []):
            # exact reference (DFS) order, e.g. t_match: [sensor/+/#, sensor/#]
            assert tr.match(topic.encode()) == [e.encode() for e in exp], (case["name"], topic)
        for topic, n in case.get("match_len", []):
            assert len(tr.match(topic.encode())) == n
        for node, exp in case.get("lookup", []):
            got = tr.lookup(node.encode())
            if exp is None:
                assert got == [], (case["name"], node)
            else:
                assert got[0][1] == exp[0], (case["name"], node, got)
                assert got[0][2] == (None if exp[1] is None else exp[1].encode())


def test_kat_triples():
    kat = load_golden("kat_trie.json")
    for topic, exp in kat["triples"]:
        got = O.Trie.triples(topic.encode())
        want = [(O.ROOT if p == "root" else p.encode(), w.encode(), c.encode()) for p, w, c in exp]
        assert got == want


def test_c_and_python_restatements_agree_on_churn():
    rng = random.Random(3)
    words = [b"a", b"b", b"", b"+", b"#", b"$s", b"c"]
    pool = [b"/".join(rng.choice(words) for _ in range(rng.randint(1, 5))) for _ in range(400)]
    t, c = O.Trie(), P.Oracle()
    for step in range(6000):
        f = rng.choice(pool)
        if rng.random() < 0.6:
            t.insert(f); c.insert(f)
        else:
            t.delete(f); c.delete(f)
        if step % 500 == 0:
            for topic in rng.sample(pool, 40):
                assert t.match(topic) == c.match(topic), topic
            assert t.empty() == c.empty()


@pytest.mark.parametrize("fixture", ["synth_c1_small.json", "synth_c2_small.json", "synth_adversarial.json"])
def test_golden_synth_against_c_oracle(fixture):
    g = load_golden(fixture)
    F = [lb(f) for f in g["filters"]]
    T = [lb(t) for t in g["topics"]]
    orc = P.Oracle()
    for f in F:
        orc.register(f)
        orc.insert(f)
    buf, offs = P.pack(T)
    counts, idx, _ = orc.match_batch(buf, offs, nthreads=2)
    rows = np.split(idx, np.cumsum(counts)[:-1])
    for i, t in enumerate(T):
        assert list(rows[i]) == g["expected"][i], t


def test_generated_workload_trie_vs_brute_force():
    from dataclasses import replace
    p = replace(gen.C1, n_filters=1200, seed=5)
    F = gen.gen_filters(p)
    T = gen.gen_topics(p, F, 99, 1500)
    orc = P.Oracle()
    for f in F.tolist():
        orc.register(f)
        orc.insert(f)
    c1, i1, st = orc.match_batch(T.buf, T.offs, nthreads=4)
    c2, i2 = P.brute_batch(F.tolist(), T.buf, T.offs, nthreads=4)
    assert np.array_equal(c1, c2) and np.array_equal(i1, i2)
    assert st["visits"] >= len(T)


def test_generators_c_and_python_identical():
    from dataclasses import replace
    for base in (gen.C1, gen.C2):
        p = replace(base, n_filters=700, vocab=min(base.vocab, 200))
        a = gen.py_gen_filters(p)
        b = gen.gen_filters(p).tolist()
        assert a == b
        assert gen.py_gen_topics(p, a, 17, 900) == gen.gen_topics(p, gen.Strings.from_list(a), 17, 900).tolist()
