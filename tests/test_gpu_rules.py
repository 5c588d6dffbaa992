"""Batched emqx_topic:match/2 on the device (tm_rules_match) against the
reference KATs and the host predicate, in both the binary form ('$' rule) and
the word-list form used by ACL rules."""

import random

import numpy as np
import pytest
from conftest import load_golden

from emqx_amd import emqx_topic as T
from emqx_amd.engine import Engine
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_kat_topic_match_on_device():
    kat = load_golden("kat_topic.json")
    names = sorted({n.encode() for n, _, _ in kat["match"]})
    rules = sorted({f.encode() for _, f, _ in kat["match"]})
    got = Engine(device=0).rules_match(names, rules, dollar_rule=True)
    for n, f, exp in kat["match"]:
        assert got[names.index(n.encode()), rules.index(f.encode())] == exp, (n, f)


def test_random_names_and_rules_both_forms():
    rng = random.Random(8)
    alpha = [b"a", b"b", b"", b"$a", b"%", b"!", b"c", b"x"]
    names = [b"/".join(rng.choice(alpha) for _ in range(rng.randint(1, 6))) for _ in range(3000)]
    names += [b"$SYS/x", b"$", b"", b"/"]
    rules = [b"/".join(rng.choice(alpha + [b"+", b"#"]) for _ in range(rng.randint(1, 5))) for _ in range(70)]
    rules += [b"#", b"+", b"+/#", b"$SYS/#", b"a/#", b"#/a"]
    eng = Engine(device=0)
    gb = eng.rules_match(names, rules, dollar_rule=True)
    gw = eng.rules_match(names, rules, dollar_rule=False)
    eb = np.array([[O.match(n, f) for f in rules] for n in names])
    ew = np.array([[T.match(T.words(n), T.words(f)) for f in rules] for n in names])
    assert np.array_equal(gb, eb)
    assert np.array_equal(gw, ew)
    assert (gb != gw).any()      # the '$' rule makes a difference on this set
