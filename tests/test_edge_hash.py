"""The host edge hash under heavy churn at high load (tm_engine_impl.hpp
delete_edge_of: backward-shift deletion at bucket granularity, no tombstones).
tm_debug_check verifies the table invariants the kernels' probes rely on
(buckets filled in order, every key's probe run unbroken and within
max_disp); lookups are checked against an oracle trie."""

import random

from emqx_amd.engine import Engine
from oracle import oracle as O


def _churn(seed, n_words, pool_n, live_n, steps, check_every, wild=False):
    rng = random.Random(seed)
    words = [b"w%d" % i for i in range(n_words)]
    if wild:   # '+' chains and '#' leaves: wildcard edges of every depth
        words += [b"+"] * (n_words // 2)
        pool = {b"/".join(rng.choice(words) for _ in range(rng.randint(1, 5))) for _ in range(pool_n)}
        pool = list(pool | {p + b"/#" for p in list(pool)[: pool_n // 8]})
    else:
        pool = list({b"/".join(rng.choice(words) for _ in range(rng.randint(1, 3))) for _ in range(pool_n)})
    e, t = Engine(device=-1), O.Trie()
    live = set()
    for f in pool[:live_n]:
        e.insert(f)
        t.insert(f)
        live.add(f)
    worst = e.debug_check()
    for step in range(steps):
        f = rng.choice(pool)
        if f in live:
            e.delete(f)
            t.delete(f)
            live.discard(f)
        else:
            e.insert(f)
            t.insert(f)
            live.add(f)
        if step % check_every == 0:
            worst = max(worst, e.debug_check())
    worst = max(worst, e.debug_check())
    for g in pool:
        exp = t.lookup(g)
        got = e.lookup(g)
        assert (got is None) == (not exp), g
        if got is not None:
            assert got == (exp[0][1], exp[0][2]), g
    return worst


def test_churn_keeps_every_probe_run_intact():
    # ~1/2 of the pool live: the table oscillates around its growth threshold
    worst = _churn(seed=5, n_words=300, pool_n=40000, live_n=20000, steps=40000, check_every=997)
    assert worst >= 2          # runs longer than one bucket were exercised


def test_churn_small_tables_many_seeds():
    for seed in range(12):
        _churn(seed=100 + seed, n_words=40, pool_n=3000, live_n=1500, steps=6000, check_every=97)


def test_churn_plus_chains():
    # wildcard-heavy churn: '+' chains, '#' leaves, shared prefixes
    worst = _churn(seed=7, n_words=60, pool_n=30000, live_n=15000, steps=30000, check_every=499, wild=True)
    assert worst >= 2
    for seed in range(6):
        _churn(seed=300 + seed, n_words=8, pool_n=3000, live_n=1500, steps=6000, check_every=97, wild=True)


def test_literal_signature_saturates_and_clears():
    """The slot's literal-child signature (tm_internal.hpp Slot.word top bits):
    2,000 literal children under one node saturate its per-bit counts (the
    bits then stay set), a node whose last literal child goes clears its bits
    -- tm_debug_check compares every slot's bits with the node's counts and
    checks each literal edge's bit in its parent's signature; lookups follow."""
    e, t = Engine(device=-1), O.Trie()
    wide = [b"a/b/c%d" % i for i in range(2000)]
    narrow = [b"a/n/x", b"a/n/y", b"a/n/+", b"a/n/#"]
    for f in wide + narrow:
        e.insert(f)
        t.insert(f)
    e.debug_check()
    for f in wide[:1990] + narrow[:2]:
        e.delete(f)
        t.delete(f)
    e.debug_check()
    for f in wide[1990:]:
        e.delete(f)
        t.delete(f)
    e.insert(b"a/b/z")
    t.insert(b"a/b/z")
    e.debug_check()
    for g in wide + narrow + [b"a/b/z"]:
        assert (e.lookup(g) is None) == (not t.lookup(g)), g
