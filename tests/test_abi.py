"""The C-ABI library: loads, exports exactly what include/emqx_tm.h declares, and
its host logic (trie maintenance, emqx_topic predicates) matches the oracle.
No compute calls without a GPU -- a host-only engine must refuse to match."""

import ctypes as C
import random
import re

import pytest
from conftest import load_golden

from emqx_amd import _native as N
from emqx_amd import emqx_topic as T
from emqx_amd.engine import Engine
from oracle import oracle as O


def header_symbols():
    with open(N.HEADER) as f:
        src = f.read()
    return set(re.findall(r"TM_API\s+[\w\s\*]+?\b(tm_\w+)\s*\(", src))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    declared = header_symbols()
    assert len(declared) >= 24
    for name in declared:
        assert hasattr(L, name), name
    # the Python binding binds every declared entry point, and nothing else
    assert declared == set(N.SIGNATURES), declared ^ set(N.SIGNATURES)


def test_build_info_and_no_device_match_fails_loudly():
    assert b"gfx950" in N.lib().tm_build_info()
    # the loaded library was built from the sources in this tree (not a stale .so)
    from emqx_amd import build as B
    assert N.lib().tm_build_info().decode().endswith("src " + B.source_hash())
    e = Engine(device=-1)
    e.insert(b"a/+")
    with pytest.raises(N.TmError) as ei:
        e.match_batch([b"a/b"])
    assert ei.value.rc == N.TM_ENODEV


def test_kat_trie_lookup_edge_count_host_engine():
    kat = load_golden("kat_trie.json")
    for case in kat["cases"]:
        e = Engine(device=-1)
        for op, arg, *rest in case["ops"]:
            if op == "insert":
                e.insert(arg.encode())
            elif op == "delete":
                e.delete(arg.encode())
            elif op == "empty":
                assert e.empty() is arg, case["name"]
        for node, exp in case.get("lookup", []):
            got = e.lookup(node.encode())
            if exp is None:
                assert got is None, (case["name"], node, got)
            else:
                assert got == (exp[0], None if exp[1] is None else exp[1].encode()), (case["name"], got)


def test_trie_maintenance_matches_oracle_under_churn():
    rng = random.Random(11)
    words = [b"a", b"b", b"", b"+", b"#", b"$x", b"c", b"d"]
    pool = [b"/".join(rng.choice(words) for _ in range(rng.randint(1, 6))) for _ in range(1500)]
    e, t = Engine(device=-1), O.Trie()
    for step in range(20000):
        f = rng.choice(pool)
        if rng.random() < 0.6:
            e.insert(f); t.insert(f)
        else:
            e.delete(f); t.delete(f)
        if step % 2500 == 0:
            for nid in set(list(t.nodes) + pool):
                if nid is O.ROOT:
                    continue
                b = t.lookup(nid)
                assert e.lookup(nid) == (None if not b else (b[0][1], b[0][2])), nid
            r, rb = e.lookup(None), t.lookup(O.ROOT)
            assert (r is None) == (not rb)
            assert e.empty() == t.empty()
    st = e.stats()
    assert st["edges"] == len(t.edges)
    assert st["nodes"] == len(t.nodes)
    assert st["filters"] == sum(1 for v in t.nodes.values() if v[1] is not None)


def test_filter_ids_and_bytes():
    e = Engine(device=-1)
    for f in [b"a/+/c", b"a/#", b"", b"x//y"]:
        e.insert(f)
    for f in [b"a/+/c", b"a/#", b"", b"x//y"]:
        assert e.filter_bytes(e.filter_id(f)) == f
    with pytest.raises(KeyError):
        e.filter_id(b"a/+")      # a node, but not a filter
    e.delete(b"a/#")
    with pytest.raises(KeyError):
        e.filter_id(b"a/#")


def test_version_bumps_on_mutation_only():
    e = Engine(device=-1)
    v0 = e.version
    e.insert(b"a/+")
    v1 = e.version
    e.insert(b"a/+")          # idempotent
    assert v1 > v0 and e.version == v1
    e.delete(b"zz/top")       # absent
    assert e.version == v1


def test_kat_emqx_topic_mirror():
    kat = load_golden("kat_topic.json")
    for name, flt, exp in kat["match"]:
        assert T.match(name.encode(), flt.encode()) is exp, (name, flt)
        if not name.startswith("$"):   # the $ rule applies to binaries only (src/emqx_topic.erl:68-71)
            assert T.match(T.words(name.encode()), T.words(flt.encode())) is exp, (name, flt)
    for t, exp in kat["wildcard"]:
        assert T.wildcard(t.encode()) is exp
    for t, ws in kat["words"]:
        got = T.words(t.encode())
        atoms = {"''": T.EMPTY, "'+'": T.PLUS, "'#'": T.HASH}
        assert len(got) == len(ws)
        for g, w in zip(got, ws):
            assert (g is atoms[w]) if w in atoms else (g == w.encode())
    for t, exp in kat["tokens"]:
        assert T.tokens(t.encode()) == [x.encode() for x in exp]
    for t, n in kat["levels"]:
        assert T.levels(t.encode()) == n
    atoms = {"''": T.EMPTY, "'+'": T.PLUS, "'#'": T.HASH}
    for ws, exp in kat["join"]:
        assert T.join([atoms.get(w, w.encode()) for w in ws]) == exp.encode()
    for t, exp in kat["join_words"]:
        assert T.join(T.words(t.encode())) == exp.encode()
    for parent, w, exp in kat["prepend"]:
        p = None if parent is None else atoms.get(parent, parent.encode())
        assert T.prepend(p, w.encode()) == exp.encode()
    for var, val, topic, exp in kat["feed_var"]:
        assert T.feed_var(var.encode(), val.encode(), topic.encode()) == exp.encode()


def test_kat_validate():
    kat = load_golden("kat_topic.json")
    long_topic = b"".join(b"%d/" % i for i in range(10001))   # long_topic() :193-194
    for kind, topic, exp in kat["validate"]:
        t = long_topic if topic == "LONG" else topic.encode()
        if exp == "ok":
            assert T.validate((kind, t)) is True
        else:
            with pytest.raises(T.TopicError) as ei:
                T.validate((kind, t))
            assert ei.value.reason == exp, (kind, topic)
    with pytest.raises(T.TopicError) as ei:
        T.validate(("name", b"a/\xff"))
    assert ei.value.reason == "function_clause"   # <<C/utf8, ...>> does not match


def test_kat_parse():
    kat = load_golden("kat_topic.json")
    for inp, opts, exp, share in kat["parse"]:
        if exp == "error":
            with pytest.raises(T.TopicError):
                T.parse(inp.encode(), {k: v.encode() for k, v in opts.items()})
        else:
            f, o = T.parse(inp.encode(), {})
            assert f == exp.encode()
            assert o.get("share") == (None if share is None else share.encode())


def test_predicate_matches_oracle_randomized():
    rng = random.Random(5)
    alpha = [b"a", b"b", b"", b"+", b"#", b"$a", b"%", b"!"]
    for _ in range(20000):
        n = b"/".join(rng.choice(alpha[:3] + alpha[5:]) for _ in range(rng.randint(1, 5)))
        f = b"/".join(rng.choice(alpha) for _ in range(rng.randint(1, 5)))
        assert T.match(n, f) == O.match(n, f), (n, f)


def test_c_struct_sizes_stable():
    assert C.sizeof(N.Config) == 16
    assert C.sizeof(N.TrieNode) == 12
    assert C.sizeof(N.Result) == 32       # u32 + pad + u64 + 2 pointers


def test_group_without_device_is_refused():
    from emqx_amd.engine import Group
    with pytest.raises(N.TmError) as ei:
        Group([-1])
    assert ei.value.rc == N.TM_EINVAL
    if N.lib().tm_device_count() == 0:
        with pytest.raises(N.TmError) as ei:
            Group([0, 0])
        assert ei.value.rc == N.TM_ENODEV
