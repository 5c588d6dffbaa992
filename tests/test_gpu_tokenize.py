"""The device tokeniser (tm_tokenize_device; the default tokeniser of
tm_match_batch / tm_batch_prepare) against the host one (tm_tokenize), which
restates emqx_topic:words/1 (src/emqx_topic.erl:150-164) plus interning.

Bit-exact word entries, offsets and flags on seeded, adversarial and edge-case
topics; the dictionary mirror follows subscribes between prepare and launch and
across dictionary rehashes; whole-batch results equal the host-tokenised
engine's and the oracle's."""

from dataclasses import replace

import numpy as np
import pytest
from conftest import lb, load_golden

from emqx_amd import gen
from emqx_amd.engine import Engine
from test_gpu_parity import assert_same, engine_rows, oracle_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def torch_first():
    """torch's HIP runtime must initialise before the engine's (the device
    tokens come back as torch tensors)."""
    import torch
    torch.zeros(1, device="cuda")
    yield


def edge_topics(words):
    """Empty and separator-only topics, '+'/'#'-leading and irregular words,
    '$' roots, hash-chunk boundary lengths (7/8/9/15/16/17/24 bytes), deep
    topics on both sides of the 10-level fast path, raw and UTF-8 bytes."""
    long = [w for w in words if len(w) >= 2][:4] or [b"ab"]
    out = [b"", b"/", b"//", b"///a", b"a", b"+", b"#", b"+/#", b"+x/y", b"a/+b", b"a/#/b", b"$", b"$SYS",
           b"$SYS/a/b", b"/$a", b"\x00a/b", "café/ü/漢".encode(), b"a" * 4096]
    for n in (7, 8, 9, 15, 16, 17, 24):
        out.append(b"x" * n + b"/" + b"y" * n)
        out.append((long[0] * 24)[:n])
    for d in (9, 10, 11, 12, 30):
        out.append(b"/".join(long[i % len(long)] for i in range(d)))
    out += [b"/".join([w, w]) for w in words[:64]]
    return out


def both(eng, topics):
    host = eng.tokenize(topics)
    dw, dt, df = eng.tokenize_device(topics)
    return host, (dw.cpu().numpy().view(np.uint32), dt.cpu().numpy().view(np.uint32), df.cpu().numpy())


def assert_tokens_equal(eng, topics):
    host, (dw, dt, df) = both(eng, topics)
    assert np.array_equal(dt, host.toff)
    assert np.array_equal(df, host.tflags)
    bad = np.nonzero(dw != host.words)[0]
    assert bad.size == 0, (bad[:5], dw[bad[:5]], host.words[bad[:5]])


def test_device_tokens_equal_host_tokens():
    p = replace(gen.C1, n_filters=20000)
    filters = gen.gen_filters(p).tolist()
    adv = load_golden("synth_adversarial.json")
    filters += [lb(f) for f in adv["filters"]]
    eng = Engine(device=0)
    for f in filters:
        eng.insert(f)
    words = sorted({w for f in filters for w in f.split(b"/")})
    topics = gen.gen_topics(p, gen.Strings.from_list(filters[:20000]), 7, 50000).tolist()
    topics += [lb(t) for t in adv["topics"]] + edge_topics(words)
    assert_tokens_equal(eng, topics)
    assert_tokens_equal(eng, [])
    assert_tokens_equal(eng, [b""])


def test_dictionary_follows_subscribes_and_rehash():
    eng = Engine(device=0)
    eng.insert(b"seed/#")
    fresh = [b"w%05d" % i for i in range(3000)]           # > 1024-slot table: two rehashes
    topics = [b"seed/" + w for w in fresh] + [w + b"/x" for w in fresh]
    b = eng.prepare(topics)                                # bytes only: words resolved at launch
    for i, w in enumerate(fresh):
        eng.insert(w + b"/+")
        if i % 997 == 0:
            assert_tokens_equal(eng, topics)               # incremental dictionary deltas
    b.launch().wait()
    offs, ids = b.result()
    b.free()
    got = [[eng.filter_bytes(int(i)) for i in ids[offs[t]:offs[t + 1]]] for t in range(len(topics))]
    exp = [[b"seed/#"] for _ in fresh] + [[w + b"/+"] for w in fresh]
    assert got == exp
    assert_tokens_equal(eng, topics)


def test_device_and_host_tokenised_engines_agree():
    p = replace(gen.C1, n_filters=10000)
    filters = gen.gen_filters(p)
    topics = gen.gen_topics(p, filters, 11, 100000)
    flist = filters.tolist()
    dev, host = Engine(device=0), Engine(device=0, host_tokenize=True)
    for f in flist:
        dev.insert(f)
        host.insert(f)
    rows = []
    for e in (dev, host):
        bt = e.prepare(topics)
        bt.launch().wait()
        rows.append((bt.result(), bt.stats()))
        bt.free()
    (o1, i1), s1 = rows[0]
    (o2, i2), s2 = rows[1]
    assert np.array_equal(o1, o2)
    got = [dev.filter_bytes(int(i)) for i in i1]
    exp = [host.filter_bytes(int(i)) for i in i2]
    assert got == exp
    for k in ("visits", "hash_hits", "words", "matches"):
        if k in s1:
            assert s1[k] == s2[k], k
    sample = topics.tolist()[:5000]
    exp_rows, _ = oracle_rows(flist, sample)
    assert_same(sample, engine_rows(dev, sample), exp_rows)


def test_words_cap_overflow_is_reported():
    eng = Engine(device=0)
    eng.insert(b"a/b")
    topics = [b"a/b/c/d"] * 100
    with pytest.raises(Exception):
        eng.tokenize_device(topics, words_cap=399)
    w, t, f = eng.tokenize_device(topics, words_cap=400)
    assert int(t[-1]) == 400


def test_large_batch_tokens_equal_host_tokens():
    """A batch past 65,536 topics (multi-block tile scan, full-size tiles):
    the same tokens as the host on the generated workload plus the edge cases
    (empty and separator-only topics, 7-24-byte words across the 8/16-byte
    boundaries, a 4,096-byte topic on the lane-per-topic path, UTF-8, unknown
    words) placed mid-batch and at its end, and the words-cap overflow still
    reported."""
    p = replace(gen.C1, n_filters=20000)
    filters = gen.gen_filters(p).tolist()
    adv = load_golden("synth_adversarial.json")
    filters += [lb(f) for f in adv["filters"]]
    eng = Engine(device=0)
    for f in filters:
        eng.insert(f)
    for n in (7, 8, 9, 15, 16, 17, 24):
        eng.insert(b"k" * n + b"/" + b"z" * n)
    words = sorted({w for f in filters for w in f.split(b"/")})
    topics = gen.gen_topics(p, gen.Strings.from_list(filters[:20000]), 9, 70000).tolist()
    edge = [lb(t) for t in adv["topics"]] + edge_topics(words)
    edge += [b"k" * n + b"/" + b"z" * n for n in (7, 8, 9, 15, 16, 17, 24)]
    topics = topics[:30000] + edge + topics[30000:] + edge
    assert len(topics) >= 65536
    assert_tokens_equal(eng, topics)
    big = [b"a/b/c/d"] * 70000
    with pytest.raises(Exception):
        eng.tokenize_device(big, words_cap=279999)
    w, t, f = eng.tokenize_device(big, words_cap=280000)
    assert int(t[-1]) == 280000
