"""Filter-sharded mode on CPU: host API (shared dictionary, shard rule, bulk
insert, tokenisation) and the multi-rank exchange over gloo (world_size 2 and 3)."""

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from emqx_amd import gen
from emqx_amd import _native as N
from emqx_amd.engine import Engine

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_frozen_dictionary_and_shard_rule():
    e = Engine(device=-1, frozen_dict=True)
    e.dict_load([b"a", b"b", b"c", b"$SYS"])
    e.insert(b"a/b/#")
    with pytest.raises(N.TmError) as ei:
        e.insert(b"a/zz")                      # word outside the shared dictionary
    assert ei.value.rc == N.TM_ENOENT
    G = 4
    for f in [b"+/b", b"#", b"a", b"a/+", b"a/#", b"", b"/"]:
        s = e.filter_shard(f, G)
        assert s == G or f == b"/", f          # b"/" = ''/'' : two literal levels
    s1 = e.filter_shard(b"a/b/c/#", G)
    assert 0 <= s1 < G and e.filter_shard(b"a/b", G) == s1 == e.filter_shard(b"a/b/+", G)
    with pytest.raises(N.TmError):
        e.filter_shard(b"a/q/c", G)            # unknown literal: no defined shard
    with pytest.raises(N.TmError):
        e.dict_load([b"x/y"])


def test_insert_many_partitions_every_filter_once():
    p = gen.IotParams(n_filters=5000, n_ids=600)
    F = gen.gen_iot_filters(p)
    vocab = gen.gen_iot_vocab(p)
    G = 3
    owned = []
    for r in range(G):
        e = Engine(device=-1, frozen_dict=True)
        e.dict_load(vocab)
        n = e.insert_many(F, r, G)
        assert e.stats()["filters"] == n
        owned.append({f for f in F.tolist() if e.filter_shard(f, G) in (r, G)})
        assert len(owned[-1]) == n
    repl = set.intersection(*owned)
    assert all(f.startswith(b"+/") for f in repl) and len(repl) == p.n_filters // 10
    assert set.union(*owned) == set(F.tolist())
    for a in range(G):
        for b in range(a + 1, G):
            assert owned[a] & owned[b] == repl


def test_tokenize_layout_matches_batch_semantics():
    e = Engine(device=-1)
    for f in [b"a/+", b"$SYS/#", b"x"]:
        e.insert(f)
    T = [b"a/b", b"$SYS/q", b"", b"+x/a", b"/".join([b"a"] * 12), b"zz/x"]
    tok = e.tokenize(T)
    assert list(np.diff(tok.toff.astype(np.int64))) == [2, 2, 1, 2, 12, 2]
    assert tok.tflags.tolist() == [0, 1, 0, 2, 2, 0]
    ids = tok.words & ((1 << 29) - 1)
    assert ids[tok.toff[5]] == 0                 # unseen word -> UNKNOWN
    assert ids[tok.toff[2]] == 1                 # '' -> W_EMPTY
    # a host-token batch validates its input
    b = e.prepare_tokens_host(tok)
    assert b.n == len(T)
    bad = type(tok)(tok.words, tok.toff.copy(), tok.tflags.copy())
    bad.tflags[4] = 0                            # deep topic without the generic-path flag
    with pytest.raises(N.TmError):
        e.prepare_tokens_host(bad)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_gloo(world):
    port = free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=os.path.dirname(HERE))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "sharded_worker.py"), str(r), str(world),
                               str(port), "11"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r}:\n" + outs[r][-3000:]
