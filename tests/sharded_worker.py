"""One rank of the filter-sharded CPU test (tests/test_sharded.py), gloo backend.

The exchange, partition and reassembly of emqx_amd/sharded.py run as in
production; the per-shard device walk is replaced by the CPU oracle over the
same shard's filter subset (test infrastructure only), and the topic->shard
rule by a restatement of tm_tokens_shard (cross-checked against the engine's
host tm_filter_shard).  Every rank's reassembled rows must equal the oracle's
rows over the FULL filter set.
"""

from __future__ import annotations

import os
import random
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import gen  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402
from emqx_amd.sharded import ShardedMatcher  # noqa: E402
from oracle import pyoracle as P  # noqa: E402

W_UNKNOWN, W_EMPTY, W_PLUS, W_HASH, W_FIRST = 0, 1, 2, 3, 4
WID_MASK = (1 << 29) - 1
M64 = (1 << 64) - 1


def edge_hash(p, w):
    k = ((p << 32) | w) & M64
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k & 0xFFFFFFFF


def shard_rule(ids, G):
    if len(ids) < 2:
        return G
    i0, i1 = ids[0], ids[1]
    if i0 in (W_UNKNOWN, W_PLUS, W_HASH) or i1 in (W_UNKNOWN, W_PLUS, W_HASH):
        return G
    return edge_hash(i0, i1) % G


def workload(seed):
    """IoT filters + irregular ones ('$', '' levels, deep, root wildcards), and
    topics that hit every routing case."""
    p = gen.IotParams(seed=seed, n_filters=3000, n_ids=400)
    F = gen.gen_iot_filters(p).tolist()
    rng = random.Random(seed)
    W = [b"device", b"d1", b"d2", b"d7", b"sensor", b"s3", b"m1", b"", b"$SYS", b"x", b"y"]
    extra = set()
    for _ in range(600):
        ws = [rng.choice(W + [b"+"]) for _ in range(rng.randint(1, 12))]
        if rng.random() < 0.4:
            ws[-1] = b"#"
        extra.add(b"/".join(ws))
    F = F + sorted(extra - set(F))
    T = gen.gen_iot_topics(p, seed + 100, 1500).tolist()
    for _ in range(500):
        T.append(b"/".join(rng.choice(W + [b"zz"]) for _ in range(rng.randint(1, 14))))
    T += [b"", b"/", b"$SYS", b"$SYS/x/y", b"device", b"device/d1", b"zz/d1/sensor", b"$zz/d1"]
    vocab = sorted({w for f in F for w in f.split(b"/")} - {b"", b"+", b"#"})
    return F, T, vocab


def main(rank, world, port, seed, mode="cpu"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F, T_all, vocab = workload(seed)
    G = world
    gpu = mode == "gpu"
    eng = Engine(device=0 if gpu else -1, frozen_dict=True)
    words_of = {W_EMPTY: b"", W_PLUS: b"+", W_HASH: b"#"}
    for k, w in enumerate(vocab):
        words_of[W_FIRST + k] = w

    # this shard's filters (tm_filter_shard) and the rule's restatement agree
    mine = []
    eng.dict_load(vocab)
    for f in F:
        s = eng.filter_shard(f, G)
        ws = f.split(b"/")
        ids = [W_EMPTY if w == b"" else W_PLUS if w == b"+" else W_HASH if w == b"#" else W_FIRST + vocab.index(w)
               for w in ws[:2]]
        assert s == shard_rule(ids, G) if len(ws) >= 2 else s == G, (f, s)
        if s in (rank, G):
            mine.append(f)
    n_ins = eng.insert_many(F, rank, G)
    assert n_ins == len(mine), (n_ins, len(mine))

    orc = P.Oracle()
    for f in mine:
        orc.register(f)
        orc.insert(f)

    def shard_fn(words, toff, n):
        w = words.numpy().view(np.uint32)
        o = toff.numpy()
        out = np.empty(n, np.int64)
        for t in range(n):
            ids = [int(x) & WID_MASK for x in w[o[t]:o[t + 1]][:2]]
            out[t] = shard_rule(ids, G)
        return torch.from_numpy(out)

    def local_match(words, toff, tflags):
        w = words.numpy().view(np.uint32)
        o = toff.numpy()
        fl = tflags.numpy()
        topics = []
        for t in range(len(o) - 1):
            parts = []
            for k, x in enumerate(w[o[t]:o[t + 1]]):
                i = int(x) & WID_MASK
                if i == W_UNKNOWN:
                    parts.append(b"$\x01?" if (k == 0 and fl[t] & 1) else b"\x01?")
                else:
                    parts.append(words_of[i])
            topics.append(b"/".join(parts))
        buf, offs = P.pack(topics)
        counts, idx, _ = orc.match_batch(buf, offs)
        gids = [eng.filter_id(mine[int(j)]) * G + rank for j in idx]
        return (torch.tensor(counts.astype(np.int64), dtype=torch.int32),
                torch.tensor(np.array(gids, dtype=np.int64), dtype=torch.int32))

    if gpu:     # the production path: HIP shard kernel + device walk, exchange staged over gloo
        sm = ShardedMatcher(eng, rank, world)
    else:
        sm = ShardedMatcher(eng, rank, world, shard_fn=shard_fn, local_match=local_match)
    check_step(sm, eng, F, T_all, mine, rank, world, gpu)

    # online churn under the frozen dictionary: subscribes that bring new
    # literal words (in levels 0/1, so they pick a shard, and deeper), and
    # unsubscribes; every rank applies the same batches
    rng = random.Random(seed + 7)
    new_f = sorted({b"/".join([b"nw%d" % rng.randrange(40), rng.choice([b"d1", b"nx%d" % rng.randrange(9), b"+"]),
                               rng.choice([b"#", b"k%d" % rng.randrange(5), b"sensor"])]) for _ in range(300)}
                   | {b"device/nz%d/#" % k for k in range(20)} | {b"+/+/q%d" % k for k in range(10)})
    new_f = [f for f in new_f if f not in set(F)]
    gone = F[::7]
    new_words = sm.missing_words(new_f)
    assert new_words and len(set(new_words)) == len(new_words)
    n_new = sm.subscribe(new_f)
    sm.unsubscribe(gone)
    F2 = [f for f in F if f not in set(gone)] + new_f
    # the appended words got the same ids on every rank
    wid = torch.from_numpy(eng.tokenize(new_words).words.view(np.int32).copy())
    all_wid = [torch.empty_like(wid) for _ in range(world)]
    dist.all_gather(all_wid, wid)
    assert all(torch.equal(all_wid[0], x) for x in all_wid), "dictionary deltas diverged"
    assert (wid & WID_MASK).min() >= W_FIRST + len(vocab)
    for k, w in enumerate(new_words):
        words_of[W_FIRST + len(vocab) + k] = w
    mine2 = [f for f in F2 if eng.filter_shard(f, G) in (rank, G)]
    assert n_new == sum(1 for f in new_f if f in set(mine2))
    assert eng.stats()["filters"] == len(mine2)
    mine[:] = mine2
    orc.__init__()
    for f in mine:
        orc.register(f)
        orc.insert(f)
    T2 = T_all + [b"/".join([b"nw%d" % rng.randrange(40), rng.choice([b"d1", b"nx%d" % rng.randrange(9), b"zz"]),
                             rng.choice([b"k%d" % rng.randrange(5), b"sensor", b"zz"])]) for _ in range(600)]
    T2 += [b"device/nz%d/a/b" % k for k in range(20)] + [b"x/y/q%d" % k for k in range(10)]
    check_step(sm, eng, F2, T2, mine, rank, world, gpu)
    dist.barrier()
    dist.destroy_process_group()


def check_step(sm, eng, F, T_all, mine, rank, world, gpu):
    """One exchange step over this rank's slice of T_all; rows must equal the
    oracle's over the full filter set F."""
    G = world
    T = T_all[rank::world]
    tok = eng.tokenize(T)
    words = torch.from_numpy(tok.words.view(np.int32).copy())
    toff = torch.from_numpy(tok.toff.view(np.int32).copy())
    tflags = torch.from_numpy(tok.tflags.copy())
    if gpu:
        words, toff, tflags = words.cuda(), toff.cuda(), tflags.cuda()
    row_off, gids = sm.step(words, toff, tflags)
    row_off, gids = row_off.cpu(), gids.cpu()

    # gid -> bytes from every shard
    local_map = {eng.filter_id(f) * G + rank: f for f in mine}
    maps = [None] * world
    dist.all_gather_object(maps, local_map)
    gmap = {}
    for m in maps:
        gmap.update(m)

    full = P.Oracle()
    for f in F:
        full.register(f)
        full.insert(f)
    buf, offs = P.pack(T)
    counts, idx, _ = full.match_batch(buf, offs)
    cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    ro = row_off.numpy()
    g = gids.numpy().astype(np.int64) & 0xFFFFFFFF
    bad = []
    for t in range(len(T)):
        got = [gmap[int(x)] for x in g[ro[t]:ro[t + 1]]]
        exp = [F[int(j)] for j in idx[cut[t]:cut[t + 1]]]
        if got != exp:
            bad.append((T[t], got, exp))
    assert not bad, bad[:3]
    # the exchange really moved topics between the ranks
    moved = sum(sm.last["sent_topics"]) - sm.last["sent_topics"][rank]
    stats = torch.tensor([moved, len(T)], dtype=torch.int64)
    dist.all_reduce(stats)
    assert stats[0] > 0


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
         sys.argv[5] if len(sys.argv) > 5 else "cpu")
