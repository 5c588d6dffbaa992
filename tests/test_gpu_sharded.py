"""Filter-sharded mode on the MI355X: the HIP shard kernel, device-token
batches and the export kernel, one rank in-process and two ranks sharing the
GPU (exchange over gloo, staged through host memory)."""

import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from emqx_amd import gen
from emqx_amd.engine import Engine
from emqx_amd.sharded import ShardedMatcher
from oracle import pyoracle as P
from sharded_worker import shard_rule, workload, WID_MASK
from test_sharded import free_port

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_kernel_matches_host_rule():
    F, T, vocab = workload(5)
    eng = Engine(device=0, frozen_dict=True)
    eng.dict_load(vocab)
    tok = eng.tokenize(T)
    w = torch.from_numpy(tok.words.view(np.int32).copy()).cuda()
    o = torch.from_numpy(tok.toff.view(np.int32).copy()).cuda()
    for G in (1, 2, 3, 8):
        out = torch.empty(len(T), dtype=torch.int32, device="cuda")
        eng.tokens_shard(w.data_ptr(), o.data_ptr(), len(T), G, out.data_ptr())
        got = out.cpu().numpy()
        for t in range(len(T)):
            ids = [int(x) & WID_MASK for x in tok.words[tok.toff[t]:tok.toff[t + 1]][:2]]
            assert got[t] == shard_rule(ids, G), (T[t], G)


def test_device_token_batch_equals_byte_batch():
    F, T, vocab = workload(6)
    eng = Engine(device=0, frozen_dict=True)
    eng.dict_load(vocab)
    eng.insert_many(F)
    offs_b, ids_b = eng.match_batch(T)
    tok = eng.tokenize(T)
    w = torch.from_numpy(tok.words.view(np.int32).copy()).cuda()
    o = torch.from_numpy(tok.toff.view(np.int32).copy()).cuda()
    f = torch.from_numpy(tok.tflags.copy()).cuda()
    torch.cuda.synchronize()
    b = eng.prepare_tokens(w.data_ptr(), o.data_ptr(), f.data_ptr(), len(T), tok.nwords, True)
    b.launch().wait()
    offs_t, ids_t = b.result()
    assert np.array_equal(offs_b, offs_t) and np.array_equal(ids_b, ids_t)
    counts = torch.empty(len(T), dtype=torch.int32, device="cuda")
    gids = torch.empty(len(ids_t), dtype=torch.int32, device="cuda")
    b.export(counts.data_ptr(), gids.data_ptr(), 8, 5)
    assert np.array_equal(counts.cpu().numpy(), np.diff(offs_t.astype(np.int64)))
    assert np.array_equal(gids.cpu().numpy().astype(np.int64) & 0xFFFFFFFF, ids_t.astype(np.int64) * 8 + 5)
    # malformed device tokens are refused before any walk runs
    bad = o.clone()
    bad[3] = bad[-1] + 7
    torch.cuda.synchronize()
    with pytest.raises(Exception):
        eng.prepare_tokens(w.data_ptr(), bad.data_ptr(), f.data_ptr(), len(T), tok.nwords, True)


def test_sharded_step_single_rank():
    F, T, vocab = workload(7)
    eng = Engine(device=0, frozen_dict=True)
    sm = ShardedMatcher(eng, 0, 1)
    sm.load(vocab, F)
    tok = eng.tokenize(T)
    row_off, gids = sm.step(torch.from_numpy(tok.words.view(np.int32).copy()).cuda(),
                            torch.from_numpy(tok.toff.view(np.int32).copy()).cuda(),
                            torch.from_numpy(tok.tflags.copy()).cuda())
    ro, g = row_off.cpu().numpy(), gids.cpu().numpy()
    orc = P.Oracle()
    for f in F:
        orc.register(f)
        orc.insert(f)
    buf, offs = P.pack(T)
    counts, idx, _ = orc.match_batch(buf, offs)
    cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    for t in range(len(T)):
        assert [sm.filter_bytes(int(x)) for x in g[ro[t]:ro[t + 1]]] == [F[int(j)] for j in idx[cut[t]:cut[t + 1]]]


def test_sharded_two_ranks_share_the_gpu():
    port = free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=os.path.dirname(HERE))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "sharded_worker.py"), str(r), "2", str(port),
                               "13", "gpu"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=200)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r}:\n" + outs[r][-3000:]
