"""Filter-sharded mode (BASELINE config C4).

Subscription sets too large to replicate are partitioned over the G GPUs of a
node, one process (and one engine) per GPU:

* A filter whose first two levels are literal words lives on the shard
  hash(id(w0), id(w1)) mod G (`tm_filter_shard`); every other filter ('+'/'#'
  in level 0 or 1, or a single level) is replicated on all shards.
* A publish whose first two words are interned literals can only be matched by
  filters of that same shard or by replicated ones -- literal levels must be
  equal -- so the owner shard resolves it completely: no merge of partial match
  lists, and rows stay bit-exact (sorted, deduplicated).  Any other publish is
  resolved by the rank it arrived on.  This is the "partition by leading words,
  replicate root-wildcard filters" variant of SURVEY.md §8e.
* Word ids must mean the same on every shard: the engines run with a frozen
  dictionary (`TM_CFG_FROZEN_DICT`) loaded identically everywhere
  (`tm_dict_load`), so tokenised batches can be exchanged as u32 arrays.

One step over a rank's device-resident tokenised batch:
  1. owner per topic on the device (`tm_tokens_shard`);
  2. topics grouped by owner; `all_to_all_single` of the per-destination sizes,
     the per-topic (depth << 2 | flags) words and the word ids (RCCL over xGMI);
  3. the owner's engine matches what it received (HIP frontier kernel);
  4. `all_to_all_single` back of the per-topic counts and the global filter ids
     (gid = local filter id * G + owner rank, `tm_batch_export`);
  5. rows restored to the publish order.
Steps 2 and 4 are the only collectives; there is none in replicated mode.

Reference: the filter set is the mnesia-replicated trie (src/emqx_trie.erl:53-74)
that every node matches in full (src/emqx_router.erl:127-141); sharding it is new.
"""

from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from .engine import Batch, Engine

META_SHIFT = 2            # meta = depth << 2 | tflags (TF_DOLLAR = 1, TF_SLOW = 2)
WID_MASK = (1 << 29) - 1  # word id bits of a token (tm_internal.hpp WID_BITS)


def excl_cumsum(x: torch.Tensor) -> torch.Tensor:
    out = torch.zeros_like(x)
    if x.numel() > 1:
        out[1:] = torch.cumsum(x[:-1], 0)
    return out


def gather_segments(src: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor) -> torch.Tensor:
    """concat(src[starts[i] : starts[i] + lens[i]] for i) with int64 index math."""
    total = int(lens.sum().item()) if lens.numel() else 0
    if total == 0:
        return src[:0]
    seg = torch.repeat_interleave(torch.arange(lens.numel(), device=lens.device), lens)
    within = torch.arange(total, device=lens.device) - torch.repeat_interleave(excl_cumsum(lens), lens)
    return src[starts[seg] + within]


class ShardedMatcher:
    """One rank of the filter-sharded engine.

    engine:      this rank's Engine(frozen_dict=True) (a GPU engine in production).
    shard_fn / local_match: injection points for the multi-process CPU tests only
                 (gloo, no GPU); the production path uses the engine's HIP kernels and
                 refuses to run without a device.
    """

    def __init__(self, engine: Engine, rank: int, world: int, group=None, device: Optional[torch.device] = None,
                 shard_fn: Optional[Callable] = None, local_match: Optional[Callable] = None):
        self.eng = engine
        self.rank, self.world, self.group = rank, world, group
        self.dev = device if device is not None else (
            torch.device("cuda", engine.device) if engine.device >= 0 else torch.device("cpu"))
        self._shard_fn = shard_fn
        self._local_match = local_match
        if engine.device < 0 and (shard_fn is None or local_match is None):
            raise RuntimeError("filter-sharded matching needs a HIP device (no CPU fallback)")
        self._batch: Optional[Batch] = None
        self.last = {}
        # gloo moves host tensors only: stage device tensors through host memory
        # (used when several ranks share one GPU in tests); RCCL takes them as is
        self._stage = (world > 1 and self.dev.type == "cuda" and dist.get_backend(group) == "gloo")

    # ---- loading -----------------------------------------------------------
    def load(self, vocab, filters) -> int:
        """Shared dictionary, then this shard's filters + the replicated ones."""
        self.eng.dict_load(vocab)
        return self.eng.insert_many(filters, self.rank, self.world)

    # ---- online subscribe / unsubscribe ---------------------------------------
    # Word ids must agree on every shard, so new literal words cannot be
    # interned by whichever rank happens to insert a filter first.  Every rank
    # applies the same subscribe stream (the replicated route table's events,
    # src/emqx_router_helper.erl / emqx_trie:insert/1 on each node), so the
    # words a batch introduces -- collected in first-appearance order -- are
    # appended to each rank's dictionary before its filters go in: an
    # append-only dictionary delta that gives every rank the same new ids
    # (tm_dict_load assigns ids in order), then each rank keeps its own shard.
    def missing_words(self, filters) -> list:
        """Literal words of `filters` absent from the shared dictionary, in
        first-appearance order (tm_tokenize marks them UNKNOWN)."""
        fl = list(filters)
        if not fl:
            return []
        tok = self.eng.tokenize(fl)
        ids = tok.words & WID_MASK
        unknown = np.nonzero(ids == 0)[0]
        if unknown.size == 0:
            return []
        toff = tok.toff.astype(np.int64)
        which = np.searchsorted(toff, unknown, side="right") - 1   # filter of each unknown word
        out, seen = [], set()
        for i, w in zip(which.tolist(), unknown.tolist()):
            word = fl[i].split(b"/")[w - int(toff[i])]
            if word not in seen:
                seen.add(word)
                out.append(word)
        return out

    def subscribe(self, filters) -> int:
        """emqx_trie:insert/1 of a subscribe batch, called with the same batch on
        every rank: dictionary delta first, then this shard's filters and the
        replicated ones.  Returns how many this rank inserted."""
        new = self.missing_words(filters)
        if new:
            self.eng.dict_load(new)
        return self.eng.insert_many(filters, self.rank, self.world)

    def unsubscribe(self, filters) -> int:
        """emqx_trie:delete/1 of an unsubscribe batch on every rank (filters of
        other shards are absent here: no-ops).  Words stay interned."""
        return self.eng.delete_many(filters)

    # ---- device pieces -------------------------------------------------------
    def _shards(self, words: torch.Tensor, toff: torch.Tensor, n: int) -> torch.Tensor:
        if self._shard_fn is not None:
            return self._shard_fn(words, toff, n)
        out = torch.empty(n, dtype=torch.int32, device=self.dev)
        if n:
            torch.cuda.current_stream(self.dev).synchronize()
            self.eng.tokens_shard(words.data_ptr(), toff.data_ptr(), n, self.world, out.data_ptr())
        return out

    def _match(self, words: torch.Tensor, toff: torch.Tensor, tflags: torch.Tensor):
        if self._local_match is not None:
            return self._local_match(words, toff, tflags)
        m = toff.numel() - 1
        torch.cuda.current_stream(self.dev).synchronize()
        self._batch = self.eng.prepare_tokens(words.data_ptr() if words.numel() else toff.data_ptr(),
                                              toff.data_ptr(), tflags.data_ptr() if m else toff.data_ptr(),
                                              m, int(words.numel()), True, self._batch)
        self._batch.launch().wait()
        st = self._batch.stats()
        self.last["ms_match"] = st["ms_match"]
        self.last["ms_total"] = st["ms_total"]
        total = int(st["matches"])
        counts = torch.empty(m, dtype=torch.int32, device=self.dev)
        gids = torch.empty(total, dtype=torch.int32, device=self.dev)
        self._batch.export(counts.data_ptr(), gids.data_ptr(), self.world, self.rank)
        return counts, gids

    def _a2a(self, x: torch.Tensor, send: list, recv: list) -> torch.Tensor:
        out = torch.empty(sum(recv), dtype=x.dtype, device=x.device)
        if self.world == 1:
            out.copy_(x)
            return out
        if self._stage:
            h = torch.empty(sum(recv), dtype=x.dtype)
            dist.all_to_all_single(h, x.contiguous().cpu(), recv, send, group=self.group)
            return h.to(x.device)
        dist.all_to_all_single(out, x.contiguous(), recv, send, group=self.group)
        return out

    def _gather(self, src: torch.Tensor, src_off: torch.Tensor, idx: torch.Tensor, lens: torch.Tensor,
                total: int):
        """Rows src[src_off[idx[i]] .. src_off[idx[i]+1]) concatenated -> (dst, dst_off int64 [n+1]);
        total = sum(lens), known on the host from the exchanged sizes (no sync here)."""
        n = idx.numel()
        dst_off = torch.zeros(n + 1, dtype=torch.int64, device=src.device)
        if n:
            dst_off[1:] = torch.cumsum(lens, 0)
        if self._local_match is not None or src.device.type != "cuda":   # CPU tests
            return gather_segments(src, src_off[idx], lens), dst_off
        dst = torch.empty(total, dtype=src.dtype, device=src.device)
        if n and total:
            torch.cuda.current_stream(src.device).synchronize()
            self.eng.gather_rows(src.data_ptr(), src_off.data_ptr(), idx.data_ptr(), n, dst_off.data_ptr(),
                                 dst.data_ptr())
        return dst, dst_off

    # ---- one step ------------------------------------------------------------
    def step(self, words: torch.Tensor, toff: torch.Tensor, tflags: torch.Tensor):
        """words int32 (u32 bits), toff int32 [n+1], tflags uint8 [n], all on this
        rank's device.  Returns (row_off int64 [n+1], gids int32) in publish order:
        row t = the sorted, deduplicated global ids of the filters matching topic t."""
        G, dev = self.world, self.dev
        n = toff.numel() - 1
        if G == 1:   # one shard holds every filter: no exchange, no reorder
            counts, gids = self._match(words, toff, tflags)
            row_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            if n:
                row_off[1:] = torch.cumsum(counts.to(torch.int64), 0)
            self.last.update(sent_topics=[n], recv_topics=[n], local_matches=int(gids.numel()))
            return row_off, gids
        shard = self._shards(words, toff, n).to(torch.int64)
        owner = torch.where(shard == G, torch.full_like(shard, self.rank), shard)
        # publishes grouped per destination: a stable sort by owner keeps the
        # publish order within each group (no per-owner host round trip)
        order = torch.argsort(owner, stable=True)
        toff64 = toff.to(torch.int64)
        depth = toff64[1:] - toff64[:-1]
        depth_o = depth[order]
        send_t = torch.bincount(owner, minlength=G)
        send_w = torch.zeros(G, dtype=torch.int64, device=dev).scatter_add_(0, owner, depth)
        meta_o = ((depth_o << META_SHIFT) | tflags[order].to(torch.int64)).to(torch.int32)

        # the split sizes must be host values for all_to_all: one copy out for
        # ours, one back for the peers'
        sizes = torch.stack([send_t, send_w], 1)
        hsz = sizes.cpu()
        st, sw = hsz[:, 0].tolist(), hsz[:, 1].tolist()
        words_o, _ = self._gather(words, toff64, order, depth_o, sum(sw))
        hs = hsz if self._stage else sizes
        rsizes = torch.empty_like(hs)
        dist.all_to_all_single(rsizes, hs, group=self.group)
        hr = rsizes.cpu()
        rt, rw = hr[:, 0].tolist(), hr[:, 1].tolist()
        r_meta = self._a2a(meta_o, st, rt)
        r_words = self._a2a(words_o, sw, rw)

        r_depth = (r_meta >> META_SHIFT).to(torch.int64)
        r_toff = torch.zeros(r_meta.numel() + 1, dtype=torch.int32, device=dev)
        if r_meta.numel():
            r_toff[1:] = torch.cumsum(r_depth, 0).to(torch.int32)
        r_flags = (r_meta & 3).to(torch.uint8)
        counts, gids = self._match(r_words, r_toff, r_flags)

        # back to the origins: counts per received topic, ids per source
        src = torch.repeat_interleave(torch.arange(G, device=dev), torch.tensor(rt, device=dev))
        back_g = torch.zeros(G, dtype=torch.int64, device=dev).scatter_add_(0, src, counts.to(torch.int64))
        counts_o = self._a2a(counts, rt, st)
        c_o = counts_o.to(torch.int64)
        recv_g = torch.zeros(G, dtype=torch.int64, device=dev).scatter_add_(0, owner[order], c_o)
        bg, rg = torch.stack([back_g, recv_g]).cpu().tolist()   # one copy out for both splits
        gids_o = self._a2a(gids, bg, rg)

        # publish order
        counts_orig = torch.empty(n, dtype=torch.int64, device=dev)
        counts_orig[order] = c_o
        inv = torch.empty_like(order)
        inv[order] = torch.arange(n, device=dev)
        off_o = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        if n:
            off_o[1:] = torch.cumsum(c_o, 0)
        gids_final, row_off = self._gather(gids_o, off_o, inv, counts_orig, sum(rg))
        self.last.update(sent_topics=st, recv_topics=rt, local_matches=int(gids.numel()))
        return row_off, gids_final

    # ---- filter bytes of a global id ------------------------------------------
    def owns(self, gid: int) -> bool:
        return gid % self.world == self.rank

    def filter_bytes(self, gid: int) -> bytes:
        if not self.owns(gid):
            raise KeyError(f"gid {gid} belongs to rank {gid % self.world}")
        return self.eng.filter_bytes(gid // self.world)
