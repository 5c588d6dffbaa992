"""Exact rows for BASELINE config C5 at full scale (10k hot topics x K = 1000
derived filters, 10M+ filters): the trie oracle would take minutes and ~10 GB
to build, so the check splits the filter set by construction.

* Derived filters (emqx_amd/csrc/tm_gen.c derive()) have >= 3 literal levels,
  and their literal words are the hot topics' "h<l>_<k>" words, which name
  their level.  For a hot topic t (every level literal, depth 10) a derived
  filter f matches iff every literal word of f is a word of t -- '+' matches
  any word and '#' any remaining levels (emqx_topic:match/2,
  src/emqx_topic.erl:74-87).  An inverted index word -> filters answers that
  for all 10M filters at once (a filter matches when the postings of t's
  words hit it as often as it has literal words).
* No derived filter can match a background topic: background words are
  "w<l>_<k>" or random words over alnum + '!' '%' (no '_'), never "h<l>_<k>".
* Background filters (100k C2-style) go through the trie oracle
  (oracle/tm_oracle.c) for every sampled topic; filters added by churn after
  the index was built go through the brute-force emqx_topic:match/2 batch.
Test infrastructure only: the checker of tests/test_gpu_skew_full.py,
tests/test_skew.py and of bench.py's C5 self-check (after its timed region)."""

from __future__ import annotations

import numpy as np

from oracle import pyoracle as P

LEVELS = 16      # level digit of "h<l>_<k>" (hot_depth <= 10)
VOCAB = 128      # k < vocab (64 in C5)


def _word_id(w: bytes) -> int:
    """h<l>_<k> -> l * VOCAB + k, anything else -> -1"""
    if len(w) >= 4 and w[0:1] == b"h" and w[2:3] == b"_" and w[1:2].isdigit() and w[3:].isdigit():
        return int(w[1:2]) * VOCAB + int(w[3:])
    return -1


class DerivedIndex:
    """Inverted index of packed derived filters (gen.Strings)."""

    def __init__(self, S):
        buf = np.asarray(S.buf)
        offs = np.asarray(S.offs).astype(np.int64)
        n = len(offs) - 1
        self.S, self.n = S, n
        slash = np.flatnonzero(buf == ord("/")).astype(np.int64)
        starts = np.sort(np.concatenate([offs[:-1], slash + 1]))
        ends = np.sort(np.concatenate([slash, offs[1:]]))
        first = buf[np.minimum(starts, max(len(buf) - 1, 0))]
        lit = (first == ord("h")) & (ends > starts)
        s, e = starts[lit], ends[lit]
        lvl = buf[s + 1].astype(np.int64) - 48
        d0 = buf[s + 3].astype(np.int64) - 48
        d1 = np.where(e - s >= 5, buf[np.minimum(s + 4, len(buf) - 1)].astype(np.int64) - 48, -1)
        k = np.where(d1 >= 0, d0 * 10 + d1, d0)
        assert ((e - s) <= 5).all() and (lvl >= 0).all() and (lvl < LEVELS).all() and (k < VOCAB).all()
        wid = lvl * VOCAB + k
        fidx = np.searchsorted(offs, s, side="right") - 1
        self.nlit = np.bincount(fidx, minlength=n).astype(np.int32)
        order = np.argsort(wid.astype(np.int16), kind="stable")   # (radix sort: wid < 2^11)
        self.post = fidx[order].astype(np.int64)
        self.post_off = np.concatenate([[0], np.cumsum(np.bincount(wid, minlength=LEVELS * VOCAB))]).astype(np.int64)
        self.alive = np.ones(n, bool)

    def match(self, topic: bytes) -> np.ndarray:
        """indices of the alive filters matching hot topic `topic`"""
        ids = [_word_id(w) for w in topic.split(b"/")]
        if any(i < 0 for i in ids):
            return np.zeros(0, np.int64)
        parts = [self.post[self.post_off[i]:self.post_off[i + 1]] for i in ids]
        if not parts:
            return np.zeros(0, np.int64)
        # postings per filter by sorting the ~1M hits (a bincount over all n
        # filters costs ~2x that at 10M filters, np.add.at ~6x)
        s = np.sort(np.concatenate(parts))
        if not len(s):
            return np.zeros(0, np.int64)
        head = np.flatnonzero(np.concatenate([[True], s[1:] != s[:-1]]))
        u = s[head]
        cnt = np.diff(np.concatenate([head, [len(s)]]))
        return u[(cnt == self.nlit[u]) & self.alive[u]]

    def filter(self, i: int) -> bytes:
        return bytes(self.S.buf[int(self.S.offs[i]):int(self.S.offs[i + 1])])


class SnapshotOracle:
    """Expected rows for C5 topics on the current snapshot: derived filters
    (indexed base set + churn additions), background filters (trie oracle)."""

    def __init__(self, derived, background):
        self.idx = DerivedIndex(derived)
        self.pos = {}
        for i in range(self.idx.n):   # filter -> base index, for deletes
            self.pos[self.idx.filter(i)] = i
        self.extra = set()             # derived filters added after the index was built
        self.bg = P.Oracle()
        self.background = list(background)
        for f in self.background:
            self.bg.register(f)
            self.bg.insert(f)

    def delete(self, f: bytes):
        i = self.pos.get(f)
        if i is not None and self.idx.alive[i]:
            self.idx.alive[i] = False
        else:
            self.extra.discard(f)

    def insert(self, f: bytes):
        i = self.pos.get(f)
        if i is not None:
            self.idx.alive[i] = True
        else:
            self.extra.add(f)

    def rows(self, topics):
        buf, offs = P.pack(topics)
        counts, idx, _ = self.bg.match_batch(buf, offs, nthreads=8)
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        extra = sorted(self.extra)
        ecounts, eidx = P.brute_batch(extra, buf, offs, nthreads=8) if extra else (np.zeros(len(topics), np.uint32),
                                                                                  np.zeros(0, np.int64))
        ecut = np.concatenate([[0], np.cumsum(ecounts.astype(np.int64))])
        out = []
        for i, t in enumerate(topics):
            row = [self.background[int(j)] for j in idx[cut[i]:cut[i + 1]]]
            row += [extra[int(j)] for j in eidx[ecut[i]:ecut[i + 1]]]
            row += [self.idx.filter(int(j)) for j in self.idx.match(t)]
            out.append(sorted(row))   # Erlang binary order: unsigned bytes, shorter prefix first
        return out

    def close(self):
        self.bg.close()


class FinalSnapshot:
    """Expected rows for C5 topics on ONE snapshot given by its live set,
    without replaying the churn (bench.py's C5 self-check, after the timed
    region): live = the derived filters alive now (skew.Churn.live_set),
    added = every filter the churn subscribed (some may be gone again).  A
    base derived filter found by the index counts when it is in `live`; the
    added ones that are live go through brute-force emqx_topic:match/2; the
    row is the set union (a base filter deleted and subscribed again is
    listed once), sorted.  Background filters: the trie oracle."""

    def __init__(self, derived, background, live, added, nthreads=8):
        self.idx = DerivedIndex(derived)
        self.live = live
        self.extra = sorted({f for f in added if f in live})
        self.nthreads = nthreads
        self.bg = P.Oracle()
        self.background = list(background)
        for f in self.background:
            self.bg.register(f)
            self.bg.insert(f)

    def rows(self, topics):
        buf, offs = P.pack(topics)
        counts, idx, _ = self.bg.match_batch(buf, offs, nthreads=self.nthreads)
        cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
        ex = self.extra
        if ex:
            ecounts, eidx = P.brute_batch(ex, buf, offs, nthreads=self.nthreads)
        else:
            ecounts, eidx = np.zeros(len(topics), np.uint32), np.zeros(0, np.int64)
        ecut = np.concatenate([[0], np.cumsum(ecounts.astype(np.int64))])
        out = []
        for i, t in enumerate(topics):
            row = {self.background[int(j)] for j in idx[cut[i]:cut[i + 1]]}
            row.update(ex[int(j)] for j in eidx[ecut[i]:ecut[i + 1]])
            row.update(f for f in (self.idx.filter(int(j)) for j in self.idx.match(t)) if f in self.live)
            out.append(sorted(row))   # Erlang binary order: unsigned bytes, shorter prefix first
        return out

    def close(self):
        self.bg.close()
