"""Executable model of the device algorithm (tm_kernels.hip) -- test infrastructure.

It restates, in plain Python, what tm_match_tiles computes per tile: the LIFO
probe stack shared by 64 topics, the per-level 3-bit path-code digits, the
E/L_lo patch for empty words, the literal-'#' SKIPE rule, the $-root rule and
the LDS-capacity overflow.  CPU tests run it against the oracle so that the
ORDER scheme (path codes == Erlang binary order of filters) and the walk rules
are checked exhaustively without a GPU; the GPU tests then check the HIP code
against the same oracle.
"""

from __future__ import annotations

C_BELOW, C_BETWEEN, C_ABOVE, C_EMPTY = 0, 1, 2, 3
FAST_MAX_DEPTH = 10
DIG_L = {C_BELOW: 2, C_BETWEEN: 3, C_ABOVE: 4, C_EMPTY: 4}
DIG_H = {C_BELOW: 3, C_BETWEEN: 2, C_ABOVE: 2, C_EMPTY: 2}
DIG_P = {C_BELOW: 4, C_BETWEEN: 4, C_ABOVE: 3, C_EMPTY: 3}
PLUS, HASH, EMPTY = "+", "#", ""


def word_class(w: bytes):
    """-> (class, irregular)"""
    if w == b"":
        return C_EMPTY, False
    c = w[0]
    if w == b"+":
        return C_ABOVE, False
    if c == ord("+"):
        return C_ABOVE, True
    if c < ord("#"):
        return C_BELOW, False
    if c < ord("+"):
        return C_BETWEEN, False
    return C_ABOVE, False


class Model:
    """Trie as {(parent, word): child}; words are bytes with b'+'/b'#' as wildcards."""

    def __init__(self, filters):
        self.edges = {}
        self.topic = {}      # node -> filter bytes
        self.nid = 1
        for f in filters:
            self._insert(f)

    def _insert(self, f: bytes):
        n = 0
        for w in f.split(b"/"):
            c = self.edges.get((n, w))
            if c is None:
                c = self.nid
                self.nid += 1
                self.edges[(n, w)] = c
            n = c
        self.topic[n] = f

    def probe(self, n, w):
        return self.edges.get((n, w))

    def hterm(self, n):
        h = self.edges.get((n, b"#"))
        return self.topic.get(h) if h is not None else None

    def match_tile(self, topics, qcap=512, ocap=1 << 30):
        """Returns (rows, overflow).  rows[i] = filters sorted by path code."""
        put = lambda key, lvl, d: key | (d << (61 - 3 * lvl))  # noqa: E731
        stack, out, meta = [], [], []
        for ti, t in enumerate(topics):
            ws = t.split(b"/")
            d = len(ws)
            dollar = t[:1] == b"$"
            cls, _ = word_class(ws[0])
            meta.append(ws)
            if not dollar and self.hterm(0) is not None:
                out.append((ti, DIG_H[cls] << 61, self.hterm(0)))
            w0 = ws[0]
            if w0 == b"#":
                if not dollar and self.probe(0, b"#") is not None:
                    stack.append((ti, 0, b"#", DIG_L[cls] << 61, 1, d == 1))
            elif w0 != b"+":
                stack.append((ti, 0, w0, DIG_L[cls] << 61, 1, False))
            if not dollar and self.probe(0, b"+") is not None:
                stack.append((ti, 0, b"+", DIG_P[cls] << 61, 1, False))
        if len(stack) > qcap or len(out) > ocap:
            return None, True
        while stack:
            k = min(len(stack), 64)
            popped = stack[len(stack) - k:]
            del stack[len(stack) - k:]
            pushes, emits = [], []
            for (ti, parent, w, key, lc, skipe) in popped:
                c = self.probe(parent, w)
                if c is None:
                    continue
                ws = meta[ti]
                d = len(ws)
                if lc == d:
                    if not skipe and c in self.topic:
                        kk = key
                        wc, _ = word_class(ws[lc - 1])
                        sp = 61 - 3 * (lc - 1)
                        if wc == C_EMPTY and ((kk >> sp) & 7) == 4:
                            kk = (kk & ~(7 << sp)) | (1 << sp)
                        emits.append((ti, kk, self.topic[c]))
                    if self.hterm(c) is not None:
                        emits.append((ti, put(key, lc, 2), self.hterm(c)))
                    continue
                wh = ws[lc]
                cls, _ = word_class(wh)
                if self.hterm(c) is not None:
                    emits.append((ti, put(key, lc, DIG_H[cls]), self.hterm(c)))
                if wh == b"#":
                    if self.probe(c, b"#") is not None:
                        pushes.append((ti, c, b"#", put(key, lc, DIG_L[cls]), lc + 1, lc + 1 == d))
                elif wh != b"+":
                    pushes.append((ti, c, wh, put(key, lc, DIG_L[cls]), lc + 1, False))
                if self.probe(c, b"+") is not None:
                    pushes.append((ti, c, b"+", put(key, lc, DIG_P[cls]), lc + 1, False))
            if len(stack) + len(pushes) > qcap or len(out) + len(emits) > ocap:
                return None, True
            stack.extend(pushes)
            out.extend(emits)
        rows = [[] for _ in topics]
        for (ti, key, f) in out:
            rows[ti].append((key, f))
        return [[f for _, f in sorted(r, key=lambda x: x[0])] for r in rows], False

    def match(self, topics, tile=64, qcap=512, row_cap=128):
        """Device semantics: LDS stack of qcap probes per tile; rows longer than
        row_cap (K) and overflowed tiles are redone by the slow path."""
        rows, slow = [None] * len(topics), 0
        for i in range(0, len(topics), tile):
            idx = [j for j in range(i, min(i + tile, len(topics)))
                   if len(topics[j].split(b"/")) <= FAST_MAX_DEPTH
                   and not any(word_class(w)[1] for w in topics[j].split(b"/"))]
            slow += min(tile, len(topics) - i) - len(idx)   # deep/irregular: byte-sorted slow path
            fast = [topics[j] for j in idx]
            r, ovf = self.match_tile(fast, qcap=qcap)
            if ovf:
                r, _ = self.match_tile(fast, qcap=1 << 30, ocap=1 << 30)
                slow += len(fast)
            else:
                slow += sum(1 for row in r if len(row) > row_cap)
            for j, row in zip(idx, r):
                rows[j] = row
        return rows, slow
