"""Bit-exact sample check of multi-device results against one replica on
device 0 (bench.py at N > 1, the in-process groups).

The replicated configs (C3) split a batch over devices and never bring the
rows together, so nothing would notice a device returning wrong rows.  After
the timed region every slice (or shard) takes an evenly spaced sample of
>= 3,000 of its publishes and digests each row as its filters' bytes -- ids
are local to an engine, bytes are not -- and a one-replica engine on device 0
matches the same publishes and must produce the same digests.  The reference
returns the same set for a topic on every node (src/emqx_trie.erl:53-74: the
trie is replicated; src/emqx_router.erl:127-141: every publish is matched in
full), which is exactly what is compared.
"""

from __future__ import annotations

import hashlib
import json

import numpy as np

SAMPLE = 3000


def sample_index(n: int, k: int = SAMPLE) -> np.ndarray:
    """k evenly spaced row indices of [0, n) (every row when n <= k), always
    including the first and last rows."""
    if n <= k:
        return np.arange(n, dtype=np.int64)
    return np.unique(np.linspace(0, n - 1, k).astype(np.int64))


def digest(row) -> str:
    """A row (filter byte strings, in order) -> hex digest; order matters."""
    h = hashlib.sha1()
    for f in row:
        h.update(len(f).to_bytes(4, "little"))
        h.update(f)
    return h.hexdigest()


def rows_from_csr(offs, ids, idx, names) -> list:
    """Sampled rows of a CSR as byte strings; names(ids array) -> {id: bytes}."""
    want = np.unique(np.concatenate([ids[int(offs[i]):int(offs[i + 1])] for i in idx])) if len(idx) else []
    name = names(want)
    return [[name[int(x)] for x in ids[int(offs[i]):int(offs[i + 1])]] for i in idx]


def engine_names(eng):
    """names() for an Engine: one bulk tm_filters_copy call."""
    def names(ids):
        ids = np.asarray(ids, dtype=np.uint32)
        out = {}
        for j, b in eng.filters_copy(ids):
            out[int(ids[j])] = b
        return out
    return names


def payload(topics, rows, label: str) -> str:
    """One slice's sample: its publishes (hex) and row digests, as JSON."""
    return json.dumps({"label": label, "topics": [t.hex() for t in topics], "digests": [digest(r) for r in rows]})


def check(payloads, match_rows) -> dict:
    """payloads: one JSON string per slice; match_rows(topics) -> rows from the
    device-0 replica.  -> {"parity_sample_ok", "sampled_rows", "mismatches", "slices"}."""
    ok, total, bad = True, 0, []
    slices = []
    for p in payloads:
        d = json.loads(p)
        topics = [bytes.fromhex(t) for t in d["topics"]]
        rows = match_rows(topics)
        mism = [i for i, (r, dg) in enumerate(zip(rows, d["digests"])) if digest(r) != dg]
        if len(rows) != len(d["digests"]):
            mism.append(-1)
        total += len(topics)
        slices.append({"label": d["label"], "rows": len(topics), "mismatches": len(mism)})
        if mism:
            ok = False
            bad.extend((d["label"], topics[i].decode("latin-1")) for i in mism[:3] if i >= 0)
    return {"parity_sample_ok": ok and total > 0, "sampled_rows": total, "mismatches": bad[:10], "slices": slices}
