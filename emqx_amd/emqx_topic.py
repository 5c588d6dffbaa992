"""emqx_topic mirror (src/emqx_topic.erl) -- topic algebra on the host.

Same function names, argument meaning and error behaviour as the reference:
errors raise `TopicError(reason)` where the reference calls error(Reason).
`match/2` goes through the C ABI predicate (tm_topic_match).  Batched matching
of publishes against a filter set is Engine.match_batch (the device path).
"""

from __future__ import annotations

import ctypes as C

from . import _native as N


class Atom(str):
    """Erlang atom stand-in for the words '' / '+' / '#'."""

    def __repr__(self):
        return f"'{str.__str__(self)}'"


EMPTY = Atom("")
PLUS = Atom("+")
HASH = Atom("#")
MAX_TOPIC_LEN = 4096   # src/emqx_topic.erl:45


class TopicError(Exception):
    def __init__(self, reason):
        self.reason = reason
        super().__init__(reason)


def _b(x) -> bytes:
    if isinstance(x, (bytes, bytearray)):
        return bytes(x)
    if isinstance(x, str):
        return x.encode()
    raise TypeError(x)


def tokens(topic: bytes):
    """src/emqx_topic.erl:150-154"""
    return _b(topic).split(b"/")


def word(w: bytes):
    """src/emqx_topic.erl:161-164"""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic: bytes):
    """src/emqx_topic.erl:156-159"""
    return [word(w) for w in tokens(topic)]


def levels(topic: bytes) -> int:
    """src/emqx_topic.erl:146-148"""
    return len(tokens(topic))


def _is_atom(w, a):
    return isinstance(w, Atom) and str.__eq__(w, a) and w is a


def wildcard(topic) -> bool:
    """src/emqx_topic.erl:52-62"""
    if isinstance(topic, (bytes, bytearray)):
        return bool(N.lib().tm_topic_wildcard(bytes(topic), len(topic)))
    return any(w is PLUS or w is HASH for w in topic)


def bin_(w) -> bytes:
    """src/emqx_topic.erl:140-144"""
    if w is EMPTY:
        return b""
    if w is PLUS:
        return b"+"
    if w is HASH:
        return b"#"
    if isinstance(w, str):
        return w.encode()
    return bytes(w)


def join(ws) -> bytes:
    """src/emqx_topic.erl:183-195"""
    return b"/".join(bin_(w) for w in ws)


def prepend(parent, w) -> bytes:
    """src/emqx_topic.erl:131-138"""
    if parent is None or parent == b"":
        return bin_(w)
    p = bin_(parent)
    if p.endswith(b"/"):
        return p + bin_(w)
    return p + b"/" + bin_(w)


def _words_match(n, f) -> bool:
    i = j = 0
    while True:
        if i == len(n) and j == len(f):
            return True
        if i < len(n) and j < len(f):
            a, b = n[i], f[j]
            same = (a is b) if isinstance(a, Atom) or isinstance(b, Atom) else a == b
            if same or b is PLUS:
                i += 1; j += 1
                continue
        if j + 1 == len(f) and f[j] is HASH:
            return True
        return False


def match(name, flt) -> bool:
    """src/emqx_topic.erl:65-87 (binaries via the C ABI; word lists in Python)."""
    if isinstance(name, (bytes, bytearray)) and isinstance(flt, (bytes, bytearray)):
        return bool(N.lib().tm_topic_match(bytes(name), len(name), bytes(flt), len(flt)))
    n = words(name) if isinstance(name, (bytes, bytearray)) else list(name)
    f = words(flt) if isinstance(flt, (bytes, bytearray)) else list(flt)
    return _words_match(n, f)


def validate(topic, kind=None) -> bool:
    """validate/1,2 -- src/emqx_topic.erl:90-127.  validate(T) == validate(filter, T);
    validate((kind, T)) and validate(T, kind) are both accepted."""
    if kind is None:
        if isinstance(topic, tuple):
            kind, topic = topic
        else:
            kind = "filter"
    if kind not in ("name", "filter"):
        raise TopicError("function_clause")
    t = _b(topic)
    reason = C.c_char_p()
    rc = N.lib().tm_topic_validate(1 if kind == "name" else 0, t, len(t), C.byref(reason))
    if rc != 0:
        raise TopicError(reason.value.decode())
    return True


def feed_var(var: bytes, val: bytes, topic: bytes) -> bytes:
    """src/emqx_topic.erl:173-181"""
    return join([val if w == var else w for w in words(topic)])


def systop(name, node=b"emqx@127.0.0.1") -> bytes:
    """src/emqx_topic.erl:166-171"""
    return b"$SYS/brokers/" + _b(node) + b"/" + _b(name)


def parse(topic_filter, options=None):
    """src/emqx_topic.erl:197-220 -> (filter, options)"""
    if isinstance(topic_filter, tuple):
        topic_filter, options = topic_filter
    opts = dict(options or {})
    tf = _b(topic_filter)
    if tf.startswith(b"$queue/"):
        if "share" in opts:
            raise TopicError(("invalid_topic_filter", tf))
        opts["share"] = b"$queue"
        return parse(tf[len(b"$queue/"):], opts)
    if tf.startswith(b"$share/"):
        if "share" in opts:
            raise TopicError(("invalid_topic_filter", tf))
        rest = tf[len(b"$share/"):]
        parts = rest.split(b"/", 1)
        if len(parts) == 1:
            raise TopicError(("invalid_topic_filter", tf))
        share, flt = parts
        if b"+" in share or b"#" in share:
            raise TopicError(("invalid_topic_filter", tf))
        opts["share"] = share
        return parse(flt, opts)
    return tf, opts
