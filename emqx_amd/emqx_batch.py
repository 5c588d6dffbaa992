"""emqx_batch mirror (src/emqx_batch.erl) + the publish batcher built on it.

`init/push/commit/size/items` keep the reference's semantics exactly:
  - the first push into an empty batch arms a linger timer that delivers the
    message 'batch_linger_expired' to the owner's mailbox (:56-62);
  - batch_size = 0 means no size limit (:64-66);
  - a push onto a batch already holding >= batch_size items commits all of
    them, i.e. commits happen at batch_size + 1 items (:68-70);
  - commit_fun receives the items in push order, then the batch is reset (:75-82).

`PublishBatcher` is the BASELINE's "publishes are batched through emqx_batch
into device topic arrays": commit_fun = one device match of the whole batch.
"""

from __future__ import annotations

import queue
import threading
from dataclasses import dataclass, field, replace
from typing import Any, Callable, List, Optional

LINGER_EXPIRED = "batch_linger_expired"
inbox: "queue.Queue" = queue.Queue()   # the calling process's mailbox (self())


@dataclass(frozen=True)
class Batch:
    batch_size: int
    linger_ms: int
    commit_fun: Callable[[List[Any]], Any]
    batch_q: tuple = ()                  # newest first, like the reference's list
    linger_timer: Optional[threading.Timer] = field(default=None, compare=False)
    mailbox: Any = field(default=None, compare=False)


def init(opts: dict) -> Batch:
    """init/1 (:49-54)"""
    return Batch(batch_size=opts.get("batch_size", 1000), linger_ms=opts.get("linger_ms", 1000),
                 commit_fun=opts["commit_fun"], mailbox=opts.get("mailbox", inbox))


def push(el, b: Batch) -> Batch:
    """push/2 (:56-73)"""
    if len(b.batch_q) == 0 and b.linger_timer is None:
        mb = b.mailbox
        t = threading.Timer(b.linger_ms / 1000.0, lambda: mb.put(LINGER_EXPIRED))
        t.daemon = True
        t.start()
        return replace(b, batch_q=(el,), linger_timer=t)
    if b.batch_size == 0:
        return replace(b, batch_q=(el,) + b.batch_q)
    if len(b.batch_q) >= b.batch_size:
        return commit(replace(b, batch_q=(el,) + b.batch_q))
    return replace(b, batch_q=(el,) + b.batch_q)


def commit(b: Batch) -> Batch:
    """commit/1 (:75-78)"""
    b.commit_fun(list(reversed(b.batch_q)))
    return reset(b)


def reset(b: Batch) -> Batch:
    """reset/1 (:80-82)"""
    if b.linger_timer is not None:
        b.linger_timer.cancel()
    return replace(b, batch_q=(), linger_timer=None)


def size(b: Batch) -> int:
    return len(b.batch_q)


def items(b: Batch):
    return list(reversed(b.batch_q))


class PublishBatcher:
    """Coalesces publishes (topics) with emqx_batch semantics; each commit is one
    device batch (Engine.match_batch).  `on_result(topics, row_offsets, ids)` gets
    the CSR of sorted filter ids per topic.  Thread-safe; linger commits run on
    the timer thread."""

    def __init__(self, engine, on_result, batch_size=65536, linger_ms=1):
        self.engine = engine
        self.on_result = on_result
        self._mb = queue.Queue()
        self._lock = threading.Lock()
        self._b = init({"batch_size": batch_size, "linger_ms": linger_ms,
                        "commit_fun": self._commit, "mailbox": self._mb})
        self._stop = threading.Event()
        self._thr = threading.Thread(target=self._linger_loop, daemon=True)
        self._thr.start()

    def _commit(self, topics):
        if topics:
            offs, ids = self.engine.match_batch(topics)
            self.on_result(topics, offs, ids)

    def publish(self, topic: bytes):
        with self._lock:
            self._b = push(topic, self._b)

    def flush(self):
        with self._lock:
            if size(self._b):
                self._b = commit(self._b)

    def _linger_loop(self):
        while not self._stop.is_set():
            try:
                msg = self._mb.get(timeout=0.05)
            except queue.Empty:
                continue
            if msg == LINGER_EXPIRED:
                self.flush()

    def close(self):
        self.flush()
        self._stop.set()
        self._thr.join(timeout=1)
