"""Config C5 of SURVEY.md §8d: high-fanout skew + churn.

10k hot topics receive 90 % of the publishes (Zipf 1.0 over the hot set); each
hot topic is matched by ~K distinct filters derived from it ("1M subs each"
collapses in the router to one route per (filter, node), src/emqx_router.erl:
115-118, so for matching it means many filters per hot topic).  Between
batches, `Churn` applies subscribe/unsubscribe deltas (emqx_trie:insert/1,
delete/1) that the engine uploads to the device before the next launch.
Batches are prepared with TM_BATCH_DEDUP, so each distinct topic is walked once.
"""

from __future__ import annotations

import random
from dataclasses import replace

from . import gen


def workload(p: gen.SkewParams, n_background_filters: int, n_publishes: int, seed: int = 5,
             background_pool: int = 200_000, p_hot: float = 0.9, batches: int = 0):
    """-> (all filters, hot-derived filters, hot topics, publishes) as gen.Strings;
    batches > 0: publishes is a list of that many batches, each a different
    draw (seed + 300 + j) over the same hot set and background pool."""
    hot, derived = gen.gen_skew(p)
    bp = replace(gen.C2, seed=seed + 100, n_filters=n_background_filters)
    background = gen.gen_filters(bp)
    pool = gen.gen_topics(bp, background, seed + 200, background_pool)
    allf = gen.Strings.from_list(derived.tolist() + background.tolist())
    if batches:
        pubs = [gen.gen_pick(hot, pool, seed + 300 + j, n_publishes, p_hot, 1.0) for j in range(batches)]
    else:
        pubs = gen.gen_pick(hot, pool, seed + 300, n_publishes, p_hot, 1.0)
    return allf, derived, hot, pubs


class Churn:
    """Subscribe/unsubscribe deltas over the hot-derived filters."""

    def __init__(self, hot: gen.Strings, derived, seed: int = 9):
        self.hot = hot.tolist()
        self.live = list(derived)
        self.live_set = set(self.live)
        self.rng = random.Random(seed)
        self.next_seed = seed * 1_000_003

    def step(self, n_deltas: int):
        """-> (deletes, inserts), half each, applied to the live set."""
        dels, adds = [], []
        for _ in range(n_deltas // 2):
            if not self.live:
                break
            i = self.rng.randrange(len(self.live))
            f = self.live[i]
            self.live[i] = self.live[-1]
            self.live.pop()
            self.live_set.discard(f)
            dels.append(f)
        while len(adds) < n_deltas - len(dels):
            self.next_seed += 1
            f = gen.derive_one(self.rng.choice(self.hot), self.next_seed)
            if f and f not in self.live_set:
                self.live_set.add(f)
                self.live.append(f)
                adds.append(f)
        return dels, adds

    @staticmethod
    def apply(engine, dels, adds):
        """Unsubscribes then subscribes (emqx_trie:delete/1, insert/1): one
        tm_trie_apply_many call where the engine has it (both lists planned
        together), else two bulk calls; dels / adds are lists of binaries or
        packed gen.Strings."""
        if hasattr(engine, "apply_many"):
            engine.apply_many(dels, adds)
            return
        if len(dels):
            engine.delete_many(dels)
        if len(adds):
            engine.insert_many(adds)
