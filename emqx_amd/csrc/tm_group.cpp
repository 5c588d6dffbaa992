// tm_group.cpp -- replicated multi-device matching in one process (BASELINE
// config C3: "1M filters replicated, publish batches split across 2/4/8
// MI355X, no collective").
//
// A group owns one engine (trie replica) per listed device.  The reference
// keeps a full copy of the emqx_trie tables on every node
// (src/emqx_trie.erl:53-74); here every mutation is applied to every replica
// in the same order, so node / filter ids agree across replicas and a batch
// split into contiguous slices (one per replica, no data-path collective)
// concatenates back into one CSR.  Built only on the engine's public C ABI.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/emqx_tm.h"

struct tm_group_batch {
    uint32_t n = 0;
    std::vector<uint32_t> lo;              // slice k = publishes [lo[k], lo[k + 1])
    std::vector<tm_batch*> parts;          // one per replica
    std::vector<uint32_t> row_offsets;     // merged CSR
    std::vector<uint32_t> filter_ids;
};

struct tm_group {
    std::vector<tm_engine*> engines;
    std::mutex mu;                         // orders mutations: the replicas see one sequence
    bool diverged = false;                 // a mutation returned different codes on two replicas
    tm_group_batch* last = nullptr;        // tm_group_match_batch's batch (its CSR outlives the call)
};

namespace {

// Runs f(engine index) on every replica, in parallel when there are several.
template <class F>
void each(tm_group* g, F f) {
    const size_t k = g->engines.size();
    if (k == 1) {
        f(0);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(k);
    for (size_t i = 0; i < k; ++i) th.emplace_back([&f, i] { f(i); });
    for (auto& t : th) t.join();
}

// Same mutation on every replica; replicas are identical, so the codes agree.
template <class F>
int mutate(tm_group* g, F f) {
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->diverged) return TM_EIO;
    std::vector<int> rc(g->engines.size(), TM_OK);
    each(g, [&](size_t i) { rc[i] = f(i); });
    for (int r : rc)
        if (r != rc[0]) {
            g->diverged = true;
            return TM_EIO;
        }
    return rc[0];
}

}  // namespace

extern "C" {

int tm_group_create(const int32_t* devices, uint32_t n, const tm_config* cfg, tm_group** out) {
    if (!devices || !n || !out) return TM_EINVAL;
    tm_group* g = new (std::nothrow) tm_group();
    if (!g) return TM_ENOMEM;
    for (uint32_t i = 0; i < n; ++i) {
        tm_config c = cfg ? *cfg : tm_config{0, 0, 0, 0};
        c.device = devices[i];
        if (c.device < 0) {
            tm_group_destroy(g);
            return TM_EINVAL;
        }
        tm_engine* e = nullptr;
        int rc = tm_create(&c, &e);
        if (rc) {
            tm_group_destroy(g);
            return rc;
        }
        g->engines.push_back(e);
    }
    *out = g;
    return TM_OK;
}

void tm_group_destroy(tm_group* g) {
    if (!g) return;
    if (g->last) tm_group_batch_free(g, g->last);
    for (tm_engine* e : g->engines) tm_destroy(e);
    delete g;
}

uint32_t tm_group_size(tm_group* g) { return g ? (uint32_t)g->engines.size() : 0; }

tm_engine* tm_group_engine(tm_group* g, uint32_t i) {
    return (g && i < g->engines.size()) ? g->engines[i] : nullptr;
}

int tm_group_trie_insert(tm_group* g, const uint8_t* t, size_t len) {
    if (!g) return TM_EINVAL;
    return mutate(g, [&](size_t i) { return tm_trie_insert(g->engines[i], t, len); });
}

int tm_group_trie_delete(tm_group* g, const uint8_t* t, size_t len) {
    if (!g) return TM_EINVAL;
    return mutate(g, [&](size_t i) { return tm_trie_delete(g->engines[i], t, len); });
}

int tm_group_insert_many(tm_group* g, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                         uint64_t* n_inserted) {
    if (!g) return TM_EINVAL;
    std::vector<uint64_t> done(g->engines.size(), 0);
    int rc = mutate(g, [&](size_t i) { return tm_trie_insert_many(g->engines[i], filters, offsets, n, 0, 1, &done[i]); });
    if (n_inserted) *n_inserted = done[0];
    return rc;
}

int tm_group_route_apply(tm_group* g, const uint8_t* topics, const uint64_t* offsets, const uint32_t* dests,
                         const uint8_t* ops, uint32_t n, uint64_t* n_changed) {
    if (!g) return TM_EINVAL;
    std::vector<uint64_t> ch(g->engines.size(), 0);
    int rc = mutate(g, [&](size_t i) { return tm_route_apply(g->engines[i], topics, offsets, dests, ops, n, &ch[i]); });
    if (n_changed) *n_changed = ch[0];
    return rc;
}

int tm_group_sync(tm_group* g) {
    if (!g) return TM_EINVAL;
    std::vector<int> rc(g->engines.size(), TM_OK);
    each(g, [&](size_t i) { rc[i] = tm_sync(g->engines[i]); });
    for (int r : rc)
        if (r) return r;
    return TM_OK;
}

int tm_group_prepare(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                     tm_group_batch** out) {
    if (!g || !offsets || !out || (!topics && n)) return TM_EINVAL;
    const size_t k = g->engines.size();
    const bool fresh = *out == nullptr;
    tm_group_batch* b = fresh ? new (std::nothrow) tm_group_batch() : *out;
    if (!b) return TM_ENOMEM;
    if (b->parts.size() != k) b->parts.assign(k, nullptr);
    b->n = n;
    b->lo.assign(k + 1, 0);
    for (size_t i = 0; i <= k; ++i) b->lo[i] = (uint32_t)((uint64_t)n * i / k);
    std::vector<int> rc(k, TM_OK);
    each(g, [&](size_t i) {
        const uint32_t lo = b->lo[i], cnt = b->lo[i + 1] - lo;
        rc[i] = tm_batch_prepare(g->engines[i], topics, offsets + lo, cnt, &b->parts[i]);
    });
    for (int r : rc)
        if (r) {
            if (fresh) tm_group_batch_free(g, b);
            return r;
        }
    b->row_offsets.clear();
    b->filter_ids.clear();
    *out = b;
    return TM_OK;
}

int tm_group_launch(tm_group* g, tm_group_batch* b) {
    if (!g || !b || b->parts.size() != g->engines.size()) return TM_EINVAL;
    // launches are asynchronous (one stream per replica): one thread issues all
    for (size_t i = 0; i < g->engines.size(); ++i) {
        int rc = tm_batch_launch(g->engines[i], b->parts[i]);
        if (rc) return rc;
    }
    return TM_OK;
}

int tm_group_wait(tm_group* g, tm_group_batch* b) {
    if (!g || !b || b->parts.size() != g->engines.size()) return TM_EINVAL;
    int first = TM_OK;
    for (size_t i = 0; i < g->engines.size(); ++i) {   // every slice is drained, even after an error
        int rc = tm_batch_wait(g->engines[i], b->parts[i]);
        if (rc && !first) first = rc;
    }
    return first;
}

int tm_group_result(tm_group* g, tm_group_batch* b, tm_result* out) {
    if (!g || !b || !out || b->parts.size() != g->engines.size()) return TM_EINVAL;
    const size_t k = g->engines.size();
    std::vector<tm_result> r(k);
    std::vector<int> rc(k, TM_OK);
    each(g, [&](size_t i) { rc[i] = tm_batch_result(g->engines[i], b->parts[i], &r[i]); });
    uint64_t total = 0;
    for (size_t i = 0; i < k; ++i) {
        if (rc[i]) return rc[i];
        total += r[i].n_matches;
    }
    if (total > 0xFFFFFFF0ull) return TM_EOVERFLOW;   // u32 CSR offsets
    b->row_offsets.resize((size_t)b->n + 1);
    b->filter_ids.resize(std::max<uint64_t>(total, 1));
    std::vector<uint64_t> base(k + 1, 0);
    for (size_t i = 0; i < k; ++i) base[i + 1] = base[i] + r[i].n_matches;
    each(g, [&](size_t i) {
        const uint32_t lo = b->lo[i], cnt = b->lo[i + 1] - lo, add = (uint32_t)base[i];
        for (uint32_t t = 0; t < cnt; ++t) b->row_offsets[lo + t] = r[i].row_offsets[t] + add;
        if (r[i].n_matches)
            memcpy(b->filter_ids.data() + base[i], r[i].filter_ids, r[i].n_matches * sizeof(uint32_t));
    });
    b->row_offsets[b->n] = (uint32_t)total;
    out->n_topics = b->n;
    out->n_matches = total;
    out->row_offsets = b->row_offsets.data();
    out->filter_ids = b->filter_ids.data();
    return TM_OK;
}

int tm_group_batch_stats(tm_group* g, tm_group_batch* b, tm_batch_stats* out) {
    if (!g || !b || !out || b->parts.size() != g->engines.size()) return TM_EINVAL;
    tm_batch_stats s{};
    for (size_t i = 0; i < g->engines.size(); ++i) {
        tm_batch_stats p{};
        int rc = tm_batch_stats_get(g->engines[i], b->parts[i], &p);
        if (rc) return rc;
        s.topics += p.topics; s.visits += p.visits; s.hash_hits += p.hash_hits; s.words += p.words;
        s.matches += p.matches; s.slow_topics += p.slow_topics; s.overflow_tiles += p.overflow_tiles;
        s.ms_match = std::max(s.ms_match, p.ms_match);
        s.ms_total = std::max(s.ms_total, p.ms_total);
        s.ms_tokenize = std::max(s.ms_tokenize, p.ms_tokenize);
        s.probes += p.probes;
    }
    *out = s;
    return TM_OK;
}

void tm_group_batch_free(tm_group* g, tm_group_batch* b) {
    if (!b) return;
    for (size_t i = 0; i < b->parts.size(); ++i)
        if (b->parts[i]) tm_batch_free(g && i < g->engines.size() ? g->engines[i] : nullptr, b->parts[i]);
    delete b;
}

int tm_group_match_batch(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_result* out) {
    if (!g || !out) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(g->mu);   // g->last is reused: one call at a time
    int rc = tm_group_prepare(g, topics, offsets, n, &g->last);
    if (rc) return rc;
    if (!(rc = tm_group_launch(g, g->last)) && !(rc = tm_group_wait(g, g->last))) rc = tm_group_result(g, g->last, out);
    return rc;
}

}  // extern "C"
