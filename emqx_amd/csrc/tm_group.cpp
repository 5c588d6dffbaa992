// tm_group.cpp -- the replicated multi-device group (BASELINE config C3: "1M
// filters replicated, publish batches split across 2/4/8 MI355X, no
// collective") as a view of ONE replicated engine.
//
// The reference keeps a full copy of the emqx_trie tables on every node
// (src/emqx_trie.erl:53-74).  Here the group's engine holds one host trie and
// one HBM replica per listed device (tm_create_replicated): a mutation is made
// once on the host and its delta uploaded to every device, so node / filter
// ids agree across devices by construction, and a batch split into contiguous
// slices (one per replica, no data-path collective) concatenates back into one
// CSR.  Every tm_* call on tm_group_engine(g, i) already spans the replicas
// (per-publish calls are dealt over them, whole batches split); the tm_group_*
// split form below keeps one slice per device explicit for callers that
// pipeline batches themselves.  Built only on the engine's public C ABI.
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
    std::vector<uint64_t> d_rows;          // merged deliveries (tm_group_dispatch)
    std::vector<uint32_t> d_subs;
    std::vector<uint32_t> s_off, s_ids;    // tm_group_sample's last result
};

struct tm_group {
    tm_engine* e = nullptr;
    std::mutex mu;                         // g->last is reused: one tm_group_match_batch at a time
    tm_group_batch* last = nullptr;
};

extern "C" {

int tm_group_create(const int32_t* devices, uint32_t n, const tm_config* cfg, tm_group** out) {
    if (!devices || !n || !out) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (devices[i] < 0) return TM_EINVAL;
    tm_group* g = new (std::nothrow) tm_group();
    if (!g) return TM_ENOMEM;
    tm_config c = cfg ? *cfg : tm_config{0, 0, 0, 0};
    c.device = devices[0];
    int rc = tm_create_replicated(&c, devices, n, &g->e);
    if (rc) {
        delete g;
        return rc;
    }
    *out = g;
    return TM_OK;
}

void tm_group_destroy(tm_group* g) {
    if (!g) return;
    if (g->last) tm_group_batch_free(g, g->last);
    tm_destroy(g->e);
    delete g;
}

uint32_t tm_group_size(tm_group* g) { return g ? tm_replica_count(g->e) : 0; }

tm_engine* tm_group_engine(tm_group* g, uint32_t i) {
    return (g && i < tm_replica_count(g->e)) ? g->e : nullptr;
}

int tm_group_trie_insert(tm_group* g, const uint8_t* t, size_t len) {
    return g ? tm_trie_insert(g->e, t, len) : TM_EINVAL;
}

int tm_group_trie_delete(tm_group* g, const uint8_t* t, size_t len) {
    return g ? tm_trie_delete(g->e, t, len) : TM_EINVAL;
}

int tm_group_insert_many(tm_group* g, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                         uint64_t* n_inserted) {
    return g ? tm_trie_insert_many(g->e, filters, offsets, n, 0, 1, n_inserted) : TM_EINVAL;
}

int tm_group_route_apply(tm_group* g, const uint8_t* topics, const uint64_t* offsets, const uint32_t* dests,
                         const uint8_t* ops, uint32_t n, uint64_t* n_changed) {
    return g ? tm_route_apply(g->e, topics, offsets, dests, ops, n, n_changed) : TM_EINVAL;
}

int tm_group_sync(tm_group* g) { return g ? tm_sync(g->e) : TM_EINVAL; }

int tm_group_prepare(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                     tm_group_batch** out) {
    if (!g || !offsets || !out || (!topics && n)) return TM_EINVAL;
    const size_t k = tm_replica_count(g->e);
    const bool fresh = *out == nullptr;
    tm_group_batch* b = fresh ? new (std::nothrow) tm_group_batch() : *out;
    if (!b) return TM_ENOMEM;
    if (b->parts.size() != k) b->parts.assign(k, nullptr);
    b->n = n;
    b->lo.assign(k + 1, 0);
    for (size_t i = 0; i <= k; ++i) b->lo[i] = (uint32_t)((uint64_t)n * i / k);
    for (size_t i = 0; i < k; ++i) {
        const uint32_t lo = b->lo[i], cnt = b->lo[i + 1] - lo;
        int rc = tm_batch_prepare_on(g->e, (uint32_t)i, topics, offsets + lo, cnt, 0, &b->parts[i]);
        if (rc) {
            if (fresh) tm_group_batch_free(g, b);
            return rc;
        }
    }
    b->row_offsets.clear();
    b->filter_ids.clear();
    *out = b;
    return TM_OK;
}

int tm_group_launch(tm_group* g, tm_group_batch* b) {
    if (!g || !b || b->parts.size() != tm_replica_count(g->e)) return TM_EINVAL;
    // launches are asynchronous (each replica's stream): one thread issues all
    for (tm_batch* p : b->parts) {
        int rc = tm_batch_launch(g->e, p);
        if (rc) return rc;
    }
    return TM_OK;
}

int tm_group_wait(tm_group* g, tm_group_batch* b) {
    if (!g || !b || b->parts.size() != tm_replica_count(g->e)) return TM_EINVAL;
    int first = TM_OK;
    for (tm_batch* p : b->parts) {   // every slice is drained, even after an error
        int rc = tm_batch_wait(g->e, p);
        if (rc && !first) first = rc;
    }
    return first;
}

int tm_group_result(tm_group* g, tm_group_batch* b, tm_result* out) {
    if (!g || !b || !out || b->parts.size() != tm_replica_count(g->e)) return TM_EINVAL;
    const size_t k = b->parts.size();
    std::vector<tm_result> r(k);
    uint64_t total = 0;
    for (size_t i = 0; i < k; ++i) {
        int rc = tm_batch_result(g->e, b->parts[i], &r[i]);
        if (rc) return rc;
        total += r[i].n_matches;
    }
    if (total > 0xFFFFFFF0ull) return TM_EOVERFLOW;   // u32 CSR offsets
    b->row_offsets.resize((size_t)b->n + 1);
    b->filter_ids.resize(std::max<uint64_t>(total, 1));
    std::vector<uint64_t> base(k + 1, 0);
    for (size_t i = 0; i < k; ++i) base[i + 1] = base[i] + r[i].n_matches;
    std::vector<std::thread> th;
    for (size_t i = 0; i < k; ++i)
        th.emplace_back([&, i] {
            const uint32_t lo = b->lo[i], cnt = b->lo[i + 1] - lo, add = (uint32_t)base[i];
            for (uint32_t t = 0; t < cnt; ++t) b->row_offsets[lo + t] = r[i].row_offsets[t] + add;
            if (r[i].n_matches)
                memcpy(b->filter_ids.data() + base[i], r[i].filter_ids, r[i].n_matches * sizeof(uint32_t));
        });
    for (auto& t : th) t.join();
    b->row_offsets[b->n] = (uint32_t)total;
    out->n_topics = b->n;
    out->n_matches = total;
    out->row_offsets = b->row_offsets.data();
    out->filter_ids = b->filter_ids.data();
    return TM_OK;
}

int tm_group_sample(tm_group* g, tm_group_batch* b, const uint32_t* publishes, uint32_t k, tm_result* out) {
    if (!g || !b || !out || (!publishes && k) || b->parts.size() != tm_replica_count(g->e)) return TM_EINVAL;
    const size_t np = b->parts.size();
    // each slice samples its own publishes (local row indices), in one call
    std::vector<std::vector<uint32_t>> local(np), where(np);
    for (uint32_t i = 0; i < k; ++i) {
        const uint32_t t = publishes[i];
        if (t >= b->n) return TM_EINVAL;
        const size_t s = (size_t)(std::upper_bound(b->lo.begin(), b->lo.end(), t) - b->lo.begin()) - 1;
        local[s].push_back(t - b->lo[s]);
        where[s].push_back(i);
    }
    std::vector<uint32_t> cnt(k, 0);
    std::vector<std::vector<uint32_t>> rows(k);
    for (size_t s = 0; s < np; ++s) {
        if (local[s].empty()) continue;
        tm_result r{};
        int rc = tm_batch_sample(g->e, b->parts[s], local[s].data(), (uint32_t)local[s].size(), &r);
        if (rc) return rc;
        for (size_t j = 0; j < local[s].size(); ++j)
            rows[where[s][j]].assign(r.filter_ids + r.row_offsets[j], r.filter_ids + r.row_offsets[j + 1]);
    }
    b->s_off.assign((size_t)k + 1, 0);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < k; ++i) {
        tot += rows[i].size();
        if (tot > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        b->s_off[i + 1] = (uint32_t)tot;
    }
    b->s_ids.clear();
    b->s_ids.reserve(std::max<uint64_t>(tot, 1));
    for (auto& r : rows) b->s_ids.insert(b->s_ids.end(), r.begin(), r.end());
    if (b->s_ids.empty()) b->s_ids.push_back(0);
    out->n_topics = k;
    out->n_matches = tot;
    out->row_offsets = b->s_off.data();
    out->filter_ids = b->s_ids.data();
    return TM_OK;
}

int tm_group_dispatch(tm_group* g, tm_group_batch* b, tm_deliveries* out) {
    if (!g || !b || !out || b->parts.size() != tm_replica_count(g->e)) return TM_EINVAL;
    const size_t k = b->parts.size();
    std::vector<tm_deliveries> d(k);
    uint64_t total = 0, nm = 0;
    float fill = 0.f;
    for (size_t i = 0; i < k; ++i) {
        int rc = tm_batch_dispatch(g->e, b->parts[i], 0, &d[i]);
        if (rc) return rc;
        total += d[i].n_deliveries;
        nm += d[i].n_matches;
        fill = std::max(fill, d[i].fill_ms);
    }
    b->d_rows.resize((size_t)b->n + 1);
    b->d_subs.resize(std::max<uint64_t>(total, 1));
    uint64_t base = 0;
    for (size_t i = 0; i < k; ++i) {
        const uint32_t lo = b->lo[i], cnt = b->lo[i + 1] - lo;
        for (uint32_t t = 0; t < cnt; ++t) b->d_rows[lo + t] = d[i].row_offsets[t] + base;
        if (d[i].n_deliveries)
            memcpy(b->d_subs.data() + base, d[i].subscribers, d[i].n_deliveries * sizeof(uint32_t));
        base += d[i].n_deliveries;
    }
    b->d_rows[b->n] = total;
    out->n_topics = b->n;
    out->n_matches = nm;
    out->n_deliveries = total;
    out->row_offsets = b->d_rows.data();
    out->match_offsets = nullptr;
    out->subscribers = b->d_subs.data();
    out->fill_ms = fill;
    return TM_OK;
}

int tm_group_batch_stats(tm_group* g, tm_group_batch* b, tm_batch_stats* out) {
    if (!g || !b || !out || b->parts.size() != tm_replica_count(g->e)) return TM_EINVAL;
    tm_batch_stats s{};
    for (tm_batch* part : b->parts) {
        tm_batch_stats p{};
        int rc = tm_batch_stats_get(g->e, part, &p);
        if (rc) return rc;
        s.topics += p.topics; s.visits += p.visits; s.hash_hits += p.hash_hits; s.words += p.words;
        s.matches += p.matches; s.slow_topics += p.slow_topics; s.overflow_tiles += p.overflow_tiles;
        s.ms_match = std::max(s.ms_match, p.ms_match);
        s.ms_total = std::max(s.ms_total, p.ms_total);
        s.ms_tokenize = std::max(s.ms_tokenize, p.ms_tokenize);
        s.probes += p.probes;
        s.iterations += p.iterations;
        s.publishes += p.publishes;
        s.delivered += p.delivered;
    }
    *out = s;
    return TM_OK;
}

void tm_group_batch_free(tm_group* g, tm_group_batch* b) {
    if (!b) return;
    for (tm_batch* p : b->parts)
        if (p) tm_batch_free(g ? g->e : nullptr, p);
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

int tm_group_match_async(tm_group* g, const uint8_t* topic, size_t len, tm_match_cb cb, void* ctx) {
    return g ? tm_match_async(g->e, topic, len, cb, ctx) : TM_EINVAL;
}

int tm_group_match_coalesced(tm_group* g, const uint8_t* topic, size_t len, uint32_t* ids, uint32_t cap,
                             uint32_t* n_out) {
    return g ? tm_match_coalesced(g->e, topic, len, ids, cap, n_out) : TM_EINVAL;
}

int tm_group_match_routes_batch(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                                tm_routes* out) {
    return g ? tm_match_routes_batch(g->e, topics, offsets, n, out) : TM_EINVAL;
}

int tm_group_rules_match(tm_group* g, const uint8_t* names, const uint64_t* name_offsets, uint32_t n,
                         const uint8_t* rules, const uint64_t* rule_offsets, uint32_t r, int dollar_rule,
                         uint32_t* bits) {
    return g ? tm_rules_match(g->e, names, name_offsets, n, rules, rule_offsets, r, dollar_rule, bits) : TM_EINVAL;
}

}  // extern "C"
