// tm_engine.cpp -- host side of the MI355X topic-matching engine: the C ABI.
// (The engine itself: tm_engine_impl.hpp and the modules it lists.)
#include "tm_engine_impl.hpp"

// ====================================================== emqx_topic predicates

namespace {

// emqx_topic:match/2 on word lists (src/emqx_topic.erl:74-87)
bool words_match(const std::vector<TWord>& n, const std::vector<TWord>& f) {
    size_t i = 0, j = 0;
    auto kind = [](const TWord& w) { return w.n == 0 ? 1 : is_plus(w) ? 2 : is_hash(w) ? 3 : 0; };
    for (;;) {
        if (i == n.size() && j == f.size()) return true;
        if (i < n.size() && j < f.size()) {
            const int kn = kind(n[i]), kf = kind(f[j]);
            const bool eq = kn == kf && (kn != 0 || (n[i].n == f[j].n && memcmp(n[i].p, f[j].p, n[i].n) == 0));
            if (eq || kf == 2) { ++i; ++j; continue; }
        }
        if (j + 1 == f.size() && kind(f[j]) == 3) return true;
        return false;
    }
}

// strict UTF-8 (Erlang's <<C/utf8, _/binary>>): returns bytes consumed or 0
size_t utf8_char(const uint8_t* p, size_t n, uint32_t& cp) {
    const uint8_t c = p[0];
    if (c < 0x80) { cp = c; return 1; }
    size_t len;
    uint32_t min;
    if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; min = 0x80; }
    else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; min = 0x800; }
    else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; min = 0x10000; }
    else return 0;
    if (len > n) return 0;
    for (size_t i = 1; i < len; ++i) {
        if ((p[i] & 0xC0) != 0x80) return 0;
        cp = (cp << 6) | (p[i] & 0x3F);
    }
    if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return 0;
    return len;
}

}  // namespace

// ======================================================================= ABI

extern "C" {

int tm_create_replicated(const tm_config* cfg, const int32_t* devices, uint32_t n_devices, tm_engine** out) {
    if (!out || (n_devices && !devices)) return TM_EINVAL;
    if (cfg && (cfg->flags & ~(TM_CFG_FROZEN_DICT | TM_CFG_HOST_TOKENIZE))) return TM_EINVAL;
    tm_engine* e = new (std::nothrow) tm_engine();
    if (!e) return TM_ENOMEM;
    int rc;
    try {
        rc = e->init(cfg, devices, n_devices);
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (rc) { e->destroy(); delete e; return rc; }
    *out = e;
    return TM_OK;
}

int tm_create(const tm_config* cfg, tm_engine** out) {
    const int32_t dev = cfg ? cfg->device : -1;
    return tm_create_replicated(cfg, &dev, dev >= 0 ? 1u : 0u, out);
}

uint32_t tm_replica_count(tm_engine* e) { return e ? (uint32_t)e->reps.size() : 0; }

int tm_async_start(tm_engine* e) {
    if (!e) return TM_EINVAL;
    if (e->reps.empty()) return TM_ENODEV;
    for (Replica* R : e->reps) {
        std::lock_guard<std::mutex> lk(R->amu);
        if (R->a_stop) return TM_ENODEV;
        int rc;
        try {
            rc = e->async_start(*R);
        } catch (...) {
            rc = TM_ENOMEM;
        }
        if (rc) return rc;
    }
    return TM_OK;
}

void tm_destroy(tm_engine* e) {
    if (!e) return;
    e->destroy();
    delete e;
}

uint64_t tm_version(tm_engine* e) {
    std::lock_guard<std::recursive_mutex> g(e->mu);
    return e->version;
}

int tm_stats(tm_engine* e, tm_engine_stats* o) {
    if (!e || !o) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    o->version = e->version;
    o->nodes = e->live_nodes;
    o->edges = e->live_edges;
    o->filters = e->n_filters;
    o->words = e->dict.size();
    o->slots = e->slots.size();
    if (!e->reps.empty()) {   // per replica (each device holds the same)
        const Replica& R = *e->reps[0];
        o->device_bytes = R.d_nslots * sizeof(Slot) + R.c_foff * 8 + R.c_flen * 4 + R.c_fbytes;
    } else {
        o->device_bytes = 0;
    }
    o->uploads_full = e->uploads_full;
    o->uploads_delta = e->uploads_delta;
    o->delta_slots = e->delta_slots;
    o->graph_launches = e->graph_launches;
    return TM_OK;
}

int tm_sync(tm_engine* e) {
    if (!e) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    if ((rc = e->sync_device())) return rc;
    for (Replica* R : e->reps) {
        HIP_OK(hipSetDevice(R->device));
        HIP_OK(hipStreamSynchronize(R->stream));
        R->delta_inflight = false;
    }
    return e->set_device();
}

int tm_sync_async(tm_engine* e) {
    if (!e) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    if ((rc = e->sync_device())) return rc;
    return e->set_device();
}

int tm_trie_insert(tm_engine* e, const uint8_t* t, size_t len) {
    if (!e || (!t && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->trie_insert(t, len);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_trie_delete(tm_engine* e, const uint8_t* t, size_t len) {
    if (!e || (!t && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->trie_delete(t, len);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_trie_lookup(tm_engine* e, const uint8_t* id, size_t len, int is_root, tm_trie_node* out) {
    if (!e || !out) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    uint32_t n;
    if (is_root) {
        n = e->nd[ROOT].live ? ROOT : NONE;
    } else {
        std::vector<uint32_t> ids;
        if (!e->filter_words(id, len, false, ids)) return 0;
        n = e->walk(ids);
    }
    if (n == NONE) return 0;
    out->edge_count = e->nd[n].ec;
    out->has_topic = e->nd[n].topic;
    out->filter_id = e->nd[n].topic ? n : TM_NONE;
    return 1;
}

int tm_trie_empty(tm_engine* e) {
    std::lock_guard<std::recursive_mutex> g(e->mu);
    return e->live_edges == 0;
}

int tm_match_batch_packed(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                          tm_result_packed* out) {
    if (!e || !offsets || !out || (!topics && n)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    Replica& R = e->pick();
    if ((rc = e->use(&R))) return rc;
    // 3 bytes while every node id fits 24 bits (the ids a result can hold)
    const uint32_t pack = e->nd.size() <= (1u << 24) ? 3u : 4u;
    tm_result r{};
    try {
        rc = e->match_batch_pipelined(R, topics, offsets, n, &r, pack);
    } catch (...) {
        return TM_ENOMEM;
    }
    if (rc) return rc;
    out->n_topics = r.n_topics;
    out->id_bytes = pack;
    out->n_matches = r.n_matches;
    out->row_offsets = r.row_offsets;
    out->ids = pack == 3 ? R.h_pids8 : reinterpret_cast<const uint8_t*>(r.filter_ids);
    return TM_OK;
}

int tm_match_batch(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_result* out) {
    if (!e || !offsets || !out || (!topics && n)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    // a large batch is split over every replica (no collective); a small one
    // runs on one of them, round-robin
    if (e->reps.size() > 1 && n >= 65536) {
        try {
            return e->match_batch_split(topics, offsets, n, out);
        } catch (...) {
            return TM_ENOMEM;
        }
    }
    Replica& R = e->pick();
    if ((rc = e->use(&R))) return rc;
    if (n > tm_engine::ONESHOT_MAX) {
        try {
            return e->match_batch_pipelined(R, topics, offsets, n, out);
        } catch (...) {
            return TM_ENOMEM;
        }
    }
    // prepare's H2D of the caller's buffers is not waited for (the pipeline is,
    // below); on any early exit the stream is drained before returning, so
    // the borrowed buffers are never read after the caller frees them
    struct Drain {
        tm_engine* e;
        Replica& R;
        bool armed = true;
        ~Drain() {
            e->upload_nosync = false;
            R.scratch.oneshot = false;   // (the scratch batch serves other calls too)
            if (armed) (void)hipStreamSynchronize(R.stream);
        }
    } drain{e, R};
    try {
        e->upload_nosync = true;
        rc = e->prepare(&R.scratch, topics, offsets, n);
        e->upload_nosync = false;
        if (rc) return rc;
        // latency-sized batches: CSR and its host copy enqueued with the walk
        R.scratch.oneshot = n <= tm_engine::ONESHOT_MAX;
        if ((rc = e->launch(&R.scratch))) return rc;
        if ((rc = e->wait(&R.scratch))) return rc;
        if (e->oneshot_result(&R.scratch, out) == TM_OK) {
            drain.armed = false;   // wait() synchronised past the copy
            return TM_OK;
        }
        rc = e->result(&R.scratch, out);
        drain.armed = rc != TM_OK;   // result() synchronised the stream
        return rc;
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_trie_match(tm_engine* e, const uint8_t* topic, size_t len, uint32_t* ids, uint32_t cap, uint32_t* n_out) {
    if (!e || !n_out || (!topic && len)) return TM_EINVAL;
    const uint64_t offs[2] = {0, len};
    tm_result r;
    static const uint8_t zero = 0;
    int rc = tm_match_batch(e, topic ? topic : &zero, offs, 1, &r);
    if (rc) return rc;
    const uint32_t m = r.row_offsets[1] - r.row_offsets[0];
    for (uint32_t i = 0; i < m && i < cap; ++i) ids[i] = r.filter_ids[r.row_offsets[0] + i];
    *n_out = m;
    return TM_OK;
}

int tm_batch_prepare(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_batch** out) {
    return tm_batch_prepare_ex(e, topics, offsets, n, 0, out);
}

// tm_match_coalesced = tm_match_async + a wait: the callback copies the row
// and releases the caller (brief spin, then a futex sleep).
namespace {
struct SyncWait {
    std::atomic<int> state{0};   // 0 pending, 1 done, 2 caller asleep
    uint32_t* ids;
    uint32_t cap;
    uint32_t n = 0;
    int rc = TM_OK;
    uint32_t word = 0;           // the caller's syncwake word
};

void sync_cb(void* ctx, int rc, const uint32_t* ids, uint32_t n) {
    SyncWait* w = static_cast<SyncWait*>(ctx);
    w->rc = rc;
    w->n = n;
    if (rc == TM_OK && n && w->cap) memcpy(w->ids, ids, (size_t)std::min(n, w->cap) * 4);
    const uint32_t k = w->word;   // (w is the caller's: gone once state reads 1)
    if (w->state.exchange(1, std::memory_order_acq_rel) == 2) {
        if (syncwake::in_batch) syncwake::pending |= 1u << k;
        else syncwake::wake(k);
    }
}
}  // namespace

int tm_match_async(tm_engine* e, const uint8_t* topic, size_t len, tm_match_cb cb, void* ctx) {
    if (!e || !cb || (!topic && len)) return TM_EINVAL;
    if (len > TM_MAX_TOPIC_LEN) return TM_EINVAL;
    try {
        return e->match_async(topic, len, cb, ctx);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_match_coalesced(tm_engine* e, const uint8_t* topic, size_t len, uint32_t* ids, uint32_t cap, uint32_t* n_out) {
    if (!e || !n_out || (!topic && len) || (cap && !ids)) return TM_EINVAL;
    if (len > TM_MAX_TOPIC_LEN) return TM_EINVAL;
    SyncWait w;
    w.ids = ids;
    w.cap = cap;
    static std::atomic<uint32_t> next_word{0};
    static thread_local uint32_t my_word = next_word.fetch_add(1) % syncwake::WAKE_WORDS;
    w.word = my_word;
    int rc = tm_match_async(e, topic, len, sync_cb, &w);
    if (rc) return rc;
    // A short spin before the futex: the box runs under a CFS CPU quota, and
    // dozens of callers spinning for long burn it and get the whole process
    // throttled for the rest of the period (tens of ms for every thread).
    // (A/B on the box, 64 blocking callers: 4,000 pauses 0.25 M calls/s with
    // 40-60 ms outliers, 200 pauses 0.62 M calls/s, none 0.53 M calls/s)
    for (int i = 0; i < 200 && w.state.load(std::memory_order_acquire) != 1; ++i) __builtin_ia32_pause();
    int expect = 0;
    if (w.state.compare_exchange_strong(expect, 2, std::memory_order_acq_rel)) {
        std::atomic<uint32_t>& seq = syncwake::words[w.word].seq;
        for (;;) {
            const uint32_t s0 = seq.load(std::memory_order_acquire);   // before the state check: no lost wake-up
            if (w.state.load(std::memory_order_acquire) != 2) break;
            syncwake::futex(&seq, FUTEX_WAIT, s0);
        }
    }
    *n_out = w.n;
    return w.rc;
}

int tm_coalesce_config(tm_engine* e, uint32_t max_batch, uint32_t linger_us, uint64_t* batches, uint64_t* requests) {
    if (!e) return TM_EINVAL;
    uint64_t nb = 0, nr = 0;
    for (Replica* R : e->reps) {
        std::lock_guard<std::mutex> lk(R->amu);
        if (max_batch) R->a_max = max_batch;
        if (linger_us != TM_NONE) R->a_linger_us = linger_us;
        nb += R->a_batches;
        nr += R->a_requests;
    }
    if (batches) *batches = nb;
    if (requests) *requests = nr;
    return TM_OK;
}

int tm_async_stats_get(tm_engine* e, tm_async_stats* out) {
    if (!e || !out) return TM_EINVAL;
    *out = tm_async_stats{};
    for (Replica* R : e->reps) {   // summed over the replicas' pipelines
        std::lock_guard<std::mutex> lk(R->amu);
        out->batches += R->a_batches;
        out->requests += R->a_requests;
        out->recoveries += R->a_recoveries;
        out->max_batch = std::max<uint64_t>(out->max_batch, R->a_max_seen);
        out->depth += R->a_depth;
        out->queued += (uint32_t)R->q_count.load();
        out->us_launch += R->a_us_launch;
        out->us_wait += R->a_us_wait;
        out->us_deliver += R->a_us_deliver;
        out->inline_launches += R->a_inline_launches;
    }
    return TM_OK;
}

namespace {
int prepare_on(tm_engine* e, Replica* R, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t flags,
               tm_batch** out) {
    if (!e || !offsets || !out || (!topics && n) || (flags & ~(TM_BATCH_DEDUP | TM_BATCH_STREAM))) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    const bool fresh = *out == nullptr;   // non-NULL: re-prepared in place (buffers only grow)
    if (!fresh) {
        if (R && (*out)->rep != R) return TM_EINVAL;   // a batch's buffers live on its replica's device
        R = (*out)->rep;
    } else if (!R && !e->reps.empty()) {
        R = &e->pick();   // a fresh batch goes to the next replica, round-robin
    }
    if (R) {
        int rc = e->use(R);
        if (rc) return rc;
    }
    tm_batch* b = fresh ? new (std::nothrow) tm_batch() : *out;
    if (!b) return TM_ENOMEM;
    b->rep = R;
    bool made_stream = false;
    if ((flags & TM_BATCH_STREAM) && R && !b->own) {
        // a stream of its own: its launches overlap other batches' (a CSR
        // pass with the next walk); trie uploads wait for it (readers)
        if (hipStreamCreateWithFlags(&b->own, hipStreamNonBlocking) != hipSuccess) {
            b->own = nullptr;
            if (fresh) delete b;
            return TM_EIO;
        }
        b->own_user = true;
        R->readers.push_back(b);
        made_stream = true;
    }
    int rc;
    try {
        rc = e->prepare(b, topics, offsets, n, flags & TM_BATCH_DEDUP);
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (rc) {
        if (b->own) (void)hipStreamSynchronize(b->own);
        if (fresh) {
            if (made_stream) e->drop_user_stream(b);
            b->release();
            delete b;
        } else {
            b->launched = b->done = false;
        }
        return rc;
    }
    if (R) HIP_OK(hipStreamSynchronize(R->stream));
    if (b->own) HIP_OK(hipStreamSynchronize(b->own));   // the caller's buffers were only borrowed
    *out = b;
    return TM_OK;
}
}  // namespace

int tm_batch_prepare_ex(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t flags,
                        tm_batch** out) {
    return prepare_on(e, nullptr, topics, offsets, n, flags, out);
}

int tm_batch_prepare_on(tm_engine* e, uint32_t replica, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                        uint32_t flags, tm_batch** out) {
    if (!e || replica >= e->reps.size()) return TM_EINVAL;
    return prepare_on(e, e->reps[replica], topics, offsets, n, flags, out);
}

uint32_t tm_batch_replica(tm_engine* e, tm_batch* b) {
    return (e && b && b->rep) ? b->rep->index : TM_NONE;
}

int tm_batch_row_map(tm_engine* e, tm_batch* b, const uint32_t** row_of, uint32_t* n_rows) {
    if (!e || !b || !row_of) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    if (b->dedup_dev) {   // the device's map, once per dedup pass (the rows exist after the wait)
        if (!b->done) return TM_EINVAL;
        if (!b->rowof_host) {
            int rc = e->use(b->rep);
            if (rc) return rc;
            b->row_of.resize(b->n_pub);
            if (b->n_pub) {
                HIP_OK(launch_dedup_rowof(e->dedup_args(b), e->st(b)));
                HIP_OK(hipMemcpyAsync(b->row_of.data(), b->d_rowof, (size_t)b->n_pub * 4, hipMemcpyDeviceToHost,
                                      e->st(b)));
                HIP_OK(hipStreamSynchronize(e->st(b)));
            }
            b->rowof_host = true;
        }
        static const uint32_t none = 0;
        *row_of = b->row_of.empty() ? &none : b->row_of.data();
        if (n_rows) *n_rows = b->n;
        return TM_OK;
    }
    if (!b->dedup && b->row_of.size() != b->n) {
        b->row_of.resize(b->n);
        for (uint32_t i = 0; i < b->n; ++i) b->row_of[i] = i;
    }
    static const uint32_t none = 0;
    *row_of = b->row_of.empty() ? &none : b->row_of.data();
    if (n_rows) *n_rows = b->n;
    return TM_OK;
}

int tm_batch_launch(tm_engine* e, tm_batch* b) {
    if (!e || !b) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    return e->launch(b);
}

int tm_batch_wait(tm_engine* e, tm_batch* b) {
    if (!e || !b) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    // The walk is waited for without the engine lock, so other callers
    // (mutations, other replicas' launches, the async launcher's inline
    // launches) proceed meanwhile; the caller owns b.  A launch that recorded
    // its end event is waited for on that event -- an event wait does not
    // touch the stream, which another thread may be capturing a graph on (a
    // synchronize on a capturing stream is refused and breaks the capture).
    // A batch on a stream of its own without an end event drains its stream.
    // Only a shared-stream batch without an end event waits under the lock
    // (in wait()).  wait() then finds the work done: its own sync is a check.
    if (b->launched && !b->done && (b->end_recorded || b->own)) {
        HIP_OK(hipSetDevice(b->rep->device));
        if (b->end_recorded) HIP_OK(hipEventSynchronize(b->ev_end));
        else HIP_OK(hipStreamSynchronize(b->own));
    }
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    return e->wait(b);
}

int tm_batch_result(tm_engine* e, tm_batch* b, tm_result* out) {
    if (!e || !b || !out) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    return e->result(b, out);
}

int tm_batch_result_packed(tm_engine* e, tm_batch* b, tm_result_packed* out) {
    if (!e || !b || !out) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    try {
        return e->result_packed(b, out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_batch_sample(tm_engine* e, tm_batch* b, const uint32_t* rows, uint32_t k, tm_result* out) {
    if (!e || !b || !out || (!rows && k)) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    try {
        return e->sample(b, rows, k, out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_batch_stats_get(tm_engine* e, tm_batch* b, tm_batch_stats* out) {
    if (!e || !b || !out) return TM_EINVAL;
    *out = b->st;
    return TM_OK;
}

int tm_batch_device_csr(tm_engine* e, tm_batch* b, const uint32_t** d_row, const uint32_t** d_ids, uint64_t* n) {
    if (!e || !b || !b->done) return TM_EINVAL;
    {
        std::lock_guard<std::recursive_mutex> g(e->mu);
        int rc = e->use(b->rep);
        if (rc) return rc;
        if ((rc = e->ensure_dense(b))) return rc;
    }
    if (d_row) *d_row = b->d_rowoff;
    if (d_ids) *d_ids = b->d_ids;
    if (n) *n = b->total;
    return TM_OK;
}

int tm_batch_rows(tm_engine* e, tm_batch* b, const uint32_t** d_count, const uint64_t** d_start,
                  const uint32_t** d_ids, uint64_t* n_matches) {
    if (!e || !b || !b->done || !b->csr) return TM_EINVAL;
    if (d_count) *d_count = b->d_count;
    if (d_start) *d_start = reinterpret_cast<const uint64_t*>(b->d_src);
    if (d_ids) *d_ids = b->d_sfids;
    if (n_matches) *n_matches = b->total;
    return TM_OK;
}

int tm_batch_publish_rows(tm_engine* e, tm_batch* b, const uint32_t** d_count, const uint64_t** d_start,
                          const uint32_t** d_ids, uint64_t* n_delivered) {
    if (!e || !b || !b->done || !b->csr) return TM_EINVAL;
    if (b->dedup && !b->dedup_dev) return TM_EINVAL;   // host-deduplicated: rows per distinct topic only
    if (d_count) *d_count = b->dedup_dev ? b->d_pcount : b->d_count;
    if (d_start) *d_start = reinterpret_cast<const uint64_t*>(b->dedup_dev ? b->d_psrc : b->d_src);
    if (d_ids) *d_ids = b->d_sfids;
    if (n_delivered) *n_delivered = b->st.delivered;
    return TM_OK;
}

int tm_batch_retokenize(tm_engine* e, tm_batch* b) {
    if (!e || !b) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    if (!b->dev_tok) return TM_EINVAL;
    b->tok_dict = ~0ull;
    b->dedup_stale = b->dedup_dev;   // a fresh pass over the resident bytes: deduplicated again
    return TM_OK;
}

void tm_batch_free(tm_engine* e, tm_batch* b) {
    if (!b) return;
    if (e) {
        std::lock_guard<std::recursive_mutex> g(e->mu);
        if (b->rep) {
            (void)hipSetDevice(b->rep->device);
            (void)hipStreamSynchronize(b->rep->stream);
        }
        e->forget_launch(b);
        if (b->own_user) {
            (void)hipStreamSynchronize(b->own);
            e->drop_user_stream(b);
        }
        b->release();
    } else {
        b->release();
    }
    delete b;
}

int tm_route_add(tm_engine* e, const uint8_t* topic, size_t len, uint32_t dest) {
    if (!e || (!topic && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->route_add(topic, len, dest);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_route_delete(tm_engine* e, const uint8_t* topic, size_t len, uint32_t dest) {
    if (!e || (!topic && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->route_delete(topic, len, dest);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_route_apply(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, const uint32_t* dests,
                   const uint8_t* ops, uint32_t n, uint64_t* n_changed) {
    if (n_changed) *n_changed = 0;
    if (!e || (n && (!offsets || !dests || !ops))) return TM_EINVAL;
    if (n && offsets[n] && !topics) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i] || ops[i] > TM_ROUTE_WRITE) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    uint64_t changed = 0;
    try {
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t* t = topics + offsets[i];
            const size_t len = (size_t)(offsets[i + 1] - offsets[i]);
            int rc = ops[i] == TM_ROUTE_WRITE ? e->route_add(t, len, dests[i]) : e->route_delete(t, len, dests[i]);
            if (rc == TM_ENOENT && ops[i] == TM_ROUTE_DELETE) continue;   // delete_object of no record: no-op
            if (rc) {
                if (n_changed) *n_changed = changed;
                return rc;
            }
            ++changed;
        }
    } catch (...) {
        if (n_changed) *n_changed = changed;
        return TM_ENOMEM;
    }
    if (n_changed) *n_changed = changed;
    return TM_OK;
}

int tm_subscribe(tm_engine* e, const uint8_t* topic, size_t len, uint32_t subscriber, uint32_t node_dest) {
    if (!e || (!topic && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->subscribe(topic, len, subscriber, node_dest);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_unsubscribe(tm_engine* e, const uint8_t* topic, size_t len, uint32_t subscriber, uint32_t node_dest) {
    if (!e || (!topic && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->unsubscribe(topic, len, subscriber, node_dest);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_subscriber_down(tm_engine* e, uint32_t subscriber, uint32_t node_dest, uint64_t* n_removed) {
    if (!e) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->subscriber_down(subscriber, node_dest, n_removed);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_batch_dispatch(tm_engine* e, tm_batch* b, uint32_t flags, tm_deliveries* out) {
    if (!e || !b || !out) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    try {
        return e->batch_dispatch(b, flags, out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_batch_routes(tm_engine* e, tm_batch* b, tm_routes* out) {
    if (!e || !b || !out) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    try {
        return e->batch_routes(b, out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_match_routes_batch(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_routes* out) {
    if (!e || !offsets || !out || (!topics && n)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    try {
        if (e->reps.size() > 1 && n >= 65536) return e->match_routes_split(topics, offsets, n, out);
        Replica& R = e->pick();
        if ((rc = e->use(&R))) return rc;
        if ((rc = e->prepare(&R.scratch, topics, offsets, n))) return rc;
        if ((rc = e->launch(&R.scratch))) return rc;
        if ((rc = e->wait(&R.scratch))) return rc;
        return e->batch_routes(&R.scratch, out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_rules_match(tm_engine* e, const uint8_t* names, const uint64_t* name_offsets, uint32_t n,
                   const uint8_t* rules, const uint64_t* rule_offsets, uint32_t r, int dollar_rule, uint32_t* bits) {
    if (!e || !name_offsets || !rule_offsets || (n && !names) || (r && !rules) || (n && r && !bits)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    if (!n || !r) return TM_OK;
    try {
        rc = e->rules_match_split(names, name_offsets, n, rules, rule_offsets, r, dollar_rule != 0, bits);
    } catch (...) {
        rc = TM_ENOMEM;
    }
    (void)e->set_device();
    return rc;
}

int tm_trie_insert_many(tm_engine* e, const uint8_t* filters, const uint64_t* offsets, uint32_t n, uint32_t shard,
                        uint32_t nshards, uint64_t* n_inserted) {
    if (!e || !offsets || (!filters && n)) return TM_EINVAL;
    if (nshards > 1 && shard >= nshards) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    WorkPool::Linger linger(e->pool);   // (the workers spin between this call's phases)
    uint64_t done = 0;
    int rc = TM_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return TM_EINVAL;
    try {
        if (nshards <= 1) {
            const auto tq0 = std::chrono::steady_clock::now();
            e->make_plan(filters, offsets, n, false);
            if (e->kn.par_trace)
                fprintf(stderr, "[plan ins n=%u] %.2f ms\n", n,
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
            if (n >= tm_engine::PAR_MIN && !e->mutate_parallel(false, filters, offsets, n, &done, &rc)) {
                if (n_inserted) *n_inserted = done;
                if (e->kn.par_trace)
                    fprintf(stderr, "[insert_many n=%u] %.2f ms in the call\n", n,
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
                return rc;
            }
            for (uint32_t i = 0; i < n && rc == TM_OK; ++i) {
                e->prefetch_insert(i, n);
                rc = e->insert_planned(filters, offsets, i);
                if (rc == TM_OK) ++done;
            }
            // a bulk build leaves the filter-bytes arena half empty: the churn
            // that follows appends to it for a long while before one growth
            // step (a copy of the whole arena, ~1 ms per 10 MB) lands inside a
            // delta batch
            if (n >= tm_engine::PAR_MIN && e->fbytes.capacity() < 2 * e->fbytes.size())
                e->fbytes.reserve(2 * e->fbytes.size());
            if (n_inserted) *n_inserted = done;
            return rc;
        }
        for (uint32_t i = 0; i < n && rc == TM_OK; ++i) {
            const uint8_t* f = filters + offsets[i];
            const size_t len = offsets[i + 1] - offsets[i];
            if (nshards > 1) {
                const int s = e->filter_shard(f, len, nshards);
                if (s < 0) { rc = s; break; }
                if ((uint32_t)s != shard && (uint32_t)s != nshards) continue;
            }
            rc = e->trie_insert(f, len);
            if (rc == TM_OK) ++done;
        }
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (n_inserted) *n_inserted = done;
    return rc;
}

int tm_trie_delete_many(tm_engine* e, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                        uint64_t* n_deleted) {
    if (!e || !offsets || (!filters && n)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    WorkPool::Linger linger(e->pool);   // (the workers spin between this call's phases)
    uint64_t done = 0;
    int rc = TM_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return TM_EINVAL;
    try {
        const auto tq0 = std::chrono::steady_clock::now();
        e->make_plan(filters, offsets, n, true);
        if (e->kn.par_trace)
            fprintf(stderr, "[plan del n=%u] %.2f ms\n", n,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
        if (n >= tm_engine::PAR_MIN && !e->mutate_parallel(true, filters, offsets, n, &done, &rc)) {
            if (n_deleted) *n_deleted = done;
            if (e->kn.par_trace)
                fprintf(stderr, "[delete_many n=%u] %.2f ms in the call\n", n,
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
            return rc;
        }
        for (uint32_t i = 0; i < n && rc == TM_OK; ++i) {
            e->prefetch_delete(i, n);
            rc = e->delete_planned(i);
            if (rc == TM_OK) ++done;
        }
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (n_deleted) *n_deleted = done;
    return rc;
}

int tm_trie_apply_many(tm_engine* e, const uint8_t* del_filters, const uint64_t* del_offsets, uint32_t n_del,
                       const uint8_t* ins_filters, const uint64_t* ins_offsets, uint32_t n_ins, uint64_t* n_deleted,
                       uint64_t* n_inserted) {
    if (n_deleted) *n_deleted = 0;
    if (n_inserted) *n_inserted = 0;
    if (!e || !del_offsets || !ins_offsets || (!del_filters && n_del) || (!ins_filters && n_ins)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    WorkPool::Linger linger(e->pool);   // (the workers spin between this call's phases)
    for (uint32_t i = 0; i < n_del; ++i)
        if (del_offsets[i + 1] < del_offsets[i]) return TM_EINVAL;
    for (uint32_t i = 0; i < n_ins; ++i)
        if (ins_offsets[i + 1] < ins_offsets[i]) return TM_EINVAL;
    const bool trace = e->kn.par_trace;
    uint64_t done = 0;
    int rc = TM_OK;
    try {
        const auto tq0 = std::chrono::steady_clock::now();
        e->tr_mark(nullptr);
        e->make_plan_pair(del_filters, del_offsets, n_del, ins_filters, ins_offsets, n_ins);
        e->tr_mark("plan");
        if (trace)
            fprintf(stderr, "[plan apply del=%u ins=%u] %.2f ms\n", n_del, n_ins,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
        // Both lists big enough for the parallel pass: the deletes' node
        // records (phase 1), the inserts' (their plan checked against the
        // deletes: an edge to a node that died is a miss), then ONE edge phase
        // and merge for both -- the deletes' edge work runs first in it, as in
        // the two calls.  Otherwise the two passes one after the other.
        tm_engine::ParRun RD, RI;
        bool del_open = false;
        if (n_del >= tm_engine::PAR_MIN && n_ins >= tm_engine::PAR_MIN &&
            !e->par_begin(true, del_filters, del_offsets, n_del, e->mut_w, RD)) {
            del_open = true;
            for (const Mut& m : e->mut_w)
                if (m.rc) {   // a delete failed: finish the deletes alone and stop
                    tm_engine::ParRun* runs[1] = {&RD};
                    e->par_finish(runs, 1);
                    if (n_deleted) *n_deleted = RD.done;
                    return RD.rc;
                }
        } else if (n_del < tm_engine::PAR_MIN || e->mutate_parallel(true, del_filters, del_offsets, n_del, &done, &rc)) {
            done = 0;
            for (uint32_t i = 0; i < n_del && rc == TM_OK; ++i) {
                e->prefetch_delete(i, n_del);
                rc = e->delete_planned(i);
                if (rc == TM_OK) ++done;
            }
        }
        if (!del_open) {
            if (n_deleted) *n_deleted = done;
            if (rc != TM_OK) return rc;
        }
        // the inserts, their plan moved to the front and checked against the
        // deletes.  With the deletes' edge work still pending, anything thrown
        // before the inserts' phase 1 has run must not leave it undone.
        bool ins_open = false;
        int irc = TM_OK;
        try {
            e->plan.erase(e->plan.begin(), e->plan.begin() + n_del);
            e->tr_mark("erase");
            const uint32_t again = e->replan_dead_inserts(n_ins);
            e->tr_mark("replan");
            if (trace)
                fprintf(stderr, "[apply: %u of %u inserts walked again after the deletes] %.2f ms in the call\n", again,
                        n_ins, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
            if (del_open) ins_open = !e->par_begin(false, ins_filters, ins_offsets, n_ins, e->mut_w2, RI);
        } catch (...) {
            if (!del_open) throw;
            // par_begin's setup allocates everything before it commits (takes
            // free ids, grows the node arrays); what it did before that --
            // new words interned, pending ids released -- leaves a consistent
            // engine, so the deletes' edge work can still be finished below
            irc = TM_ENOMEM;
        }
        done = 0;
        if (del_open) {
            if (ins_open) {
                tm_engine::ParRun* runs[2] = {&RD, &RI};
                e->par_finish(runs, 2);
                if (n_deleted) *n_deleted = RD.done;
                if (n_inserted) *n_inserted = RI.done;
                if (trace) {
                    fprintf(stderr, "[apply_many del=%u ins=%u, one edge phase] %.2f ms in the call\n", n_del, n_ins,
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
                    fprintf(stderr, "[pool] %llu runs, %.0f us in them, %.0f us of it before the last worker started\n",
                            (unsigned long long)e->pool.t_runs, e->pool.t_wall_us, e->pool.t_lag_us);
                    e->pool.t_runs = 0;
                    e->pool.t_wall_us = e->pool.t_lag_us = 0;
                    e->tr_print();
                }
                return RD.rc ? RD.rc : RI.rc;
            }
            tm_engine::ParRun* runs[1] = {&RD};   // the inserts run serially: the deletes end first
            e->par_finish(runs, 1);
            if (n_deleted) *n_deleted = RD.done;
            if (RD.rc) return RD.rc;
            if (irc) return irc;
            for (uint32_t i = 0; i < n_ins && rc == TM_OK; ++i) {
                e->prefetch_insert(i, n_ins);
                rc = e->insert_planned(ins_filters, ins_offsets, i);
                if (rc == TM_OK) ++done;
            }
        } else if (n_ins < tm_engine::PAR_MIN || e->mutate_parallel(false, ins_filters, ins_offsets, n_ins, &done, &rc)) {
            done = 0;
            for (uint32_t i = 0; i < n_ins && rc == TM_OK; ++i) {
                e->prefetch_insert(i, n_ins);
                rc = e->insert_planned(ins_filters, ins_offsets, i);
                if (rc == TM_OK) ++done;
            }
        }
        if (n_inserted) *n_inserted = done;
        if (trace)
            fprintf(stderr, "[apply_many del=%u ins=%u] %.2f ms in the call\n", n_del, n_ins,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
    } catch (...) {
        rc = TM_ENOMEM;
    }
    return rc;
}

int tm_dict_load(tm_engine* e, const uint8_t* words, const uint64_t* offsets, uint32_t n) {
    if (!e || !offsets || (!words && n)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->dict_load(words, offsets, n);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_filter_shard(tm_engine* e, const uint8_t* filter, size_t len, uint32_t nshards) {
    if (!e || (!filter && len)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    return e->filter_shard(filter, len, nshards);
}

int tm_tokenize(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t* words,
                uint64_t words_cap, uint32_t* toff, uint8_t* tflags, uint64_t* nwords_out) {
    if (!e || !offsets || !toff || !nwords_out || (!topics && n) || (!tflags && n) || (!words && words_cap))
        return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    try {
        return e->tokenize_into(topics, offsets, n, words, words_cap, toff, tflags, nwords_out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_tokenize_device(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t* d_words,
                       uint64_t words_cap, uint32_t* d_toff, uint8_t* d_tflags, uint64_t* nwords_out) {
    if (!e || !offsets || !d_toff || !nwords_out || (n && (!topics || !d_words || !d_tflags))) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    try {
        return e->tokenize_device(topics, offsets, n, d_words, words_cap, d_toff, d_tflags, nwords_out);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_batch_prepare_tokens(tm_engine* e, const uint32_t* words, const uint32_t* toff, const uint8_t* tflags,
                            uint32_t n, uint64_t nwords, int on_device, tm_batch** out) {
    if (!e || !out || !toff || (!tflags && n) || (!words && nwords)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    if (on_device) {
        int rc = e->set_device();
        if (rc) return rc;
    }
    const bool fresh = *out == nullptr;   // a non-NULL *out is reused (its buffers only grow)
    tm_batch* b = fresh ? new (std::nothrow) tm_batch() : *out;
    if (!b) return TM_ENOMEM;
    if (fresh) b->rep = e->reps.empty() ? nullptr : e->reps[0];   // device tokens live on the first replica's device
    if (b->rep) (void)e->use(b->rep);
    int rc;
    try {
        rc = e->prepare_tokens(b, words, toff, tflags, n, nwords, on_device != 0);
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (rc) {
        if (fresh) { b->release(); delete b; }
        else b->launched = b->done = false;
        return rc;
    }
    if (b->rep) HIP_OK(hipStreamSynchronize(b->rep->stream));
    *out = b;
    return TM_OK;
}

}  // extern "C"

namespace etm {

int tokenize_device_staged(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint64_t base,
                           uint64_t nbytes, uint64_t off_item0, const TokStaged& st, uint32_t* d_words,
                           uint64_t words_cap, uint32_t* d_toff, uint8_t* d_tflags, uint64_t* nwords_out) {
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    try {
        rc = e->tokenize_device(topics, offsets, n, d_words, words_cap, d_toff, d_tflags, nwords_out, &st, base,
                                nbytes, off_item0);
        // a failure may leave copies from the caller's staging in flight: they
        // finish before the caller can free it
        if (rc && !e->reps.empty()) (void)hipStreamSynchronize(e->reps[0]->stream);
        return rc;
    } catch (...) {
        return TM_ENOMEM;
    }
}


int part_batch_buffers(tm_engine* e, tm_batch** io, uint32_t n, uint64_t nwords, PartBuffers* out) {
    if (!e || !io || !out) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    if (e->reps.empty()) return TM_ENODEV;
    const bool fresh = *io == nullptr;
    tm_batch* b = fresh ? new (std::nothrow) tm_batch() : *io;
    if (!b) return TM_ENOMEM;
    if (fresh) b->rep = e->reps[0];
    int rc = e->use(b->rep);
    if (!rc) {
        try {
            rc = e->part_buffers(b, n, nwords, out);
        } catch (...) {
            rc = TM_ENOMEM;
        }
    }
    if (rc) {
        if (fresh) { b->release(); delete b; }
        else b->launched = b->done = false;
        return rc;
    }
    *io = b;
    return TM_OK;
}

int part_batch_finish(tm_engine* e, tm_batch* b, uint32_t* relaunched) {
    if (!e || !b || !b->rep) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    return e->wait(b, true, relaunched);
}

}  // namespace etm

extern "C" {

int tm_gather_rows(tm_engine* e, const uint32_t* d_src, const int64_t* d_src_off, const int64_t* d_idx, uint32_t n,
                   const int64_t* d_dst_off, uint32_t* d_dst) {
    if (!e || (n && (!d_src_off || !d_idx || !d_dst_off))) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    HIP_OK(launch_gather_rows(d_src, d_src_off, d_idx, n, d_dst_off, d_dst, e->reps[0]->stream));
    HIP_OK(hipStreamSynchronize(e->reps[0]->stream));
    return TM_OK;
}

int tm_tokens_shard(tm_engine* e, const uint32_t* d_words, const uint32_t* d_toff, uint32_t n, uint32_t nshards,
                    uint32_t* d_shard) {
    if (!e || !d_toff || nshards == 0 || (n && (!d_words || !d_shard))) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->set_device();
    if (rc) return rc;
    HIP_OK(launch_tokens_shard(d_words, d_toff, n, nshards, d_shard, e->reps[0]->stream));
    HIP_OK(hipStreamSynchronize(e->reps[0]->stream));
    return TM_OK;
}

int tm_batch_export(tm_engine* e, tm_batch* b, uint32_t* d_counts, uint32_t* d_ids, uint32_t mul, uint32_t add) {
    if (!e || !b || (!d_counts && b->n) || (!d_ids && b->total)) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    return e->export_batch(b, d_counts, d_ids, mul, add);
}

const uint8_t* tm_filter_bytes(tm_engine* e, uint32_t id, size_t* len) {
    if (!e) return nullptr;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    if (id >= e->nd.size() || !e->nd[id].hasbytes) return nullptr;   // matched ids keep their bytes
    if (len) *len = e->n_flen[id];
    static const uint8_t empty = 0;
    return e->n_flen[id] ? e->fbytes.data() + e->n_foff[id] : &empty;
}

int tm_filter_copy(tm_engine* e, uint32_t id, uint8_t* buf, size_t cap, size_t* len) {
    if (!e || !len || (cap && !buf)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    if (id >= e->nd.size() || !e->nd[id].hasbytes) return TM_ENOENT;
    *len = e->n_flen[id];
    if (*len <= cap && *len) memcpy(buf, e->fbytes.data() + e->n_foff[id], *len);
    return TM_OK;
}

extern "C++" {
namespace {
// ids read in place: u32 ids, or packed little-endian ids of 3 / 4 bytes
template <class Id>
int filters_copy(tm_engine* e, Id id_at, uint32_t n, uint8_t* buf, size_t cap, uint64_t* offs, uint32_t* keep,
                 uint32_t* n_out, uint64_t* need) {
    std::lock_guard<std::recursive_mutex> g(e->mu);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t id = id_at(i);
        if (id < e->nd.size() && e->nd[id].hasbytes) total += e->n_flen[id];
    }
    *need = total;
    if (total > cap) return TM_OK;   // nothing copied: the caller grows buf and asks again
    uint32_t k = 0;
    uint64_t at = 0;
    offs[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t id = id_at(i);
        if (id >= e->nd.size() || !e->nd[id].hasbytes) continue;
        const uint32_t len = e->n_flen[id];
        if (len) memcpy(buf + at, e->fbytes.data() + e->n_foff[id], len);
        at += len;
        if (keep) keep[k] = i;
        offs[++k] = at;
    }
    *n_out = k;
    return TM_OK;
}
}  // namespace
}  // extern "C++"

int tm_filters_copy(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, size_t cap, uint64_t* offs,
                    uint32_t* keep, uint32_t* n_out, uint64_t* need) {
    if (!e || !offs || !n_out || !need || (n && !ids) || (cap && !buf)) return TM_EINVAL;
    return filters_copy(e, [ids](uint32_t i) { return ids[i]; }, n, buf, cap, offs, keep, n_out, need);
}

int tm_filters_copy_packed(tm_engine* e, const uint8_t* ids, uint32_t id_bytes, uint32_t n, uint8_t* buf, size_t cap,
                           uint64_t* offs, uint32_t* keep, uint32_t* n_out, uint64_t* need) {
    if (!e || !offs || !n_out || !need || (n && !ids) || (cap && !buf) || (id_bytes != 3 && id_bytes != 4))
        return TM_EINVAL;
    if (id_bytes == 4)
        return filters_copy(e, [ids](uint32_t i) { uint32_t v; memcpy(&v, ids + 4ull * i, 4); return v; }, n, buf,
                            cap, offs, keep, n_out, need);
    return filters_copy(
        e, [ids](uint32_t i) {
            const uint8_t* p = ids + 3ull * i;
            return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16;
        },
        n, buf, cap, offs, keep, n_out, need);
}

int tm_filter_id(tm_engine* e, const uint8_t* f, size_t len, uint32_t* id) {
    if (!e || !id) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    std::vector<uint32_t> ids;
    if (!e->filter_words(f, len, false, ids)) return TM_ENOENT;
    const uint32_t n = e->walk(ids);
    if (n == NONE || !e->nd[n].topic) return TM_ENOENT;
    *id = n;
    return TM_OK;
}

int tm_topic_match(const uint8_t* name, size_t nl, const uint8_t* flt, size_t fl) {
    // match(<<$$, _/binary>>, <<$+, _/binary>>) -> false; ... <<$#, ...>> -> false
    if (nl > 0 && name[0] == '$' && fl > 0 && (flt[0] == '+' || flt[0] == '#')) return 0;
    std::vector<TWord> a, b;
    split_words(name, nl, a);
    split_words(flt, fl, b);
    return words_match(a, b) ? 1 : 0;
}

int tm_topic_wildcard(const uint8_t* t, size_t len) {
    std::vector<TWord> ws;
    split_words(t, len, ws);
    for (const TWord& w : ws)
        if (is_plus(w) || is_hash(w)) return 1;
    return 0;
}

int tm_topic_validate(int is_name, const uint8_t* t, size_t len, const char** reason) {
    const char* dummy;
    if (!reason) reason = &dummy;
    *reason = nullptr;
    if (len == 0) { *reason = "empty_topic"; return TM_EINVAL; }
    if (len > TM_MAX_TOPIC_LEN) { *reason = "topic_too_long"; return TM_EINVAL; }
    std::vector<TWord> ws;
    split_words(t, len, ws);
    // validate2/1 (src/emqx_topic.erl:109-120)
    bool wild = false;
    for (size_t i = 0; i < ws.size(); ++i) {
        const TWord& w = ws[i];
        if (is_hash(w)) {
            if (i + 1 != ws.size()) { *reason = "topic_invalid_#"; return TM_EINVAL; }
            wild = true;
            continue;
        }
        if (w.n == 0) continue;
        if (is_plus(w)) { wild = true; continue; }
        // validate3/1 (:122-127): utf8 chars, none of '#', '+', 0
        size_t k = 0;
        while (k < w.n) {
            uint32_t cp;
            size_t c = utf8_char(w.p + k, w.n - k, cp);
            if (!c) { *reason = "function_clause"; return TM_EINVAL; }
            if (cp == '#' || cp == '+' || cp == 0) { *reason = "topic_invalid_char"; return TM_EINVAL; }
            k += c;
        }
    }
    if (is_name && wild) { *reason = "topic_name_error"; return TM_EINVAL; }
    return TM_OK;
}

int tm_debug_check(tm_engine* e, uint64_t* max_disp_out) {
    if (!e) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    const uint32_t nb = e->nbuckets();
    uint64_t live = 0, md = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        bool hole = false;
        for (uint32_t k = 0; k < BUCKET; ++k) {
            const Slot& sl = e->slots[b * BUCKET + k];
            if (sl.parent == SLOT_EMPTY) { hole = true; continue; }
            if (hole) {
                snprintf(last_error(), 512, "bucket %u not filled in order", b);
                return TM_EIO;
            }
            ++live;
            const uint32_t sp = sl.parent & ID_MASK;
            const uint32_t h = home_bucket(sp, sl.word & WID_MASK, nb);
            const uint32_t d = (b + nb - h) % nb;
            md = std::max<uint64_t>(md, d);
            if (d > e->max_disp) {
                snprintf(last_error(), 512, "slot %u displaced %u > max_disp %u", b * BUCKET + k, d, e->max_disp);
                return TM_EIO;
            }
            for (uint32_t x = h; x != b; x = (x + 1 == nb) ? 0 : x + 1)
                if (e->slots[x * BUCKET + BUCKET - 1].parent == SLOT_EMPTY) {
                    snprintf(last_error(), 512, "run of slot %u (home %u) broken at bucket %u", b * BUCKET + k, h, x);
                    return TM_EIO;
                }
            if (e->find_slot(sp, sl.word & WID_MASK) != b * BUCKET + k || e->nd[sl.child & ID_MASK].inslot != b * BUCKET + k) {
                snprintf(last_error(), 512, "slot %u not found by its key", b * BUCKET + k);
                return TM_EIO;
            }
            // the child's literal signature: the node's own, and the parent's
            // covers this edge's word (a clear bit must prove the edge absent)
            const uint32_t c = sl.child & ID_MASK, w = sl.word & WID_MASK;
            if (slot_lsig(sl.parent, sl.word) != e->nd[c].lsig() ||
                (!(sl.hash & B_HASH) && sl.hash != e->n_lext[c])) {
                snprintf(last_error(), 512, "slot %u: literal signature %u / %#x, node %u has %u / %#x", b * BUCKET + k,
                         slot_lsig(sl.parent, sl.word), sl.hash, c, e->nd[c].lsig(), e->n_lext[c]);
                return TM_EIO;
            }
            if (sp != ROOT && w != W_PLUS && w != W_HASH) {
                const uint32_t pi = e->nd[sp].inslot;
                const Slot* ps = pi == NONE ? nullptr : &e->slots[pi];
                if (!ps || !(slot_lsig(ps->parent, ps->word) >> lsig_pos(w) & 1u) ||
                    (!(ps->hash & B_HASH) && !(ps->hash >> lext_pos(w) & 1u))) {
                    snprintf(last_error(), 512, "slot %u: word %u missing from its parent's literal signature",
                             b * BUCKET + k, w);
                    return TM_EIO;
                }
            }
        }
    }
    if (live != e->live_edges) {
        snprintf(last_error(), 512, "live slots %llu != live edges %llu", (unsigned long long)live,
                 (unsigned long long)e->live_edges);
        return TM_EIO;
    }
    if (max_disp_out) *max_disp_out = md;
    return TM_OK;
}

const char* tm_last_error(void) { return last_error(); }

}  // extern "C"

char* etm::error_buf() {
    static thread_local char buf[512] = "";
    return buf;
}

extern "C" {

int tm_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

#ifndef TM_SRC_HASH
#define TM_SRC_HASH "unstamped"
#endif
// ends with the digest of the sources it was built from (emqx_amd/build.py source_hash)
const char* tm_build_info(void) {
    return "emqx_tm gfx950 frontier-tile kernel; 16-B slots, 64-B buckets; path-code sort; src " TM_SRC_HASH;
}

}  // extern "C"
