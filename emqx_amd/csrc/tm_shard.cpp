// tm_shard.cpp -- the filter-sharded group in one process (BASELINE config C4:
// "100M IoT-style filters filter-sharded across 8 GPUs"), no torch, no
// collective.
//
// Subscription sets too large to replicate are partitioned over G shard
// engines (one per listed device; a device may repeat):
//   * a filter whose first two levels are literal words lives on shard
//     hash(id(w0), id(w1)) mod G; every other filter is replicated on all
//     shards (tm_filter_shard);
//   * a publish whose first two words are interned literals can only be
//     matched by filters of that shard or replicated ones -- literal levels
//     must be equal -- so its owner shard resolves it completely: no merge of
//     partial lists, rows stay bit-exact; any other publish can be resolved by
//     any shard and is dealt round-robin;
//   * word ids mean the same on every shard: the engines run with a frozen
//     dictionary that grows only by tm_sharded_insert_many's dictionary deltas
//     (new literal words appended in first-appearance order on every shard).
// One step over a batch tokenised on the home device (shard 0's):
//   owner per publish (tm_tokens_shard) -> a stable counting sort by owner on
//   the device (tm_part_*: each owner's publishes and words contiguous, in
//   publish order) -> every owner matches its part (token batches of its
//   engine, launched together) -> counts and global ids (local id * G + shard)
//   back on the home device -> rows restored to publish order (tm_unpart_*).
// The multi-process form with RCCL all_to_all is emqx_amd/sharded.py; in one
// process the exchange is a device-to-device copy per part.
//
// Reference: the filter set is the mnesia-replicated trie
// (src/emqx_trie.erl:53-74) that every node matches in full
// (src/emqx_router.erl:127-141); sharding it is new.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/emqx_tm.h"
#include "tm_internal.hpp"

using namespace etm;

namespace {

#define SH_HIP(expr)                                                                 \
    do {                                                                             \
        hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess) {                                                      \
            snprintf(error_buf(), 512, "%s at tm_shard.cpp:%d (%s)", hipGetErrorString(_e), __LINE__, #expr); \
            return TM_EIO;                                                           \
        }                                                                            \
    } while (0)

// device buffer on a fixed device, growing only
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    int dev = -1;
    int reserve(size_t n) {
        if (n <= cap && p) return TM_OK;
        const size_t nc = std::max<size_t>(n + n / 4, 256);
        SH_HIP(hipSetDevice(dev));
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        SH_HIP(hipMalloc((void**)&p, nc * sizeof(T)));
        cap = nc;
        return TM_OK;
    }
    void release() {
        if (p) {
            (void)hipSetDevice(dev);
            (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
};

template <class T>
int host_pinned(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return TM_OK;
    const size_t nc = std::max<size_t>(n + n / 4, 1024);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    SH_HIP(hipHostMalloc((void**)&p, nc * sizeof(T), hipHostMallocPortable));
    cap = nc;
    return TM_OK;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct tm_sharded_batch {
    uint32_t n = 0;
    uint64_t nwords = 0;
    uint64_t dict_words = ~0ull;          // dictionary size the tokens were made with
    std::vector<uint8_t> bytes;           // the publishes (re-tokenised if the dictionary grew)
    std::vector<uint64_t> offs;
    // home device
    DBuf<uint32_t> words, toff, owner, cnt, wcnt, cnt_off, cnt_bs, w_off, w_bs, segs, order, ptoff, pwords;
    DBuf<uint32_t> counts_p, ids_p, counts_o, src_off, src_bs, dst_off, dst_bs, rowg, out;
    DBuf<uint8_t> tflags, ptflags;
    uint32_t* h_segs = nullptr;
    size_t ch_segs = 0;
    // per shard: its part (a token batch of its engine) and export staging on its device
    std::vector<tm_batch*> part;
    std::vector<DBuf<uint32_t>> xcnt, xids;
    std::vector<uint32_t> tseg, wseg;     // first publish / word of each part (+ totals)
    std::vector<uint64_t> mseg;           // first match of each part's rows (+ total)
    uint64_t total = 0;
    bool done = false;
    bool direct = false;   // one shard: the result is the part's own CSR (no partition, no reorder)
    // host result
    uint32_t *h_row = nullptr, *h_ids = nullptr;
    size_t ch_row = 0, ch_ids = 0;
    tm_batch_stats st{};
    float ms_partition = 0, ms_parts = 0, ms_unpartition = 0;

    void release() {
        for (DBuf<uint32_t>* b : {&words, &toff, &owner, &cnt, &wcnt, &cnt_off, &cnt_bs, &w_off, &w_bs, &segs, &order,
                                  &ptoff, &pwords, &counts_p, &ids_p, &counts_o, &src_off, &src_bs, &dst_off, &dst_bs,
                                  &rowg, &out})
            b->release();
        tflags.release();
        ptflags.release();
        for (auto& x : xcnt) x.release();
        for (auto& x : xids) x.release();
        for (uint32_t* h : {h_segs, h_row, h_ids})
            if (h) (void)hipHostFree(h);
        h_segs = h_row = h_ids = nullptr;
    }
};

struct tm_sharded {
    std::vector<tm_engine*> sh;
    std::vector<int32_t> dev;
    uint32_t G = 0;
    int home = -1;
    hipStream_t s = nullptr;   // home device: partition / un-partition kernels
    std::mutex mu;             // one step (and one mutation) at a time
    tm_sharded_batch* last = nullptr;

    template <class F>
    void each(F f) {
        if (G == 1) { f(0); return; }
        std::vector<std::thread> th;
        for (uint32_t g = 0; g < G; ++g) th.emplace_back([&f, g] { f(g); });
        for (auto& t : th) t.join();
    }

    uint64_t dict_words() {
        tm_engine_stats st{};
        return tm_stats(sh[0], &st) == TM_OK ? st.words : 0;
    }

    // publishes -> tokens on the home device (shard 0's device tokeniser)
    int tokenize(tm_sharded_batch* b) {
        const uint32_t n = b->n;
        const uint64_t nbytes = b->offs[n];
        int rc;
        for (DBuf<uint32_t>* x : {&b->words, &b->toff}) x->dev = home;
        b->tflags.dev = home;
        if ((rc = b->words.reserve(std::max<uint64_t>(nbytes + n, 1)))) return rc;
        if ((rc = b->toff.reserve((size_t)n + 1))) return rc;
        if ((rc = b->tflags.reserve(std::max<size_t>(n, 1)))) return rc;
        static const uint8_t zero = 0;
        uint64_t nw = 0;
        b->dict_words = dict_words();
        if ((rc = tm_tokenize_device(sh[0], b->bytes.empty() ? &zero : b->bytes.data(), b->offs.data(), n, b->words.p,
                                     b->words.cap, b->toff.p, b->tflags.p, &nw)))
            return rc;
        b->nwords = nw;
        return TM_OK;
    }

    // One shard: every publish is its own part and the rows come back in
    // publish order -- no owner kernel, no partition, no reorder; global ids
    // are the local ones (local * 1 + 0).
    int step_one(tm_sharded_batch* b) {
        int rc;
        const uint32_t n = b->n;
        const double t1 = now_ms();
        if (b->part.size() != 1) b->part.assign(1, nullptr);
        static const uint32_t zero_off = 0;
        if (!n) {
            SH_HIP(hipSetDevice(home));
            SH_HIP(hipMemcpy(b->toff.p, &zero_off, 4, hipMemcpyHostToDevice));
        }
        if ((rc = tm_batch_prepare_tokens(sh[0], b->words.p, b->toff.p, b->tflags.p, n, b->nwords, 1, &b->part[0])))
            return rc;
        if ((rc = tm_batch_launch(sh[0], b->part[0]))) return rc;
        if ((rc = tm_batch_wait(sh[0], b->part[0]))) return rc;
        tm_batch_stats p{};
        if ((rc = tm_batch_stats_get(sh[0], b->part[0], &p))) return rc;
        if (p.matches > MAX_RESULT) return TM_EOVERFLOW;
        b->st = p;
        b->st.topics = n;
        b->tseg.assign(2, 0);
        b->tseg[1] = n;
        b->wseg.assign(2, 0);
        b->wseg[1] = (uint32_t)b->nwords;
        b->mseg.assign(2, 0);
        b->mseg[1] = p.matches;
        b->ms_partition = 0;
        b->ms_parts = (float)(now_ms() - t1);
        b->ms_unpartition = 0;
        b->total = p.matches;
        b->direct = true;
        b->done = true;
        return TM_OK;
    }

    int step(tm_sharded_batch* b) {
        int rc;
        const uint32_t n = b->n;
        b->done = false;
        b->direct = false;
        if (b->dict_words != dict_words() && (rc = tokenize(b))) return rc;   // new words since tokenisation
        if (G == 1) return step_one(b);
        const double t0 = now_ms();
        // ---- owner and partition (home device)
        const uint32_t nb = std::max<uint32_t>(1, (n + PART_BLOCK - 1) / PART_BLOCK);
        const uint32_t gb = G * nb;
        for (DBuf<uint32_t>* x : {&b->owner, &b->cnt, &b->wcnt, &b->cnt_off, &b->cnt_bs, &b->w_off, &b->w_bs, &b->segs,
                                  &b->order, &b->ptoff, &b->pwords})
            x->dev = home;
        b->ptflags.dev = home;
        if ((rc = b->owner.reserve(std::max<size_t>(n, 1)))) return rc;
        if ((rc = b->cnt.reserve(gb))) return rc;
        if ((rc = b->wcnt.reserve(gb))) return rc;
        if ((rc = b->cnt_off.reserve((size_t)gb + 1))) return rc;
        if ((rc = b->w_off.reserve((size_t)gb + 1))) return rc;
        if ((rc = b->cnt_bs.reserve(scan_block_count(gb) + 1))) return rc;
        if ((rc = b->w_bs.reserve(scan_block_count(gb) + 1))) return rc;
        if ((rc = b->segs.reserve(2 * ((size_t)G + 1)))) return rc;
        if ((rc = b->order.reserve(std::max<size_t>(n, 1)))) return rc;
        if ((rc = b->ptoff.reserve((size_t)n + G))) return rc;
        if ((rc = b->pwords.reserve(std::max<uint64_t>(b->nwords, 1)))) return rc;
        if ((rc = b->ptflags.reserve(std::max<size_t>(n, 1)))) return rc;
        if ((rc = host_pinned(b->h_segs, b->ch_segs, 2 * ((size_t)G + 1)))) return rc;
        b->tseg.assign(G + 1, 0);
        b->wseg.assign(G + 1, 0);
        if (n) {
            if ((rc = tm_tokens_shard(sh[0], b->words.p, b->toff.p, n, G, b->owner.p))) return rc;
            SH_HIP(hipSetDevice(home));
            PartArgs a{};
            a.owner = b->owner.p; a.words = b->words.p; a.toff = b->toff.p; a.tflags = b->tflags.p;
            a.n = n; a.G = G; a.nb = nb;
            a.cnt = b->cnt.p; a.wcnt = b->wcnt.p;
            a.cnt_off = b->cnt_off.p; a.cnt_bs = b->cnt_bs.p; a.w_off = b->w_off.p; a.w_bs = b->w_bs.p;
            a.segs = b->segs.p; a.order = b->order.p; a.ptoff = b->ptoff.p; a.ptflags = b->ptflags.p;
            a.pwords = b->pwords.p;
            SH_HIP(launch_part_count(a, s));
            ScanArgs sc{};
            sc.count = b->cnt.p; sc.row_off = b->cnt_off.p; sc.block_sums = b->cnt_bs.p; sc.n = gb;
            SH_HIP(launch_scan(sc, s, nullptr));
            ScanArgs sw{};
            sw.count = b->wcnt.p; sw.row_off = b->w_off.p; sw.block_sums = b->w_bs.p; sw.n = gb;
            SH_HIP(launch_scan(sw, s, nullptr));
            SH_HIP(launch_part_segs(a, s));
            SH_HIP(launch_part_scatter(a, s));
            SH_HIP(hipMemcpyAsync(b->h_segs, b->segs.p, 2 * ((size_t)G + 1) * 4, hipMemcpyDeviceToHost, s));
            SH_HIP(hipStreamSynchronize(s));
            for (uint32_t g = 0; g <= G; ++g) {
                b->tseg[g] = b->h_segs[g];
                b->wseg[g] = b->h_segs[G + 1 + g];
            }
            if (b->tseg[G] != n || b->wseg[G] != b->nwords) {
                snprintf(error_buf(), 512, "partition lost publishes: %u of %u, %u of %llu words", b->tseg[G], n,
                         b->wseg[G], (unsigned long long)b->nwords);
                return TM_EIO;
            }
        }
        const double t1 = now_ms();
        // ---- every owner matches its part (token batches of its engine)
        if (b->part.size() != G) b->part.assign(G, nullptr);
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t ng = b->tseg[g + 1] - b->tseg[g];
            const uint64_t nw = b->wseg[g + 1] - b->wseg[g];
            static const uint32_t zero_off = 0;
            const uint32_t* w = n ? b->pwords.p + b->wseg[g] : b->words.p;
            const uint32_t* o = n ? b->ptoff.p + b->tseg[g] + g : nullptr;
            const uint8_t* f = n ? b->ptflags.p + b->tseg[g] : b->tflags.p;
            if (!n) {   // an empty batch: one zero offset per part
                SH_HIP(hipSetDevice(home));
                SH_HIP(hipMemcpy(b->toff.p, &zero_off, 4, hipMemcpyHostToDevice));
                o = b->toff.p;
            }
            if ((rc = tm_batch_prepare_tokens(sh[g], w, o, f, ng, nw, 1, &b->part[g]))) return rc;
        }
        for (uint32_t g = 0; g < G; ++g)
            if ((rc = tm_batch_launch(sh[g], b->part[g]))) return rc;
        int first = TM_OK;
        for (uint32_t g = 0; g < G; ++g) {   // every part is drained, even after an error
            rc = tm_batch_wait(sh[g], b->part[g]);
            if (rc && !first) first = rc;
        }
        if (first) return first;
        b->mseg.assign(G + 1, 0);
        b->st = tm_batch_stats{};
        for (uint32_t g = 0; g < G; ++g) {
            tm_batch_stats p{};
            if ((rc = tm_batch_stats_get(sh[g], b->part[g], &p))) return rc;
            b->mseg[g + 1] = b->mseg[g] + p.matches;
            b->st.topics += p.topics; b->st.visits += p.visits; b->st.hash_hits += p.hash_hits;
            b->st.words += p.words; b->st.matches += p.matches; b->st.slow_topics += p.slow_topics;
            b->st.overflow_tiles += p.overflow_tiles; b->st.probes += p.probes;
            b->st.ms_match = std::max(b->st.ms_match, p.ms_match);
            b->st.ms_total = std::max(b->st.ms_total, p.ms_total);
        }
        const uint64_t total = b->mseg[G];
        if (total > MAX_RESULT) return TM_EOVERFLOW;   // u32 CSR offsets
        // counts and global ids of every part -> the home device, in partition order
        for (DBuf<uint32_t>* x : {&b->counts_p, &b->ids_p, &b->counts_o, &b->src_off, &b->src_bs, &b->dst_off,
                                  &b->dst_bs, &b->rowg, &b->out})
            x->dev = home;
        if ((rc = b->counts_p.reserve(std::max<size_t>(n, 1)))) return rc;
        if ((rc = b->ids_p.reserve(std::max<uint64_t>(total, 1)))) return rc;
        if (b->xcnt.size() != G) {
            b->xcnt.resize(G);
            b->xids.resize(G);
        }
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t ng = b->tseg[g + 1] - b->tseg[g];
            const uint64_t mg = b->mseg[g + 1] - b->mseg[g];
            if (!ng) continue;
            if (dev[g] == home) {   // same device: export straight into place
                if ((rc = tm_batch_export(sh[g], b->part[g], b->counts_p.p + b->tseg[g], b->ids_p.p + b->mseg[g], G, g)))
                    return rc;
                continue;
            }
            b->xcnt[g].dev = b->xids[g].dev = dev[g];
            if ((rc = b->xcnt[g].reserve(ng))) return rc;
            if ((rc = b->xids[g].reserve(std::max<uint64_t>(mg, 1)))) return rc;
            if ((rc = tm_batch_export(sh[g], b->part[g], b->xcnt[g].p, b->xids[g].p, G, g))) return rc;
            SH_HIP(hipSetDevice(home));
            SH_HIP(hipMemcpyAsync(b->counts_p.p + b->tseg[g], b->xcnt[g].p, (size_t)ng * 4, hipMemcpyDeviceToDevice, s));
            if (mg) SH_HIP(hipMemcpyAsync(b->ids_p.p + b->mseg[g], b->xids[g].p, mg * 4, hipMemcpyDeviceToDevice, s));
        }
        const double t2 = now_ms();
        // ---- rows back in publish order (home device)
        if ((rc = b->counts_o.reserve(std::max<size_t>(n, 1)))) return rc;
        if ((rc = b->src_off.reserve((size_t)n + 1))) return rc;
        if ((rc = b->dst_off.reserve((size_t)n + 1))) return rc;
        if ((rc = b->src_bs.reserve(scan_block_count(n) + 1))) return rc;
        if ((rc = b->dst_bs.reserve(scan_block_count(n) + 1))) return rc;
        if ((rc = b->rowg.reserve((size_t)n + 1))) return rc;
        if ((rc = b->out.reserve(std::max<uint64_t>(total, 1)))) return rc;
        SH_HIP(hipSetDevice(home));
        SH_HIP(launch_unpart_counts(b->order.p, b->counts_p.p, n, b->counts_o.p, s));
        ScanArgs ss{};
        ss.count = b->counts_p.p; ss.row_off = b->src_off.p; ss.block_sums = b->src_bs.p; ss.n = n;
        SH_HIP(launch_scan(ss, s, nullptr));
        ScanArgs sd{};
        sd.count = b->counts_o.p; sd.row_off = b->dst_off.p; sd.block_sums = b->dst_bs.p; sd.n = n;
        SH_HIP(launch_scan(sd, s, nullptr));
        SH_HIP(launch_unpart_rows(b->order.p, b->counts_p.p, n, b->src_off.p, b->src_bs.p, b->dst_off.p, b->dst_bs.p,
                                  b->ids_p.p, b->out.p, b->rowg.p, s));
        SH_HIP(hipStreamSynchronize(s));
        const double t3 = now_ms();
        b->ms_partition = (float)(t1 - t0);
        b->ms_parts = (float)(t2 - t1);
        b->ms_unpartition = (float)(t3 - t2);
        b->st.topics = n;
        b->total = total;
        b->done = true;
        return TM_OK;
    }
};

extern "C" {

int tm_sharded_create(const int32_t* devices, uint32_t n, const tm_config* cfg, tm_sharded** out) {
    if (!devices || !n || n > PART_MAX_G || !out) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (devices[i] < 0) return TM_EINVAL;
    tm_sharded* s = new (std::nothrow) tm_sharded();
    if (!s) return TM_ENOMEM;
    s->G = n;
    s->home = devices[0];
    for (uint32_t i = 0; i < n; ++i) {
        tm_config c = cfg ? *cfg : tm_config{0, 0, 0, 0};
        c.device = devices[i];
        c.flags = (c.flags | TM_CFG_FROZEN_DICT) & ~TM_CFG_HOST_TOKENIZE;   // ids agree across shards
        tm_engine* e = nullptr;
        int rc = tm_create(&c, &e);
        if (rc) {
            tm_sharded_destroy(s);
            return rc;
        }
        s->sh.push_back(e);
        s->dev.push_back(devices[i]);
    }
    if (hipSetDevice(s->home) != hipSuccess || hipStreamCreateWithFlags(&s->s, hipStreamNonBlocking) != hipSuccess) {
        tm_sharded_destroy(s);
        return TM_EIO;
    }
    *out = s;
    return TM_OK;
}

void tm_sharded_destroy(tm_sharded* s) {
    if (!s) return;
    if (s->last) tm_sharded_batch_free(s, s->last);
    if (s->s) {
        (void)hipSetDevice(s->home);
        (void)hipStreamSynchronize(s->s);
        (void)hipStreamDestroy(s->s);
    }
    for (tm_engine* e : s->sh) tm_destroy(e);
    delete s;
}

uint32_t tm_sharded_size(tm_sharded* s) { return s ? s->G : 0; }

tm_engine* tm_sharded_engine(tm_sharded* s, uint32_t shard) {
    return (s && shard < s->G) ? s->sh[shard] : nullptr;
}

int tm_sharded_dict_load(tm_sharded* s, const uint8_t* words, const uint64_t* offsets, uint32_t n) {
    if (!s) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    for (tm_engine* e : s->sh) {
        int rc = tm_dict_load(e, words, offsets, n);
        if (rc) return rc;
    }
    return TM_OK;
}

int tm_sharded_insert_many(tm_sharded* s, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                           uint64_t* n_inserted) {
    if (n_inserted) *n_inserted = 0;
    if (!s || !offsets || (!filters && n)) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    try {
        // dictionary delta: the literal words no shard knows, in first-appearance
        // order, appended on every shard (tm_dict_load assigns ids in order)
        uint64_t nwords = 0;
        for (uint32_t i = 0; i < n; ++i) nwords += 1 + std::count(filters + offsets[i], filters + offsets[i + 1], '/');
        std::vector<uint32_t> w(std::max<uint64_t>(nwords, 1)), toff((size_t)n + 1);
        std::vector<uint8_t> fl(std::max<uint32_t>(n, 1));
        uint64_t got = 0;
        int rc = tm_tokenize(s->sh[0], filters, offsets, n, w.data(), w.size(), toff.data(), fl.data(), &got);
        if (rc) return rc;
        std::vector<uint8_t> nb;
        std::vector<uint64_t> no(1, 0);
        std::unordered_set<std::string> seen;
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t* f = filters + offsets[i];
            const size_t len = offsets[i + 1] - offsets[i];
            size_t start = 0;
            uint32_t k = toff[i];
            for (size_t j = 0; j <= len; ++j)
                if (j == len || f[j] == '/') {
                    const uint32_t id = w[k++] & WID_MASK;
                    const size_t wl = j - start;
                    const bool special = wl == 0 || (wl == 1 && (f[start] == '+' || f[start] == '#'));
                    if (id == W_UNKNOWN && !special) {
                        std::string word((const char*)f + start, wl);
                        if (seen.insert(word).second) {
                            nb.insert(nb.end(), f + start, f + j);
                            no.push_back(nb.size());
                        }
                    }
                    start = j + 1;
                }
        }
        if (no.size() > 1) {
            static const uint8_t zero = 0;
            for (tm_engine* e : s->sh)
                if ((rc = tm_dict_load(e, nb.empty() ? &zero : nb.data(), no.data(), (uint32_t)(no.size() - 1))))
                    return rc;
        }
        // each shard keeps its filters and the replicated ones
        std::vector<int> rcs(s->G, TM_OK);
        std::vector<uint64_t> done(s->G, 0);
        s->each([&](uint32_t g) { rcs[g] = tm_trie_insert_many(s->sh[g], filters, offsets, n, g, s->G, &done[g]); });
        uint64_t tot = 0;
        for (uint32_t g = 0; g < s->G; ++g) {
            if (rcs[g]) return rcs[g];
            tot += done[g];
        }
        if (n_inserted) *n_inserted = tot;
        return TM_OK;
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_sharded_delete_many(tm_sharded* s, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                           uint64_t* n_deleted) {
    if (n_deleted) *n_deleted = 0;
    if (!s || !offsets || (!filters && n)) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    // counted like tm_sharded_insert_many: one deletion per shard a present
    // filter lives on (its owner, or every shard for a replicated one)
    uint64_t tot = 0;
    try {
        std::unordered_set<std::string> seen;   // a filter listed twice is deleted once
        for (uint32_t i = 0; i < n; ++i) {
            if (!seen.insert(std::string((const char*)filters + offsets[i], offsets[i + 1] - offsets[i])).second) continue;
            const int o = tm_filter_shard(s->sh[0], filters + offsets[i], offsets[i + 1] - offsets[i], s->G);
            if (o == TM_ENOENT) continue;   // a word no shard knows: the filter is nowhere
            if (o < 0) return o;
            const bool repl = (uint32_t)o >= s->G;
            uint32_t id;   // absent filters are no-ops, not deletions
            if (tm_filter_id(s->sh[repl ? 0 : o], filters + offsets[i], offsets[i + 1] - offsets[i], &id) != TM_OK)
                continue;
            tot += repl ? s->G : 1;
        }
        std::vector<int> rcs(s->G, TM_OK);
        s->each([&](uint32_t g) { rcs[g] = tm_trie_delete_many(s->sh[g], filters, offsets, n, nullptr); });
        for (int rc : rcs)
            if (rc) return rc;
    } catch (...) {
        return TM_ENOMEM;
    }
    if (n_deleted) *n_deleted = tot;
    return TM_OK;
}

int tm_sharded_prepare(tm_sharded* s, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                       tm_sharded_batch** out) {
    if (!s || !offsets || !out || (!topics && n)) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > TM_MAX_TOPIC_LEN) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    const bool fresh = *out == nullptr;
    tm_sharded_batch* b = fresh ? new (std::nothrow) tm_sharded_batch() : *out;
    if (!b) return TM_ENOMEM;
    int rc;
    try {
        b->n = n;
        b->done = false;
        const uint64_t base = offsets[0];
        b->offs.assign(offsets, offsets + (size_t)n + 1);
        for (auto& o : b->offs) o -= base;
        b->bytes.assign(topics + base, topics + base + b->offs[n]);
        rc = s->tokenize(b);
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (rc) {
        if (fresh) tm_sharded_batch_free(s, b);
        return rc;
    }
    *out = b;
    return TM_OK;
}

int tm_sharded_run(tm_sharded* s, tm_sharded_batch* b) {
    if (!s || !b) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    try {
        return s->step(b);
    } catch (...) {
        return TM_ENOMEM;
    }
}

int tm_sharded_result(tm_sharded* s, tm_sharded_batch* b, tm_result* out) {
    if (!s || !b || !out) return TM_EINVAL;
    if (!b->done) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    int rc;
    if ((rc = host_pinned(b->h_row, b->ch_row, (size_t)b->n + 1))) return rc;
    if ((rc = host_pinned(b->h_ids, b->ch_ids, std::max<uint64_t>(b->total, 1)))) return rc;
    const uint32_t* d_row = b->rowg.p;
    const uint32_t* d_ids = b->out.p;
    if (b->direct) {   // one shard: the part's CSR (built here on first use)
        uint64_t m = 0;
        if ((rc = tm_batch_device_csr(s->sh[0], b->part[0], &d_row, &d_ids, &m))) return rc;
    }
    SH_HIP(hipSetDevice(s->home));
    SH_HIP(hipMemcpyAsync(b->h_row, d_row, ((size_t)b->n + 1) * 4, hipMemcpyDeviceToHost, s->s));
    if (b->total) SH_HIP(hipMemcpyAsync(b->h_ids, d_ids, b->total * 4, hipMemcpyDeviceToHost, s->s));
    SH_HIP(hipStreamSynchronize(s->s));
    if (b->h_row[b->n] != b->total) {
        snprintf(error_buf(), 512, "inconsistent sharded CSR: %u vs %llu", b->h_row[b->n], (unsigned long long)b->total);
        return TM_EIO;
    }
    out->n_topics = b->n;
    out->n_matches = b->total;
    out->row_offsets = b->h_row;
    out->filter_ids = b->h_ids;
    return TM_OK;
}

int tm_sharded_device_csr(tm_sharded* s, tm_sharded_batch* b, const uint32_t** d_row_offsets, const uint32_t** d_ids,
                          uint64_t* n_matches) {
    if (!s || !b || !b->done) return TM_EINVAL;
    if (b->direct) {
        std::lock_guard<std::mutex> lk(s->mu);
        return tm_batch_device_csr(s->sh[0], b->part[0], d_row_offsets, d_ids, n_matches);
    }
    if (d_row_offsets) *d_row_offsets = b->rowg.p;
    if (d_ids) *d_ids = b->out.p;
    if (n_matches) *n_matches = b->total;
    return TM_OK;
}

int tm_sharded_batch_stats(tm_sharded* s, tm_sharded_batch* b, tm_sharded_stats* out) {
    if (!s || !b || !out) return TM_EINVAL;
    out->match = b->st;
    out->ms_partition = b->ms_partition;
    out->ms_parts = b->ms_parts;
    out->ms_unpartition = b->ms_unpartition;
    for (uint32_t g = 0; g < 64; ++g) out->part_topics[g] = g < s->G && !b->tseg.empty() ? b->tseg[g + 1] - b->tseg[g] : 0;
    return TM_OK;
}

void tm_sharded_batch_free(tm_sharded* s, tm_sharded_batch* b) {
    if (!b) return;
    if (s) {
        for (size_t g = 0; g < b->part.size() && g < s->sh.size(); ++g)
            if (b->part[g]) tm_batch_free(s->sh[g], b->part[g]);
        if (s->last == b) s->last = nullptr;
    }
    b->release();
    delete b;
}

int tm_sharded_match_batch(tm_sharded* s, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                           tm_result* out) {
    if (!s || !out) return TM_EINVAL;
    int rc = tm_sharded_prepare(s, topics, offsets, n, &s->last);
    if (!rc) rc = tm_sharded_run(s, s->last);
    if (!rc) rc = tm_sharded_result(s, s->last, out);
    return rc;
}

int tm_sharded_filter_copy(tm_sharded* s, uint32_t gid, uint8_t* buf, size_t cap, size_t* len) {
    if (!s || !len) return TM_EINVAL;
    return tm_filter_copy(s->sh[gid % s->G], gid / s->G, buf, cap, len);
}

}  // extern "C"
