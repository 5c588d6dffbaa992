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
//
// A batch is cut into G contiguous slices; slice i lives on shard i's device
// (its bytes tokenised there at prepare), so no device handles more than 1/G
// of the batch outside its own walk.  One step, all of it queued before the
// host waits once:
//   source i (its own stream):  owner per publish (tm_tokens_shard) -> a
//     stable counting sort by owner (tm_part_*) whose scatter writes every
//     publish's tokens straight into its owner's batch, after the parts of
//     slices < i (same device: local stores; another device: stores into the
//     peer's HBM over xGMI); when peer access is unavailable the part of
//     slice i owned by shard j is kept contiguous here and staged through
//     pinned host memory;
//   dest j (its part batch's stream): waits for every source (and copies in
//     the staged parts), then walks its batch (the launch checks the tokens
//     on the device);
//   the home stream joins every part: ONE host wait, then each part's control
//     words are checked (a capacity miss relaunches that part: another wait).
// The sizes of the (slice i -> shard j) parts are the batch's plan, made at
// prepare (the same kernels plus one read-back), and re-checked against the
// device's counts after every step.  A step leaves each shard's rows where its
// walk wrote them; the publish-order CSR with global ids (local id * G +
// shard) is built on request (tm_sharded_result / device_csr), like the
// single engine's dense CSR.
// The multi-process form with RCCL all_to_all is emqx_amd/sharded.py.
//
// Reference: the filter set is the mnesia-replicated trie
// (src/emqx_trie.erl:53-74) that every node matches in full
// (src/emqx_router.erl:127-141); sharding it is new.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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

float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

// Peer access between two devices, both ways: LINK_PEER when the runtime
// grants it (xGMI on an MI355X node), LINK_STAGED otherwise (copies bounce
// through pinned host memory).  Test knob TM_SHARD_LINK (so that a one-GPU
// box runs every link kind's code): "staged" forces the staged path (alias
// TM_SHARD_STAGED=1); "peer" takes the peer path for a pair on one device
// (a peer store / hipMemcpyPeer into the same HBM); "probe" runs the
// runtime's peer probe even for a device paired with itself, where peer
// access is refused -- the denied branch, which must fall back to staged.
uint8_t open_link(int a, int b, const std::string& mode) {
    if (mode == "staged") return TM_LINK_STAGED;
    if (a == b && mode == "peer") return TM_LINK_PEER;
    if (a == b && mode != "probe") return TM_LINK_SAME;
    int ab = 0, ba = 0;
    if (hipDeviceCanAccessPeer(&ab, a, b) != hipSuccess || hipDeviceCanAccessPeer(&ba, b, a) != hipSuccess || !ab ||
        !ba) {
        (void)hipGetLastError();
        return TM_LINK_STAGED;
    }
    const int pairs[2][2] = {{a, b}, {b, a}};
    for (const auto& p : pairs) {
        if (hipSetDevice(p[0]) != hipSuccess) {
            (void)hipGetLastError();
            return TM_LINK_STAGED;
        }
        const hipError_t e = hipDeviceEnablePeerAccess(p[1], 0);
        (void)hipGetLastError();
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return TM_LINK_STAGED;
    }
    return TM_LINK_PEER;
}

}  // namespace

// Slice i of a batch: its publishes, tokenised and partitioned on shard i's device.
struct Slice {
    uint32_t lo = 0, n = 0;        // publishes [lo, lo + n) of the batch
    uint64_t nwords = 0;
    DBuf<uint32_t> words, toff, owner, cnt, wcnt, cnt_off, cnt_bs, w_off, w_bs, segs, order, ptoff, pwords;
    DBuf<uint8_t> tflags, ptflags;
    uint32_t* h_segs = nullptr;    // the last step's partition counts (read back with its wait)
    size_t ch_segs = 0;
    std::vector<uint32_t> seg;     // the plan: [0..G] first publish of each owner's part, [G+1..2G+1] first word

    void on(int d) {
        for (DBuf<uint32_t>* x : {&words, &toff, &owner, &cnt, &wcnt, &cnt_off, &cnt_bs, &w_off, &w_bs, &segs, &order,
                                  &ptoff, &pwords})
            x->dev = d;
        tflags.dev = ptflags.dev = d;
    }
    void release() {
        for (DBuf<uint32_t>* x : {&words, &toff, &owner, &cnt, &wcnt, &cnt_off, &cnt_bs, &w_off, &w_bs, &segs, &order,
                                  &ptoff, &pwords})
            x->release();
        tflags.release();
        ptflags.release();
        if (h_segs) (void)hipHostFree(h_segs);
        h_segs = nullptr;
        ch_segs = 0;
    }
    uint32_t part_n(uint32_t j) const { return seg[j + 1] - seg[j]; }
    uint32_t part_w(uint32_t G, uint32_t j) const { return seg[G + 2 + j] - seg[G + 1 + j]; }
};

struct tm_sharded_batch {
    uint32_t n = 0;
    uint64_t dict_words = ~0ull;          // dictionary size the plan was made with
    // the publishes, rebased (re-planned if the dictionary grew), in pinned
    // memory: the tokenisers' uploads run at the DMA's rate, not through the
    // runtime's staging of pageable memory
    uint8_t* bytes = nullptr;
    uint64_t* offs = nullptr;
    size_t c_bytes = 0, c_offs = 0;
    std::vector<Slice> src;               // G slices (G > 1)
    std::vector<tm_batch*> part;          // shard j's part batch (its engine)
    std::vector<PartBuffers> pb;
    std::vector<uint32_t> pn;             // shard j: publishes it walks
    std::vector<uint64_t> pw;             //          their words
    std::vector<uint32_t> R, W;           // [i * G + j]: where slice i's part lands in shard j's batch
    uint32_t* h_close = nullptr;          // pinned: shard j's closing word offset
    size_t ch_close = 0;
    std::vector<uint8_t*> bounce;         // staged links: [i * G + j] pinned [toff | words | tflags]
    std::vector<size_t> cbounce;
    // publish-order CSR with global ids on the home device (built on request)
    DBuf<uint32_t> counts_p, ids_p, gorder, counts_o, src_off, src_bs, dst_off, dst_bs, rowg, out;
    std::vector<DBuf<uint32_t>> xcnt, xids;
    std::vector<uint64_t> mseg;           // first match of each part (+ total), in shard order
    uint64_t total = 0;
    bool done = false;
    bool ordered = false;
    uint32_t *h_row = nullptr, *h_ids = nullptr;
    size_t ch_row = 0, ch_ids = 0;
    tm_batch_stats st{};
    float ms_partition = 0, ms_exchange = 0, ms_step = 0, ms_unpartition = 0;
    float ms_stage = 0, ms_plan = 0;      // the last prepare: bytes into pinned memory; the plan (uploads, tokenisers)
    uint32_t host_waits = 0;

    void release() {
        for (auto& sl : src) sl.release();
        for (DBuf<uint32_t>* b : {&counts_p, &ids_p, &gorder, &counts_o, &src_off, &src_bs, &dst_off, &dst_bs, &rowg,
                                  &out})
            b->release();
        for (auto& x : xcnt) x.release();
        for (auto& x : xids) x.release();
        for (uint8_t* p : bounce)
            if (p) (void)hipHostFree(p);
        bounce.clear();
        for (uint32_t* h : {h_row, h_ids, h_close})
            if (h) (void)hipHostFree(h);
        h_row = h_ids = h_close = nullptr;
        if (bytes) (void)hipHostFree(bytes);
        if (offs) (void)hipHostFree(offs);
        bytes = nullptr;
        offs = nullptr;
        c_bytes = c_offs = 0;
    }
};

struct tm_sharded {
    std::vector<tm_engine*> sh;
    std::vector<int32_t> dev;
    uint32_t G = 0;
    int home = -1;
    hipStream_t s = nullptr;                 // home device: the step's join, the on-request reorder
    std::vector<hipStream_t> ss;             // shard g's device: its slice's partition
    std::vector<hipEvent_t> ev_p0, ev_p1, ev_x0, ev_x1, ev_done;   // per shard, on its device
    std::vector<uint8_t> link;               // [i * G + j]: TM_LINK_*
    std::mutex mu;                           // one step (and one mutation) at a time
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

    // a blocking copy between shards' devices (the on-request reorder)
    int copy_now(uint32_t i, uint32_t j, void* dst, const void* src, size_t bytes) {
        if (!bytes) return TM_OK;
        const uint8_t l = link[i * G + j];
        if (l == TM_LINK_STAGED) {
            std::vector<uint8_t> tmp(bytes);
            SH_HIP(hipSetDevice(dev[i]));
            SH_HIP(hipMemcpy(tmp.data(), src, bytes, hipMemcpyDeviceToHost));
            SH_HIP(hipSetDevice(dev[j]));
            SH_HIP(hipMemcpy(dst, tmp.data(), bytes, hipMemcpyHostToDevice));
        } else if (l == TM_LINK_PEER) {
            SH_HIP(hipSetDevice(dev[j]));
            SH_HIP(hipMemcpyPeer(dst, dev[j], src, dev[i], bytes));
        } else {
            SH_HIP(hipSetDevice(dev[j]));
            SH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
        }
        return TM_OK;
    }

    PartArgs part_args(Slice& S) {
        PartArgs a{};
        a.owner = S.owner.p; a.words = S.words.p; a.toff = S.toff.p; a.tflags = S.tflags.p;
        a.n = S.n; a.G = G; a.nb = std::max<uint32_t>(1, (S.n + PART_BLOCK - 1) / PART_BLOCK);
        a.cnt = S.cnt.p; a.wcnt = S.wcnt.p;
        a.cnt_off = S.cnt_off.p; a.cnt_bs = S.cnt_bs.p; a.w_off = S.w_off.p; a.w_bs = S.w_bs.p;
        a.segs = S.segs.p; a.order = S.order.p; a.ptoff = S.ptoff.p; a.ptflags = S.ptflags.p;
        a.pwords = S.pwords.p;
        return a;
    }

    // owner + counts of slice i's parts (no scatter), on shard i's stream
    int enqueue_counts(Slice& S, const PartArgs& a, hipStream_t st) {
        const uint32_t gb = G * a.nb;
        SH_HIP(launch_tokens_shard(S.words.p, S.toff.p, S.n, G, S.owner.p, st));
        SH_HIP(launch_part_count(a, st));
        ScanArgs sc{};
        sc.count = S.cnt.p; sc.row_off = S.cnt_off.p; sc.block_sums = S.cnt_bs.p; sc.n = gb;
        SH_HIP(launch_scan(sc, st, nullptr));
        ScanArgs sw{};
        sw.count = S.wcnt.p; sw.row_off = S.w_off.p; sw.block_sums = S.w_bs.p; sw.n = gb;
        SH_HIP(launch_scan(sw, st, nullptr));
        SH_HIP(launch_part_segs(a, st));
        return TM_OK;
    }

    // Prepare-time: every slice tokenised on its shard's device, its parts
    // counted (the plan: how many publishes and words of slice i shard j
    // walks, and where they land in shard j's batch), every shard's part batch
    // sized.  One shard: the slice is tokenised straight into the part batch.
    //
    // uoffs / st: called by tm_sharded_prepare while the staging threads are
    // still copying the batch into b->bytes / b->offs (TokStaged); the slice
    // bounds then come from the caller's own offsets uoffs.
    int plan(tm_sharded_batch* b, const uint64_t* uoffs = nullptr, const TokStaged* st = nullptr) {
        int rc;
        const uint32_t n = b->n;
        const uint8_t* bytes = b->bytes;
        // the bytes of topics [lo, hi) and where they start in b->bytes
        auto span = [&](uint32_t lo, uint32_t hi, uint64_t& at) -> uint64_t {
            at = st ? uoffs[lo] - uoffs[0] : b->offs[lo];
            return (st ? uoffs[hi] - uoffs[0] : b->offs[hi]) - at;
        };
        auto tokenize = [&](uint32_t i, uint32_t lo, uint32_t cnt, uint32_t* w, uint64_t wcap, uint32_t* toff,
                            uint8_t* tfl, uint64_t* nw) {
            if (!st) return tm_tokenize_device(sh[i], bytes, b->offs + lo, cnt, w, wcap, toff, tfl, nw);
            uint64_t at;
            const uint64_t nb = span(lo, lo + cnt, at);
            return tokenize_device_staged(sh[i], bytes, b->offs + lo, cnt, at, nb, lo, *st, w, wcap, toff, tfl, nw);
        };
        b->dict_words = dict_words();
        b->done = b->ordered = false;
        if (b->part.size() != G) {
            b->part.assign(G, nullptr);
            b->pb.assign(G, PartBuffers{});
        }
        b->pn.assign(G, 0);
        b->pw.assign(G, 0);
        if (G == 1) {
            uint64_t at;
            const uint64_t cap = span(0, n, at) + n + 1;
            if ((rc = part_batch_buffers(sh[0], &b->part[0], n, cap, &b->pb[0]))) return rc;
            uint64_t nw = 0;
            if ((rc = tokenize(0, 0, n, b->pb[0].words, b->pb[0].words_cap, b->pb[0].toff, b->pb[0].tflags, &nw)))
                return rc;
            b->pn[0] = n;
            b->pw[0] = nw;
            return part_batch_buffers(sh[0], &b->part[0], n, nw, &b->pb[0]);
        }
        b->src.resize(G);
        std::vector<int> rcs(G, TM_OK);
        each([&](uint32_t i) {   // slices in parallel: each tokeniser waits on its own device
            Slice& S = b->src[i];
            S.lo = (uint32_t)((uint64_t)n * i / G);
            S.n = (uint32_t)((uint64_t)n * (i + 1) / G) - S.lo;
            S.on(dev[i]);
            S.seg.assign(2 * ((size_t)G + 1), 0);
            uint64_t at;
            const uint64_t nbytes = span(S.lo, S.lo + S.n, at);
            int r;
            const uint32_t nb = std::max<uint32_t>(1, (S.n + PART_BLOCK - 1) / PART_BLOCK), gb = G * nb;
            if ((r = S.words.reserve(nbytes + S.n + 1)) || (r = S.toff.reserve((size_t)S.n + 1)) ||
                (r = S.tflags.reserve(std::max<size_t>(S.n, 1))) || (r = S.owner.reserve(std::max<size_t>(S.n, 1))) ||
                (r = S.cnt.reserve(gb)) || (r = S.wcnt.reserve(gb)) || (r = S.cnt_off.reserve((size_t)gb + 1)) ||
                (r = S.w_off.reserve((size_t)gb + 1)) || (r = S.cnt_bs.reserve(scan_block_count(gb) + 1)) ||
                (r = S.w_bs.reserve(scan_block_count(gb) + 1)) || (r = S.segs.reserve(2 * ((size_t)G + 1))) ||
                (r = S.order.reserve(std::max<size_t>(S.n, 1))) || (r = S.ptoff.reserve((size_t)S.n + G)) ||
                (r = S.ptflags.reserve(std::max<size_t>(S.n, 1))) ||
                (r = host_pinned(S.h_segs, S.ch_segs, 2 * ((size_t)G + 1)))) {
                rcs[i] = r;
                return;
            }
            uint64_t nw = 0;
            if ((r = tokenize(i, S.lo, S.n, S.words.p, S.words.cap, S.toff.p, S.tflags.p, &nw))) {
                rcs[i] = r;
                return;
            }
            S.nwords = nw;
            if ((r = S.pwords.reserve(std::max<uint64_t>(nw, 1)))) { rcs[i] = r; return; }
            if (!S.n) return;
            if (hipSetDevice(dev[i]) != hipSuccess) { rcs[i] = TM_EIO; return; }
            const PartArgs a = part_args(S);
            if ((r = enqueue_counts(S, a, ss[i]))) { rcs[i] = r; return; }
            if (hipMemcpyAsync(S.h_segs, S.segs.p, 2 * ((size_t)G + 1) * 4, hipMemcpyDeviceToHost, ss[i]) !=
                    hipSuccess ||
                hipStreamSynchronize(ss[i]) != hipSuccess) {
                snprintf(error_buf(), 512, "partition plan of slice %u failed", i);
                rcs[i] = TM_EIO;
                return;
            }
            S.seg.assign(S.h_segs, S.h_segs + 2 * ((size_t)G + 1));
            if (S.seg[G] != S.n || S.seg[2 * G + 1] != nw) {
                snprintf(error_buf(), 512, "partition of slice %u lost publishes: %u of %u, %u of %llu words", i,
                         S.seg[G], S.n, S.seg[2 * G + 1], (unsigned long long)nw);
                rcs[i] = TM_EIO;
            }
        });
        for (int r : rcs)
            if (r) return r;
        // where slice i's part lands in shard j's batch: after the parts of slices < i
        b->R.assign((size_t)G * G, 0);
        b->W.assign((size_t)G * G, 0);
        for (uint32_t j = 0; j < G; ++j) {
            uint64_t rn = 0, rw = 0;
            for (uint32_t i = 0; i < G; ++i) {
                const Slice& S = b->src[i];
                b->R[i * G + j] = (uint32_t)rn;
                b->W[i * G + j] = (uint32_t)rw;
                rn += S.n ? S.part_n(j) : 0;
                rw += S.n ? S.part_w(G, j) : 0;
                // (after every slice, the last included: shard j's part batch
                // and the scatter's word offsets are u32)
                if (rn > 0xFFFFFFF0ull || rw > 0xFFFFFFF0ull) {
                    snprintf(error_buf(), 512, "shard %u's part exceeds u32 offsets: %llu publishes, %llu words", j,
                             (unsigned long long)rn, (unsigned long long)rw);
                    return TM_EOVERFLOW;
                }
            }
            b->pn[j] = (uint32_t)rn;
            b->pw[j] = rw;
        }
        if ((rc = host_pinned(b->h_close, b->ch_close, G))) return rc;
        for (uint32_t j = 0; j < G; ++j) {
            b->h_close[j] = (uint32_t)b->pw[j];
            if ((rc = part_batch_buffers(sh[j], &b->part[j], b->pn[j], b->pw[j], &b->pb[j]))) return rc;
        }
        // staged links bounce through pinned host memory: [toff | words | tflags]
        b->bounce.resize((size_t)G * G, nullptr);
        b->cbounce.resize((size_t)G * G, 0);
        for (uint32_t i = 0; i < G; ++i)
            for (uint32_t j = 0; j < G; ++j) {
                if (link[i * G + j] != TM_LINK_STAGED || !b->src[i].n) continue;
                const Slice& S = b->src[i];
                const size_t need = (size_t)S.part_n(j) * 5 + (size_t)S.part_w(G, j) * 4 + 16;
                if ((rc = host_pinned(b->bounce[i * G + j], b->cbounce[i * G + j], need))) return rc;
            }
        return TM_OK;
    }

    int step(tm_sharded_batch* b) {
        int rc;
        const double t0 = now_ms();
        b->done = b->ordered = false;
        b->host_waits = 0;
        if (b->dict_words != dict_words() && (rc = plan(b))) return rc;   // new words since the plan
        uint32_t waits = 0;
        // ---- sources: owner + partition of every slice on its own device
        if (G > 1) {
            for (uint32_t i = 0; i < G; ++i) {
                Slice& S = b->src[i];
                SH_HIP(hipSetDevice(dev[i]));
                SH_HIP(hipEventRecord(ev_p0[i], ss[i]));
                if (S.n) {
                    PartArgs a = part_args(S);
                    a.tbase = S.lo;
                    for (uint32_t j = 0; j < G; ++j) {
                        a.wbase[j] = b->W[i * G + j];
                        if (link[i * G + j] == TM_LINK_STAGED) continue;
                        // same device or a peer: the scatter writes into shard j's batch itself
                        a.dtoff[j] = b->pb[j].toff;
                        a.dflags[j] = b->pb[j].tflags;
                        a.dwords[j] = b->pb[j].words;
                        a.rbase[j] = b->R[i * G + j];
                    }
                    if ((rc = enqueue_counts(S, a, ss[i]))) return rc;
                    SH_HIP(launch_part_scatter(a, ss[i]));
                    SH_HIP(hipMemcpyAsync(S.h_segs, S.segs.p, 2 * ((size_t)G + 1) * 4, hipMemcpyDeviceToHost, ss[i]));
                    for (uint32_t j = 0; j < G; ++j) {   // staged links: the part goes out to pinned memory
                        if (link[i * G + j] != TM_LINK_STAGED) continue;
                        const uint32_t pn = S.part_n(j), pw = S.part_w(G, j);
                        uint8_t* bb = b->bounce[i * G + j];
                        if (pn) SH_HIP(hipMemcpyAsync(bb, S.ptoff.p + S.seg[j] + j, (size_t)pn * 4, hipMemcpyDeviceToHost, ss[i]));
                        if (pw) SH_HIP(hipMemcpyAsync(bb + (size_t)pn * 4, S.pwords.p + S.seg[G + 1 + j], (size_t)pw * 4,
                                                      hipMemcpyDeviceToHost, ss[i]));
                        if (pn) SH_HIP(hipMemcpyAsync(bb + (size_t)pn * 4 + (size_t)pw * 4, S.ptflags.p + S.seg[j], pn,
                                                      hipMemcpyDeviceToHost, ss[i]));
                    }
                }
                SH_HIP(hipEventRecord(ev_p1[i], ss[i]));
            }
        }
        // ---- shards: their parts land in their batches, which walk them
        for (uint32_t j = 0; j < G; ++j) {
            const PartBuffers& P = b->pb[j];
            SH_HIP(hipSetDevice(dev[j]));
            if (G > 1) {
                for (uint32_t i = 0; i < G; ++i) SH_HIP(hipStreamWaitEvent(P.stream, ev_p1[i], 0));
                SH_HIP(hipEventRecord(ev_x0[j], P.stream));
                for (uint32_t i = 0; i < G; ++i) {
                    const Slice& S = b->src[i];
                    if (!S.n) continue;
                    const uint32_t pn = S.part_n(j), pw = S.part_w(G, j);
                    uint32_t* dtoff = P.toff + b->R[i * G + j];
                    uint32_t* dwords = P.words + b->W[i * G + j];
                    uint8_t* dflags = P.tflags + b->R[i * G + j];
                    if (link[i * G + j] == TM_LINK_STAGED) {
                        const uint8_t* bb = b->bounce[i * G + j];
                        if (pn) SH_HIP(hipMemcpyAsync(dtoff, bb, (size_t)pn * 4, hipMemcpyHostToDevice, P.stream));
                        if (pw) SH_HIP(hipMemcpyAsync(dwords, bb + (size_t)pn * 4, (size_t)pw * 4, hipMemcpyHostToDevice,
                                                      P.stream));
                        if (pn) SH_HIP(hipMemcpyAsync(dflags, bb + (size_t)pn * 4 + (size_t)pw * 4, pn,
                                                      hipMemcpyHostToDevice, P.stream));
                    }
                    // (same device or a peer: written there by the source's scatter)
                }
                SH_HIP(hipMemcpyAsync(P.toff + b->pn[j], b->h_close + j, 4, hipMemcpyHostToDevice, P.stream));
                SH_HIP(hipEventRecord(ev_x1[j], P.stream));
            }
            if ((rc = tm_batch_launch(sh[j], b->part[j]))) return rc;
            SH_HIP(hipSetDevice(dev[j]));
            SH_HIP(hipEventRecord(ev_done[j], P.stream));
        }
        // ---- one host wait: the home stream joins every part
        SH_HIP(hipSetDevice(home));
        for (uint32_t j = 0; j < G; ++j) SH_HIP(hipStreamWaitEvent(s, ev_done[j], 0));
        SH_HIP(hipStreamSynchronize(s));
        ++waits;
        if (G > 1)
            for (uint32_t i = 0; i < G; ++i) {   // the device's partition must be the plan
                const Slice& S = b->src[i];
                if (S.n && !std::equal(S.seg.begin(), S.seg.end(), S.h_segs)) {
                    snprintf(error_buf(), 512, "slice %u partitioned differently from its plan", i);
                    return TM_EIO;
                }
            }
        int first = TM_OK;
        for (uint32_t j = 0; j < G; ++j) {   // every part is checked, even after an error
            rc = part_batch_finish(sh[j], b->part[j], &waits);
            if (rc && !first) first = rc;
        }
        if (first) return first;
        b->st = tm_batch_stats{};
        b->mseg.assign(G + 1, 0);
        for (uint32_t j = 0; j < G; ++j) {
            tm_batch_stats p{};
            if ((rc = tm_batch_stats_get(sh[j], b->part[j], &p))) return rc;
            b->mseg[j + 1] = b->mseg[j] + p.matches;
            b->st.topics += p.topics; b->st.visits += p.visits; b->st.hash_hits += p.hash_hits;
            b->st.words += p.words; b->st.matches += p.matches; b->st.slow_topics += p.slow_topics;
            b->st.overflow_tiles += p.overflow_tiles; b->st.probes += p.probes;
            b->st.ms_match = std::max(b->st.ms_match, p.ms_match);
            b->st.ms_total = std::max(b->st.ms_total, p.ms_total);
        }
        b->total = b->mseg[G];
        if (b->total > MAX_RESULT) return TM_EOVERFLOW;   // u32 CSR offsets
        b->ms_partition = b->ms_exchange = 0;
        if (G > 1)
            for (uint32_t g = 0; g < G; ++g) {
                b->ms_partition = std::max(b->ms_partition, elapsed(ev_p0[g], ev_p1[g]));
                b->ms_exchange = std::max(b->ms_exchange, elapsed(ev_x0[g], ev_x1[g]));
            }
        b->ms_step = (float)(now_ms() - t0);
        b->host_waits = waits;
        b->st.topics = b->n;
        b->done = true;
        return TM_OK;
    }

    // The publish-order CSR with global ids on the home device, from the
    // shards' rows: each part's counts and ids (id * G + shard) to the home
    // device, the slices' partition orders as one publish index per walked
    // position, and the rows moved into publish order (tm_unpart_*).
    int order_rows(tm_sharded_batch* b) {
        if (b->ordered) return TM_OK;
        int rc;
        const double t0 = now_ms();
        const uint32_t n = b->n;
        const uint64_t total = b->total;
        for (DBuf<uint32_t>* x : {&b->counts_p, &b->ids_p, &b->gorder, &b->counts_o, &b->src_off, &b->src_bs,
                                  &b->dst_off, &b->dst_bs, &b->rowg, &b->out})
            x->dev = home;
        if ((rc = b->counts_p.reserve(std::max<size_t>(n, 1))) || (rc = b->ids_p.reserve(std::max<uint64_t>(total, 1))) ||
            (rc = b->gorder.reserve(std::max<size_t>(n, 1))) || (rc = b->counts_o.reserve(std::max<size_t>(n, 1))) ||
            (rc = b->src_off.reserve((size_t)n + 1)) || (rc = b->dst_off.reserve((size_t)n + 1)) ||
            (rc = b->src_bs.reserve(scan_block_count(n) + 1)) || (rc = b->dst_bs.reserve(scan_block_count(n) + 1)) ||
            (rc = b->rowg.reserve((size_t)n + 1)) || (rc = b->out.reserve(std::max<uint64_t>(total, 1))))
            return rc;
        if (b->xcnt.size() != G) {
            b->xcnt.resize(G);
            b->xids.resize(G);
        }
        uint64_t pbase = 0;
        for (uint32_t j = 0; j < G; ++j) {
            const uint32_t nj = b->pn[j];
            const uint64_t mj = b->mseg[j + 1] - b->mseg[j];
            if (nj) {
                if (dev[j] == home && link[j * G + 0] != TM_LINK_STAGED) {   // export straight into place
                    if ((rc = tm_batch_export(sh[j], b->part[j], b->counts_p.p + pbase, b->ids_p.p + b->mseg[j], G, j)))
                        return rc;
                } else {
                    b->xcnt[j].dev = b->xids[j].dev = dev[j];
                    if ((rc = b->xcnt[j].reserve(nj)) || (rc = b->xids[j].reserve(std::max<uint64_t>(mj, 1)))) return rc;
                    if ((rc = tm_batch_export(sh[j], b->part[j], b->xcnt[j].p, b->xids[j].p, G, j))) return rc;
                    if ((rc = copy_now(j, 0, b->counts_p.p + pbase, b->xcnt[j].p, (size_t)nj * 4))) return rc;
                    if ((rc = copy_now(j, 0, b->ids_p.p + b->mseg[j], b->xids[j].p, mj * 4))) return rc;
                }
            }
            // the publish walked at each position of shard j's batch
            for (uint32_t i = 0; i < G; ++i) {
                const Slice& S = b->src[i];
                if (!S.n || !S.part_n(j)) continue;
                if ((rc = copy_now(i, 0, b->gorder.p + pbase + b->R[i * G + j], S.order.p + S.seg[j],
                                   (size_t)S.part_n(j) * 4)))
                    return rc;
            }
            pbase += nj;
        }
        SH_HIP(hipSetDevice(home));
        SH_HIP(launch_unpart_counts(b->gorder.p, b->counts_p.p, n, b->counts_o.p, s));
        ScanArgs ss_{};
        ss_.count = b->counts_p.p; ss_.row_off = b->src_off.p; ss_.block_sums = b->src_bs.p; ss_.n = n;
        SH_HIP(launch_scan(ss_, s, nullptr));
        ScanArgs sd{};
        sd.count = b->counts_o.p; sd.row_off = b->dst_off.p; sd.block_sums = b->dst_bs.p; sd.n = n;
        SH_HIP(launch_scan(sd, s, nullptr));
        SH_HIP(launch_unpart_rows(b->gorder.p, b->counts_p.p, n, b->src_off.p, b->src_bs.p, b->dst_off.p, b->dst_bs.p,
                                  b->ids_p.p, b->out.p, b->rowg.p, s));
        SH_HIP(hipStreamSynchronize(s));
        b->ms_unpartition = (float)(now_ms() - t0);
        b->ordered = true;
        return TM_OK;
    }

    // device pointers of the publish-order CSR (built on first use)
    int device_csr(tm_sharded_batch* b, const uint32_t** d_row, const uint32_t** d_ids) {
        if (G == 1) {   // one shard: the part's own CSR, global id = local id
            uint64_t m = 0;
            return tm_batch_device_csr(sh[0], b->part[0], d_row, d_ids, &m);
        }
        int rc = order_rows(b);
        if (rc) return rc;
        *d_row = b->rowg.p;
        *d_ids = b->out.p;
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
    s->ss.assign(n, nullptr);
    for (auto* v : {&s->ev_p0, &s->ev_p1, &s->ev_x0, &s->ev_x1, &s->ev_done}) v->assign(n, nullptr);
    for (uint32_t i = 0; i < n; ++i) {
        tm_config c = cfg ? *cfg : tm_config{0, 0, 0, 0};
        c.device = devices[i];
        // the shards mutate in parallel (each()): their host workers share the
        // process's CPUs instead of 16 per shard
        if (!c.host_threads && n > 1) {
            const unsigned hw = std::thread::hardware_concurrency();
            c.host_threads = std::max(1u, std::min(hw ? hw : 1u, 16u) / n);
        }
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
    // every shard copies parts to every other: open the links both ways
    s->link.assign((size_t)n * n, TM_LINK_SAME);
    const Knobs kn = Knobs::read();
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = i; j < n; ++j)
            s->link[i * n + j] = s->link[j * n + i] = open_link(devices[i], devices[j], kn.shard_link);
    bool ok = hipSetDevice(s->home) == hipSuccess && hipStreamCreateWithFlags(&s->s, hipStreamNonBlocking) == hipSuccess;
    for (uint32_t g = 0; ok && g < n; ++g) {
        ok = hipSetDevice(devices[g]) == hipSuccess &&
             hipStreamCreateWithFlags(&s->ss[g], hipStreamNonBlocking) == hipSuccess;
        for (auto* v : {&s->ev_p0, &s->ev_p1, &s->ev_x0, &s->ev_x1, &s->ev_done})
            ok = ok && hipEventCreate(&(*v)[g]) == hipSuccess;
    }
    if (!ok) {
        (void)hipGetLastError();
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
    for (size_t g = 0; g < s->ss.size() && g < s->dev.size(); ++g) {
        (void)hipSetDevice(s->dev[g]);
        if (s->ss[g]) {
            (void)hipStreamSynchronize(s->ss[g]);
            (void)hipStreamDestroy(s->ss[g]);
        }
        for (auto* v : {&s->ev_p0, &s->ev_p1, &s->ev_x0, &s->ev_x1, &s->ev_done})
            if ((*v)[g]) (void)hipEventDestroy((*v)[g]);
    }
    for (tm_engine* e : s->sh) tm_destroy(e);
    delete s;
}

uint32_t tm_sharded_size(tm_sharded* s) { return s ? s->G : 0; }

int tm_sharded_link(tm_sharded* s, uint32_t i, uint32_t j) {
    if (!s || i >= s->G || j >= s->G) return TM_EINVAL;
    return s->link[i * s->G + j];
}

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
    if (offsets[n] < offsets[0]) return TM_EINVAL;   // (each topic is checked while the offsets are staged)
    std::lock_guard<std::mutex> lk(s->mu);
    const bool fresh = *out == nullptr;
    tm_sharded_batch* b = fresh ? new (std::nothrow) tm_sharded_batch() : *out;
    if (!b) return TM_ENOMEM;
    int rc;
    try {
        b->n = n;
        b->done = b->ordered = false;
        const uint64_t base = offsets[0], nbytes = offsets[n] - base;
        const double t0 = now_ms();
        if ((rc = host_pinned(b->offs, b->c_offs, (size_t)n + 1)) ||
            (rc = host_pinned(b->bytes, b->c_bytes, nbytes + 16)))   // (+16: the tokenisers' 16-B windows)
            throw std::bad_alloc();
        // copied by several threads (one would take ~30 ms for a 10M-publish
        // batch), which check every topic on the way: offsets that do not
        // decrease, names of at most ?MAX_TOPIC_LEN bytes (src/emqx_topic.erl:45).
        // The copy is cut into items taken in order (the bytes, then the
        // offsets), and the plan's tokenisers upload each item as soon as it is
        // in place: the DMA runs behind the copy instead of after it.
        constexpr uint64_t CB = 4ull << 20, CO = 512ull << 10;
        const uint64_t nbi = (nbytes + CB - 1) / CB, noi = ((uint64_t)n + 1 + CO - 1) / CO;
        std::vector<uint8_t> ready(nbi + noi, 0);
        bool bad = false;
        std::atomic<uint64_t> next{0};
        std::mutex staged_mu;
        float staged_ms = 0;   // when the last staging thread ran out of items
        auto stage = [&] {
            for (uint64_t it; (it = next.fetch_add(1, std::memory_order_relaxed)) < nbi + noi;) {
                if (it < nbi) {
                    const uint64_t c0 = it * CB, c1 = std::min(nbytes, c0 + CB);
                    memcpy(b->bytes + c0, topics + base + c0, c1 - c0);
                } else {
                    const uint64_t o0 = (it - nbi) * CO, o1 = std::min<uint64_t>((uint64_t)n + 1, o0 + CO);
                    bool ok = true;
                    for (uint64_t i = o0; i < o1; ++i) {
                        b->offs[i] = offsets[i] - base;
                        if (i < n) ok &= offsets[i + 1] >= offsets[i] && offsets[i + 1] - offsets[i] <= TM_MAX_TOPIC_LEN;
                    }
                    if (!ok) __atomic_store_n(&bad, true, __ATOMIC_RELEASE);
                }
                __atomic_store_n(&ready[it], (uint8_t)1, __ATOMIC_RELEASE);
            }
            const float t = (float)(now_ms() - t0);
            std::lock_guard<std::mutex> g(staged_mu);
            staged_ms = std::max(staged_ms, t);
        };
        const unsigned T = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(16, (nbytes + n * 8) >> 22));
        std::vector<std::thread> th;
        // joins the staging threads on every way out of this scope (a throw
        // from plan() or from a thread's creation included): a joinable
        // std::thread destroyed by the unwind would std::terminate, and the
        // threads use the locals above, which outlive this guard
        struct Joiner {
            std::vector<std::thread>& th;
            ~Joiner() {
                for (auto& t : th)
                    if (t.joinable()) t.join();
            }
        } joiner{th};
        for (unsigned k = 0; k < T; ++k) th.emplace_back(stage);
        b->dict_words = ~0ull;
        const TokStaged st{ready.data(), &bad, CB, CO, (uint32_t)nbi};
        const double t1 = now_ms();
        rc = s->plan(b, offsets, &st);
        b->ms_plan = (float)(now_ms() - t1);
        for (auto& t : th) t.join();
        b->ms_stage = staged_ms;
        if (bad) {
            b->n = 0;                 // (a re-prepared batch keeps nothing of the refused one:
            b->dict_words = ~0ull;    //  its next step re-plans)
            rc = TM_EINVAL;
        }
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
    const uint32_t *d_row = nullptr, *d_ids = nullptr;
    try {
        if ((rc = s->device_csr(b, &d_row, &d_ids))) return rc;
    } catch (...) {
        return TM_ENOMEM;
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
    std::lock_guard<std::mutex> lk(s->mu);
    const uint32_t *r = nullptr, *i = nullptr;
    int rc;
    try {
        rc = s->device_csr(b, &r, &i);
    } catch (...) {
        rc = TM_ENOMEM;
    }
    if (rc) return rc;
    if (d_row_offsets) *d_row_offsets = r;
    if (d_ids) *d_ids = i;
    if (n_matches) *n_matches = b->total;
    return TM_OK;
}

int tm_sharded_batch_stats(tm_sharded* s, tm_sharded_batch* b, tm_sharded_stats* out) {
    if (!s || !b || !out) return TM_EINVAL;
    memset(out, 0, sizeof *out);
    out->match = b->st;
    out->ms_partition = b->ms_partition;
    out->ms_exchange = b->ms_exchange;
    out->ms_step = b->ms_step;
    out->ms_unpartition = b->ms_unpartition;
    out->host_waits = b->host_waits;
    out->ms_stage = b->ms_stage;
    out->ms_plan = b->ms_plan;
    for (uint32_t g = 0; g < 64; ++g) out->part_topics[g] = g < s->G && g < b->pn.size() ? b->pn[g] : 0;
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
