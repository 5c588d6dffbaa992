// tm_engine_impl.hpp -- the engine's host-side state (struct tm_engine) and
// the helpers its modules share.  Internal: included by the engine's modules
// only, never by callers of the C ABI (include/emqx_tm.h).
//
// The engine's code is split by concern:
//   tm_engine.cpp    the C ABI entry points, emqx_topic predicates
//   tm_churn.cpp     trie mutations: emqx_trie insert/delete, the parallel
//                    mutation pass (plan, edge phase, summaries)
//   tm_upload.cpp    delta uploads of the host trie to every HBM replica
//   tm_batch.cpp     batches: tokenise, dedup, upload, launch, wait, the CSR
//   tm_async.cpp     the per-publish async pipeline (launcher, completers)
//   tm_pipeline.cpp  engine setup, multi-replica splits, chunked host pipelines
//   tm_fanout.cpp    routes, subscriptions, fan-out dispatch, rule predicates
//
// Owns: the word interner (emqx_topic:words/1 tokens -> u32 ids), the host
// mirror of the compiled trie (node table + the open-addressed edge hash that is
// byte-identical to the HBM replica), the delta log that keeps the replica in
// sync (read-your-writes: deltas are applied on the engine stream before every
// match launch), batch tokenisation, and the orchestration of the device
// pipeline in tm_kernels.hip.
//
// Trie semantics follow src/emqx_trie.erl exactly (insert/1 :81-93, add_path/1
// :145-158, delete/1 :107-116, delete_path/1 :190-204, lookup/1, empty/0); the
// node record's edge_count is kept so that emqx_trie:lookup/1 answers match
// the reference's tests (test/emqx_trie_SUITE.erl:49-142).
#pragma once

#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <deque>
#include <functional>
#include <set>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/emqx_tm.h"
#include "tm_internal.hpp"

using namespace etm;

namespace etm_host {

#define HIP_OK(expr)                                                        \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) {                                             \
            snprintf(last_error(), 512, "%s at %s:%d (%s)", hipGetErrorString(_e), \
                     __FILE_NAME__, __LINE__, #expr);               \
            return TM_EIO;                                                  \
        }                                                                   \
    } while (0)

// text of the last TM_EIO on this thread (one buffer for every module: etm::error_buf)
inline char* last_error() { return error_buf(); }

// word hash (tm_internal.hpp hw_*; the device tokeniser computes the same)
inline uint64_t hash_word(const uint8_t* p, size_t n, uint32_t seed = HW_SEED) {
    uint32_t h = seed;
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
        uint32_t v;
        memcpy(&v, p + i, 4);
        h = hw_step(h, v);
    }
    if (i < n) {
        uint32_t t = 0;
        for (size_t k = 0; i + k < n; ++k) t |= (uint32_t)p[i + k] << (8 * k);
        h = hw_step(h, t);
    }
    return hw_final(h, (uint32_t)n);
}

// 64-bit hash of a whole topic (TM_BATCH_DEDUP)
inline uint64_t hash_bytes(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull ^ (n * 0x9E3779B97F4A7C15ull);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v;
        memcpy(&v, p + i, 8);
        h = (h ^ (v * 0xBF58476D1CE4E5B9ull)) * 0x94D049BB133111EBull;
        h ^= h >> 29;
    }
    uint64_t t = 0;
    for (size_t k = 0; i < n; ++i, ++k) t |= (uint64_t)p[i] << (8 * k);
    h = (h ^ (t * 0xBF58476D1CE4E5B9ull)) * 0x94D049BB133111EBull;
    return h ^ (h >> 31);
}

// ------------------------------------------------------------- word interner
// Open-addressed string -> id map; bytes live in an append-only arena.  The
// device tokeniser gets its own mirror: a 2-choice cuckoo table of probe keys
// (tm_internal.hpp DictKey) at load <= 1/4 plus the per-id tails; ck_dirty_
// lists the cuckoo slots written since the last upload, ck_gen_ counts
// rebuilds (full upload); tails and arena only grow.
class WordDict {
  public:
    WordDict() {
        rehash(1024);
        ck_rebuild(1024);
    }

    uint32_t find(const uint8_t* p, size_t n) const { return find_h(p, n, hash_word(p, n)); }

    // the hash of a word, its home entry prefetched (batched lookups: hash
    // and prefetch a group of words, then find_h each)
    uint64_t prefetch(const uint8_t* p, size_t n) const {
        const uint64_t h = hash_word(p, n);
        __builtin_prefetch(&tab_[h & mask_]);
        return h;
    }

    uint32_t find_h(const uint8_t* p, size_t n, uint64_t h) const {
        size_t i = h & mask_;
        for (;;) {
            const DictEnt& e = tab_[i];
            if (e.h == 0) return W_UNKNOWN;
            if (e.h == h && e.len == n) {
                // up to 16 bytes compare inline (head, head2), longer words in the arena
                if (n <= 16) {
                    if (e.head == le_bytes(p, (uint32_t)std::min<size_t>(n, 8)) &&
                        e.head2 == (n > 8 ? le_bytes(p + 8, (uint32_t)(n - 8)) : 0))
                        return e.id;
                } else if (memcmp(arena_.data() + e.off, p, n) == 0) {
                    return e.id;
                }
            }
            i = (i + 1) & mask_;
        }
    }

    uint32_t intern(const uint8_t* p, size_t n) {
        uint32_t id = find(p, n);
        if (id != W_UNKNOWN) return id;
        if (next_id_ > WID_MASK) throw std::bad_alloc();   // word ids fill WID_BITS (slot + topic entries)
        if ((count_ + 1) * 2 > tab_.size()) rehash(tab_.size() * 2);
        id = next_id_++;
        const uint64_t h = hash_word(p, n);
        size_t i = h & mask_;
        while (tab_[i].h) i = (i + 1) & mask_;
        tab_[i] = DictEnt{h, le_bytes(p, (uint32_t)std::min<size_t>(n, 8)),
                          n > 8 ? le_bytes(p + 8, (uint32_t)std::min<size_t>(n - 8, 8)) : 0, (uint32_t)n, id,
                          arena_.size(), 0};
        arena_.insert(arena_.end(), p, p + n);
        ++count_;
        if (tails_.size() <= id) tails_.resize((size_t)id + 1, DictTail{0, 0});
        tails_[id] = DictTail{tab_[i].head2, tab_[i].off};
        const uint64_t hh = (uint32_t)h | (hash_word(p, n, HW_SEED2) << 32);
        if (count_ * 4 > ck_.size()) ck_rebuild(ck_.size() * 2);
        else if (!ck_put(DictKey{tab_[i].head, (uint32_t)n, id}, hh)) ck_rebuild(ck_.size() * 2);
        return id;
    }

    size_t size() const { return count_; }
    const std::vector<uint8_t>& arena() const { return arena_; }
    const std::vector<DictKey>& keys() const { return ck_; }
    const std::vector<DictTail>& tails() const { return tails_; }
    uint64_t gen() const { return ck_gen_; }
    std::vector<uint32_t>& dirty() { return ck_dirty_; }

  private:
    // cuckoo insert with a random walk of evictions; h = h1 | h2 << 32; false:
    // the table must grow
    bool ck_put(DictKey k, uint64_t h) {
        const uint32_t m = (uint32_t)ck_.size() - 1;
        uint32_t from = ~0u;
        for (int kick = 0; kick < 512; ++kick) {
            const uint32_t a = (uint32_t)h & m, b = (uint32_t)(h >> 32) & m;
            const uint32_t i = ck_[a].id == 0 ? a : ck_[b].id == 0 ? b : (a != from ? a : b);
            std::swap(k, ck_[i]);
            std::swap(h, ck_h_[i]);
            ck_dirty_.push_back(i);
            if (k.id == 0) return true;
            from = i;
        }
        return false;   // k is homeless: the rebuild reinserts every word from tab_
    }

    void ck_rebuild(size_t cap) {
        for (;;) {
            // independent hashes place any set at load 1/4; never grow without bound
            if (cap > 64 * std::max<size_t>(count_, 1024)) throw std::bad_alloc();
            ck_.assign(cap, DictKey{0, 0, 0});
            ck_h_.assign(cap, 0);
            bool ok = true;
            for (const DictEnt& e : tab_)
                if (e.h && !ck_put(DictKey{e.head, e.len, e.id},
                                   (uint32_t)e.h | (hash_word(arena_.data() + e.off, e.len, HW_SEED2) << 32))) {
                    ok = false;
                    break;
                }
            if (ok) break;
            cap *= 2;
        }
        ck_dirty_.clear();
        ++ck_gen_;
    }

    void rehash(size_t cap) {
        std::vector<DictEnt> old;
        old.swap(tab_);
        tab_.assign(cap, DictEnt{0, 0, 0, 0, 0, 0, 0});
        mask_ = cap - 1;
        for (const DictEnt& e : old)
            if (e.h) {
                size_t i = e.h & mask_;
                while (tab_[i].h) i = (i + 1) & mask_;
                tab_[i] = e;
            }
    }
    std::vector<DictEnt> tab_;
    std::vector<uint8_t> arena_;
    size_t mask_ = 0, count_ = 0;
    uint32_t next_id_ = W_FIRST;
    std::vector<DictKey> ck_;
    std::vector<uint64_t> ck_h_;   // h1 | h2 << 32 of each slot's key (relocation)
    std::vector<uint32_t> ck_dirty_;
    std::vector<DictTail> tails_;
    uint64_t ck_gen_ = 0;
};

struct TWord {
    const uint8_t* p;
    uint32_t n;
};

// binary:split(T, <<"/">>, [global]) (src/emqx_topic.erl:153-154)
inline void split_words(const uint8_t* t, size_t len, std::vector<TWord>& out) {
    out.clear();
    size_t start = 0;
    for (size_t i = 0; i <= len; ++i) {
        if (i == len || t[i] == '/') {
            out.push_back(TWord{t + start, (uint32_t)(i - start)});
            start = i + 1;
        }
    }
}

inline bool is_plus(const TWord& w) { return w.n == 1 && w.p[0] == '+'; }
inline bool is_hash(const TWord& w) { return w.n == 1 && w.p[0] == '#'; }

// word class for the path-code digits (tm_internal.hpp C_*), and whether the
// word makes the topic irregular (starts with '+' but is not '+').
inline uint32_t word_class(const TWord& w, bool& irregular) {
    if (w.n == 0) return C_EMPTY;
    const uint8_t c = w.p[0];
    if (w.n == 1 && c == '+') return C_ABOVE;
    if (c == '+') { irregular = true; return C_ABOVE; }
    if (c < '#') return C_BELOW;
    if (c < '+') return C_BETWEEN;
    return C_ABOVE;
}

template <class T>
void dev_free(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

template <class T>
int dev_reserve(T*& p, size_t& cap, size_t n, bool keep = false, size_t keep_n = 0) {
    if (n <= cap && p) return TM_OK;
    size_t nc = std::max<size_t>(n + n / 4, 1024);
    T* np = nullptr;
    HIP_OK(hipMalloc((void**)&np, nc * sizeof(T)));
    if (keep && p && keep_n) HIP_OK(hipMemcpy(np, p, keep_n * sizeof(T), hipMemcpyDeviceToDevice));
    dev_free(p);
    p = np;
    cap = nc;
    return TM_OK;
}

template <class T>
int host_reserve(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return TM_OK;
    size_t nc = std::max<size_t>(n + n / 4, 1024);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    HIP_OK(hipHostMalloc((void**)&p, nc * sizeof(T), hipHostMallocDefault));
    cap = nc;
    return TM_OK;
}

// pinned host memory the device writes directly (tm_export_host): coherent,
// so a kernel's stores are visible to the host once its completion is
inline int host_reserve_coherent(uint8_t*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap && p) return TM_OK;
    const size_t nc = std::max<size_t>(bytes + bytes / 4, 4096);
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    HIP_OK(hipHostMalloc((void**)&p, nc, hipHostMallocCoherent | hipHostMallocMapped));
    cap = nc;
    return TM_OK;
}

// Allocator of the host mirror's big random-access tables (edge hash, node
// records): blocks of 4 MB and more are mapped 2-MB aligned with
// MADV_HUGEPAGE before first touch, so a churn delta's random lines do not
// each cost a page walk (THP is "madvise" on these hosts).
template <class T>
struct HugeAlloc {
    using value_type = T;
    static constexpr size_t HUGE = 2u << 20, MIN_BYTES = 4u << 20;
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U>&) {}
    T* allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < MIN_BYTES) return std::allocator<T>().allocate(n);
        const size_t span = (bytes + HUGE - 1) / HUGE * HUGE;
        const size_t len = span + HUGE;   // room to align
        void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        const uintptr_t p0 = (uintptr_t)p, a = (p0 + HUGE - 1) & ~(uintptr_t)(HUGE - 1);
        if (a > p0) munmap(p, a - p0);                                  // head before the aligned start
        if (p0 + len > a + span) munmap((void*)(a + span), p0 + len - (a + span));   // and the tail
        (void)madvise((void*)a, span, MADV_HUGEPAGE);
        return reinterpret_cast<T*>(a);
    }
    void deallocate(T* p, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < MIN_BYTES) { std::allocator<T>().deallocate(p, n); return; }
        munmap(p, (bytes + HUGE - 1) / HUGE * HUGE);   // exactly the mapping allocate() kept
    }
    template <class U>
    bool operator==(const HugeAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const HugeAlloc<U>&) const { return false; }
};

// host worker threads when tm_config.host_threads is 0: TM_HOST_THREADS, else
// min(hardware threads, 16) -- the GPU box leases 16 CPUs of cgroup bandwidth
// out of 256 hardware threads, so hardware_concurrency() alone overcounts.
inline unsigned default_threads(const Knobs& k) {
    if (k.host_threads) return k.host_threads;
    unsigned h = std::thread::hardware_concurrency();
    return std::max(1u, std::min(h ? h : 1u, 16u));
}

// The CPUs of the NUMA node `device` is attached to (sysfs), within this
// process's affinity, for the churn workers -- so the host mirror's pages they
// first-touch and their random reads stay on one socket.  On by default since
// late round 4 (C5 K = 100 churn, three processes each on the 2-socket box:
// unpinned 1.72 / 2.18 / 1.95 ms per step, pinned 1.40 / 1.50 / 1.77,
// profiles/r04/aj/); TM_POOL_PIN=0 turns it off.  False (no pinning) for a
// host-only engine, a node-less device or fewer CPUs than `need`.
inline bool device_node_cpus(int device, unsigned need, bool pin, cpu_set_t& out) {
    if (device < 0 || !pin) return false;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus - 1, device) != hipSuccess) return false;
    for (char* c = bus; *c; ++c) *c = (char)tolower((unsigned char)*c);
    auto read_line = [](const std::string& path) {
        std::string s;
        if (FILE* f = fopen(path.c_str(), "r")) {
            char buf[4096];
            if (fgets(buf, sizeof buf, f)) s = buf;
            fclose(f);
        }
        return s;
    };
    const std::string nodes = read_line(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
    if (nodes.empty()) return false;
    const int node = atoi(nodes.c_str());
    if (node < 0) return false;
    const std::string list = read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
    cpu_set_t mine;
    CPU_ZERO(&mine);
    if (list.empty() || sched_getaffinity(0, sizeof mine, &mine) != 0) return false;
    CPU_ZERO(&out);
    for (const char* p = list.c_str(); *p && *p != '\n';) {   // "0-63,128-191"
        char* e;
        const long a = strtol(p, &e, 10);
        long b = a;
        if (e == p) return false;
        if (*e == '-') b = strtol(e + 1, &e, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET(c, &mine)) CPU_SET(c, &out);
        p = *e == ',' ? e + 1 : e;
    }
    return (unsigned)CPU_COUNT(&out) >= need;
}

}  // namespace etm_host
using namespace etm_host;

#ifndef TM_SLOW_WAVES_MAX
#define TM_SLOW_WAVES_MAX 4096   // C5 K=1000 device: 512 waves 7.75 ms, 2048 4.54, 4096 4.03 (round 2, tools/ab_slow.sh); with 8 KB of LDS per wave (round 6) 3072 1.81, 4096 1.66, 5120 1.87, 8192 1.90 (tools/ab_slow_waves.sh)
#endif

// ===================================================================== batch

struct tm_batch {
    uint32_t n = 0;
    uint64_t nwords = 0;
    uint64_t dict_size = 0;     // interner size at tokenisation (re-tokenise if it grew)
    // host copy of the input (to re-tokenise after concurrent subscribes)
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs;
    // host tokens
    std::vector<uint32_t> h_words, h_toff, h_slow;
    // TM_BATCH_DEDUP: rows are per distinct topic; row_of[i] = row of publish i
    bool dedup = false;
    uint32_t n_pub = 0;
    std::vector<uint32_t> row_of;
    std::vector<uint8_t> h_tflags;
    // device inputs
    uint32_t *d_words = nullptr, *d_toff = nullptr, *d_slow = nullptr;
    uint8_t* d_tflags = nullptr;
    size_t c_words = 0, c_toff = 0, c_slow = 0, c_tflags = 0;
    // device outputs
    uint32_t *d_sfids = nullptr, *d_rowoff = nullptr, *d_ids = nullptr;
    unsigned long long* d_rows = nullptr;
    unsigned long long* d_wstats = nullptr;   // the walk waves' partial stats
    size_t c_wstats = 0;
    uint8_t* d_pack = nullptr;                // the dense ids packed 3 bytes each (tm_match_batch_packed)
    size_t c_pack = 0;
    uint32_t *d_bsums = nullptr, *d_ovf = nullptr, *d_total = nullptr;
    size_t c_sfids = 0, c_rows = 0, c_rowoff = 0, c_ids = 0, c_bsums = 0, c_ovf = 0;
    uint32_t* h_total = nullptr;
    size_t ch_total = 0;
    size_t c_total = 0;
    // Per-topic outputs in ONE block, [ctrl CTRL_WORDS u32 | stats ST_N u64 |
    // src cap u64 | count cap u32], mirrored in pinned memory: the async path
    // reads a whole batch's control words and row descriptors back in one copy.
    uint8_t *d_hdr = nullptr, *h_hdr = nullptr;
    size_t hdr_cap = 0;   // topics the block holds
    uint32_t *d_count = nullptr, *d_ctrl = nullptr, *h_ctrl = nullptr, *h_count = nullptr;
    unsigned long long *d_src = nullptr, *d_stats = nullptr, *h_src = nullptr, *h_stats = nullptr;
    static constexpr size_t HDR_FIXED = ((size_t)XG_WORD + TICKET_GROUPS * TICKET_STRIDE) * 4;
    static size_t hdr_bytes(size_t n) { return HDR_FIXED + n * 12; }
    // pinned host results
    uint32_t* h_rowoff = nullptr;
    uint32_t* h_ids = nullptr;
    size_t ch_rowoff = 0, ch_ids = 0;
    uint8_t* h_ids8 = nullptr;                // the ids 3 bytes each (tm_batch_result_packed)
    size_t ch_ids8 = 0;
    // the replica (device copy of the trie) the batch runs on; fixed for the
    // batch's life: its buffers live on that replica's device
    struct Replica* rep = nullptr;
    // the stream the batch runs on: async slots own one, other batches use the replica's
    hipStream_t own = nullptr;
    hipEvent_t ev_read = nullptr;   // own-stream batches: marks their walk for the replica's next upload
    // the batch's whole pipeline (header clear, walk, generic path, scan,
    // finalize, read-back of the control words) captured as a HIP graph and
    // replayed while its launch arguments stay the same (small batches: one
    // launch instead of ten API calls and their gaps)
    hipGraphExec_t gexec = nullptr;
    std::vector<uint8_t> gkey;      // the arguments gexec was captured with, or of the last direct launch
    bool gbad = false;              // capture failed once: this batch launches directly
    // A bounded batch (the async slots' fresh batches, tm_async.cpp): sized
    // for n topics and bytes_cap bytes once, its input read by the tokeniser
    // straight from mapped pinned memory and its count from *d_nb (pinned
    // too), so every launch has the same arguments and replays one captured
    // graph: tokeniser, walk, generic path and `tail` (the slot's export).
    bool bounded = false;
    uint32_t* d_nb = nullptr;
    std::function<hipError_t(hipStream_t)> tail;
    std::vector<uint8_t> tail_key;  // the tail's arguments (part of the graph key)
    bool tail_done = false;         // the last launch enqueued the tail (in the graph)
    bool own_user = false;   // TM_BATCH_STREAM: a caller's batch on a stream of its own (async slots: false)
    // generic-path scratch, per batch (batches on different streams run concurrently)
    uint32_t s_waves = 0, s_qcap = 1u << 13, s_ocap = 1u << 14;
    uint32_t *d_sqpar = nullptr, *d_sqpw = nullptr, *d_sqmeta = nullptr, *d_sofid = nullptr;
    unsigned long long *d_sqkey = nullptr, *d_sokey = nullptr;
    size_t c_sq = 0, c_so = 0, c_sq2 = 0, c_sq3 = 0, c_so2 = 0, c_sq4 = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    hipEvent_t evt = nullptr;   // before the device tokeniser (fresh launches)
    hipEvent_t evc0 = nullptr, evc1 = nullptr;   // around the dense-CSR pass (ensure_dense)
    // after the launch's last read-back: wait() syncs on it, not on the stream,
    // so work queued behind the batch (a trie delta upload) does not hold it
    hipEvent_t ev_end = nullptr;
    bool end_recorded = false;
    // one-shot launch (tm_match_batch): the dense CSR is built and copied into
    // mapped host memory behind the walk, so the batch costs one host wait
    bool oneshot = false;
    bool eager_dense = false;       // scan + finalize enqueued by launch (oneshot implies it)
    uint64_t dense_cap = 0;         // ids the enqueued finalize could hold
    bool dense_enq = false;         // the LAST launch enqueued scan + finalize (set by launch, read by wait)
    std::vector<uint32_t> h_smp_off, h_smp_ids;   // tm_batch_sample's last result (host CSR)
    uint8_t* d_smp_meta = nullptr;   // tm_batch_sample's device scratch, kept (a hipFree per call
    uint32_t* d_smp_ids = nullptr;   //  would synchronise the device under the other streams)
    size_t c_smp_meta = 0, c_smp_ids = 0;
    // TM_BATCH_DEDUP on the device (device-tokenised batches, etm::DedupArgs):
    // the n_pub publishes are deduplicated by their bytes, and only the rows
    // (distinct topics) are tokenised and walked; n becomes the row count once
    // a launch has been waited
    bool dedup_dev = false;
    bool dedup_stale = false;       // fresh bytes (prepare / retokenize): the next launch deduplicates
    bool dedup_timed = false;       // the last launch deduplicated: evd.. is its time
    bool rowof_host = false;        // row_of holds the device map of the last dedup pass
    unsigned long long *d_dtab = nullptr, *d_psrc = nullptr, *d_dbits = nullptr;
    uint32_t *d_dslot = nullptr, *d_dbc = nullptr, *d_dbb = nullptr, *d_drbs = nullptr, *d_dbbs = nullptr;
    uint32_t *d_dsrow = nullptr, *d_drrep = nullptr;
    uint4* d_dsmeta = nullptr;
    size_t c_dsmeta = 0;
    unsigned long long* d_dbsum = nullptr;
    size_t c_dbsum = 0;
    uint32_t *d_rowof = nullptr, *d_dd = nullptr, *d_pcount = nullptr;
    uint8_t* d_cbytes = nullptr;
    uint64_t* d_coffs = nullptr;
    size_t c_drrep = 0;
    size_t c_dtab = 0, c_psrc = 0, c_dsrow = 0, c_dbits = 0, c_dslot = 0, c_dbc = 0, c_dbb = 0, c_drbs = 0,
           c_dbbs = 0, c_rowof = 0;
    size_t c_dd = 0, c_pcount = 0, c_cbytes = 0, c_coffs = 0;
    uint64_t dtab_mask = 0, dd_bytes = 0;
    // the table is zero between passes (the expansion clears the claimed
    // slots); dirty: a pass was enqueued and its expansion not yet waited
    // for, or the table is new -- the next pass clears it first
    bool dtab_dirty = true;
    hipEvent_t evd = nullptr, evx0 = nullptr, evx1 = nullptr;   // before the dedup pass; around the expand
    uint64_t x_cap = 0;             // ids the last one-shot copy could hold
    uint8_t *h_xrow = nullptr, *h_xids = nullptr;
    size_t c_xrow = 0, c_xids = 0;
    hipEvent_t evq = nullptr;   // at the launch call: evq..ev0 (or evt) is the queueing ahead of it
    // the waited result is the walk's own: row i = sfids[src[i] .. + count[i]);
    // dense = the CSR (row_off, ids) has been built from it since the last launch
    bool dense = false;
    bool tok_timed = false;     // the last launch tokenised: evt..ev0 is its time
    bool graphed = false;       // the last launch replayed a captured dedup graph (expand untimed)
    bool launched = false, done = false;
    // staging as one region shared by every walk group (set when one group's
    // reservation alone would need more than the staging limit / TICKET_GROUPS)
    bool one_region = false;
    bool csr = true;   // the last launch built the CSR (false: async, rows left in staging)
    uint64_t seq = 0;  // launch sequence number while its results may be read (0: none)
    uint64_t total = 0;
    tm_batch_stats st{};
    ScanArgs scan_args{};
    // token batches (tm_batch_prepare_tokens): no bytes to re-tokenise; with
    // device-resident tokens the generic-path list is built on the device
    bool tokens_only = false;
    bool dev_slow = false;
    // a part batch of the in-process sharded group: its token buffers are
    // written by the group's copies, checked on the device by every launch
    // (tm_token_check) and the verdict read back with the header
    bool check_tokens = false;
    // device tokenisation: the topic bytes are uploaded by prepare and tokenised
    // on the engine stream by the first launch, after the dictionary deltas; a
    // later launch re-tokenises only if the dictionary grew meanwhile (ids of
    // existing words never change), like the host path's re-tokenise
    bool dev_tok = false;
    uint64_t tok_dict = ~0ull;   // dict.size() the device tokens were made with
    uint8_t* d_bytes = nullptr;
    uint64_t* d_boffs = nullptr;
    // the tokeniser's inputs: d_bytes / d_boffs, or both inside d_in when the
    // batch came as one packed [offs | bytes] block (async slots: one H2D)
    uint8_t* d_in = nullptr;
    size_t c_in = 0;
    const uint8_t* in_bytes = nullptr;
    const uint64_t* in_offs = nullptr;
    uint64_t seen_upload = 0;   // own-stream batches: the last trie upload this batch's stream waited for
    uint32_t* d_wcount = nullptr;
    size_t c_bytes = 0, c_boffs = 0, c_wcount = 0;
    uint64_t tok_base = 0;
    uint32_t *d_nslow = nullptr, *h_bad = nullptr;
    size_t c_nslow = 0, ch_bad = 0;
    // route resolution (tm_batch_routes)
    uint32_t *d_rcount = nullptr, *d_rrow = nullptr, *d_rbsums = nullptr, *d_rfid = nullptr, *d_rdest = nullptr;
    uint32_t* d_reoff = nullptr;   // route scan over match entries
    size_t c_reoff = 0;
    uint32_t *d_rtotal = nullptr, *h_rtotal = nullptr, *h_rrow = nullptr, *h_rfid = nullptr, *h_rdest = nullptr;
    size_t c_rcount = 0, c_rrow = 0, c_rbsums = 0, c_rfid = 0, c_rdest = 0, c_rtotal = 0;
    size_t ch_rtotal = 0, ch_rrow = 0, ch_rfid = 0, ch_rdest = 0;
    // subscriber fan-out (tm_batch_dispatch)
    uint64_t *d_moff = nullptr, *d_fbsums = nullptr, *d_ftotal = nullptr, *d_drow = nullptr, *d_ftile = nullptr;
    uint32_t* d_moff32 = nullptr;
    uint8_t* d_fbig = nullptr;
    size_t c_moff32 = 0, c_fbig = 0;
    uint32_t* d_dcount = nullptr;   // TM_DISPATCH_ROWS: deliveries of each row
    size_t c_dcount = 0;
    uint64_t *d_fmeta = nullptr, *h_fmeta = nullptr;   // TM_DISPATCH_ROWS: staging regions (vb, rtop)
    size_t c_fmeta = 0, ch_fmeta = 0;
    uint64_t *h_ftotal = nullptr, *h_drow = nullptr, *h_moff = nullptr;
    uint32_t *d_fout = nullptr, *h_fout = nullptr;
    size_t c_moff = 0, c_fbsums = 0, c_ftotal = 0, c_drow = 0, c_fout = 0, c_ftile = 0;
    size_t ch_ftotal = 0, ch_drow = 0, ch_moff = 0, ch_fout = 0;
    hipEvent_t fev0 = nullptr, fev1 = nullptr;

    void release() {
        dev_free(d_moff); dev_free(d_moff32); dev_free(d_fbig); dev_free(d_dcount); dev_free(d_fmeta);
        if (h_fmeta) (void)hipHostFree(h_fmeta);
        h_fmeta = nullptr; dev_free(d_fbsums); dev_free(d_ftotal); dev_free(d_drow); dev_free(d_fout);
        dev_free(d_ftile);
        for (uint64_t** h : {&h_ftotal, &h_drow, &h_moff}) {
            if (*h) (void)hipHostFree(*h);
            *h = nullptr;
        }
        if (h_fout) (void)hipHostFree(h_fout);
        h_fout = nullptr;
        if (fev0) (void)hipEventDestroy(fev0);
        if (fev1) (void)hipEventDestroy(fev1);
        fev0 = fev1 = nullptr;
        dev_free(d_reoff);
        dev_free(d_rcount); dev_free(d_rrow); dev_free(d_rbsums); dev_free(d_rfid); dev_free(d_rdest); dev_free(d_rtotal);
        for (uint32_t** h : {&h_rtotal, &h_rrow, &h_rfid, &h_rdest}) {
            if (*h) (void)hipHostFree(*h);
            *h = nullptr;
        }
        dev_free(d_nslow);
        dev_free(d_drrep); dev_free(d_dbsum); dev_free(d_dsmeta);
        c_drrep = c_dbsum = c_dsmeta = 0;
        dev_free(d_dtab); dev_free(d_psrc); dev_free(d_dsrow); dev_free(d_dbits); dev_free(d_dslot); dev_free(d_dbc);
        dev_free(d_dbb); dev_free(d_drbs); dev_free(d_dbbs); dev_free(d_rowof); dev_free(d_dd); dev_free(d_pcount);
        dev_free(d_cbytes); dev_free(d_coffs);
        dtab_dirty = true;
        dev_free(d_smp_meta); dev_free(d_smp_ids);
        c_smp_meta = c_smp_ids = 0;
        c_dtab = c_psrc = c_dsrow = c_dbits = c_dslot = c_dbc = c_dbb = c_drbs = c_dbbs = c_rowof = 0;
        c_dd = c_pcount = c_cbytes = c_coffs = 0;
        for (hipEvent_t* ev : {&evd, &evx0, &evx1}) {
            if (*ev) (void)hipEventDestroy(*ev);
            *ev = nullptr;
        }
        dev_free(d_bytes); dev_free(d_boffs); dev_free(d_wcount); dev_free(d_in);
        in_bytes = nullptr;
        in_offs = nullptr;
        if (h_bad) (void)hipHostFree(h_bad);
        h_bad = nullptr;
        dev_free(d_words); dev_free(d_toff); dev_free(d_slow); dev_free(d_tflags);
        dev_free(d_sfids); dev_free(d_rows); dev_free(d_rowoff); dev_free(d_ids);
        dev_free(d_wstats); dev_free(d_pack);
        c_wstats = c_pack = 0;
        if (h_total) (void)hipHostFree(h_total);
        h_total = nullptr;
        dev_free(d_bsums); dev_free(d_ovf); dev_free(d_total);
        dev_free(d_hdr);
        if (h_hdr) (void)hipHostFree(h_hdr);
        h_hdr = nullptr;
        hdr_cap = 0;
        d_count = d_ctrl = h_ctrl = h_count = nullptr;
        d_src = d_stats = h_src = h_stats = nullptr;
        dev_free(d_sqpar); dev_free(d_sqpw); dev_free(d_sqmeta); dev_free(d_sqkey); dev_free(d_sofid); dev_free(d_sokey);
        c_sq = c_so = c_sq2 = c_sq3 = c_so2 = c_sq4 = 0;
        if (h_rowoff) (void)hipHostFree(h_rowoff);
        if (h_ids) (void)hipHostFree(h_ids);
        h_rowoff = h_ids = nullptr;
        if (h_ids8) (void)hipHostFree(h_ids8);
        h_ids8 = nullptr;
        ch_ids8 = 0;
        if (h_xrow) (void)hipHostFree(h_xrow);
        if (h_xids) (void)hipHostFree(h_xids);
        h_xrow = h_xids = nullptr;
        c_xrow = c_xids = 0;
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (ev2) (void)hipEventDestroy(ev2);
        if (evt) (void)hipEventDestroy(evt);
        if (ev_read) (void)hipEventDestroy(ev_read);
        if (evc0) (void)hipEventDestroy(evc0);
        if (evc1) (void)hipEventDestroy(evc1);
        if (ev_end) (void)hipEventDestroy(ev_end);
        if (evq) (void)hipEventDestroy(evq);
        ev0 = ev1 = ev2 = evt = ev_read = evc0 = evc1 = ev_end = evq = nullptr;
        end_recorded = false;
        if (gexec) (void)hipGraphExecDestroy(gexec);
        gexec = nullptr;
        gkey.clear();
    }
};

// ==================================================================== engine

// ------------------------------------------------------------ async matching
// One tm_match_async call.
struct AsyncCall {
    tm_match_cb cb;
    void* ctx;
};

// One device batch of the async pipeline: a tm_batch on a stream of its own,
// its inputs in pinned memory, and the read-back of its rows.
struct AsyncSlot {
    tm_batch b;
    std::vector<uint8_t> bytes;          // the calls' topics, concatenated
    std::vector<uint64_t> offs;
    std::vector<AsyncCall> calls;
    uint8_t* h_in = nullptr;             // pinned [offs (n+1) u64 | bytes] (H2D source)
    size_t c_in = 0;
    // the bounded batch's input, mapped and coherent: [n | pad | offs (bound + 1) u64 | bytes]
    uint8_t* h_bin = nullptr;
    size_t c_bin = 0;
    uint32_t bound = 0;                  // topics the bounded batch is sized for (0: not set up)
    uint64_t bytes_cap = 0;
    // the bounded batch's captured graphs, one per size class (a batch of n
    // calls runs in the smallest class >= n: a 20-call batch would otherwise
    // launch the grids of a 16,384-call one); swapped into b.gexec / b.gkey
    // around each launch
    static constexpr uint32_t NCLASS = 4;
    struct GraphCache {
        hipGraphExec_t exec = nullptr;
        std::vector<uint8_t> key;
    } gc[NCLASS];
    // written by tm_export_host: [ctrl | stats | src n u64 | count n u32] and the rows
    uint8_t* h_out = nullptr;
    size_t c_out = 0;
    uint32_t* h_rows = nullptr;
    size_t c_rows = 0;
    hipEvent_t ev_done = nullptr;
    // polled completion (TM_ASYNC_SPIN_US): the stream writes seq into this
    // pinned word after the export, the completer spins on it before it
    // falls back to the event
    uint32_t* h_flag = nullptr;
    uint32_t* d_flag = nullptr;
    uint32_t seq = 0;
    int rc = TM_OK;                      // launch failure (delivered to every call)
    bool claimed = false;                // a completer waits for it / it is being delivered
    // Delivery in chunks: once waited and checked (ready), the batch's calls
    // are delivered DELIVER_CHUNK at a time by whichever completers are idle
    // (the calls are independent), so a batch's last caller does not wait for
    // one thread to run every callback before it.  Under the replica's amu.
    static constexpr uint32_t DELIVER_CHUNK = 512;
    bool ready = false;
    uint32_t nchunks = 0, next_chunk = 0, chunks_done = 0;
    const uint32_t* d_count = nullptr;   // (ready) the per-call counts and row starts in h_out
    const unsigned long long* d_src = nullptr;
};

// One device copy of the trie (a replica): the HBM tables, the stream the
// engine's own work runs on, the batches that read the tables from streams of
// their own, and the async per-publish pipeline that feeds this device.  An
// engine owns one replica per device it was created on (tm_create: one;
// tm_create_replicated: one per listed device, a device may repeat); they all
// mirror the engine's ONE host trie, so a mutation is made once on the host
// and its delta uploaded to every replica (sync_device), and node / filter
// ids are the same on every device by construction.
struct Replica {
    uint32_t index = 0;
    int device = -1;
    hipStream_t stream = nullptr;
    hipEvent_t ev_delta = nullptr;       // end of the last async delta upload (staging reusable after it)
    hipEvent_t ev_sync = nullptr;        // end of the delta uploads, waited for by own-stream batches
    bool delta_inflight = false;
    uint64_t upload_seq = 0;             // async trie uploads recorded on ev_sync
    // batches on streams of their own (async slots, TM_BATCH_STREAM) read the
    // tables concurrently with the replica stream: uploads wait for their walks
    std::vector<tm_batch*> readers;
    tm_batch scratch;   // tm_match_batch / tm_trie_match / tm_match_routes_batch slices
    tm_batch tokb;      // staging of tm_tokenize_device
    // tm_match_batch of more than ONESHOT_MAX topics: chunks alternate over two
    // batches on streams of their own, so chunk j's copy to the host overlaps
    // chunk j + 1's upload and walk; the merged CSR lands in h_prow / h_pids
    tm_batch pipe[2];
    bool pipe_ready = false;
    hipStream_t pipe_copy = nullptr;                      // the results' copies to the host
    hipEvent_t pipe_h2d[2] = {nullptr, nullptr};          // staging k uploaded
    hipEvent_t pipe_cp[2] = {nullptr, nullptr};           // pipe[k]'s last result copied out
    hipEvent_t pipe_pk[2] = {nullptr, nullptr};           // pipe[k]'s ids packed (tm_match_batch_packed)
    uint8_t* h_stage[2] = {nullptr, nullptr};             // pinned packed chunk (offsets | bytes)
    size_t ch_stage[2] = {0, 0};
    uint32_t *h_prow = nullptr, *h_pids = nullptr;
    uint8_t* h_pids8 = nullptr;                             // the merged ids packed 3 bytes each
    size_t ch_pids8 = 0;
    size_t ch_prow = 0, ch_pids = 0;

    // trie tables
    Slot* d_slots = nullptr;
    size_t d_nslots = 0;
    uint64_t* d_foff = nullptr;
    uint32_t* d_flen = nullptr;
    size_t c_foff = 0, c_flen = 0;
    uint8_t* d_fbytes = nullptr;
    size_t c_fbytes = 0;
    uint64_t fbytes_uploaded = 0;
    uint8_t* d_dblob = nullptr;   // the engine's delta blob (h_dblob), uploaded in one copy
    size_t cd_dblob = 0;
    // word dictionary mirror (device tokeniser): cuckoo key table, tails, arena
    DictKey* d_dkey = nullptr;
    size_t d_dict_n = 0;            // cuckoo slots on the device
    uint64_t d_dict_gen = ~0ull;    // dict.gen() of the device table
    DictTail* d_tail = nullptr;
    size_t c_tail = 0, tails_uploaded = 0;
    uint8_t* d_arena = nullptr;
    size_t c_arena = 0, arena_uploaded = 0;
    uint32_t* d_dxidx = nullptr;
    DictKey* d_dxval = nullptr;
    size_t cd_dxidx = 0, cd_dxval = 0;
    // bounds-checked variant's report
    uint32_t* d_dbg = nullptr;
    uint32_t* h_dbg = nullptr;
    size_t c_dbg = 0, ch_dbg = 0;
    // pinned staging of the appended tails (filter bytes, dictionary tails and
    // arena) of one delta upload: small appends go out asynchronously instead
    // of as pageable copies the host must wait for
    uint8_t* h_app = nullptr;
    size_t ch_app = 0;
    // routes: dests CSR by node id (engine routes_gen when uploaded)
    uint32_t *d_roff = nullptr, *d_rdest = nullptr;
    size_t c_roff = 0, c_rdest = 0;
    uint64_t routes_gen = ~0ull;
    // subscribers: soff / subs / scnt / sone by node id (engine subs_gen when uploaded)
    uint64_t* d_soff = nullptr;
    uint32_t* d_subs = nullptr;
    uint8_t* d_scnt = nullptr;
    uint32_t* d_sone = nullptr;
    size_t c_soff = 0, c_subs = 0, c_scnt = 0, c_sone = 0;
    uint64_t subs_gen = ~0ull;
    // tm_rules_match
    uint32_t* d_rl = nullptr;
    size_t c_rl = 0;

    // async pipeline (tm_match_async / tm_match_coalesced): calls queue on amu;
    // the launcher thread turns the queue into a device batch on a free slot
    // (under the engine mutex, like every other engine operation), the
    // completer threads wait for slots in launch order and deliver the rows
    std::mutex amu;
    std::condition_variable a_work, a_done;
    // submissions go to one of QSHARDS queues picked by the calling thread, so
    // concurrent submitters (the NIF's scheduler threads) rarely share a lock;
    // the launcher drains them into a batch
    struct alignas(64) QShard {
        std::mutex mu;
        std::vector<uint8_t> bytes;
        std::vector<uint32_t> lens;
        std::vector<AsyncCall> calls;
        size_t head = 0;                 // calls before head were taken
        size_t head_bytes = 0;
    };
    static constexpr uint32_t QSHARDS = 16;
    QShard qs[QSHARDS];
    std::atomic<uint64_t> q_count{0};    // calls queued in all shards
    std::atomic<bool> a_live{false};     // pipeline threads running and accepting calls
    std::vector<AsyncSlot*> a_slots, a_free;
    std::deque<AsyncSlot*> a_inflight;
    uint64_t a_inflight_calls = 0;   // calls of the batches in a_inflight (under amu)
    // the queue length the gathering launcher waits for (callers reaching it
    // wake it; ~0: not gathering)
    std::atomic<uint64_t> a_gather_at{~0ull};
    std::thread a_launcher;
    std::vector<std::thread> a_completers;
    bool a_started = false, a_stop = false, a_launcher_done = false;
    // a batch launches when a slot is free and either nothing is in flight or
    // at least a_busy_min calls queued: under load, calls accumulate while the
    // device works instead of trickling out as tiny batches
    uint32_t a_max = 16384, a_linger_us = 0, a_depth = 4, a_busy_min = 128, a_ncompleters = 6;   // (depth / completers: TM_ASYNC_DEPTH / TM_ASYNC_COMPLETERS)
    uint32_t a_spin_us = 0;   // completers poll a pinned flag this long before blocking on the event (0: off)
    // (while batches are in flight and fewer than a_busy_min calls wait, the
    // launcher waits for the pipeline to idle or a_busy_min calls; a bounded
    // gather -- launch after 20 / 40 / 80 us -- was measured, profiles/r04/d/:
    // blocking leg unchanged, 4,096-in-flight leg 6.2 -> 4.6-4.7 M calls/s)
    // a call that finds the queue empty and the whole pipeline idle launches
    // its batch itself, on the calling thread (no launcher wake-up)
    const bool a_inline = true;
    uint64_t a_batches = 0, a_requests = 0, a_recoveries = 0, a_max_seen = 0, a_inline_launches = 0;
    // where the pipeline's time goes (host microseconds, summed over batches)
    double a_us_launch = 0, a_us_wait = 0, a_us_deliver = 0;
};

// Persistent host workers of the bulk mutations: run(f) calls f(0..n-1) with
// f(0) on the calling thread, so a delta batch pays no thread start-up for
// each of its phases.
// The engine's host workers (bulk plans and parallel churn).  A bulk call
// runs several short jobs back to back (plan, node records, edge ranges,
// summaries, merges: 0.1-1 ms each), so starting a job must be cheap: the
// workers sleep on a futex over the job counter (one FUTEX_WAKE starts them
// all, no mutex for them to queue on after waking) and the caller sleeps on
// the busy count.  Only a short spin before each sleep: the box runs under a
// CFS CPU quota, where spinning threads would burn the quota and throttle.
struct WorkPool {
    unsigned n = 1;
    std::vector<std::thread> th;
    const std::function<void(unsigned)>* job = nullptr;
    std::atomic<uint32_t> gen{0};
    std::atomic<uint32_t> busy{0};
    std::atomic<bool> stop{false};

    static long futex(std::atomic<uint32_t>* a, int op, uint32_t v) {
        return syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), op | FUTEX_PRIVATE_FLAG, v, nullptr, nullptr, 0);
    }
    // How long an idle worker (or the caller waiting for them) spins before
    // it sleeps on the futex.  Short by default: the box runs under a CFS CPU
    // quota, where spinning threads would burn it.  A bulk mutation keeps
    // them spinning for its duration and a short grace after (Linger): its
    // phases follow each other within tens of µs, and a futex wake-up per
    // phase and worker cost ~25 µs each (host-only K = 10 churn 1.97 -> 1.71
    // ms on the box); the deadline is re-read while spinning, so the workers
    // sleep soon after the grace.
    // (the grace after a mutation covers the delta gather that usually
    // follows it, tm_sync_async: its fork-joins find the workers awake)
    // Inside a mutation the deadline is pushed to now + PHASE_GAP_NS at the
    // start and the end of every run(): the workers spin across the short
    // gaps between phases but sleep through a long serial stretch of the
    // calling thread (a bulk build's merge of 10^8 filters, say).
    static constexpr int SPIN_IDLE = 2048;
    static constexpr int64_t GRACE_NS = 150000;
    static constexpr int64_t PHASE_GAP_NS = 300000;
    std::atomic<int64_t> linger_until{0};   // steady-clock ns
    std::atomic<int> lingering{0};          // mutations in progress (Linger scopes)
    // TM_PAR_TRACE: per run, how late the last worker started its share
    bool trace = false;
    std::atomic<int64_t> last_start{0};
    uint64_t t_runs = 0;
    double t_wall_us = 0, t_lag_us = 0;
    static int64_t now_ns() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    bool spin_until_changed(const std::atomic<uint32_t>& a, uint32_t v) const {
        for (int i = 0;; ++i) {
            if (a.load(std::memory_order_acquire) != v) return true;
            if ((i & 255) == 0 && i >= SPIN_IDLE && now_ns() > linger_until.load(std::memory_order_relaxed))
                return false;
            __builtin_ia32_pause();
        }
    }
    struct Linger {   // scope of a bulk mutation
        WorkPool& p;
        explicit Linger(WorkPool& q) : p(q) {
            p.lingering.fetch_add(1, std::memory_order_relaxed);
            p.linger_until.store(now_ns() + PHASE_GAP_NS, std::memory_order_relaxed);
        }
        ~Linger() {
            p.lingering.fetch_sub(1, std::memory_order_relaxed);
            p.linger_until.store(now_ns() + GRACE_NS, std::memory_order_relaxed);
        }
    };
    void refresh_linger() {
        if (lingering.load(std::memory_order_relaxed))
            linger_until.store(now_ns() + PHASE_GAP_NS, std::memory_order_relaxed);
    }
    // `cpus` (may be null): the CPUs the workers run on
    void start(unsigned k, const cpu_set_t* cpus) {
        n = std::max(1u, k);
        for (unsigned i = 1; i < n; ++i) {
            th.emplace_back([this, i] { loop(i); });
            if (cpus) (void)pthread_setaffinity_np(th.back().native_handle(), sizeof(cpu_set_t), cpus);
        }
    }
    void loop(unsigned i) {
        uint32_t seen = 0;
        for (;;) {
            while (gen.load(std::memory_order_acquire) == seen && !stop.load(std::memory_order_acquire))
                if (!spin_until_changed(gen, seen)) futex(&gen, FUTEX_WAIT, seen);
            if (stop.load(std::memory_order_acquire)) return;
            seen = gen.load(std::memory_order_acquire);
            if (trace) {
                const int64_t t = now_ns();
                for (int64_t o = last_start.load(std::memory_order_relaxed);
                     o < t && !last_start.compare_exchange_weak(o, t, std::memory_order_relaxed);) {
                }
            }
            (*job)(i);
            if (busy.fetch_sub(1, std::memory_order_acq_rel) == 1) futex(&busy, FUTEX_WAKE, 1);
        }
    }
    void run(const std::function<void(unsigned)>& f) {
        if (n <= 1) { f(0); return; }
        refresh_linger();
        const int64_t t0 = trace ? now_ns() : 0;
        if (trace) last_start.store(t0, std::memory_order_relaxed);
        job = &f;
        busy.store(n - 1, std::memory_order_release);
        gen.fetch_add(1, std::memory_order_acq_rel);
        futex(&gen, FUTEX_WAKE, INT32_MAX);
        f(0);
        for (uint32_t b; (b = busy.load(std::memory_order_acquire)) != 0;)
            if (!spin_until_changed(busy, b)) futex(&busy, FUTEX_WAIT, b);
        refresh_linger();
        if (trace) {
            ++t_runs;
            t_wall_us += 1e-3 * (double)(now_ns() - t0);
            t_lag_us += 1e-3 * (double)(last_start.load(std::memory_order_relaxed) - t0);
        }
    }
    ~WorkPool() {
        stop.store(true, std::memory_order_release);
        gen.fetch_add(1, std::memory_order_acq_rel);
        futex(&gen, FUTEX_WAKE, INT32_MAX);
        for (auto& t : th) t.join();
    }
};

// One worker's share of a parallel bulk mutation (tm_engine::mutate_parallel).
// Phase 1 (defer): node records change in place -- each worker owns the
// subtrees of its first words, ROOT is shared under root_mu -- while the
// edge-hash work (insert / delete an edge, rewrite a child summary) is only
// recorded; the counters, dirty lists, filter bytes and freed ids collect
// here and are merged afterwards.  Phase 2 applies the recorded edge work by
// bucket ranges.
struct alignas(64) Mut {   // (one cache line boundary per worker: no false sharing of counters)
    bool defer = false;
    std::vector<uint32_t>* ids = nullptr;               // the batch's node ids: free ones, then fresh ones
    std::atomic<size_t>* next_id = nullptr;             //   (shared by the workers)
    size_t n_free = 0, fresh_base = 0, n_fresh = 0;
    static constexpr size_t ID_CHUNK = 16;
    size_t id_lo = 0, id_hi = 0;                        // this worker's current chunk of the batch's ids
    std::vector<std::array<uint32_t, 3>> ins;           // deferred insert_edge(p, w, c)
    std::vector<std::pair<uint32_t, uint32_t>> del;     // deferred delete_edge_of(c): (c, its slot then)
    std::vector<uint32_t> sum;                          // deferred write_summary(c)
    // (parent << 32 | word) -> child made in phase 1: open addressing, keys + 1
    std::vector<std::pair<uint64_t, uint32_t>> made;
    size_t made_n = 0;
    uint32_t made_get(uint64_t k) const {
        if (made.empty()) return NONE;
        const size_t m = made.size() - 1;
        for (size_t i = (size_t)((k * 0x9E3779B97F4A7C15ull) >> 20) & m;; i = (i + 1) & m) {
            if (made[i].first == 0) return NONE;
            if (made[i].first == k + 1) return made[i].second;
        }
    }
    void made_put(uint64_t k, uint32_t c) {
        if ((made_n + 1) * 2 > made.size()) {
            std::vector<std::pair<uint64_t, uint32_t>> old;
            old.swap(made);
            made.assign(std::max<size_t>(1024, old.size() * 2), {0, 0});
            made_n = 0;
            for (const auto& e : old)
                if (e.first) made_put(e.first - 1, e.second);
        }
        const size_t m = made.size() - 1;
        size_t i = (size_t)((k * 0x9E3779B97F4A7C15ull) >> 20) & m;
        while (made[i].first && made[i].first != k + 1) i = (i + 1) & m;
        if (!made[i].first) ++made_n;
        made[i] = {k + 1, c};
    }
    std::vector<uint8_t> fb;                            // filter bytes appended
    std::vector<std::pair<uint32_t, uint64_t>> foff;    // (node, offset into fb)
    std::vector<uint32_t> dirty, dirty_f;
    std::vector<uint32_t> pend;                         // freed ids (pending_free, at the call's launch_seq)
    int64_t live_nodes = 0, n_filters = 0, live_edges = 0, used_slots = 0, route_entries = 0;
    uint32_t max_disp = 0;
    uint64_t version = 0, done = 0;
    double t_us = 0;                                    // phase-1 time (TM_PAR_TRACE)
    size_t n_items = 0;
    bool routes_dirty = false;
    int rc = TM_OK;
    // back to a fresh worker state for the next batch, keeping the vectors'
    // capacity: no allocation, page faults or table growth per churn batch
    void reset() {
        if (made_n) std::fill(made.begin(), made.end(), std::pair<uint64_t, uint32_t>{0, 0});
        Mut n;
        n.ins.swap(ins); n.del.swap(del); n.sum.swap(sum); n.made.swap(made); n.fb.swap(fb);
        n.foff.swap(foff); n.dirty.swap(dirty); n.dirty_f.swap(dirty_f); n.pend.swap(pend);
        n.ins.clear(); n.del.clear(); n.sum.clear(); n.fb.clear();
        n.foff.clear(); n.dirty.clear(); n.dirty_f.clear(); n.pend.clear();
        *this = std::move(n);
    }
};
inline thread_local Mut* tl_mut = nullptr;

// Wake-ups of blocked tm_match_coalesced callers.  A caller that stops
// spinning sleeps on one of WAKE_WORDS shared futex words (chosen by its
// thread); a completer delivering a batch marks each call done without a
// syscall and notes the words whose sleepers it finished, then wakes each
// noted word once after the batch (~8-16 FUTEX_WAKEs instead of one per
// call; a woken caller whose call is not done yet sleeps again).  Callbacks
// run outside a completer's batch wake their caller at once.
namespace syncwake {
constexpr uint32_t WAKE_WORDS = 16;
struct alignas(64) Word {
    std::atomic<uint32_t> seq{0};
};
inline Word words[WAKE_WORDS];
inline thread_local bool in_batch = false;        // a completer is delivering a batch
inline thread_local uint32_t pending = 0;         // words to wake at the batch's end
inline long futex(std::atomic<uint32_t>* a, int op, uint32_t v) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), op | FUTEX_PRIVATE_FLAG, v, nullptr, nullptr, 0);
}
inline void wake(uint32_t k) {
    words[k].seq.fetch_add(1, std::memory_order_acq_rel);
    futex(&words[k].seq, FUTEX_WAKE, INT32_MAX);
}
inline void flush() {
    for (uint32_t m = pending; m; m &= m - 1) wake((uint32_t)__builtin_ctz(m));
    pending = 0;
}
}  // namespace syncwake

struct tm_engine {
    std::recursive_mutex mu;
    std::vector<Replica*> reps;   // empty: host-only engine (trie ops, no match)
    bool upload_nosync = false;   // set by tm_match_batch (prepare -> launch -> wait in one call)
    int device = -1;              // the first replica's device, -1 = host-only
    unsigned threads = 1;
    std::atomic<uint32_t> rr{0};  // round-robin over replicas for calls that pick one

    WordDict dict;

    // node table (host): the fields a mutation touches in one 32-B record
    // (one cache line per node on the churn path), the filter-bytes index
    // (uploads, tm_filter_bytes) apart
    struct alignas(32) NodeRec {
        uint32_t parent = 0, word = 0;   // incoming edge
        uint32_t ec = 0;                 // edge_count (src/emqx_trie.erl:145-158)
        uint32_t plus = NONE, hash = NONE;   // '+' / '#' child
        uint32_t inslot = NONE;          // edge-hash slot of the incoming edge
        uint8_t live = 0, topic = 0;
        uint8_t hasbytes = 0;            // n_foff / n_flen name this id's filter (until the id is reused)
        // literal children per signature bit (lsig_pos of their words),
        // saturating: a count that reached 255 keeps its bit set for good
        uint8_t lcnt[LSIG_BITS] = {};
        uint32_t lsig() const {
            uint32_t s = 0;
            for (uint32_t i = 0; i < LSIG_BITS; ++i) s |= lcnt[i] ? 1u << i : 0u;
            return s;
        }
        void lsig_add(uint32_t w) {
            uint8_t& k = lcnt[lsig_pos(w)];
            if (k < 255) ++k;
        }
        void lsig_del(uint32_t w) {
            uint8_t& k = lcnt[lsig_pos(w)];
            if (k && k < 255) --k;
        }
    };
    static_assert(sizeof(NodeRec) == 32, "two node records per cache line");
    std::vector<NodeRec, HugeAlloc<NodeRec>> nd;
    std::vector<uint32_t> n_flen;
    std::vector<uint64_t> n_foff;
    // 30-bit Bloom filter of each node's literal children (lext_pos), carried
    // in its slot's '#'-id field when it has no '#' child; only grows between
    // re-packs (rebuild_lext)
    std::vector<uint32_t> n_lext;
    std::vector<uint32_t> free_nodes;
    // A freed node id (== filter id) is not reused while a batch launched
    // before the free may still hand it out: results are read (ids mapped to
    // filter bytes) after the walk, possibly after later deletes, and a
    // recycled id would name another filter.  Batches hold their launch
    // sequence number from launch until re-launch or free; an id freed at
    // sequence L returns to free_nodes once every live batch is newer than L.
    // (blocks of ids freed at one sequence number, oldest first)
    struct PendBlock {
        uint64_t seq;
        std::vector<uint32_t> ids;
    };
    std::deque<PendBlock> pending_free;
    size_t pending_n = 0;   // ids in pending_free
    void pend_ids(uint64_t seq, const uint32_t* ids, size_t k) {
        if (!k) return;
        if (pending_free.empty() || pending_free.back().seq != seq) pending_free.push_back({seq, {}});
        std::vector<uint32_t>& v = pending_free.back().ids;
        v.insert(v.end(), ids, ids + k);
        pending_n += k;
    }
    std::multiset<uint64_t> live_launches;
    uint64_t launch_seq = 0;
    uint64_t live_nodes = 0, live_edges = 0, n_filters = 0;
    std::vector<uint8_t, HugeAlloc<uint8_t>> fbytes;   // (2-MB pages: a growth step faults ~512x fewer pages)

    // edge hash (host mirror of the HBM replica)
    std::vector<Slot, HugeAlloc<Slot>> slots;
    uint64_t used_slots = 0;   // live + tombstones
    uint32_t max_disp = 0;

    // delta log
    std::vector<uint32_t> dirty;
    std::vector<uint64_t> dirty_mark;   // bitset over slots: in `dirty` already (0.8 MB per 6.7M slots)
    std::vector<uint32_t> dirty_f;
    std::vector<uint8_t> dirty_f_mark;
    bool full_dirty = true;
    bool full_f_dirty = true;
    // delta staging in pinned host memory, filled once per upload and copied to every replica
    // the gathered slot and filter-metadata deltas: one pinned blob, so a
    // replica's delta upload is one copy (six used to cost ~0.1 ms of device
    // time per upload in H2D setup gaps); the arrays point into it
    uint8_t* h_dblob = nullptr;
    size_t ch_dblob = 0, blob_bytes = 0;
    size_t blob_off[5] = {0, 0, 0, 0, 0};   // didx | dval | fidx | foffv | flenv
    uint32_t* h_didx = nullptr;
    Slot* h_dval = nullptr;
    uint32_t* h_fidx = nullptr;
    uint64_t* h_foffv = nullptr;
    uint32_t* h_flenv = nullptr;
    uint32_t* h_dxidx = nullptr;
    DictKey* h_dxval = nullptr;
    size_t ch_dxidx = 0, ch_dxval = 0;
    bool dev_tok = true;            // TM_CFG_HOST_TOKENIZE / TM_HOST_TOKENIZE=1: tokenise on the host


    uint64_t version = 1;
    uint64_t uploads_full = 0, uploads_delta = 0, delta_slots = 0, graph_launches = 0;
    bool frozen = false;           // TM_CFG_FROZEN_DICT: words only via tm_dict_load
    bool checked = false;          // TM_CHECKED=1: bounds-checked kernel variant
    uint32_t row_cap = 128;        // K: fast-path row slots per topic (TM_ROWCAP)
    uint32_t qcap = 384;           // LDS probe stack per wave (C2 tiles peak at ~340; 512 measured no faster)
    double static_frac = 0.5;       // share of tiles scheduled round-robin before per-XCD tickets
    uint64_t fan_big_limit = 0xFFFFFFFFull;   // fan-out scan blocks above this use u64 offsets (TM_FAN_BIG: tests)
    double target_load = 0.35;     // edge-hash load after a re-pack
    uint64_t result_limit = MAX_RESULT;   // matches per batch (TM_RESULT_LIMIT: test-only knob to lower it)
    uint64_t staging_min = 1u << 16;      // initial staging entries of a batch (TM_STAGING_MIN: test-only)

    // routes (the emqx_route bag, aggregated per destination by the caller):
    // node id -> [(dest, count)] in first-added order; total routes per node
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> n_dests;
    std::vector<uint32_t> n_nroutes;
    bool routes_dirty = true;
    uint64_t route_entries = 0;
    uint64_t routes_gen = 0;   // bumped when h_roff / h_rdest are rebuilt
    std::vector<uint32_t> h_roff, h_rdest;

    // ------------------------------------------------------------ hash
    uint32_t nslots() const { return (uint32_t)slots.size(); }
    uint32_t nbuckets() const { return nslots() / BUCKET; }

    // (parent, word) lookup: the same probe sequence as the kernel's probe()
    uint32_t find_slot(uint32_t p, uint32_t w) const {
        const uint32_t nb = nbuckets();
        uint32_t b = home_bucket(p, w, nb);
        for (uint32_t i = 0; i <= max_disp; ++i) {
            for (uint32_t s = 0; s < BUCKET; ++s) {
                const Slot& e = slots[b * BUCKET + s];
                if ((e.parent & ID_MASK) == p && (e.word & WID_MASK) == w) return b * BUCKET + s;
            }
            if (slots[b * BUCKET + BUCKET - 1].parent == SLOT_EMPTY) return NONE;
            b = (b + 1 == nb) ? 0 : b + 1;
        }
        return NONE;
    }

    // first free slot (empty or tombstone) along the probe sequence; slots of a
    // bucket are taken in order, so "last slot empty" <=> "bucket has a hole"
    uint32_t place_slot(std::vector<Slot, HugeAlloc<Slot>>& tab, uint32_t p, uint32_t w, uint32_t& disp,
                        bool& was_empty) const {
        const uint32_t nb = (uint32_t)(tab.size() / BUCKET);
        uint32_t b = home_bucket(p, w, nb);
        for (uint32_t i = 0;; ++i) {
            for (uint32_t s = 0; s < BUCKET; ++s) {
                Slot& e = tab[b * BUCKET + s];
                if (e.parent == SLOT_EMPTY) {
                    disp = i;
                    was_empty = true;
                    return b * BUCKET + s;
                }
            }
            b = (b + 1 == nb) ? 0 : b + 1;
        }
    }

    // the 30-bit literal signatures from the edges as they are (clears the
    // stale bits deletes leave); the slots change: callers upload in full
    void rebuild_lext() {
        std::fill(n_lext.begin(), n_lext.end(), 0u);
        for (const Slot& e : slots) {
            if (e.parent == SLOT_EMPTY) continue;
            const uint32_t w = e.word & WID_MASK;
            if (w != W_PLUS && w != W_HASH) n_lext[e.parent & ID_MASK] |= 1u << lext_pos(w);
        }
        for (Slot& e : slots)
            if (e.parent != SLOT_EMPTY && !(e.hash & B_HASH)) e.hash = n_lext[e.child & ID_MASK];
        full_dirty = true;
    }

    // rebuild at load <= 0.6 (any bucket count: home_bucket is multiply-shift)
    void rehash(size_t want_slots) {
        size_t nb = std::max<size_t>((want_slots + BUCKET - 1) / BUCKET, 256);
        const size_t ns = nb * BUCKET;
        std::vector<Slot, HugeAlloc<Slot>> tab(ns);
        for (Slot& s : tab) { memset(&s, 0, sizeof(s)); s.parent = SLOT_EMPTY; }
        uint32_t md = 0;
        uint64_t used = 0;
        for (const Slot& e : slots) {
            if (e.parent == SLOT_EMPTY) continue;
            uint32_t disp;
            bool was_empty;
            uint32_t i = place_slot(tab, e.parent & ID_MASK, e.word & WID_MASK, disp, was_empty);
            tab[i] = e;
            nd[e.child & ID_MASK].inslot = i;
            md = std::max(md, disp);
            ++used;
        }
        slots.swap(tab);
        max_disp = md;
        used_slots = used;
        full_dirty = true;
        dirty.clear();
        dirty_mark.assign((slots.size() + 63) / 64, 0);
    }

    void mark_dirty(uint32_t i) {
        if (full_dirty) return;
        uint64_t& w = dirty_mark[i >> 6];
        const uint64_t m = 1ull << (i & 63);
        if (!(w & m)) { w |= m; (tl_mut ? tl_mut->dirty : dirty).push_back(i); }
    }

    uint32_t insert_edge(uint32_t p, uint32_t w, uint32_t c) {
        Mut* M = tl_mut;
        if (M && M->defer) {   // phase 1 of a parallel batch: recorded, placed in phase 2
            M->ins.push_back({p, w, c});
            M->made_put((uint64_t)p << 32 | w, c);
            return NONE;
        }
        if (!M && ((used_slots + 1) * 4 > slots.size() * 3 || max_disp > 48))   // (phase 2 checks capacity first)
            rehash(std::max<size_t>((size_t)((live_edges + 1) / 0.55), slots.size() * (max_disp > 48 ? 2 : 1)));
        uint32_t disp;
        bool was_empty;
        uint32_t i = place_slot(slots, p, w, disp, was_empty);
        if (M) {
            if (was_empty) ++M->used_slots;
            M->max_disp = std::max(M->max_disp, disp);
            ++M->live_edges;
        } else {
            if (was_empty) ++used_slots;
            max_disp = std::max(max_disp, disp);
            ++live_edges;
        }
        Slot& e = slots[i];
        e.parent = p; e.word = w; e.child = c;
        nd[c].inslot = i;
        write_summary(c);
        return i;
    }

    // Removes the edge into c without tombstones.  The table keeps two
    // invariants the lookups (host find_slot, the kernels' probes) rely on:
    // a bucket's slots fill in order, and every key stored in bucket c with
    // home bucket h has all of [h, c) full -- so a bucket with a free last slot
    // ends every probe run through it.  The hole is closed by compacting its
    // bucket and pulling back the nearest later key whose run crosses it
    // (backward-shift deletion at bucket granularity); churn then leaves probe
    // runs as short as a fresh build's instead of lengthening them with
    // tombstones until a full rebuild.
    void move_slot(uint32_t to, uint32_t from) {
        slots[to] = slots[from];
        nd[slots[to].child & ID_MASK].inslot = to;
        Slot& e = slots[from];
        memset(&e, 0, sizeof(e));
        e.parent = SLOT_EMPTY;
        mark_dirty(to);
        mark_dirty(from);
    }

    // compacts bucket b after slot i was emptied; returns the bucket's
    // (now last) free slot
    uint32_t compact_bucket(uint32_t b, uint32_t i) {
        uint32_t last = b * BUCKET + BUCKET - 1;
        while (last > i && slots[last].parent == SLOT_EMPTY) --last;
        if (last > i) {
            move_slot(i, last);
            return last;
        }
        return i;
    }

    void delete_edge_of(uint32_t c) {
        Mut* M = tl_mut;
        if (M && M->defer) {   // phase 1 of a parallel batch: recorded, removed in phase 2
            M->del.emplace_back(c, nd[c].inslot);
            return;
        }
        uint32_t i = nd[c].inslot;
        nd[c].inslot = NONE;
        if (M) {
            --M->live_edges;
            --M->used_slots;
        } else {
            --live_edges;
            --used_slots;
        }
        const uint32_t nb = nbuckets();
        uint32_t hb = i / BUCKET;
        const bool was_full = slots[hb * BUCKET + BUCKET - 1].parent != SLOT_EMPTY;
        {
            Slot& e = slots[i];
            memset(&e, 0, sizeof(e));
            e.parent = SLOT_EMPTY;
            mark_dirty(i);
        }
        uint32_t hole = compact_bucket(hb, i);
        if (!was_full) return;   // no run crossed hb
        uint32_t cb = hb;
        // a key crossing the hole lives at most max_disp buckets past it
        for (uint32_t dist = 1; dist <= max_disp + 1; ++dist) {
            cb = (cb + 1 == nb) ? 0 : cb + 1;
            bool moved = false;
            for (uint32_t k = 0; k < BUCKET; ++k) {
                const uint32_t j = cb * BUCKET + k;
                const Slot& e = slots[j];
                if (e.parent == SLOT_EMPTY) break;
                const uint32_t h = home_bucket(e.parent & ID_MASK, e.word & WID_MASK, nb);
                // the run of e goes h .. cb; it crosses hb iff hb lies in [h, cb)
                const uint32_t dist_e = (cb + nb - h) % nb, dist_hole = (cb + nb - hb) % nb;
                if (dist_e >= dist_hole) {
                    const bool cb_full = slots[cb * BUCKET + BUCKET - 1].parent != SLOT_EMPTY;
                    move_slot(hole, j);
                    hole = compact_bucket(cb, j);
                    hb = cb;
                    dist = 0;   // the hole moved: measure from here
                    moved = true;
                    if (!cb_full) return;   // cb had room: nothing beyond it crossed it
                    break;
                }
            }
            if (!moved && slots[cb * BUCKET + BUCKET - 1].parent == SLOT_EMPTY) return;   // runs end here
        }
    }

    // ------------------------------------------------------------ nodes
    bool node_capacity_left() const { return !free_nodes.empty() || nd.size() < MAX_NODES; }

    void release_pending_ids() {
        const uint64_t watermark = live_launches.empty() ? ~0ull : *live_launches.begin();
        while (!pending_free.empty() && pending_free.front().seq < watermark) {
            const std::vector<uint32_t>& v = pending_free.front().ids;
            free_nodes.insert(free_nodes.end(), v.begin(), v.end());
            pending_n -= v.size();
            pending_free.pop_front();
        }
    }

    // batch b's ids stay valid from this launch until its next launch or free
    void note_launch(tm_batch* b) {
        forget_launch(b);
        b->seq = ++launch_seq;
        live_launches.insert(b->seq);
    }
    void forget_launch(tm_batch* b) {
        if (!b->seq) return;
        auto it = live_launches.find(b->seq);
        if (it != live_launches.end()) live_launches.erase(it);
        b->seq = 0;
    }

    uint32_t new_node(uint32_t parent, uint32_t word) {
        uint32_t id;
        if (Mut* M = tl_mut) {   // a parallel batch: the free ids of the batch first, then fresh ones
            if (M->id_lo == M->id_hi) {
                // a chunk of ids at a time (no line shared with another worker's
                // fresh records), their records prefetched when taken
                M->id_lo = M->next_id->fetch_add(Mut::ID_CHUNK, std::memory_order_relaxed);
                M->id_hi = M->id_lo + Mut::ID_CHUNK;
                for (size_t k = M->id_lo; k < M->id_hi; ++k) {
                    const size_t j = k < M->n_free ? (*M->ids)[k] : M->fresh_base + (k - M->n_free);
                    if (j >= nd.size()) break;
                    __builtin_prefetch(&nd[j], 1);
                    __builtin_prefetch(&n_lext[j], 1);
                    __builtin_prefetch(&n_flen[j], 1);
                    if (j < dirty_f_mark.size()) __builtin_prefetch(&dirty_f_mark[j], 1);
                }
            }
            const size_t k = M->id_lo++;
            if (k >= M->n_free + M->n_fresh) throw std::bad_alloc();   // (the batch's need was counted up front)
            id = k < M->n_free ? (*M->ids)[k] : (uint32_t)(M->fresh_base + (k - M->n_free));
            nd[id].hasbytes = 0;
            nd[id].parent = parent; nd[id].word = word; nd[id].ec = 0; nd[id].plus = NONE; nd[id].hash = NONE;
            nd[id].inslot = NONE; nd[id].live = 1; nd[id].topic = 0;
            for (uint8_t& k : nd[id].lcnt) k = 0;
            n_lext[id] = 0;
            ++M->live_nodes;
            return id;
        }
        if (free_nodes.empty()) release_pending_ids();
        if (!free_nodes.empty()) {
            id = free_nodes.back();
            free_nodes.pop_back();
            nd[id].hasbytes = 0;
        }
        else {
            id = (uint32_t)nd.size();
            nd.push_back(NodeRec{});
            n_flen.push_back(0);
            n_foff.push_back(0);
            n_lext.push_back(0);
        }
        nd[id].parent = parent; nd[id].word = word; nd[id].ec = 0; nd[id].plus = NONE; nd[id].hash = NONE;
        nd[id].inslot = NONE; nd[id].live = 1; nd[id].topic = 0;
        for (uint8_t& k : nd[id].lcnt) k = 0;
        n_lext[id] = 0;
        ++live_nodes;
        return id;
    }

    void kill_node(uint32_t id) {
        Mut* M = tl_mut;
        if (id < n_dests.size() && !n_dests[id].empty()) {
            if (M) {
                M->route_entries -= (int64_t)n_dests[id].size();
                M->routes_dirty = true;
            } else {
                route_entries -= n_dests[id].size();
                routes_dirty = true;
            }
            n_dests[id].clear();
            n_nroutes[id] = 0;
        }
        nd[id].live = 0;
        nd[id].topic = 0;
        nd[id].ec = 0;
        for (uint8_t& k : nd[id].lcnt) k = 0;
        if (M) {
            --M->live_nodes;
            if (id != ROOT) M->pend.push_back(id);
        } else {
            --live_nodes;
            if (id != ROOT) pend_ids(launch_seq, &id, 1);
        }
    }

    uint32_t summary_flags(uint32_t c) const {
        return (nd[c].plus != NONE ? NF_PLUS : 0) | (nd[c].hash != NONE ? NF_HASH : 0);
    }
    uint32_t hterm_of(uint32_t c) const {
        const uint32_t h = nd[c].hash;
        return (h != NONE && nd[h].topic) ? h : NONE;
    }

    // rewrite c's summary into its incoming slot (or the root record)
    void write_summary(uint32_t c) {
        if (c == ROOT) return;   // root record is rebuilt at every launch
        if (tl_mut && tl_mut->defer) {   // phase 1 of a parallel batch: rewritten in phase 2
            // (a node made by this batch has no slot yet: phase 2's insert_edge
            // writes its summary, from the final record)
            if (nd[c].inslot != NONE) tl_mut->sum.push_back(c);
            return;
        }
        const uint32_t i = nd[c].inslot;
        if (i == NONE) return;
        Slot& e = slots[i];
        slot_set_lsig(e, nd[c].lsig());
        e.child = c | (nd[c].topic ? B_TOPIC : 0u) | (nd[c].plus != NONE ? B_PLUS : 0u);
        const uint32_t h = nd[c].hash;
        e.hash = h != NONE ? h | (nd[h].topic ? B_HTERM : 0u) | B_HASH : n_lext[c];
        mark_dirty(i);
    }

    RootRec root_rec() const {
        RootRec r;
        r.live = nd[ROOT].live;
        r.hterm = hterm_of(ROOT);
        r.flags = summary_flags(ROOT);
        r.pad = 0;
        return r;
    }

    void set_topic(uint32_t c, const uint8_t* bytes, size_t len) {
        nd[c].topic = 1;
        nd[c].hasbytes = 1;
        n_flen[c] = (uint32_t)len;
        if (Mut* M = tl_mut) {   // bytes land in the arena at the merge (n_foff fixed up there)
            ++M->n_filters;
            M->foff.emplace_back(c, M->fb.size());
            M->fb.insert(M->fb.end(), bytes, bytes + len);
            if (!full_f_dirty && !dirty_f_mark[c]) { dirty_f_mark[c] = 1; M->dirty_f.push_back(c); }   // (pre-sized)
        } else {
            ++n_filters;
            n_foff[c] = fbytes.size();
            fbytes.insert(fbytes.end(), bytes, bytes + len);
            if (!full_f_dirty) {
                if (dirty_f_mark.size() < nd.size()) dirty_f_mark.resize(nd.size(), 0);
                if (!dirty_f_mark[c]) { dirty_f_mark[c] = 1; dirty_f.push_back(c); }
            }
        }
        write_summary(c);
        if (c != ROOT && nd[c].word == W_HASH) write_summary(nd[c].parent);
    }

    void clear_topic(uint32_t c) {
        if (!nd[c].topic) return;
        nd[c].topic = 0;
        if (tl_mut) --tl_mut->n_filters;
        else --n_filters;
        write_summary(c);
        if (c != ROOT && nd[c].word == W_HASH) write_summary(nd[c].parent);
    }

    // intern (insert=true) or look up the words of a filter / node id
    bool filter_words(const uint8_t* t, size_t len, bool insert, std::vector<uint32_t>& ids) {
        static thread_local std::vector<TWord> ws;
        split_words(t, len, ws);
        ids.clear();
        for (const TWord& w : ws) {
            uint32_t id;
            if (w.n == 0) id = W_EMPTY;
            else if (is_plus(w)) id = W_PLUS;
            else if (is_hash(w)) id = W_HASH;
            else id = (insert && !frozen) ? dict.intern(w.p, w.n) : dict.find(w.p, w.n);
            if (id == W_UNKNOWN) return false;
            ids.push_back(id);
        }
        return true;
    }

    // tm_dict_load: intern words in order ('', '+', '#' have fixed ids)
    int dict_load(const uint8_t* buf, const uint64_t* offs, uint32_t n) {
        for (uint32_t i = 0; i < n; ++i) {
            const uint8_t* p = buf + offs[i];
            const size_t len = offs[i + 1] - offs[i];
            if (offs[i + 1] < offs[i] || memchr(p, '/', len)) return TM_EINVAL;
            if (len == 0 || (len == 1 && (p[0] == '+' || p[0] == '#'))) continue;
            dict.intern(p, len);
        }
        return TM_OK;
    }

    // tm_filter_shard: shard of the literal (w0, w1) prefix, or nshards
    int filter_shard(const uint8_t* t, size_t len, uint32_t nshards) {
        if (nshards == 0) return TM_EINVAL;
        static thread_local std::vector<TWord> ws;
        split_words(t, len, ws);
        if (ws.size() < 2 || is_plus(ws[0]) || is_hash(ws[0]) || is_plus(ws[1]) || is_hash(ws[1]))
            return (int)nshards;
        uint32_t id[2];
        for (int k = 0; k < 2; ++k) {
            id[k] = ws[k].n == 0 ? W_EMPTY : dict.find(ws[k].p, ws[k].n);
            if (id[k] == W_UNKNOWN) return TM_ENOENT;
        }
        return (int)prefix_shard(id[0], id[1], nshards);
    }

    uint32_t walk(const std::vector<uint32_t>& ids) const {
        if (!nd[ROOT].live) return NONE;
        uint32_t n = ROOT;
        for (uint32_t w : ids) {
            const uint32_t s = find_slot(n, w);
            if (s == NONE) return NONE;
            n = slots[s].child & ID_MASK;
        }
        return n;
    }

    // emqx_trie:insert/1 (src/emqx_trie.erl:81-93)
    int trie_insert(const uint8_t* t, size_t len) {
        static thread_local std::vector<uint32_t> ids;
        if (!filter_words(t, len, true, ids)) return TM_ENOENT;   // frozen dictionary only
        return trie_insert_ids(t, len, ids.data(), (uint32_t)ids.size(), ROOT, 0);
    }

    // insert/1 with the word ids known and the path known to exist down to
    // `from` at level k0 (ROOT, 0 for a full walk)
    // (sd: in a parallel batch, the nodes of depth < sd are shared by workers --
    // 2, or 3 for the filters of a split part, see mutate_parallel)
    int trie_insert_ids(const uint8_t* t, size_t len, const uint32_t* ids_p, uint32_t nids, uint32_t from,
                        uint32_t k0, uint32_t sd = 2);

    // emqx_trie:delete/1 (src/emqx_trie.erl:107-116), delete_path/1 (:190-204)
    int trie_delete(const uint8_t* t, size_t len);

    // delete/1 of the filter whose words are ids and whose node is n
    // (sd: as for trie_insert_ids, the shared depth of a parallel batch)
    int trie_delete_at(uint32_t n, const uint32_t* ids_p, uint32_t nids, uint32_t sd = 2);

    // ------------------------------------------------------------ bulk plan
    // Bulk mutations (tm_trie_insert_many / delete_many: subscribe churn, C5)
    // split into a read-only PLAN over the whole batch, run by `threads`
    // workers -- split into words, dictionary lookups, and the walk down the
    // existing path (the edge-hash misses) -- and a serial pass that only
    // mutates.  The plan stays valid through the serial pass: insert_many never
    // removes a node, so a planned prefix still exists (the pass resumes the
    // walk from it and sees edges earlier filters of the batch created);
    // delete_many never creates one, and a node is only killed once no live
    // filter lies below it, so a planned node that is still live is the
    // filter's node (killed ids are not reused before the pass ends).
    std::recursive_mutex shared_mus[64];   // the records of depth < 2 during a parallel batch, striped by node id
    std::recursive_mutex& shared_mu(uint32_t id) { return shared_mus[id & 63]; }
    // edges of levels 0-1 created in phase 1 of a parallel insert, by any
    // worker: (parent << 32 | word) -> child, striped like shared_mus (a
    // worker reads and writes stripe p & 63 only under shared_mu(p))
    std::unordered_map<uint64_t, uint32_t> shared_made[64];
    WorkPool pool;            // workers of parallel batches (started at the first one)
    std::vector<Mut> mut_w;   // their states (reset per batch, capacity kept)
    std::vector<std::vector<uint32_t>> parts_buf;   // a parallel batch's parts (capacity kept)
    bool pool_started = false;

    struct PlanEnt {
        uint32_t node;    // deepest existing node (insert) / the filter's node or NONE (delete)
        uint32_t depth;   // levels walked (insert)
        uint32_t woff, nw;
        uint32_t part;    // worker whose word vector holds the ids
        // (for the parallel pass, from the plan's ids -- W_UNKNOWN for a new
        // word, so filters with equal leading words still get equal values)
        uint32_t pkey;    // the first two words' part key
        uint8_t sub;      // the third word's sub-part (a split hot part)
        uint8_t unk;      // a word is not in the dictionary yet
    };
    std::vector<PlanEnt> plan;
    std::vector<std::vector<uint32_t>> plan_words;
    std::vector<std::vector<TWord>> plan_tw;   // a plan group's words, per part

    // Plans filters lo..hi-1 in groups of PLAN_G: the group's words are split
    // and hashed with their dictionary entries prefetched, then resolved; the
    // existing paths are walked level by level for the whole group, every
    // filter's next bucket prefetched before any is probed -- PLAN_G
    // independent cache misses in flight instead of one chain per filter.
    static constexpr uint32_t PLAN_G = 64;
    void plan_range(const uint8_t* buf, const uint64_t* offs, uint32_t lo, uint32_t hi, bool del, uint32_t part,
                    uint32_t pbase = 0, bool append = false);

    void make_plan(const uint8_t* buf, const uint64_t* offs, uint32_t n, bool del);

    // One plan for a delete list and an insert list (tm_trie_apply_many):
    // plan[0, ndel) the deletes, plan[ndel, ndel + nins) the inserts; each
    // worker plans its share of both lists in the same pool run.
    void make_plan_pair(const uint8_t* dbuf, const uint64_t* doffs, uint32_t ndel, const uint8_t* ibuf,
                        const uint64_t* ioffs, uint32_t nins);

    // After the deletes of an apply: an insert planned before them keeps its
    // (node, depth) unless that node died (a delete emptied it -- its ancestors
    // live as long as it does, and deletes add no edge, so the walk's stop is
    // unchanged otherwise); those walk again from the root.  Dead ids are not
    // handed out again before the inserts start, so `live` tells, and an edge
    // to a dead child (its delete still pending) counts as absent.
    // (The walks go PLAN_G at a time, level by level with every next bucket
    // prefetched, as in plan_range.)
    uint32_t replan_dead_inserts(uint32_t n);
    void replan_range(uint32_t lo, uint32_t hi, std::vector<uint32_t>& redo);
    std::vector<std::vector<uint32_t>> replan_buf;   // per worker

    // the serial passes prefetch what filter i + PF_FAR / i + PF_NEAR will
    // touch: their node records first, then the lines those records point at
    static constexpr uint32_t PF_FAR = 16, PF_NEAR = 8;
    void prefetch_insert(uint32_t i, uint32_t n);
    void prefetch_delete(uint32_t i, uint32_t n);

    int insert_planned(const uint8_t* buf, const uint64_t* offs, uint32_t i);

    int delete_planned(uint32_t i, uint32_t sd = 2) {
        const PlanEnt& pe = plan[i];
        if (pe.node == NONE) return TM_OK;   // absent
        // (removed earlier in the batch: dead.  In a split part the record
        // may be a shared depth-2 node another worker is changing: read
        // `live` under its stripe lock)
        std::unique_lock<std::recursive_mutex> l;
        if (tl_mut && pe.nw < sd) l = std::unique_lock<std::recursive_mutex>(shared_mu(pe.node));
        if (!nd[pe.node].live) return TM_OK;
        l = {};
        return trie_delete_at(pe.node, plan_words[pe.part].data() + pe.woff, pe.nw, sd);
    }

    // ------------------------------------------------------------ parallel batches
    // A bulk insert / delete of PAR_MIN+ filters (subscribe churn, C5) runs
    // its serial mutation pass on the engine's workers instead of one thread:
    //   phase 1: the batch is dealt by first word (a worker owns the subtrees
    //            of its first words; ROOT is shared under root_mu) and every
    //            worker mutates node records in place, in batch order, while
    //            the edge-hash work is recorded (Mut);
    //   phase 2: the recorded edge deletes, then inserts, run by bucket range:
    //            2T ranges, the even ones in parallel, then the odd ones, so
    //            two workers never touch neighbouring buckets (a backward-shift
    //            chain or a probe run crosses into at most the next range);
    //            a delete whose slot moved into a range of the wrong parity
    //            meanwhile runs serially at the end; then the recorded summary
    //            rewrites, by slot range.
    // Node ids are handed out per worker up front (the free list first), and
    // the counters, dirty lists, freed ids and filter bytes are merged after.
    // Filter / node ids therefore differ from a serial run's (ids are the
    // engine's own), the trie and its HBM image are the same.
    static constexpr uint32_t PAR_MIN = 2048;
    static constexpr uint32_t PART_SPLIT = 8;          // sub-parts of a hot part (by third word)
    // plan parts / edge-phase range pairs per worker, taken by whichever
    // worker is free.  (4 of each measured slower on the box: shorter
    // prefetch runs and plan groups; profiles/r06/s3/ab_parts.txt)
    static constexpr uint32_t PLAN_PARTS = 1;
    static constexpr uint32_t EDGE_PAIRS = 1;
    static constexpr uint32_t PAR_RANGE_MIN = 4096;    // buckets per phase-2 range at least (>> max_disp)

    static uint32_t mix_word(uint32_t w) {
        uint64_t k = (uint64_t)w * 0x9E3779B97F4A7C15ull;
        return (uint32_t)(k >> 32);
    }

    void ensure_pool();

    // a pass over node ids v touching each node's record and its slot: the
    // record 16 nodes ahead, the slot (from the record, by then in cache) 8 ahead
    void prefetch_edge_of(const std::vector<uint32_t>& v, size_t q) const;

    // per-range states of the edge phase: at least k of them, fresh, their
    // vectors' capacity kept across batches (the rest stay merged-empty)
    std::vector<Mut> edge_w;
    std::vector<Mut>& edge_states(size_t k) {
        if (edge_w.size() < k) edge_w.resize(k);
        for (size_t i = 0; i < k; ++i) edge_w[i].reset();
        return edge_w;
    }

    // Phase 2: the recorded edge work of the runs' states Ws, by bucket range
    // (see above): every run's edge deletes, then their inserts, then the
    // summaries.
    void edge_phase(const std::vector<std::vector<Mut>*>& Ws);

    // write_summary for a parallel pass: the dirty mark set atomically (another
    // worker may mark a slot of the same 64-slot word)
    void write_summary_at(uint32_t c, std::vector<uint32_t>& dl);

    // TM_PAR_TRACE: the named stretches of a bulk call, in order (us since
    // the previous mark), printed at its end
    std::vector<std::pair<const char*, double>> tr_spans;
    std::chrono::steady_clock::time_point tr_last;
    void tr_mark(const char* what) {
        if (!kn.par_trace) return;
        const auto t = std::chrono::steady_clock::now();
        if (what) tr_spans.emplace_back(what, std::chrono::duration<double, std::micro>(t - tr_last).count());
        tr_last = t;
    }
    void tr_print() {
        if (!kn.par_trace) return;
        fprintf(stderr, "[spans us]");
        for (const auto& s : tr_spans) fprintf(stderr, " %s %.0f", s.first, s.second);
        fprintf(stderr, "\n");
        tr_spans.clear();
    }
    // The edge phase's work lists, bucketed by one worker each from the
    // phase-1 states it owns (capacity kept across batches): deletes and
    // inserts per bucket range (+ the wrapping tail range), summaries per
    // summary worker.
    struct EdgeBins {
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> del;   // (child, its slot)
        std::vector<std::vector<std::array<uint32_t, 3>>> ins;
        std::vector<std::vector<uint32_t>> sum;
    };
    std::vector<EdgeBins> edge_bins;

    // One parallel mutation in flight between par_begin and par_finish: its
    // workers' states and the id bookkeeping of an insert.
    struct ParRun {
        bool del = false;
        uint32_t n = 0;
        std::vector<Mut>* W = nullptr;
        std::vector<uint32_t> ids;   // node ids of an insert: free ones, then fresh ones from base
        size_t fresh = 0, base = 0;
        std::chrono::steady_clock::time_point ts0, tp0, tp1, tp2;
        uint64_t done = 0;
        int rc = TM_OK;
    };
    std::vector<Mut> mut_w2;   // the insert states of tm_trie_apply_many (its deletes use mut_w)

    // tm_trie_insert_many / delete_many of n >= PAR_MIN planned filters (make_plan ran).
    // Returns 1 when the batch must run serially instead (nothing changed then).
    int mutate_parallel(bool del, const uint8_t* buf, const uint64_t* offs, uint32_t n, uint64_t* done_out,
                        int* rc_out);

    // Setup and phase 1 (node records) of a parallel mutation into the states
    // W; 1: the batch must run serially instead (nothing changed then).
    int par_begin(bool del, const uint8_t* buf, const uint64_t* offs, uint32_t n, std::vector<Mut>& W, ParRun& R);

    // Phase 2 (the edge hash) of every run at once -- their edge deletes, then
    // their inserts, then the summaries -- and the merges.
    void par_finish(ParRun* const* runs, size_t nr);

    // ------------------------------------------------------------ device sync

    uint32_t node_of(const uint8_t* t, size_t len) {
        static thread_local std::vector<uint32_t> ids;
        if (!filter_words(t, len, false, ids)) return NONE;
        const uint32_t n = walk(ids);
        return (n != NONE && nd[n].topic) ? n : NONE;
    }

    // emqx_router:do_add_route/2 (src/emqx_router.erl:113-124, 229-234)
    int route_add(const uint8_t* t, size_t len, uint32_t dest);

    // do_delete_route/2 (:163-169) + delete_trie_route/1 (:239-247)
    int route_delete(const uint8_t* t, size_t len, uint32_t dest);

    // dests CSR by node id: built on the host when routes changed (routes_gen),
    // uploaded to a replica that has an older one
    int sync_routes(Replica& R);

    // tm_batch_routes: route CSR of a waited batch, resolved on the device
    int batch_routes(tm_batch* b, tm_routes* out);

    // ---- subscribers: the emqx_subscriber / emqx_subscription bags of the
    // local node (src/emqx_broker.erl:145-158, 179-191, 332-347), non-shared.
    // topic -> subscriber ids in subscription order (an ETS bag key keeps
    // insertion order); subscriber -> its topics.  The reference splits topics
    // with > 1024 subscribers into {shard, Topic, I} keys
    // (src/emqx_broker_helper.erl:82-87); that is a storage split of the same
    // set, so here every topic keeps one run.
    std::unordered_map<std::string, std::vector<uint32_t>> subs_of;
    std::unordered_map<uint32_t, std::vector<std::string>> topics_of;
    bool subs_dirty = true;
    uint64_t sub_entries = 0, subs_version = 0;
    uint64_t subs_gen = 0;         // bumped when the host arrays below are rebuilt
    // host image of the device arrays: soff (u64), subs, scnt = per node
    // min(soff[f + 1] - soff[f], 255) (the scan's 1-B gather), sone = the
    // subscriber of a one-subscriber node (the fill's 4-B gather)
    std::vector<uint32_t> h_sone;
    std::vector<uint8_t> h_scnt;
    uint32_t subs_nn = 0;
    std::vector<uint64_t> h_soff;
    std::vector<uint32_t> h_subs;

    // do_subscribe/4, non-shared clause (:150-158): insert into the bag; the
    // topic's first subscriber adds the node's route (handle_call({subscribe,
    // Topic}) -> emqx_router:do_add_route/1, :438-440).
    int subscribe(const uint8_t* t, size_t len, uint32_t sub, uint32_t node_dest);

    // do_unsubscribe/4 (:179-191) + handle_cast({unsubscribed, Topic}) (:463-469):
    // the last subscriber of a topic deletes the node's route.
    int unsubscribe(const uint8_t* t, size_t len, uint32_t sub, uint32_t node_dest);

    // subscriber_down/1 (:332-347): drop every subscription of the subscriber.
    int subscriber_down(uint32_t sub, uint32_t node_dest, uint64_t* n_removed);

    // subscriber runs by node id: rebuilt on the host after subscription or
    // trie changes (a topic's node id is looked up at build time), uploaded to
    // a replica holding an older build
    int sync_subs(Replica& R);

    // tm_batch_dispatch: deliveries of a waited batch, resolved on the device
    int batch_dispatch(tm_batch* b, uint32_t flags, tm_deliveries* out);

    // tm_rules_match: rules tokenised with their own dictionary, names against it
    int rules_match(Replica& R, const uint8_t* names, const uint64_t* noffs, uint32_t n, const uint8_t* rules,
                    const uint64_t* roffs, uint32_t r, bool dollar_rule, uint32_t* bits);

    bool needs_repack() const {
        return live_edges > 65536 && (slots.size() > (size_t)(live_edges / target_load) * 2 ||
                                      slots.size() * target_load * 1.5 < live_edges);
    }

    // anything for sync_device to upload to replica R?
    bool upload_pending(const Replica& R);

    int ensure_delta_idle();

    // f(i0, i1) over [0, k): in contiguous chunks on the churn workers when k
    // is large (a churn batch's delta gather: random reads of lines the
    // workers just wrote), else inline.  Only under mu, like every pool use.
    template <class F>
    void par_chunks(size_t k, const F& f) {
        if (k < 8192 || threads < 2) { f(0, k); return; }
        ensure_pool();
        const size_t W = pool.n;
        pool.run([&](unsigned t) { f(k * t / W, k * (t + 1) / W); });
    }

    // Brings every replica up to the host trie: the dirty slots, filter
    // metadata and dictionary slots are gathered ONCE into pinned staging and
    // each replica gets the same copies + scatter kernels on its own stream
    // (full uploads where a replica's table was reallocated or most of it
    // changed).  Uploads to a replica wait on the device for the walks of its
    // own-stream batches in flight; those batches' next launches wait for the
    // upload (ev_sync), so read-your-writes holds on every device.  Returns
    // with the calling thread's device set to `back` (or the first replica's).
    int sync_device(const Replica* back = nullptr);

    // one replica's share of sync_device: the staged deltas (or full tables)
    int upload_to(Replica& R, bool slots_full, bool keys_full, size_t nn, bool& pageable_used, bool& async_used);
    static constexpr size_t APP_MAX = 8u << 20;

    // word dictionary -> one replica: the whole cuckoo table after a rebuild
    // (or when most of it changed), else the staged dirty slots; the tails'
    // and the arena's new ends
    template <class H2D>
    int sync_dict(Replica& R, bool keys_full, bool& pageable_used, bool& async_used, H2D&& h2d_tail) {
        int rc;
        const hipStream_t stream = R.stream;
        const std::vector<DictKey>& tab = dict.keys();
        const std::vector<DictTail>& tl = dict.tails();
        const std::vector<uint8_t>& ar = dict.arena();
        const std::vector<uint32_t>& dx = dict.dirty();
        if (R.d_dict_n != tab.size()) {
            dev_free(R.d_dkey);
            HIP_OK(hipMalloc((void**)&R.d_dkey, tab.size() * sizeof(DictKey)));
            R.d_dict_n = tab.size();
            R.d_dict_gen = ~0ull;
        }
        if (R.d_dict_gen != dict.gen() || keys_full) {
            pageable_used = true;
            HIP_OK(hipMemcpyAsync(R.d_dkey, tab.data(), tab.size() * sizeof(DictKey), hipMemcpyHostToDevice, stream));
            R.d_dict_gen = dict.gen();
        } else if (!dx.empty()) {
            const size_t k = dx.size();
            if ((rc = dev_reserve(R.d_dxidx, R.cd_dxidx, k))) return rc;
            if ((rc = dev_reserve(R.d_dxval, R.cd_dxval, k))) return rc;
            HIP_OK(hipMemcpyAsync(R.d_dxidx, h_dxidx, k * 4, hipMemcpyHostToDevice, stream));
            HIP_OK(hipMemcpyAsync(R.d_dxval, h_dxval, k * sizeof(DictKey), hipMemcpyHostToDevice, stream));
            HIP_OK(launch_scatter_keys(R.d_dkey, R.d_dxidx, R.d_dxval, (uint32_t)k, stream));
            async_used = true;
        }
        if (R.c_tail < tl.size() + 1) {
            if ((rc = dev_reserve(R.d_tail, R.c_tail, tl.size() + tl.size() / 2 + 64))) return rc;
            R.tails_uploaded = 0;
        }
        if (tl.size() > R.tails_uploaded) {
            HIP_OK(h2d_tail(R.d_tail + R.tails_uploaded, tl.data() + R.tails_uploaded,
                            (tl.size() - R.tails_uploaded) * sizeof(DictTail)));
            R.tails_uploaded = tl.size();
        }
        if (R.c_arena < ar.size() + 1) {
            if ((rc = dev_reserve(R.d_arena, R.c_arena, ar.size() + 1))) return rc;
            R.arena_uploaded = 0;
        }
        if (ar.size() > R.arena_uploaded) {
            HIP_OK(h2d_tail(R.d_arena + R.arena_uploaded, ar.data() + R.arena_uploaded, ar.size() - R.arena_uploaded));
            R.arena_uploaded = ar.size();
        }
        return TM_OK;
    }

    // generic-path scratch of a batch: one frontier + match area per slow wave;
    // 64 waves for small batches (<= 16k topics), 512 from 128k topics up: a
    // deduplicated skewed batch can send tens of thousands of long rows here
    int ensure_slow_scratch(tm_batch* b);

    // ------------------------------------------------------------ batches
    // topic t = bytes[offs[t] .. offs[t+1]); its words go to words[toff[t] ..]
    struct TokView {
        const uint8_t* bytes;
        const uint64_t* offs;
        uint32_t* words;
        const uint32_t* toff;
        uint8_t* tflags;
    };

    void tokenize_range(const TokView& v, uint32_t lo, uint32_t hi, std::vector<uint32_t>& slow_out) const;

    // word offsets (separators + 1 per topic); TM_EOVERFLOW past u32 offsets
    static int count_words(const uint8_t* bytes, const uint64_t* offs, uint32_t n, uint32_t* toff, uint64_t* total);

    void tokenize_view(const TokView& v, uint32_t n, std::vector<uint32_t>& slow_all) const;

    int tokenize(tm_batch* b);

    // tm_tokenize into caller arrays
    int tokenize_into(const uint8_t* bytes, const uint64_t* offs, uint32_t n, uint32_t* words, uint64_t cap,
                      uint32_t* toff, uint8_t* tflags, uint64_t* nwords);

    int upload_batch(tm_batch* b);

    // tm_tokenize_device: the device tokeniser into caller device arrays (st:
    // the host arrays are still being staged, see TokStaged; base / nbytes then
    // come from the caller, and offsets[i] is staged item off_item0 + i / chunk)
    int tokenize_device(const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t* d_words, uint64_t cap,
                        uint32_t* d_toff, uint8_t* d_tflags, uint64_t* nwords, const TokStaged* st = nullptr,
                        uint64_t st_base = 0, uint64_t st_nbytes = 0, uint64_t off_item0 = 0);

    // tm_batch_prepare_tokens: a batch from tokenised arrays (host or device)
    int prepare_tokens(tm_batch* b, const uint32_t* words, const uint32_t* toff, const uint8_t* tflags, uint32_t n,
                       uint64_t nwords, bool on_device);

    // A part batch of the in-process sharded group (tm_shard.cpp): token
    // buffers for n topics / nwords words that the group's copies fill on the
    // batch's stream; no staging copy and no host sync (the launch checks the
    // tokens on the device).  The stream and buffers are returned.
    int part_buffers(tm_batch* b, uint32_t n, uint64_t nwords, PartBuffers* out);

    // tm_batch_export
    int export_batch(tm_batch* b, uint32_t* d_counts, uint32_t* d_ids, uint32_t mul, uint32_t add);

    // the [ctrl | stats | src | count] block and its pinned mirror, for cap topics
    static int reserve_hdr(tm_batch* b, size_t cap);

    int reserve_outputs(tm_batch* b);

    // rows[] = K u64 emission slots per lane of every match wave (reused tile after
    // tile, so it stays cache-resident); sfids[] = sorted rows staged per tile;
    // ids[] = the CSR.  sfids/ids start at 32 per topic and grow on demand.
    int reserve_rows(tm_batch* b);

    // distinct topics of a batch in first-occurrence order; row_of maps publishes to them
    void dedup_topics(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n);

    // publish names are at most ?MAX_TOPIC_LEN bytes (src/emqx_topic.erl:45,
    // validate/2 :99-100); offsets must not decrease
    static int check_topics(const uint64_t* offsets, uint32_t n) {
        for (uint32_t t = 0; t < n; ++t)
            if (offsets[t + 1] < offsets[t] || offsets[t + 1] - offsets[t] > TM_MAX_TOPIC_LEN) return TM_EINVAL;
        return TM_OK;
    }

    int prepare(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t flags = 0);

    hipStream_t st(const tm_batch* b) const { return b->own ? b->own : b->rep->stream; }

    // a TM_BATCH_STREAM batch goes away: no longer a reader, stream destroyed
    void drop_user_stream(tm_batch* b);

    // device tokenisation: the caller's bytes and offsets go to HBM now (the
    // caller's buffers are only borrowed for the call); words are produced at launch
    int upload_bytes(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n);

    // the device tokeniser's buffers for n topics of nbytes; words at launch
    int reserve_tokens(tm_batch* b, uint32_t n, uint64_t nbytes);

    // the device dedup's buffers for b->n publishes of nbytes bytes
    int reserve_dedup(tm_batch* b, uint64_t nbytes);

    DedupArgs dedup_args(tm_batch* b) const;
    // TM_DEDUP_WEAK_HASH=1 (tests): the dedup's hash degraded to the topic's length
    Knobs kn;   // the environment knobs, read at init

    // the dedup pass over the batch's resident bytes, ahead of the tokeniser
    int enqueue_dedup(tm_batch* b, hipStream_t S);
    int clear_dedup_table(tm_batch* b, hipStream_t S);
    int prepare_bounded(tm_batch* b, uint32_t bound, uint64_t bytes_cap, const uint64_t* d_offs,
                        const uint8_t* d_bytes, uint32_t* d_n);
    int slot_export_args(AsyncSlot* sl, ExportArgs& x, uint32_t n);
    hipError_t slot_tail(AsyncSlot* sl, const ExportArgs& x, hipStream_t S);

    int tokens_pending(tm_batch* b);

    // offsets block of a packed batch, padded so the bytes start 16-B aligned
    // (the tokeniser stages tiles with 16-B loads from 16-B aligned windows)
    static size_t packed_head(uint32_t n) { return (((size_t)n + 1) * 8 + 15) & ~(size_t)15; }

    // An async slot's batch: blk = pinned [offs (n+1) u64 from 0 | pad | bytes],
    // one H2D on the slot's stream (topic lengths were checked at submit).
    int upload_packed(tm_batch* b, const uint8_t* blk, uint32_t n, uint64_t nbytes);

    // Enqueues the pipeline on the batch's stream.  csr = false (async slots):
    // stop after the walk -- rows stay in the staging area, described by the
    // per-topic (src, count) of the header block, and the caller enqueues its
    // own read-back; ev2 then marks the end of the walk.
    int launch(tm_batch* b, bool csr = true);

    // the read-back of the control words after the walk.  The batch's result is
    // then what the walk left in HBM -- row i = sfids[src[i] .. + count[i]),
    // sorted and deduplicated -- and the dense CSR (scan + finalize copy) is
    // built only for a consumer that asks for offsets (ensure_dense).
    hipError_t enqueue_csr(tm_batch* b, const ScanArgs& s, hipStream_t S, unsigned ev_flags = 0);
    hipError_t graph_replay(tm_batch* b, hipStream_t S);

    // tm_match_batch's tail, enqueued behind the walk: scan + finalize (the
    // dense CSR, ids up to their capacity) and, for a one-shot batch, its copy
    // into mapped host memory.  wait() then finds the whole result on the
    // host; a walk that needed a relaunch, or more ids than fit, takes
    // result()'s (or ensure_dense's) path instead.
    int enqueue_dense_tail(tm_batch* b, hipStream_t S);

    // the one-shot result of a waited batch, or 1 when it does not hold
    // (staging relaunch left it stale, or more ids than the copy could hold)
    int oneshot_result(tm_batch* b, tm_result* out);

    // The dense CSR of a waited batch (row_off[n + 1], ids[total] in topic
    // order) from the walk's rows: exclusive scan of the counts, then one copy
    // of every row from staging (tm_finalize).  Built once per launch, on the
    // batch's stream, for the consumers that index the result by offsets: the
    // host copy (tm_batch_result), routes, fan-out, the sharded export and
    // tm_batch_device_csr.  The per-publish path reads the rows where the walk
    // wrote them and never builds it.
    int ensure_dense(tm_batch* b);

    // Replays the batch's captured pipeline, capturing it first when its
    // arguments changed (tables moved or grew, the root record, the staging
    // capacity...).  1: capture is unavailable, launch the direct way.
    static constexpr uint32_t GRAPH_MAX = 1u << 20;
    static constexpr uint32_t ONESHOT_MAX = 1u << 20;   // tm_match_batch: one-shot result up to this many topics
    bool use_graphs = true;
    int launch_graph(tm_batch* b, const MatchArgs& a, const ScanArgs& s, hipStream_t S);

    // control words of a finished launch: TM_EOVERFLOW past the u32 CSR, the
    // retry reasons in *err (0 = clean)
    int check_ctrl(const uint32_t* ctrl, const unsigned long long* stats, uint32_t* err, uint64_t* need,
                   uint64_t* staged_out = nullptr);

    // capacity misses of the last launch: grow what overflowed (the caller relaunches)
    int grow_for(tm_batch* b, uint32_t err, uint64_t need, uint64_t staged);

    void fill_stats(tm_batch* b);

    // drained: the caller has already waited for the batch's stream (the
    // sharded group joins all its streams in one host wait), so the first
    // check needs no sync; *relaunched counts capacity-miss relaunches
    int wait(tm_batch* b, bool drained = false, uint32_t* relaunched = nullptr);

    int result(tm_batch* b, tm_result* out);
    int result_packed(tm_batch* b, tm_result_packed* out);


    // tm_batch_sample: rows rows[0..k) of a waited batch as a host CSR, gathered
    // on the device from where the walk wrote them (two small kernels and two
    // small copies: count + start of each sampled row, then its ids).
    int sample(tm_batch* b, const uint32_t* rows, uint32_t k, tm_result* out);

    // ------------------------------------------------------------ async pipeline
    // Every replica runs a pipeline of its own (slots, launcher, completers);
    // tm_match_async deals the calls over them.  Slots are created on first
    // use or by tm_async_start (under R.amu; takes mu).
    int async_start(Replica& R);

    void async_stop(Replica& R);

    // Deals calls over the replicas: a submitting thread goes round-robin,
    // starting from a replica of its own, so a few busy submitters spread
    // evenly and each replica's batches still form from whole queue shards.
    int match_async(const uint8_t* t, size_t len, tm_match_cb cb, void* ctx);

    int match_async(Replica& R, const uint8_t* t, size_t len, tm_match_cb cb, void* ctx);

    // moves exactly `take` queued calls into the slot: the caller reserved
    // them (took them off q_count under amu), and a call is in its shard before
    // it is counted, so at least that many are there beyond other drainers'
    // reservations -- passes repeat until all are found
    void drain_queue(Replica& R, AsyncSlot* sl, size_t take);

    // amu held (lk): a free slot takes up to a_max queued calls and is
    // launched; amu is released while the batch is built and launched
    void launch_locked(Replica& R, std::unique_lock<std::mutex>& lk);

    // Forms batches from the queue: everything queued while the pipeline was
    // busy (up to R.a_max), optionally after a linger, on the next free slot.
    void launcher_loop(Replica& R);

    // H2D of the slot's topics (one copy), device tokeniser, walk, and one
    // kernel writing the per-topic (src, count) and the staged rows into the
    // slot's pinned buffers -- all on the slot's stream; ev_done marks the end.
    int slot_launch(AsyncSlot* sl);

    // Completers: the oldest in-flight slot nobody waits for is claimed by
    // one completer, which waits for it and checks its control words; then
    // every idle completer takes chunks of its calls to deliver (the last
    // chunk's completer recycles the slot).  A failed or recovered batch is
    // delivered whole by the completer that waited for it.
    void completer_loop(Replica& R);

    // amu held: the slot's calls are all delivered -- back to the free list
    void slot_finish(Replica& R, AsyncSlot* sl);

    // Waits for a launched slot and checks its control words.  false: its
    // rows are ready for chunked delivery (d_count / d_src set); true: it was
    // delivered whole here (a launch failure, an error, or a capacity miss
    // re-run through the CSR path: *recovered).
    bool slot_wait(AsyncSlot* sl, double& us_wait, bool& recovered);

    // devices[ndev]: one replica per entry (ndev = 0: host-only engine)
    int init(const tm_config* cfg, const int32_t* devices, uint32_t ndev);

    void destroy();

    // the calling thread's HIP device := replica R's (the first one by default)
    int use(const Replica* R = nullptr) {
        if (reps.empty()) return TM_ENODEV;
        HIP_OK(hipSetDevice(R ? R->device : device));
        return TM_OK;
    }
    int set_device() { return use(); }
    // the replica a call that may run anywhere takes (round-robin)
    Replica& pick() { return *reps[rr.fetch_add(1, std::memory_order_relaxed) % reps.size()]; }

    // ---- whole-batch calls over every replica: a batch is split into
    // contiguous slices, one per replica, run concurrently (launched by one
    // thread: every replica's work is asynchronous until the waits), and the
    // slices' results concatenate in publish order.  No data-path collective.
    std::vector<uint32_t> m_rowoff, m_ids, m_dests;   // merged results (valid like tm_result)

    static uint32_t slice_lo(uint32_t n, size_t k, size_t i) { return (uint32_t)((uint64_t)n * i / k); }

    template <class F>
    void each_rep(F f) {
        const size_t k = reps.size();
        if (k == 1) { f(0); return; }
        std::vector<std::thread> th;
        th.reserve(k);
        for (size_t i = 0; i < k; ++i) th.emplace_back([&f, i] { f(i); });
        for (auto& t : th) t.join();
    }

    // prepare + launch every slice (scratch batches), then wait each
    int run_slices(const uint8_t* topics, const uint64_t* offsets, uint32_t n);

    // tm_match_batch of a large batch on one replica, pipelined: chunks of
    // PIPE_CHUNK topics alternate over R.pipe[0/1] (own streams).  Chunk j is
    // uploaded and walked (dense CSR enqueued behind the walk) while chunk
    // j - 1's ids go to the host by DMA, straight to their place in the merged
    // CSR (the host learns a chunk's total when it waits for it, so every copy
    // knows its offset); row offsets are rebased on the host after their copy.
    static constexpr uint32_t PIPE_CHUNK = 1u << 20;
    int pipe_setup(Replica& R);
    void pipe_teardown(Replica& R);

    // Chunk j: its offsets (rebased) and bytes are copied into pinned staging
    // by the engine's workers, uploaded in one async copy and walked on batch
    // j % 2's stream; once the host has waited for it (its total gives the
    // offset of its ids in the merged CSR), a copy stream moves its ids and row
    // offsets to the host.  So the host fills chunk j + 1 while chunk j walks
    // and chunk j - 1's result crosses PCIe.  Row offsets are rebased at the end.
    int match_batch_pipelined(Replica& R, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                              tm_result* out, uint32_t pack = 0);

    // tm_match_batch over every replica: merged CSR in m_rowoff / m_ids
    int match_batch_split(const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_result* out);

    // tm_match_routes_batch over every replica: merged route CSR
    int match_routes_split(const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_routes* out);

    // tm_rules_match over every replica: names split, each replica writes its
    // rows of the bitmap (disjoint)
    int rules_match_split(const uint8_t* names, const uint64_t* noffs, uint32_t n, const uint8_t* rules,
                          const uint64_t* roffs, uint32_t r, bool dollar_rule, uint32_t* bits);
};
