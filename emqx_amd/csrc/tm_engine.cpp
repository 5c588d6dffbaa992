// tm_engine.cpp -- host side of the MI355X topic-matching engine + C ABI.
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

namespace {

#define HIP_OK(expr)                                                        \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) {                                             \
            snprintf(last_error(), 512, "%s at tm_engine.cpp:%d (%s)",      \
                     hipGetErrorString(_e), __LINE__, #expr);               \
            return TM_EIO;                                                  \
        }                                                                   \
    } while (0)

char* last_error() {
    static thread_local char buf[512] = "";
    return buf;
}

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
int host_reserve_coherent(uint8_t*& p, size_t& cap, size_t bytes) {
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
unsigned default_threads() {
    if (const char* v = getenv("TM_HOST_THREADS")) {
        const int t = atoi(v);
        if (t > 0) return (unsigned)std::min(t, 64);
    }
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
bool device_node_cpus(int device, unsigned need, cpu_set_t& out) {
    if (device < 0) return false;
    const char* pin = getenv("TM_POOL_PIN");
    if (pin && pin[0] == '0') return false;
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

}  // namespace

#ifndef TM_SLOW_WAVES_MAX
#define TM_SLOW_WAVES_MAX 4096   // C5 K=1000 device: 512 waves 7.75 ms, 2048 4.54, 4096 4.03 (tools/ab_slow.sh)
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
    // TM_BATCH_DEDUP on the device (device-tokenised batches, etm::DedupArgs):
    // the n_pub publishes are deduplicated by their bytes, and only the rows
    // (distinct topics) are tokenised and walked; n becomes the row count once
    // a launch has been waited
    bool dedup_dev = false;
    bool dedup_stale = false;       // fresh bytes (prepare / retokenize): the next launch deduplicates
    bool dedup_timed = false;       // the last launch deduplicated: evd.. is its time
    bool rowof_host = false;        // row_of holds the device map of the last dedup pass
    unsigned long long *d_dtab = nullptr, *d_psrc = nullptr;
    uint32_t *d_drep = nullptr, *d_dflag = nullptr, *d_dblen = nullptr, *d_drbs = nullptr, *d_dbbs = nullptr;
    uint32_t *d_rowof = nullptr, *d_dd = nullptr, *d_pcount = nullptr;
    uint16_t* d_dlead = nullptr;
    uint8_t* d_cbytes = nullptr;
    uint64_t* d_coffs = nullptr;
    size_t c_dtab = 0, c_psrc = 0, c_drep = 0, c_dflag = 0, c_dblen = 0, c_drbs = 0, c_dbbs = 0, c_rowof = 0;
    size_t c_dd = 0, c_pcount = 0, c_cbytes = 0, c_coffs = 0, c_dlead = 0;
    uint64_t dtab_mask = 0, dd_bytes = 0;
    hipEvent_t evd = nullptr, evx0 = nullptr, evx1 = nullptr;   // before the dedup pass; around the expand
    uint64_t x_cap = 0;             // ids the last one-shot copy could hold
    uint8_t *h_xrow = nullptr, *h_xids = nullptr;
    size_t c_xrow = 0, c_xids = 0;
    hipEvent_t evq = nullptr;   // at the launch call: evq..ev0 (or evt) is the queueing ahead of it
    // the waited result is the walk's own: row i = sfids[src[i] .. + count[i]);
    // dense = the CSR (row_off, ids) has been built from it since the last launch
    bool dense = false;
    bool tok_timed = false;     // the last launch tokenised: evt..ev0 is its time
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
        dev_free(d_dtab); dev_free(d_psrc); dev_free(d_drep); dev_free(d_dflag); dev_free(d_dblen); dev_free(d_drbs);
        dev_free(d_dbbs); dev_free(d_rowof); dev_free(d_dd); dev_free(d_pcount); dev_free(d_cbytes); dev_free(d_coffs);
        dev_free(d_dlead);
        c_dtab = c_psrc = c_drep = c_dflag = c_dblen = c_drbs = c_dbbs = c_rowof = 0;
        c_dd = c_pcount = c_cbytes = c_coffs = c_dlead = 0;
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
    uint8_t* h_stage[2] = {nullptr, nullptr};             // pinned packed chunk (offsets | bytes)
    size_t ch_stage[2] = {0, 0};
    uint32_t *h_prow = nullptr, *h_pids = nullptr;
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
    uint32_t* d_didx = nullptr;
    Slot* d_dval = nullptr;
    size_t cd_didx = 0, cd_dval = 0;
    uint32_t* d_fidx = nullptr;
    uint64_t* d_foffv = nullptr;
    uint32_t* d_flenv = nullptr;
    size_t cd_fidx = 0, cd_foffv = 0, cd_flenv = 0;
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
    std::thread a_launcher;
    std::vector<std::thread> a_completers;
    bool a_started = false, a_stop = false, a_launcher_done = false;
    // a batch launches when a slot is free and either nothing is in flight or
    // at least a_busy_min calls queued: under load, calls accumulate while the
    // device works instead of trickling out as tiny batches
    uint32_t a_max = 16384, a_linger_us = 0, a_depth = 4, a_busy_min = 128, a_ncompleters = 6;   // tools/ab_async.sh
    uint32_t a_spin_us = 0;   // completers poll a pinned flag this long before blocking on the event (0: off)
    // (while batches are in flight and fewer than a_busy_min calls wait, the
    // launcher waits for the pipeline to idle or a_busy_min calls; a bounded
    // gather -- launch after 20 / 40 / 80 us -- was measured, profiles/r04/d/:
    // blocking leg unchanged, 4,096-in-flight leg 6.2 -> 4.6-4.7 M calls/s)
    // a call that finds the queue empty and the whole pipeline idle launches
    // its batch itself, on the calling thread (no launcher wake-up)
    bool a_inline = true;
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
    static bool spin_until_changed(const std::atomic<uint32_t>& a, uint32_t v) {
        for (int i = 0; i < 2048; ++i) {
            if (a.load(std::memory_order_acquire) != v) return true;
            __builtin_ia32_pause();
        }
        return false;
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
            (*job)(i);
            if (busy.fetch_sub(1, std::memory_order_acq_rel) == 1) futex(&busy, FUTEX_WAKE, 1);
        }
    }
    void run(const std::function<void(unsigned)>& f) {
        if (n <= 1) { f(0); return; }
        job = &f;
        busy.store(n - 1, std::memory_order_release);
        gen.fetch_add(1, std::memory_order_acq_rel);
        futex(&gen, FUTEX_WAKE, INT32_MAX);
        f(0);
        for (uint32_t b; (b = busy.load(std::memory_order_acquire)) != 0;)
            if (!spin_until_changed(busy, b)) futex(&busy, FUTEX_WAIT, b);
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
    std::vector<std::pair<uint64_t, uint32_t>> pend;    // freed ids (pending_free)
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
thread_local Mut* tl_mut = nullptr;

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
    std::deque<std::pair<uint64_t, uint32_t>> pending_free;
    std::multiset<uint64_t> live_launches;
    uint64_t launch_seq = 0;
    uint64_t live_nodes = 0, live_edges = 0, n_filters = 0;
    std::vector<uint8_t> fbytes;

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
    uint32_t* h_didx = nullptr;
    Slot* h_dval = nullptr;
    size_t ch_didx = 0, ch_dval = 0;
    uint32_t* h_fidx = nullptr;
    uint64_t* h_foffv = nullptr;
    uint32_t* h_flenv = nullptr;
    size_t ch_fidx = 0, ch_foffv = 0, ch_flenv = 0;
    uint32_t* h_dxidx = nullptr;
    DictKey* h_dxval = nullptr;
    size_t ch_dxidx = 0, ch_dxval = 0;
    bool dev_tok = true;            // TM_CFG_HOST_TOKENIZE / TM_HOST_TOKENIZE=1: tokenise on the host


    uint64_t version = 1;
    uint64_t uploads_full = 0, uploads_delta = 0, delta_slots = 0;
    bool frozen = false;           // TM_CFG_FROZEN_DICT: words only via tm_dict_load
    bool checked = false;          // TM_CHECKED=1: bounds-checked kernel variant
    uint32_t row_cap = 128;        // K: fast-path row slots per topic (TM_ROWCAP)
    uint32_t qcap = 384;           // LDS probe stack per wave, 384 or 512 (TM_QCAP); C2 tiles peak at ~340
    double static_frac = 0.5;       // share of tiles scheduled round-robin before tickets (TM_STATIC_FRAC)
    uint64_t fan_big_limit = 0xFFFFFFFFull;   // fan-out scan blocks above this use u64 offsets (TM_FAN_BIG: tests)
    double target_load = 0.35;     // edge-hash load after a re-pack (TM_LOAD)
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
        while (!pending_free.empty() && pending_free.front().first < watermark) {
            free_nodes.push_back(pending_free.front().second);
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
            if (id != ROOT) M->pend.emplace_back(launch_seq, id);
        } else {
            --live_nodes;
            if (id != ROOT) pending_free.emplace_back(launch_seq, id);
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
                        uint32_t k0, uint32_t sd = 2) {
        struct { const uint32_t* d; uint32_t n; size_t size() const { return n; } uint32_t operator[](size_t i) const { return d[i]; } } ids{ids_p, nids};
        // add_path/1 for every triple (:145-158), in one walk: existing edges
        // are followed, the missing suffix is created
        uint32_t p = from;
        bool created = false;
        Mut* const M = tl_mut;
        for (size_t k = k0; k < ids.size(); ++k) {
            const uint32_t w = ids[k];
            // (a parallel batch: the nodes of depth < sd are shared by workers)
            std::unique_lock<std::recursive_mutex> rl;
            if (M && k < sd) rl = std::unique_lock<std::recursive_mutex>(shared_mu(p));
            uint32_t c = NONE;
            if (M && M->defer) {   // an edge made earlier in this batch is not in the hash yet
                // (levels < sd: made by any worker, held in the stripe's shared map)
                if (k < sd) {
                    const auto& sm = shared_made[p & 63];
                    const auto it = sm.find((uint64_t)p << 32 | w);
                    if (it != sm.end()) c = it->second;
                } else {
                    c = M->made_get((uint64_t)p << 32 | w);
                }
            }
            // The edge hash is frozen during phase 1 of a parallel insert and the
            // plan's walk stopped at level k0 on a miss, so every deeper parent
            // is a node of this batch: only the made maps can hold its edges.
            if (c == NONE && !(M && M->defer) && !created) {
                const uint32_t s = nd[p].live ? find_slot(p, w) : NONE;
                if (s != NONE) c = slots[s].child & ID_MASK;
            }
            if (c == NONE) {
                if (!created) {
                    // node ids are 30-bit (two flag bits ride in the slot's id words); a
                    // parallel batch checked its whole need up front
                    const size_t need = ids.size() - k;
                    if (!M && nd.size() + need >= MAX_NODES && free_nodes.size() + pending_free.size() < need)
                        return TM_ENOMEM;
                    created = true;
                }
                if (!nd[p].live) {               // only the root can be absent here
                    nd[p].live = 1; nd[p].ec = 0;
                    if (M) ++M->live_nodes;
                    else ++live_nodes;
                }
                c = new_node(p, w);
                ++nd[p].ec;
                // p's slot changes with a '+' / '#' child or a new signature bit
                // (ec is not in it): only then is it rewritten (and uploaded)
                bool resum = true;
                if (w == W_PLUS) nd[p].plus = c;
                else if (w == W_HASH) nd[p].hash = c;
                else {
                    const uint32_t s0 = nd[p].lsig(), x0 = n_lext[p];
                    nd[p].lsig_add(w);
                    n_lext[p] |= 1u << lext_pos(w);
                    resum = nd[p].lsig() != s0 || n_lext[p] != x0;
                }
                insert_edge(p, w, c);
                if (M && M->defer && k < sd) shared_made[p & 63][(uint64_t)p << 32 | w] = c;   // (stripe lock held)
                if (resum) write_summary(p);
            }
            p = c;
        }
        std::unique_lock<std::recursive_mutex> tl;
        if (M && ids.size() < sd) tl = std::unique_lock<std::recursive_mutex>(shared_mu(p));
        if (!created && nd[p].topic) return TM_OK;   // inserted already: idempotent
        set_topic(p, t, len);   // write_trie_node(#trie_node{node_id = Topic, topic = Topic})
        if (M) ++M->version;
        else ++version;
        return TM_OK;
    }

    // emqx_trie:delete/1 (src/emqx_trie.erl:107-116), delete_path/1 (:190-204)
    int trie_delete(const uint8_t* t, size_t len) {
        std::vector<uint32_t> ids;
        if (!filter_words(t, len, false, ids)) return TM_OK;
        const uint32_t n = walk(ids);
        if (n == NONE) return TM_OK;
        return trie_delete_at(n, ids.data(), (uint32_t)ids.size());
    }

    // delete/1 of the filter whose words are ids and whose node is n
    int trie_delete_at(uint32_t n, const uint32_t* ids_p, uint32_t nids) {
        struct { const uint32_t* d; uint32_t n; size_t size() const { return n; } uint32_t operator[](size_t i) const { return d[i]; } } ids{ids_p, nids};
        Mut* const M = tl_mut;
        std::unique_lock<std::recursive_mutex> nl;
        if (M && ids.size() < 2) nl = std::unique_lock<std::recursive_mutex>(shared_mu(n));
        if (nd[n].ec != 0) {
            if (nd[n].topic) {
                clear_topic(n);
                if (M) ++M->version;
                else ++version;
            }
            return TM_OK;
        }
        clear_topic(n);
        uint32_t child = n;
        int rc = TM_OK;
        bool child_dead = false;
        for (size_t k = ids.size(); k-- > 0;) {
            const uint32_t p = nd[child].parent;
            const uint32_t w = ids[k];
            delete_edge_of(child);
            if (!child_dead) { kill_node(child); child_dead = true; }
            // (a parallel batch: the nodes of depth < 2 are shared by workers)
            std::unique_lock<std::recursive_mutex> rl;
            if (M && k < 2) rl = std::unique_lock<std::recursive_mutex>(shared_mu(p));
            bool sig_changed = true;
            if (w == W_PLUS) nd[p].plus = NONE;
            else if (w == W_HASH) nd[p].hash = NONE;
            else {
                const uint32_t s0 = nd[p].lsig();
                nd[p].lsig_del(w);
                sig_changed = nd[p].lsig() != s0;
            }
            if (!nd[p].live) { rc = TM_EABORT; break; }
            if (nd[p].ec == 1 && !nd[p].topic) {
                nd[p].ec = 0;
                if (p == ROOT) { kill_node(p); break; }
                kill_node(p);
                child = p;
                continue;
            }
            --nd[p].ec;
            if (sig_changed) write_summary(p);   // (a '+' / '#' child, or a signature bit gone)
            break;
        }
        if (M) ++M->version;
        else ++version;
        return rc;
    }

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
                    uint32_t pbase = 0, bool append = false) {
        // the part's vectors are worked on as locals and put back at the end:
        // the per-part vector headers share cache lines, and a push_back per
        // word on them from 8-16 threads was a false-sharing storm (plan of
        // 5,000 filters: 0.45 us per filter on one thread, 3-5x that per
        // thread on eight)
        std::vector<uint32_t> W;
        W.swap(plan_words[part]);
        if (!append) W.clear();   // (append: a second range of the same part, tm_trie_apply_many)
        std::vector<TWord> all;
        all.swap(plan_tw[part]);
        std::vector<TWord> ws;
        std::vector<uint64_t> hs;
        const bool root_live = nd[ROOT].live != 0;
        const uint32_t nb = nbuckets();
        static const bool ptrace = getenv("TM_PAR_TRACE") != nullptr;
        std::chrono::steady_clock::duration d_split{}, d_dict{}, d_walk{};
        using clk = std::chrono::steady_clock;
        for (uint32_t g0 = lo; g0 < hi; g0 += PLAN_G) {
            const auto c0 = ptrace ? clk::now() : clk::time_point{};
            const uint32_t g1 = std::min(hi, g0 + PLAN_G);
            // words and their dictionary entries
            const uint32_t wbase = (uint32_t)W.size();
            hs.clear();
            all.clear();
            for (uint32_t i = g0; i < g1; ++i) {
                PlanEnt& pe = plan[pbase + i];
                split_words(buf + offs[i], offs[i + 1] - offs[i], ws);
                pe.woff = wbase + (uint32_t)all.size();
                pe.nw = (uint32_t)ws.size();
                pe.part = part;
                for (const TWord& w : ws) {
                    all.push_back(w);
                    hs.push_back(w.n == 0 || is_plus(w) || is_hash(w) ? 0 : dict.prefetch(w.p, w.n));
                }
            }
            const auto c1 = ptrace ? clk::now() : clk::time_point{};
            for (size_t j = 0; j < all.size(); ++j) {
                const TWord& w = all[j];
                W.push_back(w.n == 0 ? W_EMPTY : is_plus(w) ? W_PLUS : is_hash(w) ? W_HASH : dict.find_h(w.p, w.n, hs[j]));
            }
            const auto c2 = ptrace ? clk::now() : clk::time_point{};
            d_split += c1 - c0;
            d_dict += c2 - c1;
            // the existing paths, level by level over the group
            uint32_t node[PLAN_G], k[PLAN_G];
            bool run[PLAN_G], known[PLAN_G];
            const uint32_t G = g1 - g0;
            for (uint32_t q = 0; q < G; ++q) {
                const PlanEnt& pe = plan[pbase + g0 + q];
                node[q] = ROOT;
                k[q] = 0;
                known[q] = true;
                for (uint32_t j = 0; j < pe.nw; ++j) known[q] &= W[pe.woff + j] != W_UNKNOWN;
                run[q] = root_live;
            }
            for (bool any = root_live; any;) {
                any = false;
                for (uint32_t q = 0; q < G; ++q) {
                    const PlanEnt& pe = plan[pbase + g0 + q];
                    if (!run[q]) continue;
                    if (k[q] >= pe.nw || W[pe.woff + k[q]] == W_UNKNOWN) { run[q] = false; continue; }
                    __builtin_prefetch(&slots[(size_t)home_bucket(node[q], W[pe.woff + k[q]], nb) * BUCKET]);
                }
                for (uint32_t q = 0; q < G; ++q) {
                    if (!run[q]) continue;
                    const PlanEnt& pe = plan[pbase + g0 + q];
                    const uint32_t sl = find_slot(node[q], W[pe.woff + k[q]]);
                    if (sl == NONE) { run[q] = false; continue; }
                    node[q] = slots[sl].child & ID_MASK;
                    ++k[q];
                    any = true;
                }
            }
            for (uint32_t q = 0; q < G; ++q) {
                PlanEnt& pe = plan[pbase + g0 + q];
                if (del) pe.node = (root_live && known[q] && k[q] == pe.nw) ? node[q] : NONE;
                else { pe.node = node[q]; pe.depth = k[q]; }
            }
            if (ptrace) d_walk += clk::now() - c2;
        }
        plan_words[part].swap(W);
        plan_tw[part].swap(all);
        if (ptrace) {
            auto us = [](auto d) { return std::chrono::duration<double, std::micro>(d).count(); };
            fprintf(stderr, "  [plan part %u: %u filters] split+hash %.0f us, dict %.0f us, walk %.0f us\n", part, hi - lo,
                    us(d_split), us(d_dict), us(d_walk));
        }
    }

    void make_plan(const uint8_t* buf, const uint64_t* offs, uint32_t n, bool del) {
        plan.resize(n);
        const unsigned nt = std::max(1u, std::min<unsigned>(threads, n / 256));
        if (plan_words.size() < nt) plan_words.resize(nt);
        if (plan_tw.size() < nt) plan_tw.resize(nt);
        if (nt == 1) { plan_range(buf, offs, 0, n, del, 0); return; }
        ensure_pool();   // the engine's workers (no thread start-up per batch)
        pool.run([&](unsigned i) {
            for (unsigned j = i; j < nt; j += pool.n) {
                const uint32_t lo = (uint32_t)((uint64_t)n * j / nt), hi = (uint32_t)((uint64_t)n * (j + 1) / nt);
                plan_range(buf, offs, lo, hi, del, j);
            }
        });
    }

    // One plan for a delete list and an insert list (tm_trie_apply_many):
    // plan[0, ndel) the deletes, plan[ndel, ndel + nins) the inserts; each
    // worker plans its share of both lists in the same pool run.
    void make_plan_pair(const uint8_t* dbuf, const uint64_t* doffs, uint32_t ndel, const uint8_t* ibuf,
                        const uint64_t* ioffs, uint32_t nins) {
        plan.resize((size_t)ndel + nins);
        const unsigned nt = std::max(1u, std::min<unsigned>(threads, (ndel + nins) / 256));
        if (plan_words.size() < nt) plan_words.resize(nt);
        if (plan_tw.size() < nt) plan_tw.resize(nt);
        auto part = [&](unsigned j) {
            plan_range(dbuf, doffs, (uint32_t)((uint64_t)ndel * j / nt), (uint32_t)((uint64_t)ndel * (j + 1) / nt), true, j);
            plan_range(ibuf, ioffs, (uint32_t)((uint64_t)nins * j / nt), (uint32_t)((uint64_t)nins * (j + 1) / nt), false, j,
                       ndel, true);
        };
        if (nt == 1) { part(0); return; }
        ensure_pool();
        pool.run([&](unsigned i) {
            for (unsigned j = i; j < nt; j += pool.n) part(j);
        });
    }

    // After the deletes of an apply: an insert planned before them keeps its
    // (node, depth) unless that node died (a delete emptied it -- its ancestors
    // live as long as it does, and deletes add no edge, so the walk's stop is
    // unchanged otherwise); those walk again from the root.  Dead ids are not
    // handed out again before the inserts start, so `live` tells, and an edge
    // to a dead child (its delete still pending) counts as absent.
    // (The walks go PLAN_G at a time, level by level with every next bucket
    // prefetched, as in plan_range.)
    uint32_t replan_dead_inserts(uint32_t n) {
        std::vector<uint32_t>& redo = replan_buf;
        redo.clear();
        for (uint32_t i = 0; i < n; ++i) {
            if (i + 16 < n && plan[i + 16].node != ROOT) __builtin_prefetch(&nd[plan[i + 16].node]);
            const PlanEnt& pe = plan[i];
            if (pe.node != ROOT && !nd[pe.node].live) redo.push_back(i);
        }
        const bool root_live = nd[ROOT].live != 0;
        const uint32_t nb = nbuckets();
        for (size_t g0 = 0; g0 < redo.size(); g0 += PLAN_G) {
            const uint32_t G = (uint32_t)std::min<size_t>(PLAN_G, redo.size() - g0);
            bool run[PLAN_G];
            for (uint32_t q = 0; q < G; ++q) {
                PlanEnt& pe = plan[redo[g0 + q]];
                pe.node = ROOT;
                pe.depth = 0;
                run[q] = root_live;
            }
            for (bool any = root_live; any;) {
                any = false;
                for (uint32_t q = 0; q < G; ++q) {
                    const PlanEnt& pe = plan[redo[g0 + q]];
                    const uint32_t* w = plan_words[pe.part].data() + pe.woff;
                    if (run[q] && (pe.depth >= pe.nw || w[pe.depth] == W_UNKNOWN)) run[q] = false;
                    if (run[q]) __builtin_prefetch(&slots[(size_t)home_bucket(pe.node, w[pe.depth], nb) * BUCKET]);
                }
                for (uint32_t q = 0; q < G; ++q) {
                    if (!run[q]) continue;
                    PlanEnt& pe = plan[redo[g0 + q]];
                    const uint32_t s = find_slot(pe.node, plan_words[pe.part][pe.woff + pe.depth]);
                    // (an edge whose child died in this apply waits for its
                    // delete in the shared edge phase: a miss)
                    if (s == NONE || !nd[slots[s].child & ID_MASK].live) { run[q] = false; continue; }
                    pe.node = slots[s].child & ID_MASK;
                    ++pe.depth;
                    any = true;
                }
            }
        }
        return (uint32_t)redo.size();
    }
    std::vector<uint32_t> replan_buf;

    // the serial passes prefetch what filter i + PF_FAR / i + PF_NEAR will
    // touch: their node records first, then the lines those records point at
    static constexpr uint32_t PF_FAR = 16, PF_NEAR = 8;
    void prefetch_insert(uint32_t i, uint32_t n) {
        if (i + PF_FAR < n) __builtin_prefetch(&nd[plan[i + PF_FAR].node]);
        if (i + PF_NEAR < n) {
            const PlanEnt& q = plan[i + PF_NEAR];
            if (q.depth < q.nw) {
                const uint32_t w = plan_words[q.part][q.woff + q.depth];
                if (w != W_UNKNOWN) __builtin_prefetch(&slots[(size_t)home_bucket(q.node, w, nbuckets()) * BUCKET]);
            }
            const size_t nf = free_nodes.size();
            if (nf > PF_NEAR) __builtin_prefetch(&nd[free_nodes[nf - 1 - PF_NEAR]]);
        }
    }
    void prefetch_delete(uint32_t i, uint32_t n) {
        if (i + PF_FAR < n && plan[i + PF_FAR].node != NONE) __builtin_prefetch(&nd[plan[i + PF_FAR].node]);
        if (i + PF_NEAR < n && plan[i + PF_NEAR].node != NONE) {
            const NodeRec& r = nd[plan[i + PF_NEAR].node];
            __builtin_prefetch(&nd[r.parent]);
            if (r.inslot != NONE) {
                __builtin_prefetch(&slots[r.inslot]);
                if ((r.inslot >> 6) < dirty_mark.size()) __builtin_prefetch(&dirty_mark[r.inslot >> 6]);
            }
        }
    }

    int insert_planned(const uint8_t* buf, const uint64_t* offs, uint32_t i) {
        PlanEnt& pe = plan[i];
        uint32_t* ids = plan_words[pe.part].data() + pe.woff;
        for (uint32_t k = pe.depth; k < pe.nw; ++k)
            if (ids[k] == W_UNKNOWN) {   // new word (or interned by an earlier filter of the batch)
                if (frozen) return TM_ENOENT;
                const uint8_t* f = buf + offs[i];
                static thread_local std::vector<TWord> ws;
                split_words(f, offs[i + 1] - offs[i], ws);
                for (uint32_t j = k; j < pe.nw; ++j)
                    if (ids[j] == W_UNKNOWN) ids[j] = dict.intern(ws[j].p, ws[j].n);
                break;
            }
        // the planned prefix was walked with the root live; a root created since
        // (empty trie at plan time) restarts at ROOT, level 0
        return trie_insert_ids(buf + offs[i], offs[i + 1] - offs[i], ids, pe.nw, pe.node, pe.depth);
    }

    int delete_planned(uint32_t i) {
        const PlanEnt& pe = plan[i];
        if (pe.node == NONE || !nd[pe.node].live) return TM_OK;   // absent, or removed earlier in the batch
        return trie_delete_at(pe.node, plan_words[pe.part].data() + pe.woff, pe.nw);
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
    static constexpr uint32_t PAR_RANGE_MIN = 4096;    // buckets per phase-2 range at least (>> max_disp)

    static uint32_t mix_word(uint32_t w) {
        uint64_t k = (uint64_t)w * 0x9E3779B97F4A7C15ull;
        return (uint32_t)(k >> 32);
    }

    void ensure_pool() {
        if (!pool_started) {
            cpu_set_t cpus;
            pool.start(threads, device_node_cpus(device, threads, cpus) ? &cpus : nullptr);
            pool_started = true;
        }
    }

    // a pass over node ids v touching each node's record and its slot: the
    // record 16 nodes ahead, the slot (from the record, by then in cache) 8 ahead
    void prefetch_edge_of(const std::vector<uint32_t>& v, size_t q) const {
        if (q + 16 < v.size()) {
            __builtin_prefetch(&nd[v[q + 16]]);
            __builtin_prefetch(&n_lext[v[q + 16]]);
        }
        if (q + 8 < v.size()) {
            const uint32_t s = nd[v[q + 8]].inslot;
            if (s != NONE && s < slots.size()) __builtin_prefetch(&slots[s], 1);
        }
    }

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
    void edge_phase(const std::vector<std::vector<Mut>*>& Ws) {
        const unsigned T = std::max(1u, threads);
        auto each = [&](auto&& fn) {
            for (std::vector<Mut>* W : Ws)
                for (Mut& m : *W) fn(m);
        };
        auto merge_edges = [&](std::vector<Mut>& X) {
            for (Mut& m : X) {
                live_edges += m.live_edges; used_slots += m.used_slots; max_disp = std::max(max_disp, m.max_disp);
                dirty.insert(dirty.end(), m.dirty.begin(), m.dirty.end());
                m.live_edges = m.used_slots = 0; m.max_disp = 0; m.dirty.clear();
            }
        };
        auto ranges = [&](unsigned& T2, uint32_t& RS, uint32_t& R) {
            const uint32_t nb = nbuckets();
            T2 = std::min<unsigned>(T, nb / (2 * PAR_RANGE_MIN));
            if (T2 < 2) { T2 = 0; return; }
            RS = ((nb + 2 * T2 - 1) / (2 * T2) + 15) / 16 * 16;   // whole 16-bucket groups: dirty-mark words stay per range
            R = (nb + RS - 1) / RS;
        };
        each([](Mut& m) { m.defer = false; });
        const bool trace = getenv("TM_PAR_TRACE") != nullptr;
        auto now = [] { return std::chrono::steady_clock::now(); };
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        const auto e0 = now();
        unsigned T2 = 0;
        uint32_t RS = 0, R = 0;
        // ---- deletes, bucketed by the slot recorded in phase 1 (nothing has moved since)
        size_t ndel = 0;
        each([&](Mut& m) { ndel += m.del.size(); });
        ranges(T2, RS, R);
        if (!ndel) {
        } else if (!T2) {
            each([&](Mut& m) {
                for (const auto& d : m.del) delete_edge_of(d.first);
            });
        } else {
            std::vector<std::vector<uint32_t>> per(2 * T2);
            std::vector<uint32_t> tail;
            each([&](Mut& m) {
                for (const auto& d : m.del) {
                    const uint32_t r = d.second / BUCKET / RS;
                    if (R % 2 && r == R - 1) tail.push_back(d.first);   // (R odd: the last range wraps onto range 0)
                    else per[r].push_back(d.first);
                }
            });
            std::vector<Mut>& X = edge_states(T2);
            std::vector<std::vector<uint32_t>> late(T2);
            for (uint32_t par = 0; par < 2; ++par)
                pool.run([&](unsigned t) {
                    if (t >= T2) return;
                    const uint32_t r = 2 * t + par;
                    tl_mut = &X[t];
                    const std::vector<uint32_t>& v = per[r];
                    for (size_t q = 0; q < v.size(); ++q) {
                        prefetch_edge_of(v, q);
                        const uint32_t c = v[q];
                        // an odd range's slot may have been pulled back into the even range before it
                        if (nd[c].inslot / BUCKET / RS != r) { late[t].push_back(c); continue; }
                        delete_edge_of(c);
                    }
                    tl_mut = nullptr;
                });
            merge_edges(X);
            for (auto& l : late) tail.insert(tail.end(), l.begin(), l.end());
            for (uint32_t c : tail) delete_edge_of(c);   // serially, global counters
        }
        // ---- inserts: room first (the serial insert_edge's rehash rule, for the whole batch)
        const auto e1 = now();
        size_t nins = 0;
        each([&](Mut& m) { nins += m.ins.size(); });
        bool rehashed = false;
        if ((used_slots + nins) * 4 > slots.size() * 3 || max_disp > 48) {
            rehash(std::max<size_t>((size_t)((live_edges + nins) / 0.55), slots.size() * (max_disp > 48 ? 2 : 1)));
            rehashed = true;
        }
        const auto e2 = now();
        ranges(T2, RS, R);
        if (!nins) {
        } else if (!T2) {
            each([&](Mut& m) {
                for (const auto& e : m.ins) insert_edge(e[0], e[1], e[2]);
            });
        } else {
            std::vector<std::vector<std::array<uint32_t, 3>>> per(2 * T2);
            std::vector<std::array<uint32_t, 3>> tail;
            const uint32_t nb = nbuckets();
            each([&](Mut& m) {
                for (const auto& e : m.ins) {
                    const uint32_t r = home_bucket(e[0], e[1], nb) / RS;
                    if (R % 2 && r == R - 1) tail.push_back(e);
                    else per[r].push_back(e);
                }
            });
            std::vector<Mut>& X = edge_states(T2);
            for (uint32_t par = 0; par < 2; ++par)
                pool.run([&](unsigned t) {
                    if (t >= T2) return;
                    tl_mut = &X[t];
                    const auto& v = per[2 * t + par];
                    for (size_t q = 0; q < v.size(); ++q) {
                        if (q + 8 < v.size()) {   // the home bucket and the child's record, a few edges ahead
                            __builtin_prefetch(&slots[(size_t)home_bucket(v[q + 8][0], v[q + 8][1], nb) * BUCKET], 1);
                            __builtin_prefetch(&nd[v[q + 8][2]], 1);
                        }
                        insert_edge(v[q][0], v[q][1], v[q][2]);
                    }
                    tl_mut = nullptr;
                });
            merge_edges(X);
            for (const auto& e : tail) insert_edge(e[0], e[1], e[2]);
        }
        if (max_disp > 48) rehash(std::max<size_t>((size_t)(live_edges / 0.55), slots.size() * 2));
        const auto e3 = now();
        // ---- summaries of the nodes whose record changed: by node (a node's
        // records are rewritten by one worker; dirty marks set atomically)
        const unsigned TS = (unsigned)std::min<size_t>(T, std::max<size_t>(1, slots.size() / 4096));
        std::vector<std::vector<uint32_t>> per(TS);
        each([&](Mut& m) {
            for (uint32_t c : m.sum) per[mix_word(c) % TS].push_back(c);
        });
        std::vector<Mut>& X = edge_states(TS);
        pool.run([&](unsigned t) {
            if (t >= TS) return;
            std::vector<uint32_t>& v = per[t];
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
            for (size_t q = 0; q < v.size(); ++q) {
                prefetch_edge_of(v, q);
                const uint32_t c = v[q];
                if (!nd[c].live || nd[c].inslot == NONE) continue;
                write_summary_at(c, X[t].dirty);
            }
        });
        merge_edges(X);
        if (trace)
            fprintf(stderr, "[par edges T2=%u nb=%u] del %.2f rehash %d %.2f ins %.2f sum %.2f ms\n", T2, nbuckets(),
                    ms(e0, e1), (int)rehashed, ms(e1, e2), ms(e2, e3), ms(e3, now()));
    }

    // write_summary for a parallel pass: the dirty mark set atomically (another
    // worker may mark a slot of the same 64-slot word)
    void write_summary_at(uint32_t c, std::vector<uint32_t>& dl) {
        const uint32_t i = nd[c].inslot;
        Slot& e = slots[i];
        slot_set_lsig(e, nd[c].lsig());
        e.child = c | (nd[c].topic ? B_TOPIC : 0u) | (nd[c].plus != NONE ? B_PLUS : 0u);
        const uint32_t h = nd[c].hash;
        e.hash = h != NONE ? h | (nd[h].topic ? B_HTERM : 0u) | B_HASH : n_lext[c];
        if (full_dirty) return;
        const uint64_t m = 1ull << (i & 63);
        if (!(__atomic_fetch_or(&dirty_mark[i >> 6], m, __ATOMIC_RELAXED) & m)) dl.push_back(i);
    }

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
                        int* rc_out) {
        ParRun R;
        if (par_begin(del, buf, offs, n, mut_w, R)) return 1;
        ParRun* runs[1] = {&R};
        par_finish(runs, 1);
        *done_out = R.done;
        *rc_out = R.rc;
        return 0;
    }

    // Setup and phase 1 (node records) of a parallel mutation into the states
    // W; 1: the batch must run serially instead (nothing changed then).
    int par_begin(bool del, const uint8_t* buf, const uint64_t* offs, uint32_t n, std::vector<Mut>& W, ParRun& R) {
        const unsigned T = std::max(1u, threads);
        if (T < 2 || (uint64_t)n * 4 > n_filters) return 1;   // bulk builds stay serial: churn on a big trie only
        if (!del) {
            // new words are interned first, serially (the dictionary is not thread-safe)
            for (uint32_t i = 0; i < n; ++i) {
                PlanEnt& pe = plan[i];
                uint32_t* ids = plan_words[pe.part].data() + pe.woff;
                bool unknown = false;
                for (uint32_t k = pe.depth; k < pe.nw; ++k) unknown |= ids[k] == W_UNKNOWN;
                if (!unknown) continue;
                if (frozen) return 1;   // TM_ENOENT semantics of the serial pass (stop at the first)
                static thread_local std::vector<TWord> ws;
                split_words(buf + offs[i], offs[i + 1] - offs[i], ws);
                for (uint32_t k = pe.depth; k < pe.nw; ++k)
                    if (ids[k] == W_UNKNOWN) ids[k] = dict.intern(ws[k].p, ws[k].n);
            }
        }
        ensure_pool();
        const auto ts0 = std::chrono::steady_clock::now();
        if (W.size() != T) W.resize(T);   // (each worker resets its own state when phase 1 starts)
        // by the first two words: one worker owns those subtrees; 8 parts per
        // worker, taken largest first by whichever worker is free (skewed
        // churn clusters under a few first words)
        const uint32_t P = 8 * T;
        std::vector<std::vector<uint32_t>>& parts = parts_buf;   // (capacity kept across batches)
        parts.resize(P);
        for (auto& v : parts) v.clear();
        for (uint32_t i = 0; i < n; ++i) {
            const PlanEnt& pe = plan[i];
            const uint32_t* w = plan_words[pe.part].data() + pe.woff;
            const uint32_t key = mix_word(pe.nw ? w[0] : 0) ^ (pe.nw > 1 ? mix_word(w[1] * 0x85EBCA6Bu + 1) : 0u);
            parts[mix_word(key) % P].push_back(i);
        }
        // An insert part far above a worker's share (a hot first-two-words
        // prefix, e.g. 10% of C5's churn under "+/+") is split by its third
        // word: its filters then share the depth-2 nodes too, under the same
        // striped locks and shared made map (parts split_from.. are those).
        const uint32_t split_from = P;
        if (!del) {
            const size_t big = std::max<size_t>(64, n / (2 * T));
            constexpr uint32_t SPLIT = 8;
            for (uint32_t q = 0; q < split_from; ++q) {
                if (parts[q].size() <= big) continue;
                std::vector<uint32_t> whole;
                whole.swap(parts[q]);
                const size_t first = parts.size();
                parts.resize(first + SPLIT);
                for (uint32_t i : whole) {
                    const PlanEnt& pe = plan[i];
                    const uint32_t* w = plan_words[pe.part].data() + pe.woff;
                    parts[first + (pe.nw > 2 ? mix_word(w[2] * 0xC2B2AE35u + 7) % SPLIT : 0)].push_back(i);
                }
            }
        }
        const uint32_t NP = (uint32_t)parts.size();
        std::vector<uint32_t> porder(NP);
        for (uint32_t q = 0; q < NP; ++q) porder[q] = q;
        std::sort(porder.begin(), porder.end(), [&](uint32_t a, uint32_t b) { return parts[a].size() > parts[b].size(); });
        std::atomic<uint32_t> next_part{0};
        // the first error stops every worker (not just the one that hit it):
        // the filters applied are then those finished before it, see the header
        std::atomic<bool> failed{false};
        // node ids: at most the levels the batch's filters lack, the free ids first
        std::vector<uint32_t>& ids = R.ids;
        ids.clear();
        std::atomic<size_t> next_id{0};
        size_t fresh = 0;
        const size_t base = nd.size();
        if (!del) {
            release_pending_ids();
            uint64_t total = 0;
            for (uint32_t i = 0; i < n; ++i) total += plan[i].nw - plan[i].depth;
            const size_t take = std::min<size_t>(total, free_nodes.size());
            fresh = total - take + (size_t)T * Mut::ID_CHUNK;   // + slack: ids are taken a chunk per worker
            if (base + fresh >= MAX_NODES) return 1;
            // Transactional: every allocation first (a bad_alloc here leaves
            // the engine as it was: the caller may still finish other work on
            // it), then the commit below, which allocates nothing.
            ids.reserve(take);
            if (fresh) {
                nd.reserve(base + fresh);
                n_flen.reserve(base + fresh);
                n_lext.reserve(base + fresh);
                n_foff.reserve(base + fresh);
            }
            if (!full_f_dirty) dirty_f_mark.reserve(base + fresh);
            ids.assign(free_nodes.end() - (long)take, free_nodes.end());
            free_nodes.resize(free_nodes.size() - take);
            if (fresh) {
                nd.resize(base + fresh);   // dead records until handed out; the unused tail is cut after
                n_flen.resize(base + fresh, 0);
                n_lext.resize(base + fresh, 0);
                n_foff.resize(base + fresh, 0);
            }
            if (!full_f_dirty && dirty_f_mark.size() < nd.size()) dirty_f_mark.resize(nd.size(), 0);
        }
        // (shared_made was cleared at the end of the previous batch)
        const auto tp0 = std::chrono::steady_clock::now();
        // phase 1: node records, by first word
        pool.run([&](unsigned t) {
            Mut& m = W[t];
            m.reset();
            m.ids = &ids;
            m.next_id = &next_id;
            m.n_free = ids.size();
            m.n_fresh = fresh;
            m.fresh_base = base;
            m.defer = true;
            tl_mut = &m;
            const auto tw0 = std::chrono::steady_clock::now();
            try {
                for (uint32_t pi; !m.rc && !failed.load(std::memory_order_relaxed) && (pi = next_part.fetch_add(1)) < NP;) {
                    const std::vector<uint32_t>& items = parts[porder[pi]];
                    const uint32_t sd = porder[pi] >= split_from ? 3 : 2;
                    const size_t ni = items.size();
                    m.n_items += ni;
                    for (size_t q = 0; q < ni; ++q) {
                        if ((q & 63) == 63 && failed.load(std::memory_order_relaxed)) break;
                        const uint32_t i = items[q];
                        if (q + 8 < ni) {   // the record the walk starts from, a few filters ahead
                            const uint32_t f = plan[items[q + 8]].node;
                            if (f != NONE) {
                                __builtin_prefetch(&nd[f]);
                                __builtin_prefetch(&n_lext[f]);   // (a new literal child sets a bit there)
                            }
                        }
                        const PlanEnt& pe = plan[i];
                        int rc;
                        if (del) {
                            rc = delete_planned(i);
                        } else {
                            rc = trie_insert_ids(buf + offs[i], offs[i + 1] - offs[i],
                                                 plan_words[pe.part].data() + pe.woff, pe.nw, pe.node, pe.depth, sd);
                        }
                        if (rc) { m.rc = rc; failed.store(true, std::memory_order_relaxed); break; }
                        ++m.done;
                    }
                }
            } catch (...) {
                m.rc = TM_ENOMEM;
                failed.store(true, std::memory_order_relaxed);
            }
            m.t_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw0).count();
            tl_mut = nullptr;
        });
        R.del = del;
        R.n = n;
        R.W = &W;
        R.fresh = fresh;
        R.base = base;
        R.ts0 = ts0;
        R.tp0 = tp0;
        R.tp1 = std::chrono::steady_clock::now();
        return 0;
    }

    // Phase 2 (the edge hash) of every run at once -- their edge deletes, then
    // their inserts, then the summaries -- and the merges.
    void par_finish(ParRun* const* runs, size_t nr) {
        const unsigned T = std::max(1u, threads);
        std::vector<std::vector<Mut>*> Ws;
        for (size_t r = 0; r < nr; ++r) Ws.push_back(runs[r]->W);
        edge_phase(Ws);
        const auto tp2 = std::chrono::steady_clock::now();
        for (size_t r = 0; r < nr; ++r) {
            ParRun& R = *runs[r];
            R.tp2 = tp2;
            for (Mut& m : *R.W) {
                live_nodes += m.live_nodes;
                n_filters += m.n_filters;
                route_entries += m.route_entries;
                routes_dirty = routes_dirty || m.routes_dirty;
                version += m.version;
                R.done += m.done;
                if (m.rc && !R.rc) R.rc = m.rc;
                m.fresh_base = fbytes.size();   // (reused: this worker's bytes start here)
                fbytes.insert(fbytes.end(), m.fb.begin(), m.fb.end());
                dirty_f.insert(dirty_f.end(), m.dirty_f.begin(), m.dirty_f.end());
                for (const auto& q : m.pend) pending_free.push_back(q);
            }
        }
        pool.run([&](unsigned t) {   // filter byte offsets: distinct nodes per worker
            for (size_t r = 0; r < nr; ++r) {
                const std::vector<Mut>& W = *runs[r]->W;
                for (size_t j = t; j < W.size(); j += pool.n)
                    for (const auto& f : W[j].foff) n_foff[f.first] = W[j].fresh_base + f.second;
            }
            for (unsigned j = t; j < 64; j += pool.n) shared_made[j].clear();   // for the next batch
        });
        for (size_t r = 0; r < nr; ++r) {
            ParRun& R = *runs[r];
            if (R.del) continue;
            std::vector<Mut>& W = *R.W;
            const std::vector<uint32_t>& ids = R.ids;
            const size_t fresh = R.fresh, base = R.base;
            // ids not handed out: free ones back to the list, the fresh tail cut off
            // (the rest of each worker's last chunk: free-list ids go back; fresh
            // ids below the highest one handed out stay as free dead records)
            size_t used = 0;
            for (const Mut& m : W) used = std::max(used, m.id_lo);   // highest id index handed out + 1
            const size_t avail = ids.size() + fresh;
            if (used > avail) used = avail;
            for (const Mut& m : W)
                for (size_t k = m.id_lo; k < std::min(m.id_hi, used); ++k)
                    free_nodes.push_back(k < ids.size() ? ids[k] : (uint32_t)(base + (k - ids.size())));
            for (size_t k = used; k < ids.size(); ++k) free_nodes.push_back(ids[k]);
            const size_t fresh_used = used > ids.size() ? used - ids.size() : 0;
            if (fresh_used < fresh) {
                nd.resize(base + fresh_used);
                n_flen.resize(base + fresh_used);
                n_lext.resize(base + fresh_used);
                n_foff.resize(base + fresh_used);
                if (dirty_f_mark.size() > nd.size()) dirty_f_mark.resize(nd.size());
            }
        }
        if (getenv("TM_PAR_TRACE")) {
            const auto tp3 = std::chrono::steady_clock::now();
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            for (size_t r = 0; r < nr; ++r) {
                const ParRun& R = *runs[r];
                fprintf(stderr, "[par %s n=%u T=%u] setup %.2f ms phase1 %.2f ms edges %.2f ms merge %.2f ms%s; workers (items, us):",
                        R.del ? "del" : "ins", R.n, T, ms(R.ts0, R.tp0), ms(R.tp0, R.tp1), ms(R.tp1, R.tp2), ms(R.tp2, tp3),
                        nr > 1 ? " (edges + merge shared)" : "");
                for (const Mut& m : *R.W) fprintf(stderr, " (%zu, %.0f)", m.n_items, m.t_us);
                fprintf(stderr, "\n");
            }
        }
    }

    // ------------------------------------------------------------ device sync

    uint32_t node_of(const uint8_t* t, size_t len) {
        static thread_local std::vector<uint32_t> ids;
        if (!filter_words(t, len, false, ids)) return NONE;
        const uint32_t n = walk(ids);
        return (n != NONE && nd[n].topic) ? n : NONE;
    }

    // emqx_router:do_add_route/2 (src/emqx_router.erl:113-124, 229-234)
    int route_add(const uint8_t* t, size_t len, uint32_t dest) {
        uint32_t n = node_of(t, len);
        if (n == NONE || n >= n_nroutes.size() || n_nroutes[n] == 0) {
            int rc = trie_insert(t, len);     // first route: emqx_trie:insert/1 (idempotent)
            if (rc) return rc;
            n = node_of(t, len);
            if (n == NONE) return TM_EIO;
        }
        if (n_dests.size() < nd.size()) {
            n_dests.resize(nd.size());
            n_nroutes.resize(nd.size(), 0);
        }
        auto& v = n_dests[n];
        bool found = false;
        for (auto& e : v)
            if (e.first == dest) { ++e.second; found = true; break; }
        if (!found) {
            v.emplace_back(dest, 1u);
            ++route_entries;
            routes_dirty = true;
        }
        ++n_nroutes[n];
        ++version;
        return TM_OK;
    }

    // do_delete_route/2 (:163-169) + delete_trie_route/1 (:239-247)
    int route_delete(const uint8_t* t, size_t len, uint32_t dest) {
        const uint32_t n = node_of(t, len);
        if (n == NONE || n >= n_dests.size()) return TM_ENOENT;
        auto& v = n_dests[n];
        size_t k = 0;
        while (k < v.size() && v[k].first != dest) ++k;
        if (k == v.size()) return TM_ENOENT;
        if (--v[k].second == 0) {
            v.erase(v.begin() + (long)k);
            --route_entries;
            routes_dirty = true;
        }
        --n_nroutes[n];
        ++version;
        if (n_nroutes[n] == 0) return trie_delete(t, len);   // last route: emqx_trie:delete/1
        return TM_OK;
    }

    // dests CSR by node id: built on the host when routes changed (routes_gen),
    // uploaded to a replica that has an older one
    int sync_routes(Replica& R) {
        if (routes_dirty || h_roff.size() < nd.size() + 1) {
            const size_t nn = nd.size();
            h_roff.assign(nn + 1, 0);
            h_rdest.clear();
            h_rdest.reserve(route_entries);
            for (size_t i = 0; i < nn; ++i) {
                h_roff[i] = (uint32_t)h_rdest.size();
                if (i < n_dests.size())
                    for (const auto& e : n_dests[i]) h_rdest.push_back(e.first);
            }
            h_roff[nn] = (uint32_t)h_rdest.size();
            routes_dirty = false;
            ++routes_gen;
        }
        if (R.routes_gen == routes_gen) return TM_OK;
        const size_t nn = h_roff.size() - 1;
        int rc;
        if ((rc = dev_reserve(R.d_roff, R.c_roff, nn + 1))) return rc;
        if ((rc = dev_reserve(R.d_rdest, R.c_rdest, std::max<size_t>(h_rdest.size(), 1)))) return rc;
        HIP_OK(hipMemcpyAsync(R.d_roff, h_roff.data(), (nn + 1) * 4, hipMemcpyHostToDevice, R.stream));
        if (!h_rdest.empty())
            HIP_OK(hipMemcpyAsync(R.d_rdest, h_rdest.data(), h_rdest.size() * 4, hipMemcpyHostToDevice, R.stream));
        HIP_OK(hipStreamSynchronize(R.stream));
        R.routes_gen = routes_gen;
        return TM_OK;
    }

    // tm_batch_routes: route CSR of a waited batch, resolved on the device
    int batch_routes(tm_batch* b, tm_routes* out) {
        if (!b->done) return TM_EINVAL;
        Replica& R = *b->rep;
        const hipStream_t stream = R.stream;
        int rc;
        if ((rc = ensure_dense(b))) return rc;
        if ((rc = sync_routes(R))) return rc;
        const uint32_t n = b->n;
        const size_t nn = std::max<size_t>(n, 1);
        const uint64_t m64 = b->total;   // match entries (< 2^32: u32 result CSR)
        if (m64 > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        const uint32_t m = (uint32_t)m64;
        if ((rc = dev_reserve(b->d_rcount, b->c_rcount, (size_t)m + 1))) return rc;    // per-entry counts
        if ((rc = dev_reserve(b->d_reoff, b->c_reoff, (size_t)m + 1))) return rc;
        if ((rc = dev_reserve(b->d_rrow, b->c_rrow, nn + 1))) return rc;
        if ((rc = dev_reserve(b->d_rbsums, b->c_rbsums, (size_t)scan_block_count(m) + 1))) return rc;
        if ((rc = dev_reserve(b->d_rtotal, b->c_rtotal, 1))) return rc;
        if ((rc = host_reserve(b->h_rtotal, b->ch_rtotal, 1))) return rc;
        RouteArgs r{};
        r.row_off = b->d_rowoff; r.ids = b->d_ids; r.n = n; r.m = m;
        r.roff = R.d_roff; r.rdest = R.d_rdest; r.nnodes = (uint32_t)(h_roff.size() - 1);
        r.ecount = b->d_rcount; r.eoff = b->d_reoff; r.bsums = b->d_rbsums; r.total = b->d_rtotal;
        r.r_rowoff = b->d_rrow;
        HIP_OK(launch_route_count(r, stream));
        ScanArgs sa{};
        sa.count = b->d_rcount; sa.row_off = b->d_reoff; sa.block_sums = b->d_rbsums; sa.n = m;
        if (m) {
            HIP_OK(launch_scan(sa, stream, b->d_rtotal));
        } else {
            HIP_OK(hipMemsetAsync(b->d_rtotal, 0, 4, stream));
        }
        HIP_OK(launch_route_rows(r, stream));
        HIP_OK(hipMemcpyAsync(b->h_rtotal, b->d_rtotal, 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        const uint64_t total = b->h_rtotal[0];
        if ((rc = dev_reserve(b->d_rfid, b->c_rfid, std::max<uint64_t>(total, 1)))) return rc;
        if ((rc = dev_reserve(b->d_rdest, b->c_rdest, std::max<uint64_t>(total, 1)))) return rc;
        r.out_fid = b->d_rfid; r.out_dest = b->d_rdest; r.cap = total;
        HIP_OK(launch_route_fill(r, stream));
        if ((rc = host_reserve(b->h_rrow, b->ch_rrow, nn + 1))) return rc;
        if ((rc = host_reserve(b->h_rfid, b->ch_rfid, std::max<uint64_t>(total, 1)))) return rc;
        if ((rc = host_reserve(b->h_rdest, b->ch_rdest, std::max<uint64_t>(total, 1)))) return rc;
        HIP_OK(hipMemcpyAsync(b->h_rrow, b->d_rrow, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, stream));
        if (total) {
            HIP_OK(hipMemcpyAsync(b->h_rfid, b->d_rfid, total * 4, hipMemcpyDeviceToHost, stream));
            HIP_OK(hipMemcpyAsync(b->h_rdest, b->d_rdest, total * 4, hipMemcpyDeviceToHost, stream));
        }
        HIP_OK(hipStreamSynchronize(stream));
        if (b->h_rrow[n] != total) {
            snprintf(last_error(), 512, "inconsistent route CSR: %u vs %llu", b->h_rrow[n], (unsigned long long)total);
            return TM_EIO;
        }
        out->n_topics = n;
        out->n_routes = total;
        out->row_offsets = b->h_rrow;
        out->filter_ids = b->h_rfid;
        out->dests = b->h_rdest;
        return TM_OK;
    }

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
    int subscribe(const uint8_t* t, size_t len, uint32_t sub, uint32_t node_dest) {
        std::string k((const char*)t, len);
        auto it = topics_of.find(sub);
        if (it != topics_of.end() && std::find(it->second.begin(), it->second.end(), k) != it->second.end())
            return TM_OK;   // subscribed already: only subopts would change (:127-139)
        auto sit = subs_of.find(k);
        if (sit == subs_of.end()) {
            int rc = route_add(t, len, node_dest);
            if (rc) return rc;
            sit = subs_of.emplace(k, std::vector<uint32_t>()).first;
        }
        sit->second.push_back(sub);
        topics_of[sub].push_back(std::move(k));
        ++sub_entries;
        subs_dirty = true;
        return TM_OK;
    }

    // do_unsubscribe/4 (:179-191) + handle_cast({unsubscribed, Topic}) (:463-469):
    // the last subscriber of a topic deletes the node's route.
    int unsubscribe(const uint8_t* t, size_t len, uint32_t sub, uint32_t node_dest) {
        std::string k((const char*)t, len);
        auto it = topics_of.find(sub);
        if (it == topics_of.end()) return TM_ENOENT;
        auto& ts = it->second;
        auto ti = std::find(ts.begin(), ts.end(), k);
        if (ti == ts.end()) return TM_ENOENT;   // unsubscribe/1's `[] -> ok` (:170-177)
        ts.erase(ti);
        if (ts.empty()) topics_of.erase(it);
        auto sit = subs_of.find(k);
        if (sit == subs_of.end()) return TM_EIO;
        auto& v = sit->second;
        auto vi = std::find(v.begin(), v.end(), sub);
        if (vi == v.end()) return TM_EIO;
        v.erase(vi);
        --sub_entries;
        subs_dirty = true;
        if (v.empty()) {
            subs_of.erase(sit);
            int rc = route_delete(t, len, node_dest);
            if (rc && rc != TM_ENOENT) return rc;
        }
        return TM_OK;
    }

    // subscriber_down/1 (:332-347): drop every subscription of the subscriber.
    int subscriber_down(uint32_t sub, uint32_t node_dest, uint64_t* n_removed) {
        uint64_t n = 0;
        auto it = topics_of.find(sub);
        if (it != topics_of.end()) {
            const std::vector<std::string> ts = it->second;
            for (const auto& k : ts) {
                int rc = unsubscribe((const uint8_t*)k.data(), k.size(), sub, node_dest);
                if (rc) return rc;
                ++n;
            }
        }
        if (n_removed) *n_removed = n;
        return TM_OK;
    }

    // subscriber runs by node id: rebuilt on the host after subscription or
    // trie changes (a topic's node id is looked up at build time), uploaded to
    // a replica holding an older build
    int sync_subs(Replica& R) {
        const size_t nn = nd.size();
        if (subs_dirty || subs_version != version || subs_nn != nn || h_soff.empty()) {
            h_soff.assign(nn + 1, 0);
            std::vector<std::pair<uint32_t, const std::vector<uint32_t>*>> runs;
            runs.reserve(subs_of.size());
            for (const auto& kv : subs_of) {
                const uint32_t n = node_of((const uint8_t*)kv.first.data(), kv.first.size());
                if (n == NONE || n >= nn) continue;   // not in the trie: no route, no dispatch
                runs.emplace_back(n, &kv.second);
                h_soff[n + 1] += kv.second.size();
            }
            for (size_t i = 0; i < nn; ++i) h_soff[i + 1] += h_soff[i];
            h_subs.resize(h_soff[nn]);
            for (const auto& r : runs) std::copy(r.second->begin(), r.second->end(), h_subs.begin() + (long)h_soff[r.first]);
            h_scnt.resize(std::max<size_t>(nn, 1));
            for (size_t i = 0; i < nn; ++i) h_scnt[i] = (uint8_t)std::min<uint64_t>(h_soff[i + 1] - h_soff[i], 255);
            h_sone.assign(std::max<size_t>(nn, 1), NONE);
            for (size_t i = 0; i < nn; ++i)
                if (h_soff[i + 1] - h_soff[i] == 1) h_sone[i] = h_subs[h_soff[i]];
            subs_dirty = false;
            subs_version = version;
            subs_nn = (uint32_t)nn;
            ++subs_gen;
        }
        if (R.subs_gen == subs_gen) return TM_OK;
        const size_t sn = subs_nn;
        int rc;
        if ((rc = dev_reserve(R.d_soff, R.c_soff, sn + 1))) return rc;
        if ((rc = dev_reserve(R.d_scnt, R.c_scnt, std::max<size_t>(sn, 1)))) return rc;
        if ((rc = dev_reserve(R.d_sone, R.c_sone, std::max<size_t>(sn, 1)))) return rc;
        if ((rc = dev_reserve(R.d_subs, R.c_subs, std::max<size_t>(h_subs.size(), 1)))) return rc;
        HIP_OK(hipMemcpyAsync(R.d_soff, h_soff.data(), (sn + 1) * 8, hipMemcpyHostToDevice, R.stream));
        if (sn) HIP_OK(hipMemcpyAsync(R.d_scnt, h_scnt.data(), sn, hipMemcpyHostToDevice, R.stream));
        if (sn) HIP_OK(hipMemcpyAsync(R.d_sone, h_sone.data(), sn * 4, hipMemcpyHostToDevice, R.stream));
        if (!h_subs.empty())
            HIP_OK(hipMemcpyAsync(R.d_subs, h_subs.data(), h_subs.size() * 4, hipMemcpyHostToDevice, R.stream));
        HIP_OK(hipStreamSynchronize(R.stream));
        R.subs_gen = subs_gen;
        return TM_OK;
    }

    // tm_batch_dispatch: deliveries of a waited batch, resolved on the device
    int batch_dispatch(tm_batch* b, uint32_t flags, tm_deliveries* out) {
        if (!b->done) return TM_EINVAL;
        const bool rows = flags & TM_DISPATCH_ROWS;
        if (rows && ((flags & TM_DISPATCH_MATCH_OFFSETS) || !b->csr)) return TM_EINVAL;
        if (rows) flags |= TM_DISPATCH_DEVICE;
        Replica& R = *b->rep;
        const hipStream_t stream = R.stream;
        int rc;
        if (!rows && (rc = ensure_dense(b))) return rc;
        if ((rc = sync_subs(R))) return rc;
        const uint32_t n = b->n;
        FanArgs fa{};
        uint64_t nm = b->total;
        if (rows) {   // the walk's staging regions as one virtual entry space (FanArgs)
            const uint64_t cap = std::min<uint64_t>(b->c_sfids, MAX_RESULT);
            fa.nreg = b->one_region ? 1u : TICKET_GROUPS;
            fa.rcap = region_cap(cap, b->one_region);
            // [vb: TICKET_GROUPS + 1 | rtop: TICKET_GROUPS] in pinned memory -> HBM
            constexpr size_t FM = 2 * TICKET_GROUPS + 1;
            if ((rc = host_reserve(b->h_fmeta, b->ch_fmeta, FM))) return rc;
            if ((rc = dev_reserve(b->d_fmeta, b->c_fmeta, FM))) return rc;
            uint64_t* vb = b->h_fmeta;
            uint64_t* rtop = b->h_fmeta + TICKET_GROUPS + 1;
            std::fill(b->h_fmeta, b->h_fmeta + FM, 0ull);
            uint64_t v = 0, staged = 0;
            for (uint32_t g = 0; g < fa.nreg; ++g) {
                vb[g] = v;
                rtop[g] = xg_top_read(b->h_ctrl, g);
                staged += rtop[g];
                v += (rtop[g] + 15) & ~15ull;
            }
            for (uint32_t g = fa.nreg; g <= TICKET_GROUPS; ++g) vb[g] = v;
            HIP_OK(hipMemcpyAsync(b->d_fmeta, b->h_fmeta, FM * 8, hipMemcpyHostToDevice, stream));
            fa.vb = b->d_fmeta;
            fa.rtop = b->d_fmeta + TICKET_GROUPS + 1;
            if (staged != b->total) {
                snprintf(last_error(), 512, "staging holds %llu entries, the walk matched %llu",
                         (unsigned long long)staged, (unsigned long long)b->total);
                return TM_EIO;
            }
            nm = v;
            if ((rc = dev_reserve(b->d_dcount, b->c_dcount, std::max<size_t>(n, 1)))) return rc;
            fa.rcount = b->d_count;
            fa.rsrc = b->d_src;
            fa.dcount = b->d_dcount;
        }
        const uint32_t nb = (uint32_t)((nm + 1 + fan_scan_tile() - 1) / fan_scan_tile());
        if ((rc = dev_reserve(b->d_moff, b->c_moff, nm + 1))) return rc;
        if ((rc = dev_reserve(b->d_fbsums, b->c_fbsums, nb))) return rc;
        if ((rc = dev_reserve(b->d_moff32, b->c_moff32, nm + 1))) return rc;
        if ((rc = dev_reserve(b->d_fbig, b->c_fbig, nb))) return rc;
        if ((rc = dev_reserve(b->d_ftotal, b->c_ftotal, 1))) return rc;
        if ((rc = dev_reserve(b->d_drow, b->c_drow, (size_t)n + 1))) return rc;
        if ((rc = host_reserve(b->h_ftotal, b->ch_ftotal, 1))) return rc;
        if (!b->fev0) {
            HIP_OK(hipEventCreate(&b->fev0));
            HIP_OK(hipEventCreate(&b->fev1));
        }
        fa.row_off = b->d_rowoff; fa.ids = rows ? b->d_sfids : b->d_ids; fa.n = n; fa.n_matches = nm;
        fa.soff = R.d_soff; fa.scnt = R.d_scnt; fa.sone = R.d_sone; fa.subs = R.d_subs; fa.nnodes = subs_nn;
        fa.moff = b->d_moff; fa.moff32 = b->d_moff32; fa.bbig = b->d_fbig; fa.bsums = b->d_fbsums;
        fa.big_limit = fan_big_limit; fa.d_total = b->d_ftotal; fa.drow = b->d_drow;
        HIP_OK(launch_fan_scan(fa, stream));
        HIP_OK(hipMemcpyAsync(b->h_ftotal, b->d_ftotal, 8, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        const uint64_t total = b->h_ftotal[0];
        const bool counts_only = flags & TM_DISPATCH_COUNT_ONLY;
        float fill_ms = 0.f;
        if (!counts_only) {
            if ((rc = dev_reserve(b->d_fout, b->c_fout, std::max<uint64_t>(total, 1)))) return rc;
            if ((rc = dev_reserve(b->d_ftile, b->c_ftile, (size_t)(total / fan_fill_tile()) + 2))) return rc;
            fa.out = b->d_fout; fa.total = total; fa.tile_j = b->d_ftile;
            HIP_OK(hipEventRecord(b->fev0, stream));
            HIP_OK(launch_fan_fill(fa, stream));
            HIP_OK(hipEventRecord(b->fev1, stream));
        }
        const bool want_moff = flags & TM_DISPATCH_MATCH_OFFSETS;
        if (want_moff) HIP_OK(launch_fan_globalize(fa, stream));   // moff is block-relative until now
        out->n_topics = n;
        out->n_matches = b->total;
        out->n_deliveries = total;
        out->row_counts = nullptr;
        if (flags & TM_DISPATCH_DEVICE) {
            HIP_OK(hipStreamSynchronize(stream));
            if (!counts_only) HIP_OK(hipEventElapsedTime(&fill_ms, b->fev0, b->fev1));
            out->row_offsets = b->d_drow;
            out->match_offsets = want_moff ? b->d_moff : nullptr;
            out->subscribers = counts_only ? nullptr : b->d_fout;
            out->fill_ms = fill_ms;
            out->row_counts = rows ? b->d_dcount : nullptr;
            return TM_OK;
        }
        if ((rc = host_reserve(b->h_drow, b->ch_drow, (size_t)n + 1))) return rc;
        HIP_OK(hipMemcpyAsync(b->h_drow, b->d_drow, ((size_t)n + 1) * 8, hipMemcpyDeviceToHost, stream));
        if (want_moff) {
            if ((rc = host_reserve(b->h_moff, b->ch_moff, nm + 1))) return rc;
            HIP_OK(hipMemcpyAsync(b->h_moff, b->d_moff, (nm + 1) * 8, hipMemcpyDeviceToHost, stream));
        }
        if (!counts_only) {
            if ((rc = host_reserve(b->h_fout, b->ch_fout, std::max<uint64_t>(total, 1)))) return rc;
            if (total) HIP_OK(hipMemcpyAsync(b->h_fout, b->d_fout, total * 4, hipMemcpyDeviceToHost, stream));
        }
        HIP_OK(hipStreamSynchronize(stream));
        if (!counts_only) HIP_OK(hipEventElapsedTime(&fill_ms, b->fev0, b->fev1));
        if (b->h_drow[n] != total) {
            snprintf(last_error(), 512, "inconsistent delivery CSR: %llu vs %llu", (unsigned long long)b->h_drow[n],
                     (unsigned long long)total);
            return TM_EIO;
        }
        out->row_offsets = b->h_drow;
        out->match_offsets = want_moff ? b->h_moff : nullptr;
        out->subscribers = counts_only ? nullptr : b->h_fout;
        out->fill_ms = fill_ms;
        return TM_OK;
    }

    // tm_rules_match: rules tokenised with their own dictionary, names against it
    int rules_match(Replica& R, const uint8_t* names, const uint64_t* noffs, uint32_t n, const uint8_t* rules,
                    const uint64_t* roffs, uint32_t r, bool dollar_rule, uint32_t* bits) {
        const hipStream_t stream = R.stream;
        WordDict rd;
        std::vector<TWord> ws;
        std::vector<uint32_t> rw, ro(1, 0), nw, no(1, 0);
        std::vector<uint8_t> rf(r), nf(n);
        auto id_of = [](const TWord& w) -> uint32_t {
            return w.n == 0 ? W_EMPTY : is_plus(w) ? W_PLUS : is_hash(w) ? W_HASH : W_UNKNOWN;
        };
        for (uint32_t j = 0; j < r; ++j) {
            const uint8_t* p = rules + roffs[j];
            const size_t len = roffs[j + 1] - roffs[j];
            split_words(p, len, ws);
            for (const TWord& w : ws) {
                uint32_t id = id_of(w);
                if (id == W_UNKNOWN) id = rd.intern(w.p, w.n);
                rw.push_back(id);
            }
            ro.push_back((uint32_t)rw.size());
            rf[j] = (len > 0 && (p[0] == '+' || p[0] == '#')) ? 1 : 0;
        }
        for (uint32_t t = 0; t < n; ++t) {
            const uint8_t* p = names + noffs[t];
            const size_t len = noffs[t + 1] - noffs[t];
            split_words(p, len, ws);
            for (const TWord& w : ws) {
                uint32_t id = id_of(w);
                if (id == W_UNKNOWN) id = rd.find(w.p, w.n);
                nw.push_back(id);
            }
            if (nw.size() > 0xFFFFFFF0ull) return TM_EOVERFLOW;
            no.push_back((uint32_t)nw.size());
            nf[t] = (len > 0 && p[0] == '$') ? 1 : 0;
        }
        const uint32_t wpr = (r + 31) / 32;
        // one device block: [rw | ro | nw | no | bits] in u32, then rf | nf bytes
        const size_t nbits = (size_t)n * wpr;
        const size_t words = rw.size() + ro.size() + nw.size() + no.size() + nbits + (r + n + 3) / 4 + 4;
        int rc;
        if ((rc = dev_reserve(R.d_rl, R.c_rl, words))) return rc;
        uint32_t* d = R.d_rl;
        uint32_t *d_rw = d, *d_ro = d_rw + rw.size(), *d_nw = d_ro + ro.size(), *d_no = d_nw + nw.size();
        uint32_t* d_bits = d_no + no.size();
        uint8_t* d_rf = reinterpret_cast<uint8_t*>(d_bits + nbits);
        uint8_t* d_nf = d_rf + r;
        HIP_OK(hipMemcpyAsync(d_rw, rw.data(), rw.size() * 4, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(d_ro, ro.data(), ro.size() * 4, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(d_nw, nw.data(), nw.size() * 4, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(d_no, no.data(), no.size() * 4, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(d_rf, rf.data(), r, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(d_nf, nf.data(), n, hipMemcpyHostToDevice, stream));
        RulesArgs a{};
        a.nwords = d_nw; a.noff = d_no; a.nflag = d_nf; a.n = n;
        a.rwords = d_rw; a.roff = d_ro; a.rflag = d_rf; a.r = r;
        a.dollar_rule = dollar_rule ? 1u : 0u; a.wpr = wpr; a.bits = d_bits;
        HIP_OK(launch_rules_match(a, stream));
        HIP_OK(hipMemcpyAsync(bits, d_bits, nbits * 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));   // the host vectors above are freed on return
        return TM_OK;
    }

    bool needs_repack() const {
        return live_edges > 65536 && (slots.size() > (size_t)(live_edges / target_load) * 2 ||
                                      slots.size() * target_load * 1.5 < live_edges);
    }

    // anything for sync_device to upload to replica R?
    bool upload_pending(const Replica& R) {
        if (full_dirty || !dirty.empty() || R.d_nslots != slots.size() || needs_repack()) return true;
        if (full_f_dirty || !dirty_f.empty() || fbytes.size() > R.fbytes_uploaded) return true;
        if (R.c_foff < nd.size() || R.c_flen < nd.size() || R.c_fbytes < fbytes.size() + 1) return true;
        if (dev_tok && (R.d_dict_n != dict.keys().size() || R.d_dict_gen != dict.gen() || !dict.dirty().empty() ||
                        dict.tails().size() > R.tails_uploaded || dict.arena().size() > R.arena_uploaded ||
                        R.c_arena < dict.arena().size() + 1))
            return true;
        return false;
    }

    int ensure_delta_idle() {
        for (Replica* R : reps)
            if (R->delta_inflight) {
                HIP_OK(hipSetDevice(R->device));
                HIP_OK(hipEventSynchronize(R->ev_delta));
                R->delta_inflight = false;
            }
        return TM_OK;
    }

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
    int sync_device(const Replica* back = nullptr) {
        if (reps.empty()) return TM_ENODEV;
        int rc = ensure_delta_idle();
        if (rc) return rc;
        bool any = false;
        for (Replica* R : reps) any = any || upload_pending(*R);
        if (!any) {
            HIP_OK(hipSetDevice(back ? back->device : device));
            return TM_OK;
        }
        // after a bulk build or heavy churn, re-pack the host table to the
        // target load so the walk's working set stays small (a full upload)
        if (needs_repack()) {
            rehash((size_t)(live_edges / target_load));
            rebuild_lext();   // (a full upload follows the re-pack anyway)
        }
        const size_t nn = nd.size();
        // gather the deltas once
        const bool slots_full = full_dirty || dirty.size() > slots.size() / 8;
        if (!slots_full && !dirty.empty()) {
            const size_t k = dirty.size();
            if ((rc = host_reserve(h_didx, ch_didx, k))) return rc;
            if ((rc = host_reserve(h_dval, ch_dval, k))) return rc;
            par_chunks(k, [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i) {
                    if (i + 16 < i1) __builtin_prefetch(&slots[dirty[i + 16]]);
                    h_didx[i] = dirty[i];
                    h_dval[i] = slots[dirty[i]];
                }
            });
        }
        if (!full_f_dirty && !dirty_f.empty()) {
            const size_t k = dirty_f.size();
            if ((rc = host_reserve(h_fidx, ch_fidx, k))) return rc;
            if ((rc = host_reserve(h_foffv, ch_foffv, k))) return rc;
            if ((rc = host_reserve(h_flenv, ch_flenv, k))) return rc;
            par_chunks(k, [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i) {
                    const uint32_t c = dirty_f[i];
                    h_fidx[i] = c; h_foffv[i] = n_foff[c]; h_flenv[i] = n_flen[c];
                }
            });
        }
        std::vector<uint32_t>& dx = dict.dirty();
        const bool keys_full = dx.size() > dict.keys().size() / 8;
        if (dev_tok && !keys_full && !dx.empty()) {
            std::sort(dx.begin(), dx.end());
            dx.erase(std::unique(dx.begin(), dx.end()), dx.end());   // a slot may move twice: scatter it once
            const size_t k = dx.size();
            if ((rc = host_reserve(h_dxidx, ch_dxidx, k))) return rc;
            if ((rc = host_reserve(h_dxval, ch_dxval, k))) return rc;
            for (size_t i = 0; i < k; ++i) {
                h_dxidx[i] = dx[i];
                h_dxval[i] = dict.keys()[dx[i]];
            }
        }
        // apply to every replica (different devices run their copies concurrently)
        std::vector<uint8_t> pageable(reps.size(), 0), async(reps.size(), 0);
        for (size_t r = 0; r < reps.size(); ++r) {
            Replica& R = *reps[r];
            bool pg = false, as = false;
            if ((rc = upload_to(R, slots_full, keys_full, nn, pg, as))) return rc;
            pageable[r] = pg;
            async[r] = as;
        }
        // the dirty sets are consumed: every replica has them now
        if (slots_full) {
            full_dirty = false;
            for (uint32_t i : dirty) dirty_mark[i >> 6] = 0;   // every set bit is in `dirty`
            if (dirty_mark.size() != (slots.size() + 63) / 64) dirty_mark.assign((slots.size() + 63) / 64, 0);
        } else {
            for (uint32_t i : dirty) dirty_mark[i >> 6] = 0;
        }
        dirty.clear();
        if (full_f_dirty) {
            full_f_dirty = false;
            dirty_f_mark.assign(nn, 0);
        } else {
            for (uint32_t c : dirty_f) dirty_f_mark[c] = 0;
        }
        dirty_f.clear();
        if (dev_tok) dx.clear();
        for (size_t r = 0; r < reps.size(); ++r) {
            Replica& R = *reps[r];
            HIP_OK(hipSetDevice(R.device));
            if (pageable[r]) {
                // host vectors may be mutated / reallocated right after we return
                HIP_OK(hipStreamSynchronize(R.stream));
            } else if (async[r]) {
                HIP_OK(hipEventRecord(R.ev_delta, R.stream));
                R.delta_inflight = true;
                if (!R.readers.empty()) {   // own-stream batches launched from now on wait for this upload
                    HIP_OK(hipEventRecord(R.ev_sync, R.stream));
                    ++R.upload_seq;
                }
            }
        }
        HIP_OK(hipSetDevice(back ? back->device : device));
        return TM_OK;
    }

    // one replica's share of sync_device: the staged deltas (or full tables)
    int upload_to(Replica& R, bool slots_full, bool keys_full, size_t nn, bool& pageable_used, bool& async_used) {
        int rc;
        HIP_OK(hipSetDevice(R.device));
        const hipStream_t stream = R.stream;
        // tables change under the walks of this replica's own-stream batches in
        // flight: the uploads wait for them on the device, or on the host when
        // a table is reallocated (its old buffer is freed here)
        const bool realloc = R.d_nslots != slots.size() || R.c_foff < nn || R.c_flen < nn ||
                             R.c_fbytes < fbytes.size() + 1 ||
                             (dev_tok && (R.d_dict_n != dict.keys().size() || R.c_tail < dict.tails().size() + 1 ||
                                          R.c_arena < dict.arena().size() + 1));
        for (tm_batch* r : R.readers)
            if (r->launched) {
                if (realloc) {
                    HIP_OK(hipStreamSynchronize(r->own));
                    continue;
                }
                if (!r->ev_read) HIP_OK(hipEventCreateWithFlags(&r->ev_read, hipEventDisableTiming));
                HIP_OK(hipEventRecord(r->ev_read, r->own));
                HIP_OK(hipStreamWaitEvent(stream, r->ev_read, 0));
            }
        // edge hash
        bool full = slots_full;
        if (R.d_nslots != slots.size()) {
            dev_free(R.d_slots);
            HIP_OK(hipMalloc((void**)&R.d_slots, slots.size() * sizeof(Slot)));
            R.d_nslots = slots.size();
            full = true;
        }
        if (full) {
            pageable_used = true;
            HIP_OK(hipMemcpyAsync(R.d_slots, slots.data(), slots.size() * sizeof(Slot), hipMemcpyHostToDevice, stream));
            ++uploads_full;
        } else if (!dirty.empty()) {
            const size_t k = dirty.size();
            if ((rc = dev_reserve(R.d_didx, R.cd_didx, k))) return rc;
            if ((rc = dev_reserve(R.d_dval, R.cd_dval, k))) return rc;
            HIP_OK(hipMemcpyAsync(R.d_didx, h_didx, k * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
            HIP_OK(hipMemcpyAsync(R.d_dval, h_dval, k * sizeof(Slot), hipMemcpyHostToDevice, stream));
            HIP_OK(launch_scatter_slots(R.d_slots, R.d_didx, R.d_dval, (uint32_t)k, stream));
            ++uploads_delta;
            delta_slots += k;
            async_used = true;
        }
        // appended tails up to APP_MAX bytes in all go through the replica's
        // pinned staging (reserved once here: copies queued below read it until
        // the upload's event, and ensure_delta_idle waits for that before the
        // next upload reuses it)
        size_t app_need = 0, app_used = 0;
        {
            const uint64_t fb_from = R.c_fbytes < fbytes.size() + 1 ? 0 : R.fbytes_uploaded;
            app_need += fbytes.size() > fb_from ? fbytes.size() - fb_from : 0;
            if (dev_tok) {
                const size_t t_from = R.c_tail < dict.tails().size() + 1 ? 0 : R.tails_uploaded;
                const size_t a_from = R.c_arena < dict.arena().size() + 1 ? 0 : R.arena_uploaded;
                if (dict.tails().size() > t_from) app_need += (dict.tails().size() - t_from) * sizeof(DictTail) + 16;
                if (dict.arena().size() > a_from) app_need += dict.arena().size() - a_from + 16;
            }
        }
        const bool app_pinned = app_need > 0 && app_need <= APP_MAX;
        if (app_pinned && (rc = host_reserve(R.h_app, R.ch_app, app_need))) return rc;
        // a host range -> device, through the pinned staging when it fits
        auto h2d_tail = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
            if (app_pinned && app_used + bytes <= R.ch_app) {
                uint8_t* stg = R.h_app + app_used;
                memcpy(stg, src, bytes);
                app_used = (app_used + bytes + 15) & ~(size_t)15;
                async_used = true;
                return hipMemcpyAsync(dst, stg, bytes, hipMemcpyHostToDevice, stream);
            }
            pageable_used = true;
            return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream);
        };
        // filter bytes (slow-path sort): arena + per-node (off, len)
        bool f_full = full_f_dirty;
        if (R.c_foff < nn || R.c_flen < nn) {
            if ((rc = dev_reserve(R.d_foff, R.c_foff, nn))) return rc;
            if ((rc = dev_reserve(R.d_flen, R.c_flen, nn))) return rc;
            f_full = true;
        }
        if (R.c_fbytes < fbytes.size() + 1) {
            if ((rc = dev_reserve(R.d_fbytes, R.c_fbytes, fbytes.size() + 1))) return rc;
            R.fbytes_uploaded = 0;
        }
        if (fbytes.size() > R.fbytes_uploaded) {
            HIP_OK(h2d_tail(R.d_fbytes + R.fbytes_uploaded, fbytes.data() + R.fbytes_uploaded,
                            fbytes.size() - R.fbytes_uploaded));
            R.fbytes_uploaded = fbytes.size();
        }
        if (f_full) {
            pageable_used = true;
            HIP_OK(hipMemcpyAsync(R.d_foff, n_foff.data(), nn * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
            HIP_OK(hipMemcpyAsync(R.d_flen, n_flen.data(), nn * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
        } else if (!dirty_f.empty()) {
            const size_t k = dirty_f.size();
            if ((rc = dev_reserve(R.d_fidx, R.cd_fidx, k))) return rc;
            if ((rc = dev_reserve(R.d_foffv, R.cd_foffv, k))) return rc;
            if ((rc = dev_reserve(R.d_flenv, R.cd_flenv, k))) return rc;
            HIP_OK(hipMemcpyAsync(R.d_fidx, h_fidx, k * 4, hipMemcpyHostToDevice, stream));
            HIP_OK(hipMemcpyAsync(R.d_foffv, h_foffv, k * 8, hipMemcpyHostToDevice, stream));
            HIP_OK(hipMemcpyAsync(R.d_flenv, h_flenv, k * 4, hipMemcpyHostToDevice, stream));
            HIP_OK(launch_scatter_fmeta(R.d_foff, R.d_flen, R.d_fidx, R.d_foffv, R.d_flenv, (uint32_t)k, stream));
            async_used = true;
        }
        if (dev_tok && (rc = sync_dict(R, keys_full, pageable_used, async_used, h2d_tail))) return rc;
        return TM_OK;
    }
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
    int ensure_slow_scratch(tm_batch* b) {
        int rc;
        if (!b->s_waves) {
            // one wave per generic-path topic at a time, latency-bound: a
            // skewed batch (C5: ~28k rows of ~1,000 matches) needs several
            // waves per CU; idle waves exit at once (scratch ~350 KB each)
            uint32_t w = b->n < 65536 ? 64u : std::min<uint32_t>(TM_SLOW_WAVES_MAX, b->n / 32);
            if (const char* v = getenv("TM_SLOW_WAVES")) w = std::max(1, atoi(v));
            b->s_waves = w;
        }
        const size_t q = (size_t)b->s_waves * b->s_qcap, o = (size_t)b->s_waves * b->s_ocap;
        if ((rc = dev_reserve(b->d_sqpar, b->c_sq, q))) return rc;
        if ((rc = dev_reserve(b->d_sqpw, b->c_sq2, q))) return rc;
        if ((rc = dev_reserve(b->d_sqmeta, b->c_sq3, q))) return rc;
        if ((rc = dev_reserve(b->d_sqkey, b->c_sq4, q))) return rc;
        if ((rc = dev_reserve(b->d_sofid, b->c_so, o))) return rc;
        if ((rc = dev_reserve(b->d_sokey, b->c_so2, o))) return rc;
        return TM_OK;
    }

    // ------------------------------------------------------------ batches
    // topic t = bytes[offs[t] .. offs[t+1]); its words go to words[toff[t] ..]
    struct TokView {
        const uint8_t* bytes;
        const uint64_t* offs;
        uint32_t* words;
        const uint32_t* toff;
        uint8_t* tflags;
    };

    void tokenize_range(const TokView& v, uint32_t lo, uint32_t hi, std::vector<uint32_t>& slow_out) const {
        std::vector<TWord> ws;
        for (uint32_t t = lo; t < hi; ++t) {
            const uint8_t* p = v.bytes + v.offs[t];
            const size_t len = v.offs[t + 1] - v.offs[t];
            split_words(p, len, ws);
            uint32_t* out = v.words + v.toff[t];
            bool irregular = false;
            for (size_t i = 0; i < ws.size(); ++i) {
                const TWord& w = ws[i];
                const uint32_t cls = word_class(w, irregular);
                uint32_t id;
                if (w.n == 0) id = W_EMPTY;
                else if (is_plus(w)) id = W_PLUS;
                else if (is_hash(w)) id = W_HASH;
                else id = dict.find(w.p, w.n);
                out[i] = (cls << WID_BITS) | id;
            }
            uint8_t fl = 0;
            if (len > 0 && p[0] == '$') fl |= TF_DOLLAR;
            if (irregular || ws.size() > FAST_MAX_DEPTH) fl |= TF_SLOW;
            v.tflags[t] = fl;
            if (fl & TF_SLOW) slow_out.push_back(t);
        }
    }

    // word offsets (separators + 1 per topic); TM_EOVERFLOW past u32 offsets
    static int count_words(const uint8_t* bytes, const uint64_t* offs, uint32_t n, uint32_t* toff, uint64_t* total) {
        uint64_t acc = 0;
        for (uint32_t t = 0; t < n; ++t) {
            toff[t] = (uint32_t)acc;
            const uint8_t* p = bytes + offs[t];
            const size_t len = offs[t + 1] - offs[t];
            acc += 1 + (uint64_t)std::count(p, p + len, (uint8_t)'/');
            if (acc > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        }
        toff[n] = (uint32_t)acc;
        *total = acc;
        return TM_OK;
    }

    void tokenize_view(const TokView& v, uint32_t n, std::vector<uint32_t>& slow_all) const {
        slow_all.clear();
        const unsigned nt = (n >= 65536) ? threads : 1;
        if (nt <= 1) {
            tokenize_range(v, 0, n, slow_all);
            return;
        }
        std::vector<std::vector<uint32_t>> slow(nt);
        std::vector<std::thread> th;
        for (unsigned i = 0; i < nt; ++i) {
            const uint32_t lo = (uint32_t)((uint64_t)n * i / nt), hi = (uint32_t)((uint64_t)n * (i + 1) / nt);
            th.emplace_back([this, &v, lo, hi, &slow, i] { tokenize_range(v, lo, hi, slow[i]); });
        }
        for (auto& x : th) x.join();
        for (auto& s : slow) slow_all.insert(slow_all.end(), s.begin(), s.end());
    }

    int tokenize(tm_batch* b) {
        const uint32_t n = b->n;
        b->h_toff.resize((size_t)n + 1);
        b->h_tflags.resize(n);
        uint64_t acc = 0;
        int rc = count_words(b->bytes.data(), b->offs.data(), n, b->h_toff.data(), &acc);
        if (rc) return rc;
        b->nwords = acc;
        b->h_words.resize(acc ? acc : 1);
        TokView v{b->bytes.data(), b->offs.data(), b->h_words.data(), b->h_toff.data(), b->h_tflags.data()};
        tokenize_view(v, n, b->h_slow);
        b->dict_size = dict.size();
        return TM_OK;
    }

    // tm_tokenize into caller arrays
    int tokenize_into(const uint8_t* bytes, const uint64_t* offs, uint32_t n, uint32_t* words, uint64_t cap,
                      uint32_t* toff, uint8_t* tflags, uint64_t* nwords) {
        uint64_t acc = 0;
        int rc = count_words(bytes, offs, n, toff, &acc);
        if (rc) return rc;
        *nwords = acc;
        if (acc > cap) return TM_EOVERFLOW;
        std::vector<uint32_t> slow;
        TokView v{bytes, offs, words, toff, tflags};
        tokenize_view(v, n, slow);
        return TM_OK;
    }

    int upload_batch(tm_batch* b) {
        int rc;
        const uint32_t n = b->n;
        if ((rc = dev_reserve(b->d_words, b->c_words, b->h_words.size()))) return rc;
        if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
        if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(b->h_slow.size(), 1)))) return rc;
        const hipStream_t S = st(b);
        HIP_OK(hipMemcpyAsync(b->d_words, b->h_words.data(), b->h_words.size() * 4, hipMemcpyHostToDevice, S));
        HIP_OK(hipMemcpyAsync(b->d_toff, b->h_toff.data(), ((size_t)n + 1) * 4, hipMemcpyHostToDevice, S));
        if (n) HIP_OK(hipMemcpyAsync(b->d_tflags, b->h_tflags.data(), n, hipMemcpyHostToDevice, S));
        if (!b->h_slow.empty())
            HIP_OK(hipMemcpyAsync(b->d_slow, b->h_slow.data(), b->h_slow.size() * 4, hipMemcpyHostToDevice, S));
        b->dev_slow = false;
        return reserve_outputs(b);
    }

    // tm_tokenize_device: the device tokeniser into caller device arrays
    int tokenize_device(const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t* d_words, uint64_t cap,
                        uint32_t* d_toff, uint8_t* d_tflags, uint64_t* nwords) {
        if (reps.empty()) return TM_ENODEV;
        int rc;
        Replica& R = *reps[0];   // the caller's device buffers are on the first replica's device
        const hipStream_t stream = R.stream;
        tm_batch* b = &R.tokb;
        const uint64_t base = offsets[0], nbytes = offsets[n] - base;
        if (nbytes + n + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        if ((rc = sync_device(&R))) return rc;
        if ((rc = dev_reserve(b->d_bytes, b->c_bytes, nbytes + 16))) return rc;
        if ((rc = dev_reserve(b->d_boffs, b->c_boffs, (size_t)n + 1))) return rc;
        if ((rc = dev_reserve(b->d_wcount, b->c_wcount, (size_t)n + 2))) return rc;   // per tile + total
        if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
        if ((rc = dev_reserve(b->d_bsums, b->c_bsums, (size_t)scan_block_count(n) + 1))) return rc;
        if ((rc = host_reserve(b->h_total, b->ch_total, 4))) return rc;
        if (nbytes) HIP_OK(hipMemcpyAsync(b->d_bytes, topics + base, nbytes, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(b->d_boffs, offsets, ((size_t)n + 1) * 8, hipMemcpyHostToDevice, stream));
        if (!n) HIP_OK(hipMemsetAsync(d_toff, 0, 4, stream));
        TokArgs t{};
        t.bytes = b->d_bytes; t.offs = b->d_boffs; t.base = base; t.n = n;
        t.keys = R.d_dkey; t.tails = R.d_tail; t.dict_mask = R.d_dict_n - 1; t.arena = R.d_arena;
        t.wcount = b->d_wcount; t.tflags = d_tflags; t.toff = d_toff; t.words = d_words; t.words_cap = cap;
        t.slow_list = b->d_slow; t.d_nslow = b->d_nslow;
        t.tile_topics = tok_tile_topics(n, nbytes);
        ScanArgs ts{};
        ts.block_sums = b->d_bsums;
        HIP_OK(launch_tokenize(t, ts, b->d_nslow + 1, stream));
        HIP_OK(hipMemcpyAsync(b->h_total, b->d_nslow + 1, 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        *nwords = n ? b->h_total[0] : 0;
        return *nwords > cap ? TM_EOVERFLOW : TM_OK;
    }

    // tm_batch_prepare_tokens: a batch from tokenised arrays (host or device)
    int prepare_tokens(tm_batch* b, const uint32_t* words, const uint32_t* toff, const uint8_t* tflags, uint32_t n,
                       uint64_t nwords, bool on_device) {
        if (nwords > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        const hipStream_t stream = b->rep ? st(b) : nullptr;   // (host-only engine: none)
        b->n = n;
        b->nwords = nwords;
        b->tokens_only = true;
        b->dev_tok = false;
        b->launched = b->done = false;
        b->bytes.clear();
        b->offs.clear();
        int rc;
        if (!on_device) {
            if (toff[0] != 0 || toff[n] != nwords) return TM_EINVAL;
            b->h_slow.clear();
            for (uint32_t t = 0; t < n; ++t) {
                const uint8_t f = tflags[t];
                if (toff[t + 1] < toff[t] || (f & ~(TF_DOLLAR | TF_SLOW))) return TM_EINVAL;
                if (toff[t + 1] - toff[t] > FAST_MAX_DEPTH && !(f & TF_SLOW)) return TM_EINVAL;
                if (f & TF_SLOW) b->h_slow.push_back(t);
            }
            b->h_words.assign(words, words + nwords);
            if (b->h_words.empty()) b->h_words.push_back(0);
            b->h_toff.assign(toff, toff + (size_t)n + 1);
            b->h_tflags.assign(tflags, tflags + n);
            if (device < 0) return TM_OK;
            return upload_batch(b);
        }
        if (device < 0) return TM_ENODEV;
        b->h_words.clear(); b->h_toff.clear(); b->h_tflags.clear(); b->h_slow.clear();
        if ((rc = dev_reserve(b->d_words, b->c_words, std::max<uint64_t>(nwords, 1)))) return rc;
        if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
        if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
        if ((rc = host_reserve(b->h_bad, b->ch_bad, 2))) return rc;
        if (nwords) HIP_OK(hipMemcpyAsync(b->d_words, words, nwords * 4, hipMemcpyDeviceToDevice, stream));
        HIP_OK(hipMemcpyAsync(b->d_toff, toff, ((size_t)n + 1) * 4, hipMemcpyDeviceToDevice, stream));
        if (n) HIP_OK(hipMemcpyAsync(b->d_tflags, tflags, n, hipMemcpyDeviceToDevice, stream));
        HIP_OK(hipMemsetAsync(b->d_nslow, 0, 2 * 4, stream));
        // toff[0] and toff[n] checked with the rest: a walk must never read past words[]
        HIP_OK(launch_token_check(b->d_toff, b->d_tflags, n, nwords, b->d_slow, b->d_nslow, b->d_nslow + 1, stream));
        HIP_OK(hipMemcpyAsync(b->h_bad, b->d_nslow, 2 * 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipStreamSynchronize(stream));
        if (b->h_bad[1] || (n == 0 && nwords != 0)) return TM_EINVAL;
        if (n == 0) {   // no thread checked toff[0] == nwords == 0
            uint32_t t0 = 0;
            HIP_OK(hipMemcpy(&t0, b->d_toff, 4, hipMemcpyDeviceToHost));
            if (t0 != 0) return TM_EINVAL;
        }
        b->dev_slow = true;
        return reserve_outputs(b);
    }

    // A part batch of the in-process sharded group (tm_shard.cpp): token
    // buffers for n topics / nwords words that the group's copies fill on the
    // batch's stream; no staging copy and no host sync (the launch checks the
    // tokens on the device).  The stream and buffers are returned.
    int part_buffers(tm_batch* b, uint32_t n, uint64_t nwords, PartBuffers* out) {
        if (nwords > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        int rc;
        b->n = n;
        b->nwords = nwords;
        b->tokens_only = true;
        b->dev_tok = false;
        b->check_tokens = true;
        b->gbad = true;   // launched directly: the token check belongs to every launch
        b->launched = b->done = false;
        b->bytes.clear(); b->offs.clear();
        b->h_words.clear(); b->h_toff.clear(); b->h_tflags.clear(); b->h_slow.clear();
        if ((rc = dev_reserve(b->d_words, b->c_words, std::max<uint64_t>(nwords, 1)))) return rc;
        if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
        if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
        if ((rc = host_reserve(b->h_bad, b->ch_bad, 2))) return rc;
        b->h_bad[0] = b->h_bad[1] = 0;
        b->dev_slow = true;
        if ((rc = reserve_outputs(b))) return rc;
        out->words = b->d_words;
        out->toff = b->d_toff;
        out->tflags = b->d_tflags;
        out->words_cap = b->c_words;
        out->stream = st(b);
        out->device = b->rep->device;
        return TM_OK;
    }

    // tm_batch_export
    int export_batch(tm_batch* b, uint32_t* d_counts, uint32_t* d_ids, uint32_t mul, uint32_t add) {
        if (!b->done) return TM_EINVAL;
        if (int rc = ensure_dense(b)) return rc;
        const uint64_t top = (uint64_t)(nd.size() ? nd.size() - 1 : 0) * mul + add;
        if (top > 0xFFFFFFFFull) return TM_EOVERFLOW;
        HIP_OK(launch_export(b->d_rowoff, b->d_ids, b->n, b->total, d_counts, d_ids, mul, add, st(b)));
        HIP_OK(hipStreamSynchronize(st(b)));
        return TM_OK;
    }

    // the [ctrl | stats | src | count] block and its pinned mirror, for cap topics
    static int reserve_hdr(tm_batch* b, size_t cap) {
        if (b->d_hdr && b->hdr_cap >= cap) return TM_OK;
        cap = std::max<size_t>(cap + cap / 4, 1024);
        uint8_t *d = nullptr, *h = nullptr;
        HIP_OK(hipMalloc((void**)&d, tm_batch::hdr_bytes(cap)));
        if (hipHostMalloc((void**)&h, tm_batch::hdr_bytes(cap), hipHostMallocDefault) != hipSuccess) {
            (void)hipFree(d);
            snprintf(last_error(), 512, "hipHostMalloc of %zu bytes failed", tm_batch::hdr_bytes(cap));
            return TM_ENOMEM;
        }
        dev_free(b->d_hdr);
        if (b->h_hdr) (void)hipHostFree(b->h_hdr);
        b->d_hdr = d;
        b->h_hdr = h;
        b->hdr_cap = cap;
        const size_t o_stats = CTRL_WORDS * 4, o_src = tm_batch::HDR_FIXED, o_count = o_src + cap * 8;
        b->d_ctrl = (uint32_t*)d; b->h_ctrl = (uint32_t*)h;
        b->d_stats = (unsigned long long*)(d + o_stats); b->h_stats = (unsigned long long*)(h + o_stats);
        b->d_src = (unsigned long long*)(d + o_src); b->h_src = (unsigned long long*)(h + o_src);
        b->d_count = (uint32_t*)(d + o_count); b->h_count = (uint32_t*)(h + o_count);
        return TM_OK;
    }

    int reserve_outputs(tm_batch* b) {
        int rc;
        const uint32_t n = b->n;
        const size_t nn = std::max<size_t>(n, 1);
        if ((rc = reserve_hdr(b, nn))) return rc;
        if ((rc = dev_reserve(b->d_rowoff, b->c_rowoff, nn + 1))) return rc;
        if ((rc = dev_reserve(b->d_bsums, b->c_bsums, (size_t)scan_block_count(n) + 1))) return rc;
        if ((rc = dev_reserve(b->d_ovf, b->c_ovf, nn))) return rc;
        if ((rc = dev_reserve(b->d_total, b->c_total, 1))) return rc;
        if ((rc = reserve_rows(b))) return rc;
        if (!b->ev0) {
            HIP_OK(hipEventCreate(&b->ev0));
            HIP_OK(hipEventCreate(&b->ev1));
            HIP_OK(hipEventCreate(&b->ev2));
            HIP_OK(hipEventCreate(&b->evt));
            HIP_OK(hipEventCreate(&b->evc0));
            HIP_OK(hipEventCreate(&b->evc1));
            HIP_OK(hipEventCreateWithFlags(&b->ev_end, hipEventDisableTiming));
            HIP_OK(hipEventCreate(&b->evq));
        }
        return TM_OK;
    }

    // rows[] = K u64 emission slots per lane of every match wave (reused tile after
    // tile, so it stays cache-resident); sfids[] = sorted rows staged per tile;
    // ids[] = the CSR.  sfids/ids start at 32 per topic and grow on demand.
    int reserve_rows(tm_batch* b) {
        int rc;
        const uint64_t fast =
            std::max<uint64_t>((uint64_t)match_waves(b->n, b->rep->device, qcap) * tile_topics(b->n) * row_cap, 1);
        // + a byte per entry past the rows: the emission-log variant's lanes (TM_EMIT_LOG)
        if ((rc = dev_reserve(b->d_rows, b->c_rows, fast + fast / 8 + 8))) return rc;
        if ((rc = dev_reserve(b->d_sfids, b->c_sfids, std::max<uint64_t>((uint64_t)b->n * 32, staging_min)))) return rc;
        if ((rc = dev_reserve(b->d_ids, b->c_ids, std::max<uint64_t>((uint64_t)b->n * 32, 1u << 16)))) return rc;
        if ((rc = host_reserve(b->h_total, b->ch_total, 4))) return rc;
        return TM_OK;
    }

    // distinct topics of a batch in first-occurrence order; row_of maps publishes to them
    void dedup_topics(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n) {
        std::vector<uint64_t> h(n);
        const unsigned nt = (n >= 65536) ? threads : 1;
        auto hash_range = [&](uint32_t lo, uint32_t hi) {
            for (uint32_t t = lo; t < hi; ++t) h[t] = hash_bytes(topics + offsets[t], offsets[t + 1] - offsets[t]);
        };
        if (nt <= 1) hash_range(0, n);
        else {
            std::vector<std::thread> th;
            for (unsigned i = 0; i < nt; ++i)
                th.emplace_back(hash_range, (uint32_t)((uint64_t)n * i / nt), (uint32_t)((uint64_t)n * (i + 1) / nt));
            for (auto& x : th) x.join();
        }
        size_t cap = 1024;
        while (cap < (size_t)n * 2) cap <<= 1;
        std::vector<uint32_t> tab(cap, 0);          // distinct index + 1
        std::vector<uint32_t> first;                 // publish index of each distinct topic
        b->row_of.resize(n);
        for (uint32_t t = 0; t < n; ++t) {
            const uint8_t* p = topics + offsets[t];
            const size_t len = offsets[t + 1] - offsets[t];
            size_t i = h[t] & (cap - 1);
            for (;;) {
                const uint32_t u = tab[i];
                if (u == 0) {
                    first.push_back(t);
                    tab[i] = (uint32_t)first.size();
                    b->row_of[t] = (uint32_t)first.size() - 1;
                    break;
                }
                const uint32_t f = first[u - 1];
                const size_t fl = offsets[f + 1] - offsets[f];
                if (h[f] == h[t] && fl == len && memcmp(topics + offsets[f], p, len) == 0) {
                    b->row_of[t] = u - 1;
                    break;
                }
                i = (i + 1) & (cap - 1);
            }
        }
        const uint32_t nu = (uint32_t)first.size();
        b->offs.assign((size_t)nu + 1, 0);
        uint64_t tot = 0;
        for (uint32_t u = 0; u < nu; ++u) tot += offsets[first[u] + 1] - offsets[first[u]];
        b->bytes.resize(tot);
        uint64_t o = 0;
        for (uint32_t u = 0; u < nu; ++u) {
            const uint32_t f = first[u];
            const size_t len = offsets[f + 1] - offsets[f];
            if (len) memcpy(b->bytes.data() + o, topics + offsets[f], len);
            o += len;
            b->offs[u + 1] = o;
        }
        b->n = nu;
    }

    // publish names are at most ?MAX_TOPIC_LEN bytes (src/emqx_topic.erl:45,
    // validate/2 :99-100); offsets must not decrease
    static int check_topics(const uint64_t* offsets, uint32_t n) {
        for (uint32_t t = 0; t < n; ++t)
            if (offsets[t + 1] < offsets[t] || offsets[t + 1] - offsets[t] > TM_MAX_TOPIC_LEN) return TM_EINVAL;
        return TM_OK;
    }

    int prepare(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t flags = 0) {
        if (int rc = check_topics(offsets, n)) return rc;
        forget_launch(b);   // its previous results are gone
        b->dedup = (flags & TM_BATCH_DEDUP) != 0;
        b->n_pub = n;
        b->row_of.clear();
        b->dev_tok = false;
        b->dedup_dev = b->dedup_stale = b->rowof_host = false;
        if (device >= 0 && dev_tok) {
            b->launched = b->done = false;
            b->tokens_only = false;
            b->n = n;
            b->bytes.clear();
            b->offs.clear();
            int rc = upload_bytes(b, topics, offsets, n);
            if (rc || !b->dedup) return rc;
            // deduplicated on the device at launch, ahead of the tokeniser
            b->dedup_dev = b->dedup_stale = true;
            return reserve_dedup(b, offsets[n] - offsets[0]);
        }
        if (b->dedup) {
            dedup_topics(b, topics, offsets, n);
        } else {
            b->n = n;
            b->offs.assign(offsets, offsets + (size_t)n + 1);
            const uint64_t base = offsets[0];
            for (auto& o : b->offs) o -= base;
            b->bytes.assign(topics + base, topics + base + b->offs[n]);
        }
        b->launched = b->done = false;
        b->tokens_only = false;
        int rc = tokenize(b);
        if (rc) return rc;
        if (device < 0) return TM_OK;
        return upload_batch(b);
    }

    hipStream_t st(const tm_batch* b) const { return b->own ? b->own : b->rep->stream; }

    // a TM_BATCH_STREAM batch goes away: no longer a reader, stream destroyed
    void drop_user_stream(tm_batch* b) {
        auto& rd = b->rep->readers;
        rd.erase(std::remove(rd.begin(), rd.end(), b), rd.end());
        if (b->own) (void)hipStreamDestroy(b->own);
        b->own = nullptr;
        b->own_user = false;
    }

    // device tokenisation: the caller's bytes and offsets go to HBM now (the
    // caller's buffers are only borrowed for the call); words are produced at launch
    int upload_bytes(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n) {
        int rc;
        const hipStream_t S = st(b);
        const uint64_t base = offsets[0], nbytes = offsets[n] - base;
        if (nbytes + n + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;   // u32 word offsets
        b->tok_base = base;
        if ((rc = dev_reserve(b->d_bytes, b->c_bytes, nbytes + 16))) return rc;   // +16: no tail reads past
        if ((rc = dev_reserve(b->d_boffs, b->c_boffs, (size_t)n + 1))) return rc;
        if ((rc = reserve_tokens(b, n, nbytes))) return rc;
        if (nbytes) HIP_OK(hipMemcpyAsync(b->d_bytes, topics + base, nbytes, hipMemcpyHostToDevice, S));
        HIP_OK(hipMemcpyAsync(b->d_boffs, offsets, ((size_t)n + 1) * 8, hipMemcpyHostToDevice, S));
        // the caller's buffers are only borrowed for the call; tm_match_batch
        // (and the async slots, whose inputs are their own pinned buffers)
        // wait for the whole pipeline later, so they skip this sync
        if (!upload_nosync && !b->own) HIP_OK(hipStreamSynchronize(S));
        b->in_bytes = b->d_bytes;
        b->in_offs = b->d_boffs;
        return tokens_pending(b);
    }

    // the device tokeniser's buffers for n topics of nbytes; words at launch
    int reserve_tokens(tm_batch* b, uint32_t n, uint64_t nbytes) {
        int rc;
        b->nwords = nbytes + n;                  // bound: one word per byte + 1 per topic
        if ((rc = dev_reserve(b->d_wcount, b->c_wcount, (size_t)n + 2))) return rc;   // per tile + total
        if ((rc = dev_reserve(b->d_words, b->c_words, std::max<uint64_t>(b->nwords, 1)))) return rc;
        if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
        if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
        return TM_OK;
    }

    // the device dedup's buffers for b->n publishes of nbytes bytes
    int reserve_dedup(tm_batch* b, uint64_t nbytes) {
        int rc;
        const size_t n = b->n;
        uint64_t cap = 1024;
        while (cap < (uint64_t)n + n / 2) cap <<= 1;   // load <= 2/3 when every publish is distinct
        b->dtab_mask = cap - 1;
        b->dd_bytes = nbytes;
        const size_t nb = scan_block_count((uint32_t)n) + 1;
        if ((rc = dev_reserve(b->d_dtab, b->c_dtab, cap))) return rc;
        if ((rc = dev_reserve(b->d_drep, b->c_drep, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_dlead, b->c_dlead, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_dflag, b->c_dflag, n + 1))) return rc;
        if ((rc = dev_reserve(b->d_dblen, b->c_dblen, n + 1))) return rc;
        if ((rc = dev_reserve(b->d_drbs, b->c_drbs, nb))) return rc;
        if ((rc = dev_reserve(b->d_dbbs, b->c_dbbs, nb))) return rc;
        if ((rc = dev_reserve(b->d_rowof, b->c_rowof, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_cbytes, b->c_cbytes, nbytes + 32))) return rc;   // (the tokeniser's 16-B windows)
        if ((rc = dev_reserve(b->d_coffs, b->c_coffs, n + 1))) return rc;
        if ((rc = dev_reserve(b->d_dd, b->c_dd, 2))) return rc;
        if ((rc = dev_reserve(b->d_pcount, b->c_pcount, std::max<size_t>(n, 1)))) return rc;
        if ((rc = dev_reserve(b->d_psrc, b->c_psrc, std::max<size_t>(n, 1)))) return rc;
        if (!b->evd) {
            HIP_OK(hipEventCreate(&b->evd));
            HIP_OK(hipEventCreate(&b->evx0));
            HIP_OK(hipEventCreate(&b->evx1));
        }
        return TM_OK;
    }

    DedupArgs dedup_args(tm_batch* b) const {
        DedupArgs d{};
        d.bytes = b->in_bytes; d.offs = b->in_offs; d.base = b->tok_base; d.n = b->n_pub;
        d.table = b->d_dtab; d.mask = b->dtab_mask;
        d.rep = b->d_drep; d.lead = b->d_dlead; d.rflag = b->d_dflag; d.blen = b->d_dblen; d.rbs = b->d_drbs; d.bbs = b->d_dbbs;
        d.row_of = b->d_rowof; d.cbytes = b->d_cbytes; d.coffs = b->d_coffs; d.dd = b->d_dd;
        d.ctrl = b->d_ctrl; d.count = b->d_count; d.src = b->d_src; d.pcount = b->d_pcount; d.psrc = b->d_psrc;
        d.stats = b->d_stats;
        d.weak_hash = dedup_weak_hash ? 1u : 0u;
        return d;
    }
    // TM_FRESH_FUSED=1: a fresh batch's tokeniser fill inside the walk (tm_match_fresh).  Measured
    // slower on C2 (fresh 10M batch 5.35 -> 5.64 ms, profiles/r05/fused/): off by default
    const bool fresh_fused = getenv("TM_FRESH_FUSED") && atoi(getenv("TM_FRESH_FUSED")) != 0;
    // TM_DEDUP_WEAK_HASH=1 (tests): the dedup's hash degraded to the topic's length
    const bool dedup_weak_hash = getenv("TM_DEDUP_WEAK_HASH") && atoi(getenv("TM_DEDUP_WEAK_HASH")) != 0;

    // the dedup pass over the batch's resident bytes, ahead of the tokeniser
    int enqueue_dedup(tm_batch* b, hipStream_t S) {
        const DedupArgs d = dedup_args(b);
        HIP_OK(hipMemsetAsync(b->d_dtab, 0, (b->dtab_mask + 1) * 8, S));
        if (!d.n) HIP_OK(hipMemsetAsync(b->d_dd, 0, 8, S));   // (no compact kernel: zero rows)
        ScanArgs rs{}, bs{};
        rs.count = d.rflag; rs.row_off = d.rflag; rs.block_sums = b->d_drbs; rs.n = d.n;   // (in place)
        bs.count = d.blen; bs.row_off = d.blen; bs.block_sums = b->d_dbbs; bs.n = d.n;
        HIP_OK(launch_dedup(d, rs, bs, S));
        return TM_OK;
    }

    int tokens_pending(tm_batch* b) {
        b->h_words.clear(); b->h_toff.clear(); b->h_tflags.clear(); b->h_slow.clear();
        b->dev_tok = true;
        b->tok_dict = ~0ull;
        b->dev_slow = true;
        return reserve_outputs(b);
    }

    // offsets block of a packed batch, padded so the bytes start 16-B aligned
    // (the tokeniser stages tiles with 16-B loads from 16-B aligned windows)
    static size_t packed_head(uint32_t n) { return (((size_t)n + 1) * 8 + 15) & ~(size_t)15; }

    // An async slot's batch: blk = pinned [offs (n+1) u64 from 0 | pad | bytes],
    // one H2D on the slot's stream (topic lengths were checked at submit).
    int upload_packed(tm_batch* b, const uint8_t* blk, uint32_t n, uint64_t nbytes) {
        int rc;
        const size_t head = packed_head(n);
        if (nbytes + n + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;
        b->dedup = false;
        b->n_pub = n;
        b->row_of.clear();
        b->launched = b->done = false;
        b->tokens_only = false;
        b->n = n;
        b->bytes.clear();
        b->offs.clear();
        b->tok_base = 0;
        if ((rc = reserve_tokens(b, n, nbytes))) return rc;
        if ((rc = dev_reserve(b->d_in, b->c_in, head + nbytes + 16))) return rc;   // +16: no tail reads past
        HIP_OK(hipMemcpyAsync(b->d_in, blk, head + nbytes, hipMemcpyHostToDevice, b->own));
        b->in_offs = reinterpret_cast<const uint64_t*>(b->d_in);
        b->in_bytes = b->d_in + head;
        return tokens_pending(b);
    }

    // Enqueues the pipeline on the batch's stream.  csr = false (async slots):
    // stop after the walk -- rows stay in the staging area, described by the
    // per-topic (src, count) of the header block, and the caller enqueues its
    // own read-back; ev2 then marks the end of the walk.
    int launch(tm_batch* b, bool csr = true) {
        if (reps.empty()) return TM_ENODEV;
        int rc;
        Replica& R = *b->rep;
        const hipStream_t S = st(b);
        if (!b->tokens_only && !b->dev_tok && b->dict_size != dict.size()) {   // new words since tokenisation
            if ((rc = tokenize(b))) return rc;
            if ((rc = upload_batch(b))) return rc;
        }
        if (csr) HIP_OK(hipEventRecord(b->evq, S));   // (before the delta upload and the waits below)
        if ((rc = sync_device(&R))) return rc;
        if (b->own && b->seen_upload != R.upload_seq) {   // trie deltas still in flight on the replica stream land first
            HIP_OK(hipStreamWaitEvent(S, R.ev_sync, 0));
            b->seen_upload = R.upload_seq;
        }
        if ((rc = ensure_slow_scratch(b))) return rc;
        if (checked) {
            if ((rc = dev_reserve(R.d_dbg, R.c_dbg, 8))) return rc;
            if ((rc = host_reserve(R.h_dbg, R.ch_dbg, 8))) return rc;
            HIP_OK(hipMemsetAsync(R.d_dbg, 0, 8 * 4, S));
        }
        // A device-deduplicated batch: fresh bytes are deduplicated first, and
        // only the rows are tokenised (again when the dictionary grew) and
        // walked.  The rows are counted on the device, so the tokeniser and
        // the walk are sized for every publish (the bound) and read the count
        // there; wait() sets n to the rows.
        const bool dedup_now = b->dedup_dev && b->dedup_stale;
        const bool tokenize_now = b->dev_tok && (b->tok_dict != dict.size() || dedup_now);
        if (b->dedup_dev) b->n = b->n_pub;
        b->dedup_timed = dedup_now && csr;
        const bool graph = csr && !checked && !tokenize_now && use_graphs && !b->gbad && b->n <= GRAPH_MAX &&
                           !b->dedup_dev;
        if (!tokenize_now && !graph) HIP_OK(hipMemsetAsync(b->d_hdr, 0, tm_batch::HDR_FIXED, S));   // ctrl + stats
        b->tok_timed = tokenize_now && csr;
        if (dedup_now) {
            if (b->dedup_timed) HIP_OK(hipEventRecord(b->evd, S));
            if ((rc = enqueue_dedup(b, S))) return rc;
            b->dedup_stale = false;
            b->rowof_host = false;
        }
        if (b->tok_timed) HIP_OK(hipEventRecord(b->evt, S));
        // a fresh batch's tokeniser fill runs inside the walk (tm_match_fresh)
        const bool fuse = tokenize_now && !checked && !b->dedup_dev && fresh_fused;
        TokArgs t{};
        ScanArgs ts{};
        if (tokenize_now) {
            b->tok_dict = dict.size();
            t.zero = reinterpret_cast<uint32_t*>(b->d_hdr);   // the tokeniser's first kernel clears ctrl + stats
            t.zero_words = tm_batch::HDR_FIXED / 4;
            t.bytes = b->in_bytes; t.offs = b->in_offs; t.base = b->tok_base; t.n = b->n;
            t.keys = R.d_dkey; t.tails = R.d_tail; t.dict_mask = R.d_dict_n - 1; t.arena = R.d_arena;
            t.wcount = b->d_wcount; t.tflags = b->d_tflags; t.toff = b->d_toff; t.words = b->d_words;
            t.words_cap = b->c_words;
            t.slow_list = b->d_slow; t.d_nslow = b->d_nslow;
            t.tile_topics = tok_tile_topics(b->n, b->nwords - b->n);   // nwords = bytes + topics (reserve_tokens)
            t.d_n = nullptr;
            if (b->dedup_dev) {   // the rows' bytes, compacted by the dedup pass
                t.bytes = b->d_cbytes; t.offs = b->d_coffs; t.base = 0; t.d_n = b->d_dd;
            }
            // fused: one tile for both (any tile size is a valid walk tile)
            if (fuse) t.tile_topics = std::min(t.tile_topics, tile_topics(b->n));
            ts.block_sums = b->d_bsums;
            if (!fuse) HIP_OK(launch_tokenize(t, ts, b->d_nslow + 1, S));
        }
        if (b->check_tokens && b->n) {
            HIP_OK(hipMemsetAsync(b->d_nslow, 0, 2 * 4, S));
            HIP_OK(launch_token_check(b->d_toff, b->d_tflags, b->n, b->nwords, b->d_slow, b->d_nslow, b->d_nslow + 1, S));
        }
        MatchArgs a{};
        a.slots = R.d_slots;
        a.nbuckets = nbuckets();
        a.max_probe = max_disp;
        a.root = root_rec();
        a.foff = R.d_foff; a.flen = R.d_flen; a.fbytes = R.d_fbytes;
        a.words = b->d_words; a.toff = b->d_toff; a.tflags = b->d_tflags; a.n = b->n;
        a.slow_list = b->d_slow; a.n_slow = b->dev_slow ? 0u : (uint32_t)b->h_slow.size();
        a.d_nslow = b->dev_slow ? b->d_nslow : nullptr;
        a.d_n = b->dedup_dev ? b->d_dd : nullptr;   // the rows, counted by the dedup pass
        a.count = b->d_count; a.src = b->d_src; a.rows = b->d_rows; a.row_cap = row_cap;
        a.grid = match_waves(b->n, R.device, qcap);
        a.tile_topics = tile_topics(b->n);
        if (fuse) {
            a.tile_topics = t.tile_topics;
            a.grid = (uint32_t)std::min<uint64_t>(((uint64_t)b->n + a.tile_topics - 1) / a.tile_topics,
                                                  match_waves(0xFFFFFFF0u, R.device, qcap));
        }
        a.qcap = qcap;
        {   // the first static_frac of the tiles round-robin, the tail by per-XCD tickets
            const uint64_t ntiles = ((uint64_t)b->n + a.tile_topics - 1) / a.tile_topics;
            a.static_rounds = std::max<uint32_t>(1, (uint32_t)(static_frac * (double)ntiles / std::max(a.grid, 1u)));
        }
        if ((uint64_t)a.grid * a.tile_topics * row_cap > b->c_rows) {
            snprintf(last_error(), 512, "emission rows sized for fewer waves than the launch");
            return TM_EIO;
        }
        a.sfids = b->d_sfids; a.sfids_cap = std::min<uint64_t>(b->c_sfids, MAX_RESULT);
        a.rcap = region_cap(a.sfids_cap, b->one_region);
        a.sgmask = b->one_region ? 0u : TICKET_GROUPS - 1;
        a.xg = b->d_ctrl + XG_WORD;
        a.ctrl = b->d_ctrl; a.ovf_list = b->d_ovf; a.ovf_cap = (uint32_t)std::min<size_t>(b->c_ovf, 0xFFFFFFF0ull);
        a.stats = b->d_stats;
        a.s_qparent = b->d_sqpar; a.s_qpw = b->d_sqpw; a.s_qmeta = b->d_sqmeta; a.s_qkey = b->d_sqkey;
        a.s_ofid = b->d_sofid; a.s_okey = b->d_sokey;
        a.s_qcap = b->s_qcap; a.s_ocap = b->s_ocap; a.s_waves = b->s_waves;
        a.nwords = (uint32_t)std::max<uint64_t>(b->nwords, 1);
        a.nslots = (uint32_t)slots.size();
        a.nnodes = (uint32_t)nd.size();
        a.nfbytes = fbytes.size();
        a.dbg = checked ? R.d_dbg : nullptr;
        ScanArgs s{};
        s.count = b->d_count; s.src = b->d_src;
        s.sfids = b->d_sfids; s.sfids_cap = std::min<uint64_t>(b->c_sfids, MAX_RESULT);
        s.row_off = b->d_rowoff; s.ids = b->d_ids; s.block_sums = b->d_bsums;
        s.n = b->n; s.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull); s.ctrl = b->d_ctrl;
        s.dbg = checked ? R.d_dbg : nullptr;
        b->end_recorded = false;
        b->dense_enq = false;
        int grc = 1;
        if (graph) {
            grc = launch_graph(b, a, s, S);
            if (grc != 1 && grc) return grc;
            if (grc == 1) HIP_OK(hipMemsetAsync(b->d_hdr, 0, tm_batch::HDR_FIXED, S));   // capture refused: the direct way
        }
        if (grc == 1 && fuse) HIP_OK(launch_match_fresh(a, t, ts, b->d_nslow + 1, S, csr ? b->ev0 : nullptr,
                                                        csr ? b->ev1 : nullptr));
        else if (grc == 1) HIP_OK(launch_match(a, S, csr ? b->ev0 : nullptr, csr ? b->ev1 : nullptr, checked));
        if (b->dedup_dev) {   // every publish's row (count, start) + the delivered matches
            HIP_OK(hipEventRecord(b->evx0, S));
            HIP_OK(launch_dedup_expand(dedup_args(b), S));
            HIP_OK(hipEventRecord(b->evx1, S));
        }
        note_launch(b);
        b->launched = true;
        b->done = false;
        b->dense = false;
        b->csr = csr;
        if (!csr) return TM_OK;   // the async slot enqueues its read-back and event
        if (grc == 1) HIP_OK(enqueue_csr(b, s, S));   // (the graph holds it)
        b->scan_args = s;
        if (b->check_tokens) HIP_OK(hipMemcpyAsync(b->h_bad, b->d_nslow, 2 * 4, hipMemcpyDeviceToHost, S));
        if (checked) HIP_OK(hipMemcpyAsync(R.h_dbg, R.d_dbg, 8 * 4, hipMemcpyDeviceToHost, S));
        if (b->oneshot || b->eager_dense) {
            if ((rc = enqueue_dense_tail(b, S))) return rc;
            b->dense_enq = true;
        }
        HIP_OK(hipEventRecord(b->ev_end, S));
        b->end_recorded = true;
        return TM_OK;
    }

    // the read-back of the control words after the walk.  The batch's result is
    // then what the walk left in HBM -- row i = sfids[src[i] .. + count[i]),
    // sorted and deduplicated -- and the dense CSR (scan + finalize copy) is
    // built only for a consumer that asks for offsets (ensure_dense).
    // TM_EAGER_CSR=1 builds it in every launch (round-2 behaviour, for A/B).
    bool eager_csr = getenv("TM_EAGER_CSR") && atoi(getenv("TM_EAGER_CSR")) != 0;
    hipError_t enqueue_csr(tm_batch* b, const ScanArgs& s, hipStream_t S, unsigned ev_flags = 0) {
        hipError_t e;
        if (eager_csr) {
            if ((e = launch_scan(s, S, b->d_total)) != hipSuccess) return e;
            if ((e = launch_finalize(s, S, false)) != hipSuccess) return e;
        }
        if ((e = hipEventRecordWithFlags(b->ev2, S, ev_flags)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(b->h_hdr, b->d_hdr, tm_batch::HDR_FIXED, hipMemcpyDeviceToHost, S)) != hipSuccess)
            return e;   // ctrl + stats
        if (eager_csr) return hipMemcpyAsync(b->h_total, b->d_total, 4, hipMemcpyDeviceToHost, S);
        return hipSuccess;
    }

    // tm_match_batch's tail, enqueued behind the walk: scan + finalize (the
    // dense CSR, ids up to their capacity) and, for a one-shot batch, its copy
    // into mapped host memory.  wait() then finds the whole result on the
    // host; a walk that needed a relaunch, or more ids than fit, takes
    // result()'s (or ensure_dense's) path instead.
    int enqueue_dense_tail(tm_batch* b, hipStream_t S) {
        int rc;
        ScanArgs s = b->scan_args;
        s.ids = b->d_ids;
        s.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull);
        b->dense_cap = s.ids_cap;
        if (!b->oneshot) {   // the dense CSR only (the pipelined tm_match_batch copies it by DMA)
            HIP_OK(hipEventRecord(b->evc0, S));
            HIP_OK(launch_scan(s, S, b->d_total));
            HIP_OK(launch_finalize(s, S, false));
            HIP_OK(hipEventRecord(b->evc1, S));
            return TM_OK;
        }
        if ((rc = host_reserve_coherent(b->h_xrow, b->c_xrow, ((size_t)b->n + 1) * 4))) return rc;
        if ((rc = host_reserve_coherent(b->h_xids, b->c_xids, std::max<size_t>(b->c_ids, 1) * 4))) return rc;
        void *d_row = nullptr, *d_ids = nullptr;
        HIP_OK(hipHostGetDevicePointer(&d_row, b->h_xrow, 0));
        HIP_OK(hipHostGetDevicePointer(&d_ids, b->h_xids, 0));
        b->x_cap = std::min<uint64_t>(s.ids_cap, b->c_xids / 4);
        HIP_OK(hipEventRecord(b->evc0, S));
        HIP_OK(launch_scan(s, S, b->d_total));
        HIP_OK(launch_finalize(s, S, false));
        HIP_OK(hipEventRecord(b->evc1, S));
        HIP_OK(launch_csr_to_host(b->d_rowoff, b->d_ids, b->n, b->d_total, b->x_cap, static_cast<uint32_t*>(d_row),
                                  static_cast<uint32_t*>(d_ids), S));
        return TM_OK;
    }

    // the one-shot result of a waited batch, or 1 when it does not hold
    // (staging relaunch left it stale, or more ids than the copy could hold)
    int oneshot_result(tm_batch* b, tm_result* out) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(b->h_xrow);
        if (!b->oneshot || !b->done || b->total > b->x_cap || row[b->n] != b->total || row[0] != 0) return 1;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, b->evc0, b->evc1);
        b->st.ms_csr = ms;
        b->dense = true;
        out->n_topics = b->n;
        out->n_matches = b->total;
        out->row_offsets = row;
        out->filter_ids = reinterpret_cast<const uint32_t*>(b->h_xids);
        return TM_OK;
    }

    // The dense CSR of a waited batch (row_off[n + 1], ids[total] in topic
    // order) from the walk's rows: exclusive scan of the counts, then one copy
    // of every row from staging (tm_finalize).  Built once per launch, on the
    // batch's stream, for the consumers that index the result by offsets: the
    // host copy (tm_batch_result), routes, fan-out, the sharded export and
    // tm_batch_device_csr.  The per-publish path reads the rows where the walk
    // wrote them and never builds it.
    int ensure_dense(tm_batch* b) {
        if (!b->done) return TM_EINVAL;
        if (b->dense) return TM_OK;
        const hipStream_t S = st(b);
        int rc;
        if (b->total > b->c_ids) {
            if ((rc = dev_reserve(b->d_ids, b->c_ids, (size_t)b->total + b->total / 4))) return rc;
        }
        b->scan_args.ids = b->d_ids;
        b->scan_args.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull);
        HIP_OK(hipEventRecord(b->evc0, S));
        HIP_OK(launch_scan(b->scan_args, S, b->d_total));
        HIP_OK(launch_finalize(b->scan_args, S, checked));
        HIP_OK(hipEventRecord(b->evc1, S));
        HIP_OK(hipMemcpyAsync(b->h_total, b->d_total, 4, hipMemcpyDeviceToHost, S));
        HIP_OK(hipStreamSynchronize(S));
        if (b->h_total[0] != b->total) {
            snprintf(last_error(), 512, "inconsistent CSR: scanned %u entries, kernel count %llu", b->h_total[0],
                     (unsigned long long)b->total);
            return TM_EIO;
        }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, b->evc0, b->evc1);
        b->st.ms_csr = ms;
        b->dense = true;
        return TM_OK;
    }

    // Replays the batch's captured pipeline, capturing it first when its
    // arguments changed (tables moved or grew, the root record, the staging
    // capacity...).  1: capture is unavailable, launch the direct way.
    static constexpr uint32_t GRAPH_MAX = 1u << 20;
    static constexpr uint32_t ONESHOT_MAX = 1u << 20;   // tm_match_batch: one-shot result up to this many topics
    bool use_graphs = true;
    int launch_graph(tm_batch* b, const MatchArgs& a, const ScanArgs& s, hipStream_t S) {
        std::vector<uint8_t> key(sizeof(MatchArgs) + sizeof(ScanArgs));
        memcpy(key.data(), &a, sizeof a);
        memcpy(key.data() + sizeof a, &s, sizeof s);
        if (!b->gexec || b->gkey != key) {
            if (b->gexec) (void)hipGraphExecDestroy(b->gexec);
            b->gexec = nullptr;
            if (b->gkey != key) {   // captured only when a launch repeats the last one's arguments
                b->gkey.swap(key);
                return 1;
            }
            hipGraph_t g = nullptr;
            if (hipStreamBeginCapture(S, hipStreamCaptureModeRelaxed) != hipSuccess) {
                (void)hipGetLastError();
                b->gbad = true;
                return 1;
            }
            hipError_t e = hipMemsetAsync(b->d_hdr, 0, tm_batch::HDR_FIXED, S);
            // timing events as external nodes: every replay re-records them
            if (e == hipSuccess) e = launch_match(a, S, b->ev0, b->ev1, false, hipEventRecordExternal);
            if (e == hipSuccess) e = enqueue_csr(b, s, S, hipEventRecordExternal);
            const hipError_t e2 = hipStreamEndCapture(S, &g);
            if (e != hipSuccess || e2 != hipSuccess || !g ||
                hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0) != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                (void)hipGetLastError();
                b->gexec = nullptr;
                b->gbad = true;
                return 1;
            }
            (void)hipGraphDestroy(g);
            b->gkey.swap(key);
        }
        HIP_OK(hipGraphLaunch(b->gexec, S));
        return TM_OK;
    }

    // control words of a finished launch: TM_EOVERFLOW past the u32 CSR, the
    // retry reasons in *err (0 = clean)
    int check_ctrl(const uint32_t* ctrl, const unsigned long long* stats, uint32_t* err, uint64_t* need,
                   uint64_t* staged_out = nullptr) {
        *err = ctrl[CTRL_ERR];
        uint64_t staged = 0, top = 0;
        for (uint32_t g = 0; g < TICKET_GROUPS; ++g) {
            const uint64_t t = xg_top_read(ctrl, g);
            staged += t;
            top = std::max(top, t);
        }
        *need = top * TICKET_GROUPS;   // staging capacity that holds every region's reservation
        if (staged_out) *staged_out = staged;
        const uint64_t nmatch = stats[ST_MATCHES];
        // a CSR with u32 offsets cannot hold more (tm_result): refuse, never wrap
        if ((*err & ERR_CSR_RANGE) || staged > result_limit || nmatch > result_limit) {
            snprintf(last_error(), 512, "batch result too large: %llu staged / %llu matched > limit %llu",
                     (unsigned long long)staged, (unsigned long long)nmatch, (unsigned long long)result_limit);
            return TM_EOVERFLOW;
        }
        return TM_OK;
    }

    // capacity misses of the last launch: grow what overflowed (the caller relaunches)
    int grow_for(tm_batch* b, uint32_t err, uint64_t need, uint64_t staged) {
        if (err & ERR_STAGING) {
            // per-group regions of the largest group's size: unless that exceeds
            // the limit while the batch as a whole fits (skew concentrated in one
            // walk group) -- then one region for all groups, sized by the total
            const uint64_t limit = std::min<uint64_t>(MAX_RESULT, result_limit + 1024);
            if (!b->one_region && need + need / 4 + 1024 > limit && staged <= result_limit) b->one_region = true;
            if (b->one_region) need = staged;
            int rc = dev_reserve(b->d_sfids, b->c_sfids, std::min<uint64_t>(need + need / 4 + 1024, limit));
            if (rc) return rc;
        }
        if (err & ERR_SLOW_SCRATCH) {
            b->s_qcap *= 4;
            b->s_ocap *= 4;
        }
        return TM_OK;
    }

    void fill_stats(tm_batch* b) {
        float ms_match = 0, ms_total = 0, ms_tok = 0, ms_dd = 0, ms_x = 0;
        (void)hipEventElapsedTime(&ms_match, b->ev0, b->ev1);
        (void)hipEventElapsedTime(&ms_total, b->ev0, b->ev2);
        if (b->tok_timed) (void)hipEventElapsedTime(&ms_tok, b->evt, b->ev0);
        if (b->dedup_timed) (void)hipEventElapsedTime(&ms_dd, b->evd, b->tok_timed ? b->evt : b->ev0);
        if (b->dedup_dev) (void)hipEventElapsedTime(&ms_x, b->evx0, b->evx1);
        b->st.ms_tokenize = ms_tok;
        b->st.ms_dedup = ms_dd;
        b->st.ms_expand = ms_x;
        b->st.publishes = b->dedup ? b->n_pub : b->n;
        float ms_q = 0;
        (void)hipEventElapsedTime(&ms_q, b->evq, b->dedup_timed ? b->evd : b->tok_timed ? b->evt : b->ev0);
        b->st.ms_queue = ms_q;
        b->st.ms_csr = 0;   // set by ensure_dense
        b->st.topics = b->n;
        b->st.visits = b->h_stats[ST_VISITS];
        b->st.hash_hits = b->h_stats[ST_HASH];
        b->st.words = b->h_stats[ST_WORDS];
        b->st.matches = b->h_stats[ST_MATCHES];
        b->st.slow_topics = b->h_stats[ST_SLOW];
        b->st.probes = b->h_stats[ST_PROBES];
        b->st.iterations = b->h_stats[ST_ITERS];
        b->st.overflow_tiles = b->h_ctrl[CTRL_NOVF];
        b->st.ms_match = ms_match;
        b->st.ms_total = ms_total;
        b->total = b->st.matches;
        b->st.delivered = b->dedup_dev ? b->h_stats[ST_DELIVERED] : b->st.matches;
    }

    // drained: the caller has already waited for the batch's stream (the
    // sharded group joins all its streams in one host wait), so the first
    // check needs no sync; *relaunched counts capacity-miss relaunches
    int wait(tm_batch* b, bool drained = false, uint32_t* relaunched = nullptr) {
        if (!b->launched) return TM_EINVAL;
        const hipStream_t S = st(b);
        if (!b->csr) {   // an async launch stopped after the walk: redo it the CSR way
            int rc = launch(b, true);
            if (rc) return rc;
            drained = false;
        }
        for (int attempt = 0;; ++attempt) {
            if (!drained || attempt) {
                static const bool wtrace = getenv("TM_WAIT_TRACE") != nullptr;
                const auto w0 = std::chrono::steady_clock::now();
                const bool was_done = b->end_recorded && hipEventQuery(b->ev_end) == hipSuccess;
                if (b->end_recorded) HIP_OK(hipEventSynchronize(b->ev_end));
                else HIP_OK(hipStreamSynchronize(S));
                if (wtrace)
                    fprintf(stderr, "[wait] done before: %d, sync %.1f us\n", (int)was_done,
                            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count());
            }
            if (attempt && relaunched) ++*relaunched;
            if (b->dedup_dev) {   // the walk's rows: the distinct publishes counted by the dedup pass
                b->n = b->h_ctrl[CTRL_NROWS];
                b->scan_args.n = b->n;
            }
            if (b->check_tokens && b->n && b->h_bad[1]) {
                snprintf(last_error(), 512, "token batch failed the device check (word offsets or flags)");
                return TM_EINVAL;
            }
            const uint32_t* h_dbg = b->rep->h_dbg;
            if (checked && h_dbg[0]) {
                snprintf(last_error(), 512, "bounds check %u failed: index %u bound %u (count %u, extra %u)",
                         h_dbg[0], h_dbg[1], h_dbg[2], h_dbg[3], h_dbg[4]);
                return TM_EIO;
            }
            uint32_t err;
            uint64_t need, staged;
            int rc = check_ctrl(b->h_ctrl, b->h_stats, &err, &need, &staged);
            if (rc) return rc;
            if (!err) break;
            if (attempt >= 6) {
                snprintf(last_error(), 512, "capacity misses did not settle after %d relaunches (err %#x, %llu staged)",
                         attempt, err, (unsigned long long)staged);
                return TM_EOVERFLOW;
            }
            if ((rc = grow_for(b, err, need, staged))) return rc;
            if ((rc = launch(b))) return rc;
        }
        // eager CSR (TM_EAGER_CSR): the finalize pass is rerun alone when ids[] was too small
        if (eager_csr && b->h_total[0] > b->c_ids) {
            int rc = dev_reserve(b->d_ids, b->c_ids, (size_t)b->h_total[0] + b->h_total[0] / 4);
            if (rc) return rc;
            b->scan_args.ids = b->d_ids;
            b->scan_args.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull);
            // scan + finalize again (finalize turns the block-local offsets into global ones)
            HIP_OK(launch_scan(b->scan_args, S, b->d_total));
            HIP_OK(launch_finalize(b->scan_args, S, checked));
            HIP_OK(hipEventRecord(b->ev2, S));
            HIP_OK(hipStreamSynchronize(S));
        }
        fill_stats(b);
        b->done = true;
        // (dense_enq, not eager_dense: the pipelined caller clears eager_dense
        // right after launch, while the tail it asked for is already queued)
        b->dense = eager_csr || (b->dense_enq && !b->oneshot && b->total <= b->dense_cap);
        if (b->dense && !eager_csr) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, b->evc0, b->evc1);
            b->st.ms_csr = ms;
        }
        return TM_OK;
    }

    int result(tm_batch* b, tm_result* out) {
        if (!b->done) return TM_EINVAL;
        int rc;
        if ((rc = ensure_dense(b))) return rc;
        const hipStream_t S = st(b);
        // the match count is known since wait(): both copies go out behind one sync
        const uint64_t total = b->total;
        if (total > b->c_ids) {
            snprintf(last_error(), 512, "inconsistent CSR: kernel count %llu, capacity %zu",
                     (unsigned long long)total, b->c_ids);
            return TM_EIO;
        }
        if ((rc = host_reserve(b->h_rowoff, b->ch_rowoff, (size_t)b->n + 1))) return rc;
        if ((rc = host_reserve(b->h_ids, b->ch_ids, std::max<uint64_t>(total, 1)))) return rc;
        HIP_OK(hipMemcpyAsync(b->h_rowoff, b->d_rowoff, ((size_t)b->n + 1) * 4, hipMemcpyDeviceToHost, S));
        if (total) HIP_OK(hipMemcpyAsync(b->h_ids, b->d_ids, total * 4, hipMemcpyDeviceToHost, S));
        HIP_OK(hipStreamSynchronize(S));
        if (b->h_rowoff[b->n] != total) {
            snprintf(last_error(), 512, "inconsistent CSR: row offsets end at %u, kernel count %llu",
                     b->h_rowoff[b->n], (unsigned long long)total);
            return TM_EIO;
        }
        out->n_topics = b->n;
        out->n_matches = total;
        out->row_offsets = b->h_rowoff;
        out->filter_ids = b->h_ids;
        return TM_OK;
    }


    // tm_batch_sample: rows rows[0..k) of a waited batch as a host CSR, gathered
    // on the device from where the walk wrote them (two small kernels and two
    // small copies: count + start of each sampled row, then its ids).
    int sample(tm_batch* b, const uint32_t* rows, uint32_t k, tm_result* out) {
        if (!b->done || !b->csr) return TM_EINVAL;
        for (uint32_t i = 0; i < k; ++i)
            if (rows[i] >= b->n) return TM_EINVAL;
        const hipStream_t S = st(b);
        b->h_smp_off.assign((size_t)k + 1, 0);
        b->h_smp_ids.clear();
        if (k) {
            struct Scratch {
                void* p = nullptr;
                ~Scratch() { if (p) (void)hipFree(p); }
            } meta, ids;
            // [rows u32 k | cnt u32 k | pad | src u64 k | off u64 k + 1]
            const size_t o_src = (((size_t)k * 8) + 15) & ~(size_t)15, o_off = o_src + (size_t)k * 8;
            HIP_OK(hipMalloc(&meta.p, o_off + ((size_t)k + 1) * 8));
            uint8_t* m = static_cast<uint8_t*>(meta.p);
            uint32_t* d_rows = reinterpret_cast<uint32_t*>(m);
            uint32_t* d_cnt = d_rows + k;
            unsigned long long* d_src = reinterpret_cast<unsigned long long*>(m + o_src);
            uint64_t* d_off = reinterpret_cast<uint64_t*>(m + o_off);
            std::vector<uint32_t> cnt(k);
            HIP_OK(hipMemcpyAsync(d_rows, rows, (size_t)k * 4, hipMemcpyHostToDevice, S));
            HIP_OK(launch_sample_meta(b->d_count, b->d_src, d_rows, k, d_cnt, d_src, S));
            HIP_OK(hipMemcpyAsync(cnt.data(), d_cnt, (size_t)k * 4, hipMemcpyDeviceToHost, S));
            HIP_OK(hipStreamSynchronize(S));
            std::vector<uint64_t> off((size_t)k + 1, 0);
            for (uint32_t i = 0; i < k; ++i) off[i + 1] = off[i] + cnt[i];
            if (off[k] > MAX_RESULT) return TM_EOVERFLOW;   // u32 CSR offsets
            for (uint32_t i = 0; i <= k; ++i) b->h_smp_off[i] = (uint32_t)off[i];
            b->h_smp_ids.resize(off[k]);
            if (off[k]) {
                HIP_OK(hipMalloc(&ids.p, off[k] * 4));
                HIP_OK(hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, S));
                HIP_OK(launch_sample_ids(b->d_sfids, d_cnt, d_src, d_off, k, static_cast<uint32_t*>(ids.p), S));
                HIP_OK(hipMemcpyAsync(b->h_smp_ids.data(), ids.p, off[k] * 4, hipMemcpyDeviceToHost, S));
                HIP_OK(hipStreamSynchronize(S));
            }
        }
        if (b->h_smp_ids.empty()) b->h_smp_ids.push_back(0);   // (a valid pointer for an empty result)
        out->n_topics = k;
        out->n_matches = b->h_smp_off[k];
        out->row_offsets = b->h_smp_off.data();
        out->filter_ids = b->h_smp_ids.data();
        return TM_OK;
    }

    // ------------------------------------------------------------ async pipeline
    // Every replica runs a pipeline of its own (slots, launcher, completers);
    // tm_match_async deals the calls over them.  Slots are created on first
    // use or by tm_async_start (under R.amu; takes mu).
    int async_start(Replica& R) {
        if (R.a_started) return TM_OK;
        if (reps.empty()) return TM_ENODEV;
        if (const char* d = getenv("TM_ASYNC_DEPTH")) R.a_depth = (uint32_t)std::min(16, std::max(1, atoi(d)));
        if (const char* d = getenv("TM_ASYNC_BUSY_MIN")) R.a_busy_min = (uint32_t)std::max(1, atoi(d));
        if (const char* d = getenv("TM_ASYNC_COMPLETERS")) R.a_ncompleters = (uint32_t)std::min(8, std::max(1, atoi(d)));
        if (const char* d = getenv("TM_ASYNC_SPIN_US")) R.a_spin_us = (uint32_t)std::min(10000, std::max(0, atoi(d)));
        if (const char* d = getenv("TM_ASYNC_INLINE")) R.a_inline = atoi(d) != 0;
        {
            std::lock_guard<std::recursive_mutex> g(mu);
            HIP_OK(hipSetDevice(R.device));
            for (uint32_t i = 0; i < R.a_depth; ++i) {
                AsyncSlot* sl = new AsyncSlot();
                R.a_slots.push_back(sl);
                sl->b.rep = &R;
                HIP_OK(hipStreamCreateWithFlags(&sl->b.own, hipStreamNonBlocking));
                HIP_OK(hipEventCreateWithFlags(&sl->ev_done, hipEventDisableTiming));
                R.a_free.push_back(sl);
                R.readers.push_back(&sl->b);
            }
        }
        R.a_stop = false;
        R.a_launcher_done = false;
        R.a_launcher = std::thread([this, &R] { launcher_loop(R); });
        for (uint32_t i = 0; i < R.a_ncompleters; ++i) R.a_completers.emplace_back([this, &R] { completer_loop(R); });
        R.a_started = true;
        R.a_live.store(true, std::memory_order_release);
        return TM_OK;
    }

    void async_stop(Replica& R) {
        {
            std::lock_guard<std::mutex> lk(R.amu);
            if (!R.a_started && R.a_slots.empty()) return;
            R.a_stop = true;
            R.a_live.store(false, std::memory_order_release);
        }
        R.a_work.notify_all();
        R.a_done.notify_all();
        if (R.a_launcher.joinable()) R.a_launcher.join();
        for (auto& t : R.a_completers)
            if (t.joinable()) t.join();
        R.a_completers.clear();
        std::lock_guard<std::recursive_mutex> g(mu);
        (void)hipSetDevice(R.device);
        for (AsyncSlot* sl : R.a_slots) {
            if (sl->b.own) (void)hipStreamSynchronize(sl->b.own);
            forget_launch(&sl->b);
            sl->b.release();
            if (sl->b.own) (void)hipStreamDestroy(sl->b.own);
            if (sl->ev_done) (void)hipEventDestroy(sl->ev_done);
            if (sl->h_in) (void)hipHostFree(sl->h_in);
            if (sl->h_rows) (void)hipHostFree(sl->h_rows);
            if (sl->h_out) (void)hipHostFree(sl->h_out);
            if (sl->h_flag) (void)hipHostFree(sl->h_flag);
            delete sl;
        }
        R.a_slots.clear();
        R.a_free.clear();
        R.readers.erase(std::remove_if(R.readers.begin(), R.readers.end(), [](tm_batch* r) { return !r->own_user; }),
                        R.readers.end());
        R.a_started = false;
    }

    // Deals calls over the replicas: a submitting thread goes round-robin,
    // starting from a replica of its own, so a few busy submitters spread
    // evenly and each replica's batches still form from whole queue shards.
    int match_async(const uint8_t* t, size_t len, tm_match_cb cb, void* ctx) {
        if (reps.empty()) return TM_ENODEV;
        static std::atomic<uint32_t> next_sub{0};
        static thread_local uint32_t my_sub = next_sub.fetch_add(1);
        static thread_local uint32_t my_calls = 0;
        Replica& R = *reps[(my_sub + my_calls++) % reps.size()];
        return match_async(R, t, len, cb, ctx);
    }

    int match_async(Replica& R, const uint8_t* t, size_t len, tm_match_cb cb, void* ctx) {
        if (!R.a_live.load(std::memory_order_acquire)) {
            std::lock_guard<std::mutex> lk(R.amu);
            if (R.a_stop) return TM_ENODEV;
            if (!R.a_started) {
                int rc = async_start(R);
                if (rc) return rc;
            }
        }
        static std::atomic<uint32_t> next_shard{0};
        static thread_local uint32_t my_shard = next_shard.fetch_add(1) % Replica::QSHARDS;
        Replica::QShard& sh = R.qs[my_shard];
        {
            std::lock_guard<std::mutex> g(sh.mu);
            if (len) sh.bytes.insert(sh.bytes.end(), t, t + len);
            sh.lens.push_back((uint32_t)len);
            sh.calls.push_back(AsyncCall{cb, ctx});
        }
        const uint64_t q = R.q_count.fetch_add(1, std::memory_order_acq_rel) + 1;
        if (q == 1 && R.a_inline) {   // the queue was empty: launch it here if the pipeline is idle
            std::unique_lock<std::mutex> lk(R.amu, std::try_to_lock);
            if (lk.owns_lock() && R.a_started && !R.a_stop && !R.a_free.empty() &&
                R.a_free.size() == R.a_slots.size() && R.q_count.load(std::memory_order_acquire) > 0) {
                ++R.a_inline_launches;
                launch_locked(R, lk);
                return TM_OK;
            }
        }
        if (q == 1 || q == R.a_busy_min || q == R.a_max) {   // the launcher may be waiting for this
            std::lock_guard<std::mutex> lk(R.amu);
            R.a_work.notify_one();
        }
        return TM_OK;
    }

    // moves exactly `take` queued calls into the slot: the caller reserved
    // them (took them off q_count under amu), and a call is in its shard before
    // it is counted, so at least that many are there beyond other drainers'
    // reservations -- passes repeat until all are found
    void drain_queue(Replica& R, AsyncSlot* sl, size_t take) {
        constexpr uint32_t QSHARDS = Replica::QSHARDS;
        sl->calls.clear();
        sl->bytes.clear();
        sl->offs.assign(1, 0);
        static thread_local uint32_t start = 0;
        for (uint32_t k = 0; sl->calls.size() < take; ++k) {
            if (k && k % QSHARDS == 0) std::this_thread::yield();   // another drainer is mid-shard

            Replica::QShard& sh = R.qs[(start + k) % QSHARDS];
            std::lock_guard<std::mutex> g(sh.mu);
            size_t h = sh.head, hb = sh.head_bytes;
            while (h < sh.calls.size() && sl->calls.size() < take) {
                const uint32_t len = sh.lens[h];
                sl->calls.push_back(sh.calls[h]);
                sl->bytes.insert(sl->bytes.end(), sh.bytes.begin() + (long)hb, sh.bytes.begin() + (long)(hb + len));
                sl->offs.push_back(sl->bytes.size());
                hb += len;
                ++h;
            }
            if (h == sh.calls.size()) {   // shard emptied: reset, keep the capacity
                sh.calls.clear();
                sh.lens.clear();
                sh.bytes.clear();
                sh.head = sh.head_bytes = 0;
            } else {
                sh.head = h;
                sh.head_bytes = hb;
            }
        }
        start = (start + 1) % QSHARDS;   // no shard is always last
    }

    // amu held (lk): a free slot takes up to a_max queued calls and is
    // launched; amu is released while the batch is built and launched
    void launch_locked(Replica& R, std::unique_lock<std::mutex>& lk) {
        AsyncSlot* sl = R.a_free.back();
        R.a_free.pop_back();
        const size_t take =
            std::min<uint64_t>(R.q_count.load(std::memory_order_acquire), std::max<uint32_t>(R.a_max, 1));
        R.q_count.fetch_sub(take, std::memory_order_acq_rel);   // reserved: no other drainer counts on them
        lk.unlock();
        drain_queue(R, sl, take);
        const auto t0 = std::chrono::steady_clock::now();
        try {
            sl->rc = slot_launch(sl);
        } catch (...) {
            sl->rc = TM_ENOMEM;
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        lk.lock();
        R.a_max_seen = std::max<uint64_t>(R.a_max_seen, sl->calls.size());
        R.a_us_launch += us;
        R.a_inflight.push_back(sl);
        R.a_done.notify_all();
    }

    // Forms batches from the queue: everything queued while the pipeline was
    // busy (up to R.a_max), optionally after a linger, on the next free slot.
    void launcher_loop(Replica& R) {
        (void)hipSetDevice(R.device);
        std::unique_lock<std::mutex> lk(R.amu);
        auto queued = [&] { return R.q_count.load(std::memory_order_acquire); };
        for (;;) {
            R.a_work.wait(lk, [&] {
                if (R.a_stop) return queued() == 0 || !R.a_free.empty();
                return queued() && !R.a_free.empty();
            });
            if (queued() == 0) {
                if (R.a_stop) break;   // stopping, queue drained
                continue;              // an inline launch took the calls
            }
            if (!R.a_stop && R.a_free.size() != R.a_slots.size() && queued() < R.a_busy_min) {
                // batches in flight, few calls queued: gather more for a while
                auto enough = [&] {
                    return R.a_stop || R.a_free.size() == R.a_slots.size() || queued() >= R.a_busy_min;
                };
                R.a_work.wait(lk, enough);
                if (R.a_free.empty() || queued() == 0) continue;
            }
            if (R.a_linger_us && !R.a_stop && queued() < R.a_max)
                R.a_work.wait_for(lk, std::chrono::microseconds(R.a_linger_us),
                                  [&] { return R.a_stop || queued() >= R.a_max; });
            if (R.a_free.empty() || queued() == 0) continue;
            launch_locked(R, lk);
        }
        R.a_launcher_done = true;
        R.a_done.notify_all();
    }

    // H2D of the slot's topics (one copy), device tokeniser, walk, and one
    // kernel writing the per-topic (src, count) and the staged rows into the
    // slot's pinned buffers -- all on the slot's stream; ev_done marks the end.
    int slot_launch(AsyncSlot* sl) {
        const uint32_t n = (uint32_t)sl->calls.size();
        const size_t nb = sl->bytes.size(), head = packed_head(n);
        int rc;
        if ((rc = host_reserve(sl->h_in, sl->c_in, head + nb))) return rc;
        memcpy(sl->h_in, sl->offs.data(), ((size_t)n + 1) * 8);
        if (nb) memcpy(sl->h_in + head, sl->bytes.data(), nb);
        std::lock_guard<std::recursive_mutex> g(mu);
        HIP_OK(hipSetDevice(sl->b.rep->device));
        tm_batch* b = &sl->b;
        const hipStream_t S = b->own;
        rc = dev_tok ? upload_packed(b, sl->h_in, n, nb)
                     : prepare(b, sl->h_in + head, reinterpret_cast<const uint64_t*>(sl->h_in), n);
        if (rc) return rc;
        if ((rc = launch(b, false))) return rc;
        const size_t hdr_bytes = tm_batch::HDR_FIXED + (size_t)n * 8;
        if ((rc = host_reserve_coherent(sl->h_out, sl->c_out, hdr_bytes + (size_t)n * 4 + 8))) return rc;
        uint8_t* rows8 = reinterpret_cast<uint8_t*>(sl->h_rows);
        if ((rc = host_reserve_coherent(rows8, sl->c_rows, std::max<size_t>(b->c_sfids, 1) * 4))) return rc;
        sl->h_rows = reinterpret_cast<uint32_t*>(rows8);
        void *d_out = nullptr, *d_rows = nullptr;
        HIP_OK(hipHostGetDevicePointer(&d_out, sl->h_out, 0));
        HIP_OK(hipHostGetDevicePointer(&d_rows, sl->h_rows, 0));
        ExportArgs x{};
        x.hdr = reinterpret_cast<const uint32_t*>(b->d_hdr);
        x.hdr_words = hdr_bytes / 4;
        x.h_hdr = reinterpret_cast<uint32_t*>(d_out);
        x.count = b->d_count;
        x.h_count = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_out) + hdr_bytes);
        x.n = n;
        x.rows = b->d_sfids;
        x.h_rows = reinterpret_cast<uint32_t*>(d_rows);
        x.rows_cap = std::min<uint64_t>(b->c_sfids, sl->c_rows / 4);
        x.rcap = region_cap(std::min<uint64_t>(b->c_sfids, MAX_RESULT), b->one_region);
        HIP_OK(launch_export_host(x, S));
        if (b->rep->a_spin_us) {
            if (!sl->h_flag) {
                HIP_OK(hipHostMalloc((void**)&sl->h_flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
                *sl->h_flag = 0;
                HIP_OK(hipHostGetDevicePointer((void**)&sl->d_flag, sl->h_flag, 0));
            }
            HIP_OK(hipStreamWriteValue32(S, sl->d_flag, ++sl->seq, 0));
        }
        HIP_OK(hipEventRecord(sl->ev_done, S));
        return TM_OK;
    }

    // Completers: the oldest in-flight slot nobody waits for is claimed by
    // one completer, which waits for it and checks its control words; then
    // every idle completer takes chunks of its calls to deliver (the last
    // chunk's completer recycles the slot).  A failed or recovered batch is
    // delivered whole by the completer that waited for it.
    void completer_loop(Replica& R) {
        (void)hipSetDevice(R.device);
        std::unique_lock<std::mutex> lk(R.amu);
        for (;;) {
            AsyncSlot* sl = nullptr;
            bool head = false;
            R.a_done.wait(lk, [&] {
                for (AsyncSlot* x : R.a_inflight)
                    if (x->ready && x->next_chunk < x->nchunks) {
                        sl = x;
                        return true;
                    }
                for (AsyncSlot* x : R.a_inflight)
                    if (!x->claimed) {
                        sl = x;
                        head = true;
                        return true;
                    }
                return R.a_launcher_done && R.a_inflight.empty();
            });
            if (!sl) break;
            if (head) {
                sl->claimed = true;
                lk.unlock();
                bool whole = true, recovered = false;
                double us_wait = 0;
                try {
                    whole = slot_wait(sl, us_wait, recovered);
                } catch (...) {
                }
                lk.lock();
                R.a_us_wait += us_wait;
                R.a_recoveries += recovered ? 1 : 0;
                if (whole) {
                    slot_finish(R, sl);
                } else {
                    sl->nchunks = std::max<uint32_t>(
                        1, (uint32_t)((sl->calls.size() + AsyncSlot::DELIVER_CHUNK - 1) / AsyncSlot::DELIVER_CHUNK));
                    sl->next_chunk = sl->chunks_done = 0;
                    sl->ready = true;
                    R.a_done.notify_all();
                }
                continue;
            }
            const uint32_t c = sl->next_chunk++;
            lk.unlock();
            const auto t0 = std::chrono::steady_clock::now();
            const uint32_t n = (uint32_t)sl->calls.size();
            const uint32_t lo = std::min(n, c * AsyncSlot::DELIVER_CHUNK);
            const uint32_t hi = std::min(n, lo + AsyncSlot::DELIVER_CHUNK);
            syncwake::in_batch = true;
            for (uint32_t i = lo; i < hi; ++i) {
                const uint32_t k = sl->d_count[i];
                sl->calls[i].cb(sl->calls[i].ctx, TM_OK, k ? sl->h_rows + sl->d_src[i] : sl->h_rows, k);
            }
            syncwake::in_batch = false;
            syncwake::flush();
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            lk.lock();
            R.a_us_deliver += us;
            if (++sl->chunks_done == sl->nchunks) slot_finish(R, sl);
        }
    }

    // amu held: the slot's calls are all delivered -- back to the free list
    void slot_finish(Replica& R, AsyncSlot* sl) {
        R.a_inflight.erase(std::find(R.a_inflight.begin(), R.a_inflight.end(), sl));
        ++R.a_batches;
        R.a_requests += sl->calls.size();
        sl->calls.clear();
        sl->claimed = sl->ready = false;
        sl->nchunks = sl->next_chunk = sl->chunks_done = 0;
        R.a_free.push_back(sl);
        R.a_work.notify_all();
        R.a_done.notify_all();
    }

    // Waits for a launched slot and checks its control words.  false: its
    // rows are ready for chunked delivery (d_count / d_src set); true: it was
    // delivered whole here (a launch failure, an error, or a capacity miss
    // re-run through the CSR path: *recovered).
    bool slot_wait(AsyncSlot* sl, double& us_wait, bool& recovered) {
        tm_batch* b = &sl->b;
        const uint32_t n = (uint32_t)sl->calls.size();
        auto fail_all = [&](int rc) {
            syncwake::in_batch = true;
            for (const AsyncCall& c : sl->calls) c.cb(c.ctx, rc, nullptr, 0);
            syncwake::in_batch = false;
            syncwake::flush();
        };
        if (sl->rc) {
            (void)hipStreamSynchronize(b->own);   // whatever was enqueued before the failure
            fail_all(sl->rc);
            return true;
        }
        const auto tw = std::chrono::steady_clock::now();
        if (sl->h_flag && b->rep->a_spin_us) {   // poll the pinned flag first (no interrupt wake-up)
            const volatile uint32_t* f = sl->h_flag;
            const auto lim = tw + std::chrono::microseconds(b->rep->a_spin_us);
            for (uint32_t it = 0; *f != sl->seq; ++it) {
                __builtin_ia32_pause();
                if ((it & 255) == 0 && std::chrono::steady_clock::now() > lim) break;
            }
            // the flag follows the export in stream order; the event right after it
            if (*f == sl->seq)
                while (hipEventQuery(sl->ev_done) == hipErrorNotReady && std::chrono::steady_clock::now() < lim)
                    __builtin_ia32_pause();
        }
        if (hipEventSynchronize(sl->ev_done) != hipSuccess) {
            fail_all(TM_EIO);
            return true;
        }
        us_wait = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw).count();
        const size_t hdr_bytes = tm_batch::HDR_FIXED + (size_t)n * 8;
        const uint32_t* ctrl = reinterpret_cast<const uint32_t*>(sl->h_out);
        const unsigned long long* stats = reinterpret_cast<const unsigned long long*>(sl->h_out + CTRL_WORDS * 4);
        uint32_t err = 0;
        uint64_t need = 0, staged = 0;
        int rc = check_ctrl(ctrl, stats, &err, &need, &staged);
        if (rc) {
            fail_all(rc);
            return true;
        }
        if (b->one_region) need = staged;
        if (!err && need > sl->c_rows / 4) err = ERR_STAGING;   // (cannot happen: rows hold the staging area)
        if (err) {
            // capacity miss (staging, generic-path scratch): the CSR path grows
            // and re-runs, then the rows come from the CSR
            recovered = true;
            tm_result r{};
            {
                std::lock_guard<std::recursive_mutex> g(mu);
                (void)hipSetDevice(b->rep->device);
                rc = grow_for(b, err, need, staged);
                if (!rc) rc = wait(b);
                if (!rc) rc = result(b, &r);
            }
            if (rc) {
                fail_all(rc);
                return true;
            }
            syncwake::in_batch = true;
            for (uint32_t i = 0; i < n; ++i)
                sl->calls[i].cb(sl->calls[i].ctx, TM_OK, r.filter_ids + r.row_offsets[i],
                                r.row_offsets[i + 1] - r.row_offsets[i]);
            syncwake::in_batch = false;
            syncwake::flush();
            return true;
        }
        sl->d_src = reinterpret_cast<const unsigned long long*>(sl->h_out + tm_batch::HDR_FIXED);
        sl->d_count = reinterpret_cast<const uint32_t*>(sl->h_out + hdr_bytes);
        return false;
    }

    // devices[ndev]: one replica per entry (ndev = 0: host-only engine)
    int init(const tm_config* cfg, const int32_t* devices, uint32_t ndev) {
        frozen = cfg && (cfg->flags & TM_CFG_FROZEN_DICT);
        const char* ck = getenv("TM_CHECKED");
        checked = ck && ck[0] == '1';
        if (const char* rcap = getenv("TM_ROWCAP")) row_cap = std::min(128, std::max(1, atoi(rcap)));
        if (const char* qc = getenv("TM_QCAP")) qcap = atoi(qc) <= 384 ? 384u : 512u;
        if (const char* sf = getenv("TM_STATIC_FRAC")) static_frac = std::min(1.0, std::max(0.0, atof(sf)));
        if (const char* fb = getenv("TM_FAN_BIG")) fan_big_limit = std::min<uint64_t>(0xFFFFFFFFull, strtoull(fb, nullptr, 10));
        if (const char* ld = getenv("TM_LOAD")) target_load = std::min(0.75, std::max(0.1, atof(ld)));
        if (const char* rl = getenv("TM_RESULT_LIMIT"))
            result_limit = std::min<uint64_t>(MAX_RESULT, strtoull(rl, nullptr, 10));
        if (const char* sm = getenv("TM_STAGING_MIN")) staging_min = std::max<uint64_t>(64, strtoull(sm, nullptr, 10));
        threads = (cfg && cfg->host_threads) ? cfg->host_threads : default_threads();
        dev_tok = !(cfg && (cfg->flags & TM_CFG_HOST_TOKENIZE));
        if (const char* ht = getenv("TM_HOST_TOKENIZE")) dev_tok = dev_tok && !(ht[0] == '1');
        if (const char* ng = getenv("TM_NO_GRAPH")) use_graphs = ng[0] != '1';
        // root node id 0 (absent until the first add_path, like the reference)
        nd.push_back(NodeRec{});
        n_flen.push_back(0);
        n_foff.push_back(0);
        n_lext.push_back(0);
        slots.clear();
        slots.resize(1024);
        for (Slot& s : slots) { memset(&s, 0, sizeof(s)); s.parent = SLOT_EMPTY; }
        if (cfg && cfg->init_slots) rehash(cfg->init_slots);
        dirty_mark.assign((slots.size() + 63) / 64, 0);
        if (ndev) {
            int count = 0;
            if (hipGetDeviceCount(&count) != hipSuccess) return TM_ENODEV;
            for (uint32_t i = 0; i < ndev; ++i)
                if (devices[i] < 0 || devices[i] >= count) return TM_ENODEV;
            device = devices[0];
            for (uint32_t i = 0; i < ndev; ++i) {
                Replica* R = new Replica();
                R->index = i;
                R->device = devices[i];
                R->scratch.rep = R;
                R->tokb.rep = R;
                reps.push_back(R);
                HIP_OK(hipSetDevice(R->device));
                HIP_OK(hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking));
                HIP_OK(hipEventCreateWithFlags(&R->ev_delta, hipEventDisableTiming));
                HIP_OK(hipEventCreateWithFlags(&R->ev_sync, hipEventDisableTiming));
            }
            HIP_OK(hipSetDevice(device));
        }
        return TM_OK;
    }

    void destroy() {
        for (Replica* R : reps) async_stop(*R);
        for (Replica* R : reps) {
            (void)hipSetDevice(R->device);
            if (R->stream) (void)hipStreamSynchronize(R->stream);
            pipe_teardown(*R);
            R->scratch.release();
            R->tokb.release();
            dev_free(R->d_slots); dev_free(R->d_foff); dev_free(R->d_flen); dev_free(R->d_fbytes);
            dev_free(R->d_dkey); dev_free(R->d_tail); dev_free(R->d_arena); dev_free(R->d_dxidx); dev_free(R->d_dxval);
            dev_free(R->d_didx); dev_free(R->d_dval); dev_free(R->d_fidx); dev_free(R->d_foffv); dev_free(R->d_flenv);
            dev_free(R->d_dbg); dev_free(R->d_roff); dev_free(R->d_rdest); dev_free(R->d_rl);
            dev_free(R->d_soff); dev_free(R->d_subs); dev_free(R->d_scnt); dev_free(R->d_sone);
            if (R->h_dbg) (void)hipHostFree(R->h_dbg);
            if (R->h_app) (void)hipHostFree(R->h_app);
            if (R->ev_delta) (void)hipEventDestroy(R->ev_delta);
            if (R->ev_sync) (void)hipEventDestroy(R->ev_sync);
            if (R->stream) (void)hipStreamDestroy(R->stream);
            delete R;
        }
        reps.clear();
        for (void* h : {(void*)h_dxidx, (void*)h_dxval, (void*)h_didx, (void*)h_dval, (void*)h_fidx, (void*)h_foffv,
                        (void*)h_flenv})
            if (h) (void)hipHostFree(h);
        h_dxidx = nullptr; h_dxval = nullptr; h_didx = nullptr; h_dval = nullptr;
        h_fidx = nullptr; h_foffv = nullptr; h_flenv = nullptr;
    }

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
    int run_slices(const uint8_t* topics, const uint64_t* offsets, uint32_t n) {
        const size_t k = reps.size();
        int rc = TM_OK;
        upload_nosync = true;   // every slice's stream is drained by its wait below (or on failure)
        for (size_t i = 0; i < k; ++i) {
            Replica& R = *reps[i];
            const uint32_t lo = slice_lo(n, k, i), hi = slice_lo(n, k, i + 1);
            if ((rc = use(&R))) break;
            if ((rc = prepare(&R.scratch, topics, offsets + lo, hi - lo))) break;
            if ((rc = launch(&R.scratch))) break;
        }
        upload_nosync = false;
        int first = rc;
        for (size_t i = 0; i < k; ++i) {   // every slice is drained, even after an error
            Replica& R = *reps[i];
            (void)use(&R);
            if (R.scratch.launched && !R.scratch.done) rc = wait(&R.scratch);
            if (rc && !first) first = rc;
            (void)hipStreamSynchronize(R.stream);
        }
        return first;
    }

    // tm_match_batch of a large batch on one replica, pipelined: chunks of
    // PIPE_CHUNK topics alternate over R.pipe[0/1] (own streams).  Chunk j is
    // uploaded and walked (dense CSR enqueued behind the walk) while chunk
    // j - 1's ids go to the host by DMA, straight to their place in the merged
    // CSR (the host learns a chunk's total when it waits for it, so every copy
    // knows its offset); row offsets are rebased on the host after their copy.
    static constexpr uint32_t PIPE_CHUNK = 1u << 20;
    int pipe_setup(Replica& R) {
        if (R.pipe_ready) return TM_OK;
        for (int k = 0; k < 2; ++k) {
            tm_batch& b = R.pipe[k];
            b.rep = &R;
            HIP_OK(hipStreamCreateWithFlags(&b.own, hipStreamNonBlocking));
            b.own_user = true;   // (kept out of async_stop's sweep of slot batches)
            R.readers.push_back(&b);
            HIP_OK(hipEventCreateWithFlags(&R.pipe_h2d[k], hipEventDisableTiming));
            HIP_OK(hipEventCreateWithFlags(&R.pipe_cp[k], hipEventDisableTiming));
        }
        HIP_OK(hipStreamCreateWithFlags(&R.pipe_copy, hipStreamNonBlocking));
        R.pipe_ready = true;
        return TM_OK;
    }
    void pipe_teardown(Replica& R) {
        if (!R.pipe_ready) return;
        if (R.pipe_copy) (void)hipStreamSynchronize(R.pipe_copy);
        for (int k = 0; k < 2; ++k) {
            tm_batch& b = R.pipe[k];
            if (b.own) (void)hipStreamSynchronize(b.own);
            forget_launch(&b);
            b.release();
            drop_user_stream(&b);
            if (R.pipe_h2d[k]) (void)hipEventDestroy(R.pipe_h2d[k]);
            if (R.pipe_cp[k]) (void)hipEventDestroy(R.pipe_cp[k]);
            R.pipe_h2d[k] = R.pipe_cp[k] = nullptr;
            if (R.h_stage[k]) (void)hipHostFree(R.h_stage[k]);
            R.h_stage[k] = nullptr;
            R.ch_stage[k] = 0;
        }
        if (R.pipe_copy) (void)hipStreamDestroy(R.pipe_copy);
        R.pipe_copy = nullptr;
        if (R.h_prow) (void)hipHostFree(R.h_prow);
        if (R.h_pids) (void)hipHostFree(R.h_pids);
        R.h_prow = R.h_pids = nullptr;
        R.ch_prow = R.ch_pids = 0;
        R.pipe_ready = false;
    }

    // Chunk j: its offsets (rebased) and bytes are copied into pinned staging
    // by the engine's workers, uploaded in one async copy and walked on batch
    // j % 2's stream; once the host has waited for it (its total gives the
    // offset of its ids in the merged CSR), a copy stream moves its ids and row
    // offsets to the host.  So the host fills chunk j + 1 while chunk j walks
    // and chunk j - 1's result crosses PCIe.  Row offsets are rebased at the end.
    int match_batch_pipelined(Replica& R, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                              tm_result* out) {
        int rc;
        if ((rc = pipe_setup(R))) return rc;
        const uint32_t nch = (n + PIPE_CHUNK - 1) / PIPE_CHUNK;
        if ((rc = host_reserve(R.h_prow, R.ch_prow, (size_t)n + 1))) return rc;
        bool h2d_pending[2] = {false, false}, cp_pending[2] = {false, false};
        std::vector<uint64_t> cbase(nch + 1, 0);
        // every stream is drained before returning: staging and results stay consistent
        struct Drain {
            Replica& R;
            ~Drain() {
                for (tm_batch& b : R.pipe)
                    if (b.own) (void)hipStreamSynchronize(b.own);
                if (R.pipe_copy) (void)hipStreamSynchronize(R.pipe_copy);
            }
        } drain{R};
        for (uint32_t j = 0; j <= nch; ++j) {
            if (j < nch) {   // chunk j: stage, upload, walk + dense CSR
                const int k = j & 1;
                tm_batch* X = &R.pipe[k];
                const uint32_t lo = j * PIPE_CHUNK, cnt = std::min(n - lo, PIPE_CHUNK);
                const uint64_t b0 = offsets[lo], nb = offsets[lo + cnt] - b0;
                const size_t head = packed_head(cnt);
                if (h2d_pending[k]) HIP_OK(hipEventSynchronize(R.pipe_h2d[k]));   // staging k is free again
                if ((rc = host_reserve(R.h_stage[k], R.ch_stage[k], head + nb))) return rc;
                uint64_t* so = reinterpret_cast<uint64_t*>(R.h_stage[k]);
                uint8_t* sb = R.h_stage[k] + head;
                par_chunks((size_t)cnt + 1, [&](size_t i0, size_t i1) {
                    for (size_t i = i0; i < i1; ++i) so[i] = offsets[lo + i] - b0;
                });
                par_chunks(nb, [&](size_t i0, size_t i1) { memcpy(sb + i0, topics + b0 + i0, i1 - i0); });
                if (cp_pending[k]) HIP_OK(hipStreamWaitEvent(X->own, R.pipe_cp[k], 0));   // its last ids were copied out
                if (dev_tok) {
                    rc = upload_packed(X, R.h_stage[k], cnt, nb);
                } else {
                    upload_nosync = true;
                    rc = prepare(X, sb, so, cnt);
                    upload_nosync = false;
                }
                if (rc) return rc;
                HIP_OK(hipEventRecord(R.pipe_h2d[k], X->own));
                h2d_pending[k] = true;
                X->eager_dense = true;
                rc = launch(X);
                X->eager_dense = false;
                if (rc) return rc;
            }
            if (j >= 1) {    // chunk j - 1: wait, then its result to its place in the merged CSR
                const int k = (j - 1) & 1;
                tm_batch* Y = &R.pipe[k];
                const uint32_t lo = (j - 1) * PIPE_CHUNK, cnt = std::min(n - lo, PIPE_CHUNK);
                if ((rc = wait(Y))) return rc;
                if ((rc = ensure_dense(Y))) return rc;   // (built by the launch unless ids overflowed)
                const uint64_t base = cbase[j - 1], total = Y->total;
                if (base + total > MAX_RESULT) return TM_EOVERFLOW;   // u32 CSR offsets
                if (base + total > R.ch_pids) {
                    // grow the merged ids (earlier copies land first): room for the rest at this chunk's rate
                    HIP_OK(hipStreamSynchronize(R.pipe_copy));
                    const size_t want = (size_t)(base + total) +
                                        (size_t)((double)(total + 1) / cnt * (n - lo - cnt) * 1.25) + 1024;
                    uint32_t* np = nullptr;
                    HIP_OK(hipHostMalloc((void**)&np, want * sizeof(uint32_t), hipHostMallocDefault));
                    if (base) memcpy(np, R.h_pids, base * sizeof(uint32_t));
                    if (R.h_pids) (void)hipHostFree(R.h_pids);
                    R.h_pids = np;
                    R.ch_pids = want;
                }
                HIP_OK(hipStreamWaitEvent(R.pipe_copy, Y->ev_end, 0));
                if (total)
                    HIP_OK(hipMemcpyAsync(R.h_pids + base, Y->d_ids, total * 4, hipMemcpyDeviceToHost, R.pipe_copy));
                HIP_OK(hipMemcpyAsync(R.h_prow + lo, Y->d_rowoff, (size_t)cnt * 4, hipMemcpyDeviceToHost, R.pipe_copy));
                HIP_OK(hipEventRecord(R.pipe_cp[k], R.pipe_copy));
                cp_pending[k] = true;
                cbase[j] = base + total;
            }
        }
        HIP_OK(hipStreamSynchronize(R.pipe_copy));
        // chunk-local row offsets -> merged
        for (uint32_t j = 1; j < nch; ++j) {
            const uint32_t lo = j * PIPE_CHUNK, cnt = std::min(n - lo, PIPE_CHUNK), add = (uint32_t)cbase[j];
            par_chunks(cnt, [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i) R.h_prow[lo + i] += add;
            });
        }
        const uint64_t total = cbase[nch];
        R.h_prow[n] = (uint32_t)total;
        out->n_topics = n;
        out->n_matches = total;
        out->row_offsets = R.h_prow;
        out->filter_ids = total ? R.h_pids : R.h_prow;
        return TM_OK;
    }

    // tm_match_batch over every replica: merged CSR in m_rowoff / m_ids
    int match_batch_split(const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_result* out) {
        for (Replica* R : reps) R->scratch.launched = R->scratch.done = false;
        int rc = run_slices(topics, offsets, n);
        if (rc) return rc;
        const size_t k = reps.size();
        std::vector<tm_result> r(k);
        uint64_t total = 0;
        for (size_t i = 0; i < k; ++i) {
            if ((rc = use(reps[i]))) return rc;
            if ((rc = result(&reps[i]->scratch, &r[i]))) return rc;
            total += r[i].n_matches;
        }
        if (total > MAX_RESULT) return TM_EOVERFLOW;   // u32 CSR offsets
        m_rowoff.resize((size_t)n + 1);
        m_ids.resize(std::max<uint64_t>(total, 1));
        std::vector<uint64_t> base(k + 1, 0);
        for (size_t i = 0; i < k; ++i) base[i + 1] = base[i] + r[i].n_matches;
        each_rep([&](size_t i) {
            const uint32_t lo = slice_lo(n, k, i), cnt = slice_lo(n, k, i + 1) - lo, add = (uint32_t)base[i];
            for (uint32_t t = 0; t < cnt; ++t) m_rowoff[lo + t] = r[i].row_offsets[t] + add;
            if (r[i].n_matches) memcpy(m_ids.data() + base[i], r[i].filter_ids, r[i].n_matches * sizeof(uint32_t));
        });
        m_rowoff[n] = (uint32_t)total;
        out->n_topics = n;
        out->n_matches = total;
        out->row_offsets = m_rowoff.data();
        out->filter_ids = m_ids.data();
        return TM_OK;
    }

    // tm_match_routes_batch over every replica: merged route CSR
    int match_routes_split(const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_routes* out) {
        for (Replica* R : reps) R->scratch.launched = R->scratch.done = false;
        int rc = run_slices(topics, offsets, n);
        if (rc) return rc;
        const size_t k = reps.size();
        std::vector<tm_routes> r(k);
        uint64_t total = 0;
        for (size_t i = 0; i < k; ++i) {
            if ((rc = use(reps[i]))) return rc;
            if ((rc = batch_routes(&reps[i]->scratch, &r[i]))) return rc;
            total += r[i].n_routes;
        }
        if (total > MAX_RESULT) return TM_EOVERFLOW;
        m_rowoff.resize((size_t)n + 1);
        m_ids.resize(std::max<uint64_t>(total, 1));
        m_dests.resize(std::max<uint64_t>(total, 1));
        std::vector<uint64_t> base(k + 1, 0);
        for (size_t i = 0; i < k; ++i) base[i + 1] = base[i] + r[i].n_routes;
        each_rep([&](size_t i) {
            const uint32_t lo = slice_lo(n, k, i), cnt = slice_lo(n, k, i + 1) - lo, add = (uint32_t)base[i];
            for (uint32_t t = 0; t < cnt; ++t) m_rowoff[lo + t] = r[i].row_offsets[t] + add;
            if (r[i].n_routes) {
                memcpy(m_ids.data() + base[i], r[i].filter_ids, r[i].n_routes * sizeof(uint32_t));
                memcpy(m_dests.data() + base[i], r[i].dests, r[i].n_routes * sizeof(uint32_t));
            }
        });
        m_rowoff[n] = (uint32_t)total;
        out->n_topics = n;
        out->n_routes = total;
        out->row_offsets = m_rowoff.data();
        out->filter_ids = m_ids.data();
        out->dests = m_dests.data();
        return TM_OK;
    }

    // tm_rules_match over every replica: names split, each replica writes its
    // rows of the bitmap (disjoint)
    int rules_match_split(const uint8_t* names, const uint64_t* noffs, uint32_t n, const uint8_t* rules,
                          const uint64_t* roffs, uint32_t r, bool dollar_rule, uint32_t* bits) {
        const size_t k = std::min<size_t>(reps.size(), std::max<uint32_t>(1, n / 4096));   // small: one replica
        const uint32_t wpr = (r + 31) / 32;
        std::vector<int> rc(k, TM_OK);
        auto one = [&](size_t i) {
            Replica& R = *reps[i];
            const uint32_t lo = slice_lo(n, k, i), hi = slice_lo(n, k, i + 1);
            if (hipSetDevice(R.device) != hipSuccess) { rc[i] = TM_EIO; return; }
            try {
                rc[i] = rules_match(R, names, noffs + lo, hi - lo, rules, roffs, r, dollar_rule, bits + (size_t)lo * wpr);
            } catch (...) {
                rc[i] = TM_ENOMEM;
            }
        };
        if (k == 1) one(0);
        else {
            std::vector<std::thread> th;
            for (size_t i = 0; i < k; ++i) th.emplace_back(one, i);
            for (auto& t : th) t.join();
        }
        for (int x : rc)
            if (x) return x;
        return TM_OK;
    }
};

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
    if (n > tm_engine::ONESHOT_MAX && !e->eager_csr) {
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
        R.scratch.oneshot = n <= tm_engine::ONESHOT_MAX && !e->eager_csr;
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
    for (int i = 0; i < 4000 && w.state.load(std::memory_order_acquire) != 1; ++i) __builtin_ia32_pause();
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
    static const bool wtrace = getenv("TM_WAIT_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::recursive_mutex> g(e->mu);
    const auto t1 = std::chrono::steady_clock::now();
    int rc = e->use(b->rep);
    if (rc) return rc;
    rc = e->wait(b);
    if (wtrace) {
        auto us = [](auto a, auto c) { return std::chrono::duration<double, std::micro>(c - a).count(); };
        fprintf(stderr, "[tm_batch_wait] lock %.1f us, total %.1f us\n", us(t0, t1), us(t0, std::chrono::steady_clock::now()));
    }
    return rc;
}

int tm_batch_result(tm_engine* e, tm_batch* b, tm_result* out) {
    if (!e || !b || !out) return TM_EINVAL;
    if (!b->rep) return TM_ENODEV;   // host-only engine
    std::lock_guard<std::recursive_mutex> g(e->mu);
    int rc = e->use(b->rep);
    if (rc) return rc;
    return e->result(b, out);
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
    uint64_t done = 0;
    int rc = TM_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return TM_EINVAL;
    try {
        if (nshards <= 1) {
            const auto tq0 = std::chrono::steady_clock::now();
            e->make_plan(filters, offsets, n, false);
            if (getenv("TM_PAR_TRACE"))
                fprintf(stderr, "[plan ins n=%u] %.2f ms\n", n,
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
            if (n >= tm_engine::PAR_MIN && !e->mutate_parallel(false, filters, offsets, n, &done, &rc)) {
                if (n_inserted) *n_inserted = done;
                if (getenv("TM_PAR_TRACE"))
                    fprintf(stderr, "[insert_many n=%u] %.2f ms in the call\n", n,
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
                return rc;
            }
            for (uint32_t i = 0; i < n && rc == TM_OK; ++i) {
                e->prefetch_insert(i, n);
                rc = e->insert_planned(filters, offsets, i);
                if (rc == TM_OK) ++done;
            }
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
    uint64_t done = 0;
    int rc = TM_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i]) return TM_EINVAL;
    try {
        const auto tq0 = std::chrono::steady_clock::now();
        e->make_plan(filters, offsets, n, true);
        if (getenv("TM_PAR_TRACE"))
            fprintf(stderr, "[plan del n=%u] %.2f ms\n", n,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
        if (n >= tm_engine::PAR_MIN && !e->mutate_parallel(true, filters, offsets, n, &done, &rc)) {
            if (n_deleted) *n_deleted = done;
            if (getenv("TM_PAR_TRACE"))
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
    for (uint32_t i = 0; i < n_del; ++i)
        if (del_offsets[i + 1] < del_offsets[i]) return TM_EINVAL;
    for (uint32_t i = 0; i < n_ins; ++i)
        if (ins_offsets[i + 1] < ins_offsets[i]) return TM_EINVAL;
    static const bool trace = getenv("TM_PAR_TRACE") != nullptr;
    uint64_t done = 0;
    int rc = TM_OK;
    try {
        const auto tq0 = std::chrono::steady_clock::now();
        e->make_plan_pair(del_filters, del_offsets, n_del, ins_filters, ins_offsets, n_ins);
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
            const uint32_t again = e->replan_dead_inserts(n_ins);
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
                if (trace)
                    fprintf(stderr, "[apply_many del=%u ins=%u, one edge phase] %.2f ms in the call\n", n_del, n_ins,
                            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq0).count());
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

int tm_filters_copy(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, size_t cap, uint64_t* offs,
                    uint32_t* keep, uint32_t* n_out, uint64_t* need) {
    if (!e || !offs || !n_out || !need || (n && !ids) || (cap && !buf)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(e->mu);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (ids[i] < e->nd.size() && e->nd[ids[i]].hasbytes) total += e->n_flen[ids[i]];
    *need = total;
    if (total > cap) return TM_OK;   // nothing copied: the caller grows buf and asks again
    uint32_t k = 0;
    uint64_t at = 0;
    offs[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t id = ids[i];
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

char* etm::error_buf() { return last_error(); }

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
