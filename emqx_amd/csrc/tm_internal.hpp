// tm_internal.hpp -- layout shared by the host engine (tm_engine_impl.hpp and its modules) and the
// gfx950 kernels (tm_kernels.hip).  See DESIGN.md "Data layout in HBM".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

struct tm_engine;   // include/emqx_tm.h (opaque handles, defined in tm_engine_impl.hpp)
struct tm_batch;

namespace etm {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t SLOT_EMPTY = 0xFFFFFFFFu;   // slot.parent of a free slot (never a live slot's: ids < ID_MASK)
constexpr uint32_t ROOT = 0;                   // node id of the atom `root`

// Interned word ids (low 29 bits of a topic word entry).  '' is a regular word
// for the trie (a literal edge), it only gets a fixed id.
constexpr uint32_t W_UNKNOWN = 0;   // topic word absent from every filter
constexpr uint32_t W_EMPTY = 1;     // ''
constexpr uint32_t W_PLUS = 2;      // '+'
constexpr uint32_t W_HASH = 3;      // '#'
constexpr uint32_t W_FIRST = 4;
constexpr uint32_t WID_BITS = 29;
constexpr uint32_t WID_MASK = (1u << WID_BITS) - 1;

// Byte class of a topic word relative to '#' (0x23) and '+' (0x2B): decides
// where the literal branch sorts among {'#', '+'} filters at that level.
constexpr uint32_t C_BELOW = 0;     // first byte < '#'
constexpr uint32_t C_BETWEEN = 1;   // '#' <= first byte < '+'  (incl. the word '#')
constexpr uint32_t C_ABOVE = 2;     // first byte > '+'
constexpr uint32_t C_EMPTY = 3;     // ''

// Topic flags
constexpr uint8_t TF_DOLLAR = 1;    // first byte is '$' (src/emqx_trie.erl:162-163)
constexpr uint8_t TF_SLOW = 2;      // deep (> FAST_MAX_DEPTH) or irregular word

// Fast path: 3-bit sort digits for levels 0..10 packed MSB-first in bits
// 63..31 of a u64; the low 31 bits carry the filter id, so one u64 per match
// sorts by path code (== Erlang binary order of the filter).
constexpr uint32_t FAST_MAX_DEPTH = 10;
constexpr uint64_t KEY_MASK = 0xFFFFFFFF80000000ull;

// Node summary flags (RootRec.flags)
constexpr uint32_t NF_PLUS = 1;     // node has a '+' child
constexpr uint32_t NF_HASH = 2;     // node has a '#' child

// Node ids (== filter ids) are < 2^30 so that two flag bits ride in each id word.
constexpr uint32_t ID_BITS = 30;
constexpr uint32_t ID_MASK = (1u << ID_BITS) - 1;
constexpr uint32_t MAX_NODES = ID_MASK;          // ids 0 .. 2^30-2; ID_MASK = "none"
constexpr uint32_t B_TOPIC = 1u << 30;           // child word: child has topic (term = child)
constexpr uint32_t B_PLUS = 1u << 31;            // child word: child has a '+' child
constexpr uint32_t B_HTERM = 1u << 30;           // hash word: child/'#' has topic (hterm valid)
constexpr uint32_t B_HASH = 1u << 31;            // hash word: child has a '#' child

// One edge of the trie in the open-addressed hash, keyed (parent, word), and
// carrying the CHILD's summary, so one 64-B bucket read per visited node is all
// the walk needs.  16 B; four slots per 64-B bucket.
//
// The key's spare bits -- the word's top 3 (word ids are < 2^29) and the
// parent's top 2 (node ids are < 2^30) -- carry the child's 5-bit LITERAL-CHILD
// SIGNATURE: bit lsig_pos(w) is set for every literal word w under the child
// (not '+' / '#').  A clear bit proves the literal edge absent, so the walk
// skips that probe -- a third of the literal probes on C2 miss, and the
// signature settles ~45% of those without a bucket read.
struct alignas(16) Slot {
    uint32_t parent;   // key hi: parent id | signature bits 3-4 << ID_BITS; SLOT_EMPTY when free
    uint32_t word;     // key lo: word id | signature bits 0-2 << WID_BITS
    uint32_t child;    // child id | B_TOPIC | B_PLUS
    uint32_t hash;     // B_HASH: id of child/'#' | B_HTERM | B_HASH; else the 30-bit literal signature
};
constexpr uint32_t LSIG_WBITS = 32 - WID_BITS;              // signature bits in the word field
constexpr uint32_t LSIG_BITS = LSIG_WBITS + (32 - ID_BITS);   // 5
__host__ __device__ inline uint32_t lsig_pos(uint32_t w) {
    return (uint32_t)(((uint64_t)(w * 0x9E3779B1u) * LSIG_BITS) >> 32);
}
// A child with no '#' child leaves the slot's '#'-id field free: it then holds
// a 30-bit Bloom filter of the same literal words (bit lext_pos(w)), set as
// children arrive and rebuilt exactly when the table is re-packed -- a stale
// bit costs one probe, never a match.
__host__ __device__ inline uint32_t lext_pos(uint32_t w) {
    return (uint32_t)(((uint64_t)(w * 0x85EBCA6Bu) * 30u) >> 32);
}
__host__ __device__ inline uint32_t slot_lsig(uint32_t parent_field, uint32_t word_field) {
    return (word_field >> WID_BITS) | ((parent_field >> ID_BITS) << LSIG_WBITS);
}
__host__ __device__ inline void slot_set_lsig(Slot& e, uint32_t sig) {
    e.word = (e.word & WID_MASK) | ((sig & ((1u << LSIG_WBITS) - 1u)) << WID_BITS);
    e.parent = (e.parent & ID_MASK) | ((sig >> LSIG_WBITS) << ID_BITS);
}
static_assert(sizeof(Slot) == 16, "slot is 16 bytes");
constexpr uint32_t BUCKET = 4;   // slots per 64-B bucket

struct RootRec {
    uint32_t hterm;    // filter id of root/'#' or NONE
    uint32_t flags;    // NF_*
    uint32_t live;
    uint32_t pad;
};

__host__ __device__ inline uint32_t edge_hash(uint32_t parent, uint32_t word) {
    uint64_t k = ((uint64_t)parent << 32) | word;
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (uint32_t)k;
}

// home bucket for any bucket count (multiply-shift, no power-of-two rounding)
__host__ __device__ inline uint32_t home_bucket(uint32_t parent, uint32_t word, uint32_t nbuckets) {
    return (uint32_t)(((uint64_t)edge_hash(parent, word) * nbuckets) >> 32);
}

// Control words of one batch launch (device memory, zeroed per launch).
// Walk groups: one per XCD (blockIdx % 8 on the round-robin dispatch), each
// with its own 128-B header line, so no two groups ever contend for one
// address.  Group g hands out the tail tiles g, g + 8, g + 16, ... from its
// ticket and reserves staging entries in its own region of sfids[] (region g
// = [g * rcap, (g + 1) * rcap)): a single device-wide counter per tile
// serialises at one L2 line and its return stalls every in-order vmcnt wait.
constexpr uint32_t TICKET_GROUPS = 8, TICKET_STRIDE = 32;

enum Ctrl : uint32_t {
    CTRL_NOVF = 1,          // topics appended to the ovf list
    CTRL_ERR = 2,           // error bits
    CTRL_SLOW_DONE = 3,
    CTRL_TILE_NEXT = 4,     // (unused: tail tickets live in MatchArgs.xtickets)
    CTRL_NROWS = 5,         // TM_BATCH_DEDUP on the device: distinct topics (rows) of the batch
    CTRL_WORDS = 16
};
constexpr uint32_t ERR_STAGING = 1;      // staging capacity exceeded
constexpr uint32_t ERR_SLOW_SCRATCH = 2; // slow-path scratch exceeded
constexpr uint32_t ERR_OVF_LIST = 4;
constexpr uint32_t ERR_CSR_RANGE = 8;    // the batch's match count does not fit u32 CSR offsets
// Staging and CSR offsets are u32 (tm_result.row_offsets): a batch with more
// matches than this fails with TM_EOVERFLOW instead of wrapping.
constexpr uint64_t MAX_RESULT = 0xFFFFFFF0ull;


enum StatIdx : uint32_t { ST_VISITS = 0, ST_HASH = 1, ST_WORDS = 2, ST_MATCHES = 3, ST_SLOW = 4, ST_PROBES = 5, ST_ITERS = 6,
                          ST_DELIVERED = 7,   // TM_BATCH_DEDUP: sum over the publishes of their rows' lengths
                          ST_N = 8 };

// The batch header block: ctrl (CTRL_WORDS u32) | stats (ST_N u64) | one
// 128-B line per walk group (see TICKET_GROUPS): u32 tail ticket at +0, u64
// staging top at +8 | per-topic src / count.  Zeroed per launch.
constexpr uint32_t XG_WORD = CTRL_WORDS + ST_N * 2;   // first group line, in u32 of the header
// staging entries group g reserved (u64; may exceed the region -> rerun)
__host__ __device__ __forceinline__ unsigned long long* xg_top(uint32_t* xg, uint32_t g) {
    return reinterpret_cast<unsigned long long*>(xg + g * TICKET_STRIDE + 2);
}
__host__ __device__ __forceinline__ uint64_t xg_top_read(const uint32_t* hdr, uint32_t g) {
    const uint32_t* w = hdr + XG_WORD + g * TICKET_STRIDE + 2;
    return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}

constexpr uint32_t WSTATS = 8;   // u64 partial sums per walk wave (MatchArgs.wstats)
// walks of at least this many waves sum their stats by tm_stats_reduce: ~4,000
// waves ending together queued ~24k same-line device atomics (C5 K = 100 walk
// 0.48 -> 0.23 ms without them, C2 4.75 -> 4.62 ms)
constexpr uint32_t WSTATS_MIN_WAVES = 256;
struct MatchArgs {
    // trie replica
    const Slot* slots;
    uint32_t nbuckets;        // buckets of BUCKET slots
    uint32_t max_probe;       // max bucket displacement of any live key
    RootRec root;
    const uint64_t* foff;     // filter bytes offset per node id (slow-path byte sort)
    const uint32_t* flen;
    const uint8_t* fbytes;
    // batch input
    const uint32_t* words;    // (class << 29) | word id
    const uint32_t* toff;     // n + 1 word offsets
    const uint8_t* tflags;
    uint32_t n;
    uint32_t pad0_;             // (explicit padding: the struct's bytes are a graph cache key, tm_batch.cpp)
    const uint32_t* d_n;        // or null: the topic count is *d_n (<= n) -- a device-deduplicated
                                // batch's rows, known only on the device when the walk is enqueued
    const uint32_t* slow_list;  // host-flagged slow topics
    uint32_t n_slow;
    uint32_t s_lcap;            // generic path: LDS probe-stack entries to use (0 = all; TM_SLOW_LDS)
    const uint32_t* d_nslow;    // device-resident count of slow_list (token batches), or null
    // outputs
    uint32_t* count;          // per topic |M(t)|
    unsigned long long* src;  // per topic: offset of its sorted row in sfids[]
    unsigned long long* rows; // [match_waves(n) * tile_topics * row_cap] wave-private emission rows,
                              // (path code | filter id), reused by every tile of the wave
    uint32_t row_cap;         // K: per-topic row slots on the fast path
    uint32_t tile_topics;     // topics per tm_match_tiles tile (tile_topics(n): 64 .. 1)
    uint32_t grid;            // tm_match_tiles workgroups (= match_waves(n)); rows[] is sized for it
    uint32_t qcap;            // LDS probe-stack entries per wave (384 or 512)
    uint32_t static_rounds;   // round-robin tiles per wave before tickets (>= 1)
    uint32_t pad2_;
    uint32_t* xg;             // the header's group lines (header + XG_WORD)
    uint64_t rcap;            // staging entries per group region (sfids_cap / TICKET_GROUPS)
    uint32_t sgmask;          // staging group of a wave = (blockIdx % TICKET_GROUPS) & sgmask
                              // (TICKET_GROUPS - 1; 0 = one region for all: a skewed batch)
    uint32_t pad3_;
    uint32_t* sfids;          // staging: sorted filter ids, one contiguous run per tile
    uint64_t sfids_cap;
    uint32_t* ctrl;
    uint32_t* ovf_list;       // topics redone by the slow path (row > K or stack overflow)
    uint32_t ovf_cap;
    uint32_t pad4_;
    unsigned long long* stats;
    unsigned long long* wstats;   // or null: per walk wave WSTATS partial sums (tm_stats_reduce adds them up)
    // slow-path scratch
    uint32_t* s_qparent;
    uint32_t* s_qpw;
    uint32_t* s_qmeta;
    unsigned long long* s_qkey;
    uint32_t* s_ofid;
    unsigned long long* s_okey;
    uint32_t s_qcap;
    uint32_t s_ocap;
    uint32_t s_waves;
    // sizes for the bounds-checked debug variant (TM_CHECKED=1)
    uint32_t nwords;
    uint32_t nslots;
    uint32_t nnodes;
    uint64_t nfbytes;
    uint32_t* dbg;            // [0] first failing check id, [1] index, [2] bound, [3] count
};

struct ScanArgs {
    const uint32_t* count;
    const unsigned long long* src;
    const uint32_t* sfids;
    uint64_t sfids_cap;
    uint32_t* row_off;        // n + 1
    uint32_t* ids;
    uint32_t* block_sums;     // scratch
    uint32_t n;
    uint32_t ids_cap;
    uint32_t* ctrl;
    uint32_t* dbg;
};

// Route resolution over a batch's match CSR (tm_batch_routes).
// Entry-parallel: one thread per match entry, so a topic matching thousands of
// filters (C5 skew) costs no more per thread than one matching a few.
struct RouteArgs {
    const uint32_t* row_off;  // match CSR (n + 1) and filter ids (m entries)
    const uint32_t* ids;
    uint32_t n;
    uint32_t m;
    const uint32_t* roff;     // per node id: dests roff[f] .. roff[f+1] (nnodes + 1)
    const uint32_t* rdest;
    uint32_t nnodes;
    uint32_t* ecount;         // per match entry: dests of its filter
    uint32_t* eoff;           // m + 1: exclusive scan of ecount (block-local + bsums)
    uint32_t* bsums;          // scan block sums (SCAN_TILE entries per block)
    const uint32_t* total;    // routes in the batch (scan total)
    uint32_t* r_rowoff;       // n + 1: route CSR offsets
    uint32_t* out_fid;        // route i: filter id, dest
    uint32_t* out_dest;
    uint64_t cap;             // capacity of out_fid / out_dest
};

// Subscriber fan-out over a batch's match CSR (tm_batch_dispatch):
// emqx_broker:dispatch/2 (src/emqx_broker.erl:284-309) for every matched filter.
struct FanArgs {
    const uint32_t* row_off;  // match CSR (n + 1) and filter ids
    const uint32_t* ids;
    uint32_t n;
    uint64_t n_matches;
    const uint64_t* soff;     // per node id: subscribers soff[f] .. soff[f+1] (nnodes + 1)
    const uint8_t* scnt;      // per node id: min(soff[f + 1] - soff[f], 255); 255 = read soff
    const uint32_t* sone;     // per node id: the subscriber of a one-subscriber node
    const uint32_t* subs;
    uint32_t nnodes;
    uint64_t* moff;           // n_matches + 1: u64 first delivery of entry j (block-relative in "big"
                              // scan blocks; all entries, global, after tm_fan_scan_add)
    uint32_t* moff32;         // n_matches + 1: the same, u32 block-relative, in blocks under 2^32 deliveries
    uint8_t* bbig;            // per scan block: 1 = its deliveries exceed u32, read moff instead of moff32
    uint64_t big_limit;       // a block delivering more takes the u64 path (u32 max; TM_FAN_BIG test knob)
    uint64_t* bsums;          // scan block sums (FAN_SCAN_TILE entries per block)
    uint64_t* d_total;
    uint64_t* drow;           // n + 1: deliveries of publish i
    uint32_t* out;            // subscriber of delivery p
    uint64_t total;
    uint64_t* tile_j;         // total / fan_fill_tile() + 2: match entry of each fill tile's first delivery
    // Rows mode (TM_DISPATCH_ROWS): the entries are the walk's staging, read
    // where it was written.  Staging region g holds rtop[g] entries from
    // g * rcap; entry j of the virtual entry space [0, vb[nreg]) is region g's
    // entry j - vb[g] (vb[g] a multiple of 16, entries past rtop[g] padding
    // with no deliveries), so a row -- contiguous in its region -- is
    // contiguous here too.  nreg = 0: ids is the match CSR.
    // (vb / rtop live in device memory, not in the arguments: a kernel-argument
    // array indexed at run time is copied to scratch, and every pointer the
    // kernel then loads becomes a flat access -- tools/isa_check.py)
    uint32_t nreg;
    uint64_t rcap;            // a multiple of 16 (region_cap)
    const uint64_t* vb;       // TICKET_GROUPS + 1
    const uint64_t* rtop;     // TICKET_GROUPS
    const uint32_t* rcount;   // n: the walk's row lengths (tm_batch_rows)
    const unsigned long long* rsrc;   // n: the rows' first staging entries
    uint32_t* dcount;         // n: deliveries of each row (drow = its first)
};

// staging region capacity of a launch: a multiple of 16 entries per region so
// the fan-out's rows mode reads 16-entry chunks aligned and in bounds
__host__ __device__ inline uint64_t region_cap(uint64_t sfids_cap, bool one_region) {
    return (one_region ? sfids_cap : sfids_cap / TICKET_GROUPS) & ~15ull;
}

// Batched emqx_topic:match/2 (tm_rules_match): names x rules -> bitmap.
struct RulesArgs {
    const uint32_t* nwords;   // name word ids (rule dictionary; unknown = W_UNKNOWN)
    const uint32_t* noff;     // n + 1
    const uint8_t* nflag;     // bit 0: name starts with '$'
    uint32_t n;
    const uint32_t* rwords;
    const uint32_t* roff;     // r + 1
    const uint8_t* rflag;     // bit 0: rule starts with '+' or '#'
    uint32_t r;
    uint32_t dollar_rule;
    uint32_t wpr;             // u32 words per name row = ceil(r / 32)
    uint32_t* bits;
};

// text of the last TM_EIO on this thread (tm_last_error), shared by the C++ modules
char* error_buf();

// kernel launchers (tm_kernels.hip)
hipError_t launch_rules_match(const RulesArgs& a, hipStream_t s);
hipError_t launch_gather_rows(const uint32_t* src, const int64_t* src_off, const int64_t* idx, uint32_t n,
                              const int64_t* dst_off, uint32_t* dst, hipStream_t s);
hipError_t launch_route_count(const RouteArgs& a, hipStream_t s);
hipError_t launch_route_rows(const RouteArgs& a, hipStream_t s);
hipError_t launch_route_fill(const RouteArgs& a, hipStream_t s);
// fan-out: per-match delivery counts + u64 scan (moff, d_total), publish row
// offsets (drow), then the load-balanced subscriber copy (out[total])
hipError_t launch_fan_scan(const FanArgs& a, hipStream_t s);
hipError_t launch_fan_fill(const FanArgs& a, hipStream_t s);
hipError_t launch_fan_globalize(const FanArgs& a, hipStream_t s);   // block-relative moff -> global
uint32_t fan_scan_tile();   // match entries per scan block
uint32_t fan_fill_tile();   // deliveries per fill block
hipError_t launch_match(const MatchArgs& a, hipStream_t s, hipEvent_t ev_a, hipEvent_t ev_b, bool checked,
                        unsigned ev_flags = 0);
hipError_t launch_scan(const ScanArgs& a, hipStream_t s, uint32_t* d_total);
hipError_t launch_finalize(const ScanArgs& a, hipStream_t s, bool checked);
hipError_t launch_scatter_slots(Slot* slots, const uint32_t* idx, const Slot* vals, uint32_t n,
                                hipStream_t s);
hipError_t launch_scatter_fmeta(uint64_t* foff, uint32_t* flen, const uint32_t* idx,
                                const uint64_t* off, const uint32_t* len, uint32_t n, hipStream_t s);
uint32_t scan_block_count(uint32_t n);
// sampled rows of a waited batch (tm_batch_sample): per-row count + start, then the ids
hipError_t launch_sample_meta(const uint32_t* count, const unsigned long long* src, const uint32_t* rows, uint32_t k,
                              uint32_t* out_cnt, unsigned long long* out_src, hipStream_t s);
hipError_t launch_sample_ids(const uint32_t* sfids, const uint32_t* cnt, const unsigned long long* src,
                             const uint64_t* off, uint32_t k, uint32_t* out, hipStream_t s);
// token batches (filter-sharded mode)
hipError_t launch_token_check(const uint32_t* toff, const uint8_t* tflags, uint32_t n, uint64_t nwords,
                              uint32_t* slow_list, uint32_t* d_nslow, uint32_t* d_bad, hipStream_t s);
hipError_t launch_tokens_shard(const uint32_t* words, const uint32_t* toff, uint32_t n, uint32_t nshards,
                               uint32_t* shard, hipStream_t s);
hipError_t launch_export(const uint32_t* row_off, const uint32_t* ids, uint32_t n, uint64_t total,
                         uint32_t* counts, uint32_t* gids, uint32_t mul, uint32_t add, hipStream_t s);

// In-process filter-sharded group (tm_sharded, BASELINE config C4 without a
// collective): a tokenised batch on the home device is partitioned by owner
// shard (a stable counting sort: each owner's publishes contiguous, in publish
// order), every shard matches its part, and the rows come back in publish order.
constexpr uint32_t PART_BLOCK = 1024;   // publishes per partition block (one per thread)
constexpr uint32_t PART_MAX_G = 64;     // shards
struct PartArgs {
    const uint32_t* owner;    // n: tm_tokens_shard's shard, or G = any shard
    const uint32_t* words;
    const uint32_t* toff;     // n + 1
    const uint8_t* tflags;
    uint32_t n, G, nb;        // nb = partition blocks
    uint32_t* cnt;            // [G * nb]: publishes of owner g in block b (g-major), scanned by launch_scan
    uint32_t* wcnt;           // [G * nb]: their words
    const uint32_t* cnt_off;  // scans of cnt / wcnt (two-level: off[i] + bsums[i / SCAN_TILE], total at [G * nb])
    const uint32_t* cnt_bs;
    const uint32_t* w_off;
    const uint32_t* w_bs;
    uint32_t* segs;           // [2 * (G + 1)]: first publish / first word of every owner's part, then the totals
    uint32_t* order;          // n: publish index (+ tbase) at each partitioned position
    uint32_t* ptoff;          // n + G: owner g's word offsets at [tseg[g] + g ..], relative to its part + wbase[g]
    uint8_t* ptflags;         // n
    uint32_t* pwords;
    uint32_t tbase;           // added to every publish index in order[] (the slice's first publish)
    uint32_t wbase[PART_MAX_G];   // added to owner g's word offsets (where its part lands in g's batch)
    // Direct delivery: owner g's part is written straight into g's batch
    // (same device, or a peer device over xGMI) at topic rbase[g] / word
    // wbase[g] instead of into ptoff / ptflags / pwords; null = kept here
    // (staged links, and the prepare-time plan)
    uint32_t* dtoff[PART_MAX_G];
    uint8_t* dflags[PART_MAX_G];
    uint32_t* dwords[PART_MAX_G];
    uint32_t rbase[PART_MAX_G];
};
hipError_t launch_part_count(const PartArgs& a, hipStream_t s);
hipError_t launch_part_segs(const PartArgs& a, hipStream_t s);
hipError_t launch_part_scatter(const PartArgs& a, hipStream_t s);
// A part batch's token buffers (etm::part_batch_buffers): the group's copies
// write a shard's part straight into them on `stream` (device `device`).
struct PartBuffers {
    uint32_t* words;
    uint32_t* toff;
    uint8_t* tflags;
    size_t words_cap;
    hipStream_t stream;
    int device;
};
// engine internals the sharded group (tm_shard.cpp) drives: a part batch with
// buffers of its own for n topics / nwords words (no host sync; the launch
// checks the tokens on the device), and the finish of a launched part after the
// caller has waited for its stream (*relaunched += capacity-miss relaunches,
// each with its own wait)
int part_batch_buffers(tm_engine* e, tm_batch** io, uint32_t n, uint64_t nwords, PartBuffers* out);
int part_batch_finish(tm_engine* e, tm_batch* b, uint32_t* relaunched);
// Host arrays still being staged by other threads (tm_sharded_prepare): the
// topic bytes in chunks of chunk_bytes (items [0, nbyte_items)), the rebased
// offsets in chunks of chunk_offs (items after); ready[item] turns 1 once the
// item is in place (release), bad turns true first when a staged topic fails
// its check.  The tokeniser uploads each chunk it needs as soon as it is ready
// (the DMA of one overlaps the copying of the next) and refuses to launch on a
// bad batch.
struct TokStaged {
    const uint8_t* ready;   // (read with __atomic_load_n, acquire)
    const bool* bad;
    uint64_t chunk_bytes, chunk_offs;
    uint32_t nbyte_items;
};
// tm_tokenize_device with the topic bytes [base, base + nbytes) of topics and
// the n + 1 offsets at offsets (absolute, offsets[0] == base once staged)
// taken from a staging in progress
int tokenize_device_staged(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint64_t base,
                           uint64_t nbytes, uint64_t off_item0, const TokStaged& st, uint32_t* d_words,
                           uint64_t words_cap, uint32_t* d_toff, uint8_t* d_tflags, uint64_t* nwords_out);
// un-partition: counts_o[order[p]] = counts_p[p]
hipError_t launch_unpart_counts(const uint32_t* order, const uint32_t* counts_p, uint32_t n, uint32_t* counts_o,
                                hipStream_t s);
// rows back in publish order: row p of ids_p (at scan(counts_p)[p]) -> out[scan(counts_o)[order[p]]],
// and the global CSR offsets rowg[order[p]] (rowg[n] = total)
hipError_t launch_unpart_rows(const uint32_t* order, const uint32_t* counts_p, uint32_t n, const uint32_t* src_off,
                              const uint32_t* src_bs, const uint32_t* dst_off, const uint32_t* dst_bs,
                              const uint32_t* ids_p, uint32_t* out, uint32_t* rowg, hipStream_t s);

// ------------------------------------------------------------ word dictionary
// One entry of the word interner's open-addressed table (emqx_topic:words/1
// tokens -> ids).  The host table is uploaded verbatim so the device tokeniser
// probes exactly the host's slots; word bytes live in an append-only arena.
struct DictEnt {
    uint64_t h;      // hash_word(bytes) | 1; 0 = empty
    uint64_t head;   // bytes 0..7 and 8..15, little-endian, zero-padded: words of up
    uint64_t head2;  // to 16 bytes compare without touching the arena
    uint32_t len;
    uint32_t id;
    uint64_t off;    // arena offset (longer words: bytes 16.. are compared there)
    uint64_t pad;
};
static_assert(sizeof(DictEnt) == 48, "dictionary entry is 48 bytes (three 16-B loads)");

// The device tokeniser's dictionary: a 2-choice cuckoo table of probe keys
// (a word lives in slot h1 & mask or h2 & mask: hash_word with seeds HW_SEED
// and HW_SEED2), so a
// lookup is two independent 16-B loads and no probe chain; head + len are the
// whole word up to 8 bytes, longer words also compare their DictTail (by id).
// Mirrored from the host interner (tm_engine_impl.hpp WordDict).
struct DictKey {
    uint64_t head;   // bytes 0..7, little-endian, zero-padded
    uint32_t len;
    uint32_t id;     // 0 = empty slot (ids start at W_FIRST)
};
struct DictTail {
    uint64_t head2;  // bytes 8..15, zero-padded
    uint64_t off;    // arena offset of the word (bytes 16.. are compared there)
};
static_assert(sizeof(DictTail) == 16, "dictionary tail is one 16-B load");
static_assert(sizeof(DictKey) == 16, "dictionary key is one 16-B load");

__host__ __device__ inline uint64_t le_bytes(const uint8_t* p, uint32_t n) {   // n <= 8
    uint64_t v = 0;
    for (uint32_t k = 0; k < n; ++k) v |= (uint64_t)p[k] << (8 * k);
    return v;
}

// Word hash of the dictionary (host interner and device tokeniser agree):
// murmur3-style 32-bit steps over the word's little-endian dwords (the tail
// zero-padded), the length mixed in at the end.  32-bit multiplies only: the
// device tokeniser hashes ~50M words per 10M publishes.  |1: 0 marks an empty
// table slot.  (Equality is decided by length + the inline 16 bytes + arena,
// never by the hash.)
__host__ __device__ inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
// one 4-byte chunk's mixing (seed-independent) and its accumulation: split
// so the device tokeniser computes both cuckoo hashes in one pass
__host__ __device__ inline uint32_t mix_chunk(uint32_t d) {
    d *= 0xCC9E2D51u;
    d = rotl32(d, 15);
    return d * 0x1B873593u;
}
__host__ __device__ inline uint32_t hw_acc(uint32_t h, uint32_t mixed) {
    h ^= mixed;
    h = rotl32(h, 13);
    return h * 5u + 0xE6546B64u;
}
__host__ __device__ inline uint32_t hw_step(uint32_t h, uint32_t d) { return hw_acc(h, mix_chunk(d)); }
__host__ __device__ inline uint32_t hw_final(uint32_t h, uint32_t n) {
    h ^= n;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h | 1u;
}
constexpr uint32_t HW_SEED = 0x9E3779B9u;
// the second cuckoo slot comes from an independent hash of the word (another
// seed): a function of h1 alone would put every word of a full-h1 collision
// triple on the same two slots, which no table size separates
constexpr uint32_t HW_SEED2 = 0x7F4A7C15u;

// Device tokenisation of a topic batch (bytes[offs[t] - base .. offs[t+1] - base)):
// the same words, classes, flags and ids as the host tokeniser (tm_batch.cpp
// tokenize_range), against the uploaded dictionary.
// One wavefront per tile of 64 topics: a tile's bytes are contiguous, so
// pass 1 counts the tile's words ('/' + 1 per topic) with coalesced loads,
// a scan over tiles gives each tile its first word, and pass 2 stages the
// tile's bytes in LDS, splits every topic there, looks its words up in the
// dictionary with the lookups spread over the lanes, and writes the tile's
// words with coalesced stores.
struct TokArgs {
    const uint8_t* bytes;
    const uint64_t* offs;     // n + 1 absolute offsets (caller's), minus base
    uint64_t base;
    uint32_t n;
    uint32_t pad0_;           // (explicit padding: the struct's bytes are a graph cache key)
    const DictKey* keys;      // cuckoo table of probe keys (DictKey)
    const DictTail* tails;    // by word id
    uint64_t dict_mask;       // cuckoo table size - 1 (power of two)
    const uint8_t* arena;
    uint32_t* wcount;         // pass 1: words per tile (ntiles + 1 entries), scanned in place
    uint8_t* tflags;
    uint32_t* toff;           // n + 1 word offsets
    const uint32_t* bsums;    // scan block offsets of the tile scan (tm_scan_sums)
    uint32_t* words;
    uint64_t words_cap;       // entries of words[]; nothing at or past it is written
    uint32_t* slow_list;
    uint32_t* d_nslow;        // [0] generic-path topics, [1] total words; zeroed by pass 1
    uint32_t* zero;           // optional: zero[0 .. zero_words) cleared by pass 1 (the batch's ctrl + stats)
    uint32_t zero_words;
    uint32_t tile_topics;     // topics per tokeniser tile (tok_tile_topics)
    const uint32_t* d_n;      // or null: the topic count is *d_n (<= n, the launch's bound): a
                              // device-deduplicated batch's rows
};
hipError_t launch_tokenize(const TokArgs& a, ScanArgs scan, uint32_t* d_nwords, hipStream_t s);
// topics per tokeniser tile for n topics of nbytes (64 unless topics are long)
uint32_t tok_tile_topics(uint32_t n, uint64_t nbytes);

// TM_BATCH_DEDUP on the device (tm_dedup_*), before the tokeniser:
// identical publishes (equal bytes) are tokenised and walked once.  A
// publish's representative is the FIRST publish with its bytes, so rows come
// out in first-occurrence order, deterministically -- the same rows as the
// host's dedup.  The representatives' bytes are compacted (cbytes / coffs) and
// only they are tokenised and walked; after the walk, tm_dedup_expand gives
// every publish its row (row_of) and its row's (count, start): the
// per-publish result.  Passes (tm_kernels.hip):
//   claim    every distinct topic of a workgroup claims one slot of the global
//            table {1 | tag | len | byte offset}, checking the bytes of any
//            occupant with its tag and length (exact: a slot holds one topic);
//            equal topics lower the offset to the first occurrence (offsets
//            grow with the publish index) -> slot[t]
//   count    representative bits (offset == the slot's) -> repbits, and
//            per 4,096-publish block the representatives and their bytes
//   (two scans of the block sums)
//   compact  each representative: its row, its bytes into cbytes, coffs,
//            srow[slot] = row and rrep[row] = the representative
//   rowmeta  (after the walk) each row's (count, start) into smeta at its
//            slot, and the slot cleared, so the table is zero for the next
//            pass
//   expand   every publish's (count, start) from smeta[slot[t]]: two
//            dependent reads instead of three (row_of[t] = srow[slot[t]] is
//            built only when the host asks for it)
struct DedupArgs {
    const uint8_t* bytes;     // the batch's publishes: bytes[offs[t] - base .. offs[t + 1] - base)
    const uint64_t* offs;
    uint64_t base;
    uint32_t n;
    uint32_t pad0_;           // (explicit padding: the struct's bytes are a graph cache key)
    unsigned long long* table;   // mask + 1 slots, zero between passes
    uint64_t mask;
    uint32_t* slot;           // n: the table slot of each publish's topic
    unsigned long long* repbits;  // ceil(n / 64): bit t = publish t is its topic's representative
    uint32_t* bcount;         // nblk + 1: representatives per DD_TILE block; scanned in place -> row bases
    uint32_t* bbytes;         // nblk + 1: their bytes; scanned in place -> byte bases
    const uint32_t* rbs;      // block sums of the two scans (SCAN_TILE entries per block)
    const uint32_t* bbs;
    uint32_t* srow;           // mask + 1: per claimed slot, its row
    uint32_t* rrep;           // n: per row, its representative publish
    uint32_t* row_of;         // n: row of each publish (tm_dedup_rowof, when the host asks)
    uint4* smeta;             // mask + 1: per claimed slot, its row's (count, 0, start lo, start hi)
    uint8_t* cbytes;          // the rows' bytes, the tokeniser's input (16-B aligned, + 32 bytes of slack)
    uint64_t* coffs;          // rows + 1 offsets into cbytes
    uint32_t* dd;             // [0] rows: the tokeniser's and the walk's topic count (TokArgs / MatchArgs d_n)
    // after the walk
    uint32_t* ctrl;           // CTRL_NROWS for the host (written with the expansion: every launch)
    const uint32_t* count;    // per row
    const unsigned long long* src;
    uint32_t* pcount;         // n: per publish
    unsigned long long* psrc;
    unsigned long long* bsum;  // the expansion's per-block sums of delivered matches
    unsigned long long* stats;
    uint32_t weak_hash;       // test knob (TM_DEDUP_WEAK_HASH): hash = length only, every same-length
                              // topic collides -- exercises the claim's byte check and probing
    uint32_t pad1_;
};
constexpr uint32_t DD_TILE = 1024;   // publishes per count / compact block
constexpr uint32_t DD_EXPAND_TILE = 2048;   // publishes per expansion block (one partial sum each)
constexpr uint32_t DD_OFF_BITS = 40; // byte offset bits of a table slot (a batch's bytes < 2^40)
__host__ __device__ inline uint32_t dedup_blocks(uint32_t n) { return (n + DD_TILE - 1) / DD_TILE; }
hipError_t launch_dedup(const DedupArgs& a, ScanArgs rows_scan, ScanArgs bytes_scan, hipStream_t s);
hipError_t launch_dedup_expand(const DedupArgs& a, hipStream_t s);
hipError_t launch_dedup_rowof(const DedupArgs& a, hipStream_t s);
// A captured launch is keyed by the bytes of its argument structs
// (tm_batch.cpp launch / launch_graph): no implicit padding, so equal
// arguments always give equal keys (the pads are members, zeroed by `{}`)
static_assert(std::has_unique_object_representations_v<MatchArgs>, "MatchArgs has implicit padding");
static_assert(std::has_unique_object_representations_v<ScanArgs>, "ScanArgs has implicit padding");
static_assert(std::has_unique_object_representations_v<TokArgs>, "TokArgs has implicit padding");
static_assert(std::has_unique_object_representations_v<DedupArgs>, "DedupArgs has implicit padding");

// tm_export_host: an async batch's per-topic results and rows -> pinned host memory
struct ExportArgs {
    const uint32_t* hdr;      // batch header block (ctrl | stats | src ...), as u32
    uint64_t hdr_words;       // u32 words of it to copy: ctrl + stats + src[n]
    uint32_t* h_hdr;          // device-visible pointers of the pinned destinations
    const uint32_t* count;
    uint32_t* h_count;
    uint64_t n;
    const uint32_t* rows;     // staging area
    uint32_t* h_rows;
    uint64_t rows_cap;        // entries h_rows holds
    uint64_t rcap;            // entries per group region of the staging area
    // or null: the batch's topic count is *d_n (a bounded batch, n above is
    // its bound): hdr_words = fixed_words + 2 * n and the counts follow it
    const uint32_t* d_n;
    uint64_t fixed_words;
};
static_assert(std::has_unique_object_representations_v<ExportArgs>, "ExportArgs has implicit padding");
hipError_t launch_export_host(const ExportArgs& a, hipStream_t s);
// ids[0..n) (each < 2^24) packed little-endian 3 bytes each into out (3n bytes)
hipError_t launch_pack_ids(const uint32_t* ids, uint64_t n, uint8_t* out, hipStream_t s);
// the dense CSR of a batch into device-visible pinned host memory: row_off[0..n]
// and ids[0 .. min(*d_total, cap)) (tm_match_batch: one host wait per batch)
hipError_t launch_csr_to_host(const uint32_t* row_off, const uint32_t* ids, uint32_t n, const uint32_t* d_total,
                              uint64_t cap, uint32_t* h_row, uint32_t* h_ids, hipStream_t s);
// dirty cuckoo slots -> the device table
hipError_t launch_scatter_keys(DictKey* keys, const uint32_t* idx, const DictKey* vals, uint32_t n, hipStream_t s);

// shard of a (w0, w1) literal prefix; host and device agree (tm_filter_shard)
__host__ __device__ inline uint32_t prefix_shard(uint32_t id0, uint32_t id1, uint32_t nshards) {
    return edge_hash(id0, id1) % nshards;
}
// workgroups (one wave each) of tm_match_tiles for n topics on this device:
// min(tiles, resident capacity), so that every wave is resident from the start
uint32_t match_waves(uint32_t n, int device, uint32_t qcap);
uint32_t tile_topics(uint32_t n);

// Every environment knob the engine reads, in one place (INTEGRATION.md lists
// them).  Read once per engine at tm_create (tests set them around an
// engine's creation) and per sharded group at tm_sharded_create.
struct Knobs {
    // test / debug knobs
    bool checked = false;          // TM_CHECKED=1: bounds-checked kernel variants
    bool no_graph = false;         // TM_NO_GRAPH=1: no captured HIP graphs
    bool par_trace = false;        // TM_PAR_TRACE: per-phase churn timings on stderr
    bool dedup_weak_hash = false;  // TM_DEDUP_WEAK_HASH=1: the dedup's hash degraded to the length
    int row_cap = 0;               // TM_ROWCAP: fast-path row slots per topic (1..128)
    uint32_t slow_lds = 0;         // TM_SLOW_LDS: generic-path LDS stack entries (small: forces the global restart)
    uint64_t fan_big = 0;          // TM_FAN_BIG: fan-out scan blocks above this use u64 offsets
    uint64_t result_limit = 0;     // TM_RESULT_LIMIT: matches per batch
    uint64_t staging_min = 0;      // TM_STAGING_MIN: initial staging entries of a batch
    std::string shard_link;        // TM_SHARD_LINK (staged | peer | probe), TM_SHARD_STAGED=1
    // deployment knobs
    unsigned host_threads = 0;     // TM_HOST_THREADS: host workers when tm_config.host_threads is 0
    bool pool_pin = true;          // TM_POOL_PIN=0: workers not pinned to the GPU's NUMA node
    int async_depth = 0, async_completers = 0, async_spin_us = -1;   // TM_ASYNC_DEPTH / _COMPLETERS / _SPIN_US

    static Knobs read() {
        Knobs k;
        auto env = [](const char* n) { return getenv(n); };
        auto on = [&](const char* n) { const char* v = env(n); return v && atoi(v) != 0; };
        k.checked = on("TM_CHECKED");
        k.no_graph = on("TM_NO_GRAPH");
        k.par_trace = env("TM_PAR_TRACE") != nullptr;
        k.dedup_weak_hash = on("TM_DEDUP_WEAK_HASH");
        if (const char* v = env("TM_ROWCAP")) k.row_cap = std::min(128, std::max(1, atoi(v)));
        if (const char* v = env("TM_SLOW_LDS")) k.slow_lds = (uint32_t)std::max(1, atoi(v));
        if (const char* v = env("TM_FAN_BIG")) k.fan_big = std::min<uint64_t>(0xFFFFFFFFull, strtoull(v, nullptr, 10));
        if (const char* v = env("TM_RESULT_LIMIT")) k.result_limit = strtoull(v, nullptr, 10);
        if (const char* v = env("TM_STAGING_MIN")) k.staging_min = std::max<uint64_t>(64, strtoull(v, nullptr, 10));
        if (on("TM_SHARD_STAGED")) k.shard_link = "staged";
        else if (const char* v = env("TM_SHARD_LINK")) k.shard_link = v;
        if (const char* v = env("TM_HOST_THREADS")) k.host_threads = (unsigned)std::min(std::max(atoi(v), 0), 64);
        if (const char* v = env("TM_POOL_PIN")) k.pool_pin = v[0] != '0';
        if (const char* v = env("TM_ASYNC_DEPTH")) k.async_depth = std::min(16, std::max(1, atoi(v)));
        if (const char* v = env("TM_ASYNC_COMPLETERS")) k.async_completers = std::min(8, std::max(1, atoi(v)));
        if (const char* v = env("TM_ASYNC_SPIN_US")) k.async_spin_us = std::min(10000, std::max(0, atoi(v)));
        return k;
    }
};

}  // namespace etm
