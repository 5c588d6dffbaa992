// tm_kernels.hip -- gfx950 (CDNA4) kernels of the topic-matching engine.
//
// The reference walk is emqx_trie:match/1 -> match_node/3 (src/emqx_trie.erl:
// 96-99, 162-186): per visited node, emit its '#' child's topic, then follow the
// literal word and the '+' edge; at the end of the words emit the node's own
// topic and its '#' child's.  Here that recursion becomes a frontier expansion:
//
//   tm_match_tiles  one 64-lane wavefront owns a TILE of 64 topics.  Pending
//                   edge probes of all 64 topics live in an LDS stack; every
//                   iteration pops up to 64 of them (one per lane), each lane
//                   reads ONE 64-B hash bucket whose matching 16-B slot holds the
//                   child's whole summary, and the lanes push their children
//                   through ballot + mbcnt prefix sums.  Each match is one u64
//                   (3-bit-per-level path code | filter id) stored into the
//                   topic's row of the wave's private emission buffer; path-code
//                   order == Erlang binary order of the filters (DESIGN.md "Sort
//                   order").  When the tile's frontier is empty the wave sorts
//                   its 64 rows in registers (bitonic over __shfl_xor) and
//                   stages the filter ids as ONE contiguous run per tile.
//   tm_match_slow   one wavefront per topic, frontier in global scratch: deep
//                   (> 10 levels) or irregular topics (sorted by filter bytes),
//                   rows longer than K and tiles whose LDS stack overflowed.
//   scan            exclusive scan of the per-topic counts -> CSR offsets.
//   tm_finalize     one wave per tile: a tile's staged run is copied into the
//                   CSR with coalesced loads/stores (per-topic copy for tiles
//                   holding slow-path topics).
//
// No MFMA: this is a dependent irregular gather, bound by the memory system.
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include "tm_internal.hpp"

namespace etm {

constexpr int TILE = 64;
constexpr int WCAP = 512;   // LDS word cache per tile
#ifndef TM_WPE384
#define TM_WPE384 4         // waves/SIMD the 384-entry-stack kernel is register-allocated for
#endif

// queue/meta encoding (fast path): tl (6 bits) | lc << 6 (4 bits, lc <= FAST_MAX_DEPTH) | flags.
// It rides in the low 31 bits of the probe's path-code key, which are zero
// until a filter id is put there at emission.
constexpr uint32_t M_LVL_SHIFT = 6;
constexpr uint32_t M_LVL_MASK = 0xF;
constexpr uint32_t M_PLUS = 1u << 10;    // probe the '+' edge (else the literal word w[lc-1])
constexpr uint32_t M_SKIPE = 1u << 11;   // don't emit the child's own topic (literal '#' dup)
constexpr uint32_t M_DSTART = 1u << 12;  // $-rooted start probe: the node was already counted
static_assert(FAST_MAX_DEPTH <= (int)M_LVL_MASK, "level field too narrow");
constexpr uint32_t M_DISP_SHIFT = 13;    // bucket displacement of a continued probe (<= max_probe <= 48)
constexpr uint32_t M_DISP_MASK = 0x3F;
// probe-entry marks written by the quad: FOUND | the child's literal signature
// into the parent field, TAIL into the word field (never a parent / word id)
constexpr uint32_t Q_FOUND = ~((1u << LSIG_BITS) - 1u);
constexpr uint32_t Q_TAIL = 0xFFFFFFFFu;

// digit tables indexed by class (C_BELOW, C_BETWEEN, C_ABOVE, C_EMPTY):
//   L = literal branch, H = '#' terminal, P = '+' branch; E = 0, L_lo = 1.
__device__ __forceinline__ uint32_t dig_L(uint32_t c) { return (0x4432u >> (4 * c)) & 0xF; }
__device__ __forceinline__ uint32_t dig_H(uint32_t c) { return (0x2223u >> (4 * c)) & 0xF; }
__device__ __forceinline__ uint32_t dig_P(uint32_t c) { return (0x3344u >> (4 * c)) & 0xF; }

__device__ __forceinline__ int key_shift(uint32_t level) { return 61 - 3 * (int)level; }

__device__ __forceinline__ uint64_t put_digit(uint64_t key, uint32_t level, uint32_t d) {
    return level <= FAST_MAX_DEPTH ? (key | ((uint64_t)d << key_shift(level))) : key;
}

__device__ __forceinline__ uint32_t prefix_count(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Bounds-checked debug variant: an out-of-range index is recorded (first
// failing check id, index, bound) and clamped to 0 instead of faulting.
template <bool CK>
__device__ __forceinline__ uint64_t ck(uint64_t i, uint64_t bound, uint32_t* dbg, uint32_t id) {
    if (CK && i >= bound) {
        if (dbg) {
            if (atomicCAS(&dbg[0], 0u, id) == 0u) { dbg[1] = (uint32_t)i; dbg[2] = (uint32_t)bound; }
            atomicAdd(&dbg[3], 1u);
        }
        return 0;
    }
    return i;
}
#define CK_(i, bound, id) ck<CK>((i), (bound), a.dbg, (id))

// Child summary decoded from one slot.
struct Node {
    uint32_t child;   // node id
    uint32_t term;    // own filter id or NONE
    uint32_t hterm;   // filter id of child/'#' or NONE
    uint32_t flags;   // NF_*
};

// One 64-B bucket read (four 16-B slots, key compare).  max_probe bounds the scan.
// Tables under 4 GiB are read with raw buffer loads (a wave-uniform descriptor
// built from kernel arguments): four dwordx4 that the compiler cannot narrow,
// issued back to back.  Larger tables use plain global loads.
#ifndef TM_PROBE_CPOL
#define TM_PROBE_CPOL 0     // cache-policy bits of the bucket loads (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
#endif
__device__ __forceinline__ uint4 ld_b128(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, TM_PROBE_CPOL);
    return uint4{v[0], v[1], v[2], v[3]};
}

template <bool CK, bool BIG>
__device__ __forceinline__ bool probe(const MatchArgs& a, uint32_t parent, uint32_t word, Node& n) {
    uint32_t b = home_bucket(parent, word, a.nbuckets);
    const bool small = !BIG;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<Slot*>(a.slots), 0, BIG ? 0u : a.nslots * 16u, 0x00020000);
    for (uint32_t p = 0; p <= a.max_probe; ++p) {
        uint4 s0, s1, s2, s3;
        const uint64_t si = CK_((uint64_t)b * BUCKET, a.nslots, 1);
        if (small) {
            const uint32_t off = (uint32_t)si * 16u;
            s0 = ld_b128(rs, off); s1 = ld_b128(rs, off + 16); s2 = ld_b128(rs, off + 32); s3 = ld_b128(rs, off + 48);
        } else {
            const uint4* q = reinterpret_cast<const uint4*>(a.slots) + si;
            s0 = q[0]; s1 = q[1]; s2 = q[2]; s3 = q[3];
        }
        // (the key's top bits are the child's literal signature)
        const bool m0 = (s0.x & ID_MASK) == parent && (s0.y & WID_MASK) == word;
        const bool m1 = (s1.x & ID_MASK) == parent && (s1.y & WID_MASK) == word;
        const bool m2 = (s2.x & ID_MASK) == parent && (s2.y & WID_MASK) == word;
        const bool m3 = (s3.x & ID_MASK) == parent && (s3.y & WID_MASK) == word;
        const uint32_t hz = m0 ? s0.z : m1 ? s1.z : m2 ? s2.z : s3.z;
        const uint32_t hw = m0 ? s0.w : m1 ? s1.w : m2 ? s2.w : s3.w;
        if (m0 | m1 | m2 | m3) {
            n.child = hz & ID_MASK;
            n.term = (hz & B_TOPIC) ? n.child : NONE;
            n.hterm = (hw & B_HTERM) ? (hw & ID_MASK) : NONE;
            n.flags = ((hz & B_PLUS) ? NF_PLUS : 0u) | ((hw & B_HASH) ? NF_HASH : 0u);
            return true;
        }
        if (s3.x == SLOT_EMPTY) return false;   // slots fill in order: a free tail ends the run
        b = (b + 1 == a.nbuckets) ? 0 : b + 1;
    }
    return false;
}

// Expansion of one found child at level lc (= words consumed), mirroring
// match_node/3: at the end of the words the node's own topic and its '#'
// child's (src/emqx_trie.erl:168-169); otherwise the '#' child's topic, then the
// literal and '+' probes (:171-177).
struct Expand {
    uint32_t ne, np;
    uint32_t ef0, ef1;
    uint64_t ek0, ek1;
    uint32_t pf0, pf1;     // M_PLUS / M_SKIPE / M_DSTART
    uint64_t pk0, pk1;
};

__device__ __forceinline__ void add_e(Expand& x, uint32_t fid, uint64_t key) {
    if (x.ne == 0) { x.ef0 = fid; x.ek0 = key; } else { x.ef1 = fid; x.ek1 = key; }
    x.ne++;
}
__device__ __forceinline__ void add_p(Expand& x, uint64_t key, uint32_t fl) {
    if (x.np == 0) { x.pk0 = key; x.pf0 = fl; } else { x.pk1 = key; x.pf1 = fl; }
    x.np++;
}

__device__ __forceinline__ void expand(const Node& s, uint32_t lc, uint32_t d, uint32_t flags,
                                       uint64_t key, uint32_t w_here, uint32_t w_prev, Expand& x) {
    x.ne = 0; x.np = 0;
    if (lc == d) {
        if (!(flags & M_SKIPE) && s.term != NONE) {
            uint64_t k = key;
            // '' word at level lc-1 followed by the end: "P/" sorts before "P/#".
            if ((w_prev >> WID_BITS) == C_EMPTY && lc - 1 <= FAST_MAX_DEPTH) {
                const int sp = key_shift(lc - 1);
                if (((k >> sp) & 7) == 4) k = (k & ~(7ull << sp)) | (1ull << sp);
            }
            add_e(x, s.term, k);
        }
        if (s.hterm != NONE) add_e(x, s.hterm, put_digit(key, lc, 2));
        return;
    }
    const uint32_t cls = w_here >> WID_BITS, id = w_here & WID_MASK;
    if (s.hterm != NONE) add_e(x, s.hterm, put_digit(key, lc, dig_H(cls)));
    if (id == W_HASH) {
        if (s.flags & NF_HASH) add_p(x, put_digit(key, lc, dig_L(cls)), (lc + 1 == d) ? M_SKIPE : 0u);
    } else if (id != W_UNKNOWN && id != W_PLUS) {
        add_p(x, put_digit(key, lc, dig_L(cls)), 0u);
    }
    if (s.flags & NF_PLUS) add_p(x, put_digit(key, lc, dig_P(cls)), M_PLUS);
}

// Root expansion for a topic (match_node(root, Words), or the $ rule that
// starts at node W and never tries root's '+'/'#', src/emqx_trie.erl:162-166).
__device__ __forceinline__ void expand_root(const RootRec& r, bool dollar, uint32_t d, uint32_t w0, Expand& x) {
    x.ne = 0; x.np = 0;
    const uint32_t cls = w0 >> WID_BITS, id = w0 & WID_MASK;
    if (!dollar && r.hterm != NONE) add_e(x, r.hterm, (uint64_t)dig_H(cls) << 61);
    if (id == W_HASH) {
        if (!dollar && (r.flags & NF_HASH)) add_p(x, (uint64_t)dig_L(cls) << 61, (d == 1) ? M_SKIPE : 0u);
    } else if (id != W_UNKNOWN && id != W_PLUS) {
        add_p(x, (uint64_t)dig_L(cls) << 61, dollar ? M_DSTART : 0u);
    }
    if (!dollar && (r.flags & NF_PLUS)) add_p(x, (uint64_t)dig_P(cls) << 61, M_PLUS);
}

// Per-wave LDS of the tile kernel.  The probe stack holds QC 16-B entries
// {key lo | meta, key hi, parent, word to probe (the literal w[lc-1] or
// W_PLUS / W_HASH)}: one ds_write_b128 per push, one ds_read_b128 per pop.
template <int QC>
struct alignas(16) TileLds {
    static constexpr int QCAP = QC;
    uint4 q[QC];
    uint32_t words[WCAP];
    uint32_t toff[TILE];
    uint32_t depth[TILE];
    uint32_t cnt[TILE];
    uint32_t list[TILE];
    // the stack and the word cache are free once a tile's frontier is empty: the
    // epilogue reuses them as a staging area of STAGE u64
    static constexpr uint32_t STAGE = (QC * 16 + WCAP * 4) / 8;
};

__device__ __forceinline__ uint4 q_pack(uint64_t key, uint32_t meta, uint32_t parent, uint32_t pw) {
    return uint4{(uint32_t)key | meta, (uint32_t)(key >> 32), parent, pw};
}

static_assert(offsetof(TileLds<512>, words) + sizeof(uint32_t) * WCAP == TileLds<512>::STAGE * 8,
              "staging area must be contiguous");
static_assert(offsetof(TileLds<384>, words) + sizeof(uint32_t) * WCAP == TileLds<384>::STAGE * 8,
              "staging area must be contiguous");

// Lane exchange with lane ^ j in VALU (no LDS crossbar): DPP quad_perm for 1
// and 2, row_half_mirror + quad reverse for 4, row_ror:8 for 8, and gfx950's
// v_permlane16/32_swap for 16 and 32.  j is a compile-time constant after the
// bitonic loops unroll, so the switch folds (tools/shx_check.hip checks all six).
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v, uint32_t j) {
    const uint32_t lane = threadIdx.x & 63;
    switch (j) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    case 4: return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false), 0x1B, 0xF,
                                                      0xF, false);
    case 8: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
    case 16: {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? p[0] : p[1];
    }
    default: {
        const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? p[0] : p[1];
    }
    }
}

__device__ __forceinline__ unsigned long long xor_lane64(unsigned long long v, uint32_t j) {
    return ((unsigned long long)xor_lane32((uint32_t)(v >> 32), j) << 32) | xor_lane32((uint32_t)v, j);
}

// Tile epilogue: sort the 64 rows of this wave and write their filter ids to
// sfids[dst .. dst + c).  The rows are pulled into LDS a chunk of whole rows at
// a time (at most STAGE elements), eight rows per batch of independent loads:
// the rows were written moments ago but have usually left L2, so a dependent
// load per sort group would pay full memory latency ~20 times per tile.  Rows
// of size class W (W/2 < c <= W, W = 2..64) are then packed 64/W per
// wave-instruction, one element per lane, and sorted by a W-wide bitonic
// network of __shfl_xor exchanges.  65..128 elements: rank count, two per lane.
template <bool CK, class LT>
__device__ __forceinline__ void sort_classes(const MatchArgs& a, LT& L, bool keep, uint32_t c, uint32_t pos,
                                             uint32_t dst) {
    constexpr uint32_t STAGE = LT::STAGE;
    const uint32_t lane = threadIdx.x;
    const unsigned long long* stg = reinterpret_cast<const unsigned long long*>(L.q);
    if (keep && c == 1) a.sfids[CK_(dst, a.sfids_cap, 40)] = (uint32_t)(stg[CK_(pos, STAGE, 41)] & ~KEY_MASK);
#pragma unroll
    for (uint32_t W = 2; W <= 64; W <<= 1) {
        const bool mine = keep && c > W / 2 && c <= W;
        const uint64_t m = __ballot(mine);
        if (!m) continue;
        const uint32_t nrows = __popcll(m);
        if (mine) L.list[prefix_count(m)] = lane;
        __syncthreads();
        const uint32_t e = lane & (W - 1);
        const uint32_t STEP = 64 / W;
        for (uint32_t g = 0; g < nrows; g += STEP) {
            const uint32_t r = g + lane / W;
            const bool rv = r < nrows;
            const uint32_t owner = rv ? L.list[r] : 0u;
            const uint32_t cr = __shfl(c, owner, 64);
            const uint32_t pr = __shfl(pos, owner, 64);
            const uint32_t dr = __shfl(dst, owner, 64);
            unsigned long long key = ~0ull;
            if (rv && e < cr) key = stg[CK_(pr + e, STAGE, 42)];
#pragma unroll
            for (uint32_t kk = 2; kk <= W; kk <<= 1) {
#pragma unroll
                for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
                    const unsigned long long other = xor_lane64(key, j);
                    const bool up = (e & kk) == 0;
                    const bool lower = (e & j) == 0;
                    const unsigned long long lo = key < other ? key : other;
                    const unsigned long long hi = key < other ? other : key;
                    key = (lower == up) ? lo : hi;
                }
            }
            if (rv && e < cr) a.sfids[CK_((uint64_t)dr + e, a.sfids_cap, 44)] = (uint32_t)(key & ~KEY_MASK);
        }
        __syncthreads();
    }
    {
        const bool mine = keep && c > 64;
        uint64_t m = __ballot(mine);
        while (m) {
            const uint32_t owner = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t cr = __shfl(c, owner, 64);
            const uint32_t pr = __shfl(pos, owner, 64);
            const uint32_t dr = __shfl(dst, owner, 64);
            unsigned long long k0 = ~0ull, k1 = ~0ull;
            if (lane < cr) k0 = stg[CK_(pr + lane, STAGE, 45)];
            if (lane + 64 < cr) k1 = stg[CK_(pr + lane + 64, STAGE, 46)];
            uint32_t r0 = 0, r1 = 0;
            for (uint32_t j = 0; j < 64; ++j) {
                const unsigned long long kj = __shfl(k0, j, 64);
                r0 += kj < k0 ? 1u : 0u;
                r1 += kj < k1 ? 1u : 0u;
            }
            for (uint32_t j = 64; j < cr; ++j) {
                const unsigned long long kj = __shfl(k1, j - 64, 64);
                r0 += kj < k0 ? 1u : 0u;
                r1 += kj < k1 ? 1u : 0u;
            }
            if (lane < cr) a.sfids[CK_((uint64_t)dr + r0, a.sfids_cap, 47)] = (uint32_t)(k0 & ~KEY_MASK);
            if (lane + 64 < cr) a.sfids[CK_((uint64_t)dr + r1, a.sfids_cap, 48)] = (uint32_t)(k1 & ~KEY_MASK);
        }
    }
}

#ifndef TM_LOG_U
#define TM_LOG_U 12  // log entries per lane per read-back step, all in flight (4 / 8 / 12 / 16: 5.10 / 5.07 / 5.04 / 5.05 ms)
#endif
// Emission log epilogue: the tile's matches were appended
// to a wave-private log in iteration order (coalesced: one store of <= 64
// consecutive entries per emission role per iteration), each with its topic
// lane in a parallel byte log.  The rows are rebuilt in LDS a chunk of whole
// rows at a time -- the log is streamed (L2-resident: written moments ago)
// and every entry of a chunk's rows goes to its row's next free place -- and
// sorted as before.
template <bool CK, class LT>
__device__ __forceinline__ void sort_rows_log(const MatchArgs& a, LT& L, bool keep, uint32_t c, uint32_t dst,
                                              unsigned long long* wlog, uint8_t* wlane, uint32_t lcount) {
    constexpr uint32_t STAGE = LT::STAGE;
    const uint32_t lane = threadIdx.x;
    unsigned long long* stg = reinterpret_cast<unsigned long long*>(L.q);
    const uint32_t cw = keep ? c : 0u;
    uint32_t incl = cw;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += u;
    }
    const uint32_t pos = incl - cw;
    uint32_t rs = 0;
    while (rs < a.tile_topics) {
        const uint32_t p0 = __builtin_amdgcn_readlane(pos, rs);
        const uint64_t beyond = __ballot(lane >= rs && pos + cw - p0 > STAGE);
        const uint32_t re = beyond ? (uint32_t)__builtin_ctzll(beyond) : a.tile_topics;
        const bool in_chunk = keep && lane >= rs && lane < re;
        // (depth / toff are free after the frontier loop) row base in the
        // stage, NONE for rows not staged in this pass
        L.depth[lane] = in_chunk ? pos - p0 : NONE;
        L.toff[lane] = 0;                            // row fill cursor
        __syncthreads();
        for (uint32_t k0 = 0; k0 < lcount; k0 += 64 * TM_LOG_U) {
            unsigned long long e[TM_LOG_U];
            uint32_t r[TM_LOG_U];
#pragma unroll
            for (uint32_t u = 0; u < TM_LOG_U; ++u) {
                const uint32_t k = k0 + lane + 64 * u;
                r[u] = 64;
                if (k < lcount) {
                    e[u] = wlog[k];
                    r[u] = wlane[k];
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < TM_LOG_U; ++u) {
                const uint32_t base = r[u] < 64 ? L.depth[r[u]] : NONE;
                if (base == NONE) continue;
                const uint32_t at = base + atomicAdd(&L.toff[r[u]], 1u);
                stg[CK_(at, STAGE, 49)] = e[u];
            }
        }
        __syncthreads();
        sort_classes<CK, LT>(a, L, in_chunk, c, pos - p0, dst);
        __syncthreads();
        rs = re;
    }
}

template <bool CK>
__device__ __forceinline__ void send_to_slow(const MatchArgs& a, bool mine, uint32_t t) {
    const uint64_t m = __ballot(mine);
    uint32_t base = 0;
    if (threadIdx.x == 0 && m) base = atomicAdd(&a.ctrl[CTRL_NOVF], (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (mine) {
        const uint32_t slot = base + prefix_count(m);
        if (slot < a.ovf_cap) a.ovf_list[CK_(slot, a.ovf_cap, 12)] = t;
        else atomicOr(&a.ctrl[CTRL_ERR], ERR_OVF_LIST);
    }
}

// One tile.  IN_LDS: the tile's words are staged in LDS (the common case);
// otherwise they are read from HBM.  Templated so word reads are plain ds_read
// or global_load, never flat.
template <bool CK, bool BIG, bool IN_LDS, class LT>
__device__ __forceinline__ void match_tile(const MatchArgs& a, LT& L, uint32_t t0, uint32_t tend, uint32_t wbase,
                                           uint8_t fl, bool valid, unsigned long long& sV, unsigned long long& sH,
                                           unsigned long long& sW, unsigned long long& sM, unsigned long long& sP) {
    const uint32_t lane = threadIdx.x;
    const uint32_t t = t0 + lane;
    const uint32_t* wsrc = IN_LDS ? L.words : a.words;
    const uint32_t wlim = IN_LDS ? (uint32_t)WCAP : a.nwords;
    (void)wbase;

    uint32_t qn = 0;
    bool ovf = false;
    const bool active = !(fl & TF_SLOW);
    unsigned long long* const wrows = a.rows + (uint64_t)blockIdx.x * a.tile_topics * a.row_cap;
    // the wave's emission log: its rows region (entries) + a byte per entry
    // (topic lane) past the whole rows array
    const uint32_t lcap = a.tile_topics * a.row_cap;
    uint8_t* const wlane =
        reinterpret_cast<uint8_t*>(a.rows + (uint64_t)a.grid * lcap) + (uint64_t)blockIdx.x * lcap;
    uint32_t lcount = 0;
    uint32_t tV = 0, tH = 0, tW = 0, tP = 0;   // committed only if the tile does not overflow
    const uint32_t d_me = L.depth[lane];

    // ---- level 0: root expansion, one topic per lane
    {
        Expand x; x.ne = 0; x.np = 0;
        uint32_t w0 = 0;
        if (active && d_me > 0) {
            const bool dollar = fl & TF_DOLLAR;
            tV += 1;
            if (!dollar && (a.root.flags & NF_HASH)) tH += 1;
            tW += d_me;
            w0 = wsrc[CK_(L.toff[lane], wlim, 9)];
            expand_root(a.root, dollar, d_me, w0, x);
        }
        const uint64_t b0 = __ballot(x.np >= 1), b1 = __ballot(x.np >= 2);
        const uint32_t pre = prefix_count(b0) + prefix_count(b1);
        const uint32_t meta = lane | (1u << M_LVL_SHIFT);
        const uint32_t wid = w0 & WID_MASK;
        if (x.np >= 1) L.q[qn + pre] = q_pack(x.pk0, meta | x.pf0, ROOT, (x.pf0 & M_PLUS) ? W_PLUS : wid);
        if (x.np >= 2) L.q[qn + pre + 1] = q_pack(x.pk1, meta | x.pf1, ROOT, (x.pf1 & M_PLUS) ? W_PLUS : wid);
        qn += __popcll(b0) + __popcll(b1);
        const uint64_t mr = __ballot(x.ne != 0);
        if (x.ne) {   // at most one emission at the root ('#')
            L.cnt[lane] = 1;
            const uint32_t i = prefix_count(mr);
            wrows[i] = (x.ek0 & KEY_MASK) | x.ef0;
            wlane[i] = (uint8_t)lane;
        }
        lcount = (uint32_t)__popcll(mr);
    }

    // ---- frontier loop: LIFO stack, up to 64 probes per iteration
    //
    // Quad-cooperative probing: probe p (0..63) of an iteration is read by the
    // quad of lanes 4q..4q+3 in round r (p = 16r + q), each lane loading one
    // 16-B slot of the 64-B bucket, so a load instruction touches 16 cache
    // lines instead of 64 (one L1 tag lookup per probe instead of four: the
    // lookups, not the bytes, saturate the L1 at full occupancy).  The popped
    // entries stay in their LDS slots during the probe: the owner lane writes
    // the bucket index into its entry, the quads read it from there, and the
    // matching lane writes the slot's child summary back for the owner.  A key
    // that spilled past its home bucket is pushed again as a continuation
    // (displacement + 1) rather than holding the whole wave for a dependent read.
    const uint32_t qd = lane >> 2, qs = lane & 3;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<Slot*>(a.slots), 0, BIG ? 0u : a.nslots * 16u, 0x00020000);
    while (qn > 0) {
        const uint32_t k = min(qn, 64u);
        const bool has = lane < k;
        qn -= k;
        tP += lane == 0 ? k + (1u << 20) : 0u;   // bucket reads (hits, misses, continuations) | iterations << 20
        const uint32_t idx = qn + lane;
        uint4 e = uint4{0u, 0u, 0u, 0u};
        if (has) e = L.q[idx];
        const uint32_t meta = e.x & 0x7FFFFFFFu;
        const uint64_t key = ((uint64_t)e.y << 32) | (e.x & 0x80000000u);
        const uint32_t parent = e.z, pw = e.w;
        const uint32_t tl = meta & 63;
        const uint32_t lc = (meta >> M_LVL_SHIFT) & M_LVL_MASK;
        const uint32_t disp = (meta >> M_DISP_SHIFT) & M_DISP_MASK;
        if (has) {
            uint32_t hb = home_bucket(parent, pw, a.nbuckets) + disp;
            if (hb >= a.nbuckets) hb -= a.nbuckets;
            L.q[idx].x = hb;
        }
        uint32_t rp[4], rw[4];
        uint4 sl[4];
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const uint32_t p = 16 * r + qd;
            const bool v = p < k;
            const uint4 rec = L.q[qn + (v ? p : 0u)];
            rp[r] = v ? rec.z : SLOT_EMPTY;
            rw[r] = rec.w;
            const uint64_t si = CK_((uint64_t)rec.x * BUCKET + qs, a.nslots, 1);
            if (!BIG) {
                sl[r] = ld_b128(rsrc, v ? (uint32_t)si * 16u : 0xFFFFFFF0u);   // out of range: reads 0
            } else {
                sl[r] = v ? reinterpret_cast<const uint4*>(a.slots)[si] : uint4{0u, 0u, 0u, 0u};
            }
        }
        // the topic's words are read while the buckets are in flight (the
        // barrier keeps the compiler from hoisting these LDS reads, and their
        // waits, above the bucket loads)
        __builtin_amdgcn_sched_barrier(0);
        uint32_t d = 0, w_here = 0, w_prev = 0;
        if (has) {
            const uint32_t base = L.toff[tl];
            d = L.depth[tl];
            w_here = lc < d ? wsrc[CK_(base + lc, wlim, 11)] : 0u;
            w_prev = wsrc[CK_(base + lc - 1, wlim, 10)];
        }
        // The quad reports to the owner through the owner's LDS entry, not
        // through ballots: the matching lane writes the child summary and a
        // FOUND mark, the lane of the bucket's last slot a TAIL mark when that
        // slot is free (the probe run ends in this bucket).  Parent ids and
        // word ids never equal the marks.
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            const bool m = rp[r] != SLOT_EMPTY && (sl[r].x & ID_MASK) == rp[r] && (sl[r].y & WID_MASK) == rw[r];
            if (m) {
                L.q[qn + 16 * r + qd].x = sl[r].z;
                L.q[qn + 16 * r + qd].y = sl[r].w;
                L.q[qn + 16 * r + qd].z = Q_FOUND | slot_lsig(sl[r].x, sl[r].y);
            }
            if (qs == 3 && sl[r].x == SLOT_EMPTY) L.q[qn + 16 * r + qd].w = Q_TAIL;   // out-of-range loads read 0
        }
        uint4 res = uint4{0u, 0u, 0u, 0u};
        if (has) res = L.q[idx];
        // a row already longer than K goes to the generic path whole: its
        // entries are not expanded further (C5 K = 1000: ~10k rows of ~1,000
        // matches each stopped at K + 1 instead of walked to the end)
        const bool gone = has && L.cnt[tl] > a.row_cap;
        const bool found = has && !gone && res.z >= Q_FOUND;
        const bool cont = has && !gone && !found && res.w != Q_TAIL && disp < a.max_probe;
        Node s;
        s.child = 0; s.term = NONE; s.hterm = NONE; s.flags = 0;
        if (found) {
            const uint32_t hz = res.x, hw = res.y;
            s.child = hz & ID_MASK;
            s.term = (hz & B_TOPIC) ? s.child : NONE;
            s.hterm = (hw & B_HTERM) ? (hw & ID_MASK) : NONE;
            s.flags = ((hz & B_PLUS) ? NF_PLUS : 0u) | ((hw & B_HASH) ? NF_HASH : 0u);
        }
        // Expansion of the found node, match_node/3 (src/emqx_trie.erl:168-177),
        // with fixed roles instead of expand()'s packed lists: emissions A, B;
        // push L (the literal word, or the continuation) and push P ('+').
        // lc <= FAST_MAX_DEPTH here, so every level has a digit position.
        const bool at_end = lc == d;
        const uint32_t cls = w_here >> WID_BITS, id = w_here & WID_MASK;
        const int sh = key_shift(lc);
        bool eA = false, eB = false, pL = false, pP = false;
        uint32_t fA = 0;
        uint64_t kA = key;
        if (found) {
            if (!(meta & M_DSTART)) tV += 1;
            if (s.flags & NF_HASH) tH += 1;
            if (at_end) {   // end of the words: own topic, then the '#' child's
                eA = !(meta & M_SKIPE) && s.term != NONE;
                fA = s.term;
                // '' word at level lc-1 followed by the end: "P/" sorts before "P/#"
                if ((w_prev >> WID_BITS) == C_EMPTY) {
                    const int sp = key_shift(lc - 1);
                    if (((kA >> sp) & 7) == 4) kA = (kA & ~(7ull << sp)) | (1ull << sp);
                }
                eB = s.hterm != NONE;
            } else {        // '#' child's topic, then the literal and '+' edges
                eA = s.hterm != NONE;
                fA = s.hterm;
                kA = key | ((uint64_t)dig_H(cls) << sh);
                // a literal word whose signature bit is clear has no edge here
                // (and, for a node without a '#' child, its 30-bit signature)
                pL = id == W_HASH ? (s.flags & NF_HASH) != 0
                                  : (id != W_UNKNOWN && id != W_PLUS && ((res.z >> lsig_pos(id)) & 1u) &&
                                     ((res.y & B_HASH) || ((res.y >> lext_pos(id)) & 1u)));
                pP = (s.flags & NF_PLUS) != 0;
            }
        }
        const bool sL = cont || pL;
        const uint64_t bL = __ballot(sL), bP = __ballot(pP);
        const uint32_t ptot = __popcll(bL) + __popcll(bP);
        if (qn + ptot > (uint32_t)LT::QCAP) { ovf = true; break; }
        const uint32_t pre = qn + prefix_count(bL) + prefix_count(bP);
        const uint32_t nmeta = tl | ((lc + 1) << M_LVL_SHIFT);
        if (sL) {
            const uint32_t lfl = (id == W_HASH && lc + 1 == d) ? M_SKIPE : 0u;
            L.q[pre] = cont ? q_pack(key, meta + (1u << M_DISP_SHIFT), parent, pw)
                            : q_pack(key | ((uint64_t)dig_L(cls) << sh), nmeta | lfl, s.child, id);
        }
        if (pP) L.q[pre + (sL ? 1u : 0u)] = q_pack(key | ((uint64_t)dig_P(cls) << sh), nmeta | M_PLUS, s.child, W_PLUS);
        qn += ptot;
        {
            // row sizes; a row's entries past K are not logged (the row goes to
            // the generic path), so the log holds at most tile_topics * K
            uint32_t slot = 0;
            if (eA | eB) slot = atomicAdd(&L.cnt[tl], (eA ? 1u : 0u) + (eB ? 1u : 0u));
            const uint32_t slotB = slot + (eA ? 1u : 0u);
            eA = eA && slot < a.row_cap;
            eB = eB && slotB < a.row_cap;
            const uint64_t mA = __ballot(eA), mB = __ballot(eB);
            const uint32_t nA = (uint32_t)__popcll(mA), nE = nA + (uint32_t)__popcll(mB);
            if (eA) {
                const uint32_t i = lcount + prefix_count(mA);
                wrows[CK_(i, lcap, 13)] = (kA & KEY_MASK) | fA;
                wlane[i] = (uint8_t)tl;
            }
            if (eB) {
                const uint32_t i = lcount + nA + prefix_count(mB);
                wrows[CK_(i, lcap, 14)] = ((key | (2ull << sh)) & KEY_MASK) | s.hterm;
                wlane[i] = (uint8_t)tl;
            }
            lcount += nE;
        }
    }
    __syncthreads();

    if (ovf) {
        // probe stack overflow: every regular topic of the tile goes to the slow path
        send_to_slow<CK>(a, valid && active, t);
        return;
    }
    sV += tV; sH += tH; sW += tW;
    sP += (tP & 0xFFFFFu) | ((unsigned long long)(tP >> 20) << 40);   // probes | iterations << 40
    const uint32_t c_me = L.cnt[lane];
    const bool row_ovf = valid && active && c_me > a.row_cap;   // row longer than K
    send_to_slow<CK>(a, row_ovf, t);
    const bool keep = valid && active && !row_ovf;
    const uint32_t c = keep ? c_me : 0u;
    // one contiguous staging run per tile: exclusive scan of the counts
    uint32_t incl = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += u;
    }
    const uint32_t tot = __shfl(incl, 63, 64);
    // u64 ticket: a batch may reserve more than 2^32 entries; the host then
    // fails it with TM_EOVERFLOW (sfids_cap < 2^32, so dst below never wraps)
    unsigned long long base64 = 0;
    const uint32_t g = (blockIdx.x % TICKET_GROUPS) & a.sgmask;   // my group's staging region
    if (lane == 0 && tot) base64 = atomicAdd(xg_top(a.xg, g), (unsigned long long)tot);
    base64 = __shfl(base64, 0, 64);
    const bool fits = base64 + tot <= a.rcap;
    base64 += (uint64_t)g * a.rcap;
    const uint32_t base = (uint32_t)base64;
    const uint32_t dst = base + incl - c;
    if (fits) {
        sort_rows_log<CK, LT>(a, L, keep, c, dst, wrows, wlane, lcount);
    } else if (lane == 0) {
        atomicOr(&a.ctrl[CTRL_ERR], ERR_STAGING);   // host grows sfids[] and reruns
    }
    if (keep) {
        a.count[CK_(t, a.n, 16)] = c_me;
        a.src[CK_(t, a.n, 17)] = dst;
        sM += c_me;
    }
    (void)tend;
}

#ifndef TM_DN_TILES_PER_WAVE
#define TM_DN_TILES_PER_WAVE 4
#endif
// device-counted batches: tiles shrink until each wave has this many to take
constexpr uint32_t DN_TILES_PER_WAVE = TM_DN_TILES_PER_WAVE;

template <bool CK, bool BIG, int QC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(QC == 384 ? TM_WPE384 : 3, 8))) void tm_match_tiles(MatchArgs a) {
    __shared__ TileLds<QC> L;
    if (a.d_n) {
        // a device-deduplicated batch: its rows are counted on the device.
        // The grid was sized for the bound (every publish); tiles shrink
        // until the rows cover every wave (a C5 batch's ~186k rows would
        // otherwise be 2,900 tiles for 4,096 waves, the hot ones long)
        a.n = *a.d_n;
        while (a.tile_topics > 1 && (a.n + a.tile_topics - 1) / a.tile_topics < DN_TILES_PER_WAVE * gridDim.x)
            a.tile_topics >>= 1;
        // the host sized the static share for every publish: the rows take
        // half of their own tiles round-robin, the rest by tickets (a skewed
        // batch's hot rows come first, in the first tiles)
        const uint32_t nt = (a.n + a.tile_topics - 1) / a.tile_topics;
        a.static_rounds = max(1u, nt / (2u * gridDim.x));
    }
    const uint32_t lane = threadIdx.x;
    const uint32_t tt = a.tile_topics;   // topics per tile: 64, or fewer for small batches
    const uint32_t ntiles = (a.n + tt - 1) / tt;
    unsigned long long sV = 0, sH = 0, sW = 0, sM = 0, sP = 0;

    // static round-robin tiles, then tickets for the tail; a ticket is taken at
    // the start of a tile so its latency hides behind the tile's work
    uint32_t tile = blockIdx.x, round = 0;
    while (tile < ntiles) {
        // the next tile: round-robin for the first static_rounds, then from a
        // ticket (a contended counter's latency would stall every in-order vmcnt
        // wait of the tile, so only the tail balances by tickets, per XCD)
        uint32_t ticket = 0;
        if (round + 1 >= a.static_rounds && lane == 0)
            ticket = atomicAdd(&a.xg[(blockIdx.x % TICKET_GROUPS) * TICKET_STRIDE], 1u);
        const uint32_t t0 = tile * tt;
        const uint32_t tend = min(t0 + tt, a.n);
        const uint32_t t = t0 + lane;
        const bool valid = lane < tt && t < a.n;
        const uint32_t wbeg = a.toff[CK_(t0, a.n + 1, 2)], wend = a.toff[CK_(tend, a.n + 1, 3)];
        const bool in_lds = (wend - wbeg) <= (uint32_t)WCAP;
        const uint32_t my_off = valid ? a.toff[CK_(t, a.n + 1, 4)] : wend;
        const uint32_t my_end = valid ? a.toff[CK_(t + 1, a.n + 1, 5)] : wend;
        const uint8_t fl = valid ? a.tflags[CK_(t, a.n, 6)] : (uint8_t)TF_SLOW;
        if (in_lds)
            for (uint32_t i = lane; i < wend - wbeg; i += 64) L.words[CK_(i, WCAP, 7)] = a.words[CK_(wbeg + i, a.nwords, 8)];
        L.toff[lane] = in_lds ? my_off - wbeg : my_off;
        L.depth[lane] = my_end - my_off;
        L.cnt[lane] = 0;
        __syncthreads();
        if (in_lds) match_tile<CK, BIG, true>(a, L, t0, tend, wbeg, fl, valid, sV, sH, sW, sM, sP);
        else match_tile<CK, BIG, false>(a, L, t0, tend, wbeg, fl, valid, sV, sH, sW, sM, sP);
        __syncthreads();
        ++round;
        tile = round < a.static_rounds
                   ? blockIdx.x + round * gridDim.x
                   : a.static_rounds * gridDim.x + __builtin_amdgcn_readfirstlane(ticket) * TICKET_GROUPS +
                         blockIdx.x % TICKET_GROUPS;
    }

    for (int o = 32; o > 0; o >>= 1) {
        sV += __shfl_xor(sV, o, 64); sH += __shfl_xor(sH, o, 64);
        sW += __shfl_xor(sW, o, 64); sM += __shfl_xor(sM, o, 64);
        sP += __shfl_xor(sP, o, 64);
    }
    if (lane == 0 && a.wstats) {
        // the wave's sums, added up by tm_stats_reduce: ~4,000 waves ending
        // together would queue 6 same-line device atomics each (~30 ns apiece)
        unsigned long long* w = a.wstats + (uint64_t)blockIdx.x * WSTATS;
        w[0] = sV; w[1] = sH; w[2] = sW; w[3] = sM;
        w[4] = sP & ((1ull << 40) - 1); w[5] = sP >> 40;
    } else if (lane == 0) {
        atomicAdd(&a.stats[ST_VISITS], sV); atomicAdd(&a.stats[ST_HASH], sH);
        atomicAdd(&a.stats[ST_WORDS], sW); atomicAdd(&a.stats[ST_MATCHES], sM);
        atomicAdd(&a.stats[ST_PROBES], sP & ((1ull << 40) - 1));
        atomicAdd(&a.stats[ST_ITERS], sP >> 40);
    }
}

// the walk waves' sums -> the batch's stats (one block; after the walk)
__global__ __launch_bounds__(256) void tm_stats_reduce(const unsigned long long* w, uint32_t waves,
                                                       unsigned long long* stats) {
    __shared__ unsigned long long sh[4][6];
    unsigned long long v[6] = {0, 0, 0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < waves; i += 256)
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k) v[k] += w[(uint64_t)i * WSTATS + k];
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) {
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const uint32_t k = threadIdx.x;
        const unsigned long long t = sh[0][k] + sh[1][k] + sh[2][k] + sh[3][k];
        const uint32_t idx[6] = {ST_VISITS, ST_HASH, ST_WORDS, ST_MATCHES, ST_PROBES, ST_ITERS};
        if (t) atomicAdd(&stats[idx[k]], t);
    }
}

// ---------------------------------------------------------------- slow path

// Erlang binary order on two filters (unsigned bytes, shorter prefix first).
template <bool CK>
__device__ __forceinline__ bool filter_less(const MatchArgs& a, uint32_t x, uint32_t y) {
    if (x == NONE) return false;
    if (y == NONE) return true;
    x = CK_(x, a.nnodes, 20); y = CK_(y, a.nnodes, 21);
    const uint8_t* px = a.fbytes + CK_(a.foff[x], a.nfbytes + 1, 22);
    const uint8_t* py = a.fbytes + CK_(a.foff[y], a.nfbytes + 1, 23);
    const uint32_t lx = a.flen[x], ly = a.flen[y];
    const uint32_t m = min(lx, ly);
    for (uint32_t i = 0; i < m; ++i)
        if (px[i] != py[i]) return px[i] < py[i];
    return lx < ly;
}

// Bitonic sort of n (power of two) (key, fid) pairs held at kp/fp (LDS or global).
template <bool CK>
__device__ void bitonic(const MatchArgs& a, unsigned long long* kp, uint32_t* fp, uint32_t n, bool by_bytes) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < n; i += 64) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const bool up = (i & k) == 0;
                    const bool gt = by_bytes ? filter_less<CK>(a, fp[ixj], fp[i]) : (kp[i] > kp[ixj]);
                    if (gt == up) {
                        const unsigned long long tk = kp[i]; kp[i] = kp[ixj]; kp[ixj] = tk;
                        const uint32_t tf = fp[i]; fp[i] = fp[ixj]; fp[ixj] = tf;
                    }
                }
            }
            __threadfence_block();
            __syncthreads();
        }
    }
}

// Generic path LDS: the probe stack while a topic is walked (SLOW_SQ 16-B
// entries {parent, meta, key lo, key hi}), then the same 8 KB as the row's
// sort area: 1,024 u64 (path code | filter id) or 2,048 u32 filter ids (rows
// ordered by bytes); a path-coded row of up to 2,048 sorts as two LDS runs
// merged on the way out (merge_runs_out).  A topic whose frontier outgrows the
// stack restarts in global scratch.  The walk is a chain of dependent probes
// per row, so the waves per CU set its pace: 8 KB of LDS per wave allows 20
// (16 KB: 10).
#ifndef TM_SLOW_SQ
#define TM_SLOW_SQ 512
#endif
constexpr uint32_t SLOW_SQ = TM_SLOW_SQ;
constexpr uint32_t SORT_LDS = SLOW_SQ * 2;    // u64 entries of the sort area
constexpr uint32_t SM_PLUS = 1u << 29;
constexpr uint32_t SM_SKIPE = 1u << 30;
constexpr uint32_t SM_DSTART = 1u << 31;
constexpr uint32_t SM_LVL = (1u << 29) - 1;

__device__ __forceinline__ uint32_t slow_flags(uint32_t pf) {
    return ((pf & M_PLUS) ? SM_PLUS : 0u) | ((pf & M_SKIPE) ? SM_SKIPE : 0u) | ((pf & M_DSTART) ? SM_DSTART : 0u);
}

// bitonic sort of n (power of two) u64 in LDS, ascending
__device__ void bitonic_lds64(unsigned long long* k, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t kk = 2; kk <= n; kk <<= 1) {
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < n; i += 64) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = k[i], y = k[ixj];
                    if ((x > y) == ((i & kk) == 0)) { k[i] = y; k[ixj] = x; }
                }
            }
            __syncthreads();
        }
    }
}

// bitonic sort of n (power of two) filter ids in LDS by filter bytes
template <bool CK>
__device__ void bitonic_lds_bytes(const MatchArgs& a, uint32_t* f, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t kk = 2; kk <= n; kk <<= 1) {
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < n; i += 64) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t x = f[i], y = f[ixj];
                    if (filter_less<CK>(a, y, x) == ((i & kk) == 0)) { f[i] = y; f[ixj] = x; }
                }
            }
            __syncthreads();
        }
    }
}

// A row of on (SORT_LDS < on <= 2 * SORT_LDS) path-coded entries whose first
// SORT_LDS, sorted, are back in okey[] (global scratch, as code | id) and the
// rest, sorted, in sk[0, nb) (LDS): every entry's place in the merged row is
// its index in its own run plus its rank in the other (a binary search: the
// keys are distinct, as a row's filter ids are), and its id goes there.
__device__ __forceinline__ void merge_runs_out(const unsigned long long* A, const unsigned long long* sk, uint32_t nb,
                                               uint32_t* out) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < SORT_LDS; i += 64) {   // run A: rank in B (LDS)
        const unsigned long long x = A[i];
        uint32_t lo = 0, hi = nb;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (sk[m] < x) lo = m + 1; else hi = m;
        }
        out[i + lo] = (uint32_t)(x & ~KEY_MASK);
    }
    for (uint32_t j = lane; j < nb; j += 64) {         // run B: rank in A (global)
        const unsigned long long x = sk[j];
        uint32_t lo = 0, hi = SORT_LDS;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (A[m] < x) lo = m + 1; else hi = m;
        }
        out[j + lo] = (uint32_t)(x & ~KEY_MASK);
    }
}

template <bool CK, bool BIG>
__global__ __launch_bounds__(64) void tm_match_slow(MatchArgs a) {
    __shared__ uint4 sq[SLOW_SQ];
    unsigned long long* const sk = reinterpret_cast<unsigned long long*>(sq);   // (after the walk)
    uint32_t* const sfi = reinterpret_cast<uint32_t*>(sq);
    const uint32_t lane = threadIdx.x;
    const uint32_t wave = blockIdx.x;
    uint32_t* qpar = a.s_qparent + (size_t)wave * a.s_qcap;
    uint32_t* qmeta = a.s_qmeta + (size_t)wave * a.s_qcap;
    unsigned long long* qkey = a.s_qkey + (size_t)wave * a.s_qcap;
    uint32_t* ofid = a.s_ofid + (size_t)wave * a.s_ocap;
    unsigned long long* okey = a.s_okey + (size_t)wave * a.s_ocap;
    const uint32_t novf = min(a.ctrl[CTRL_NOVF], a.ovf_cap);
    const uint32_t n_slow = a.d_nslow ? min(*a.d_nslow, a.n) : a.n_slow;
    const uint32_t total_items = n_slow + novf;
    const uint32_t lcap = a.s_lcap && a.s_lcap < SLOW_SQ ? a.s_lcap : SLOW_SQ;
    unsigned long long sV = 0, sH = 0, sW = 0, sM = 0, sS = 0;

    for (uint32_t item = wave; item < total_items; item += gridDim.x) {
        uint32_t t = (item < n_slow) ? a.slow_list[CK_(item, n_slow, 24)]
                                     : a.ovf_list[CK_(item - n_slow, a.ovf_cap, 25)];
        t = CK_(t, a.n, 26);
        const uint8_t fl = a.tflags[t];
        const bool dollar = fl & TF_DOLLAR;
        const bool by_bytes = fl & TF_SLOW;   // deep or irregular: path code does not apply
        const uint32_t wb = a.toff[t];
        const uint32_t d = a.toff[t + 1] - wb;
        const uint32_t* w = a.words + wb;
        sS += 1;
        uint32_t qn = 0, on = 0;
        bool err = false;
        // the stack in LDS; a topic whose frontier outgrows it walks again
        // with the stack in its wave's global scratch (the counters of the
        // abandoned attempt are dropped)
        for (bool in_lds = true;;) {
            unsigned long long tV = 0, tH = 0, tW = 0;
            bool spill = false;
            qn = 0; on = 0;
            if (d > 0) {
                Expand x; x.ne = 0; x.np = 0;
                if (lane == 0) {
                    tV += 1; tW += d;
                    if (!dollar && (a.root.flags & NF_HASH)) tH += 1;
                    expand_root(a.root, dollar, d, w[0], x);
                    if (in_lds) {
                        if (x.np >= 1) sq[0] = uint4{ROOT, 1u | slow_flags(x.pf0), (uint32_t)x.pk0, (uint32_t)(x.pk0 >> 32)};
                        if (x.np >= 2) sq[1] = uint4{ROOT, 1u | slow_flags(x.pf1), (uint32_t)x.pk1, (uint32_t)(x.pk1 >> 32)};
                    } else {
                        if (x.np >= 1) { qpar[0] = ROOT; qkey[0] = x.pk0; qmeta[0] = 1u | slow_flags(x.pf0); }
                        if (x.np >= 2) { qpar[1] = ROOT; qkey[1] = x.pk1; qmeta[1] = 1u | slow_flags(x.pf1); }
                    }
                    if (x.ne >= 1) { ofid[0] = x.ef0; okey[0] = x.ek0; }
                }
                qn = __shfl(x.np, 0, 64);
                on = __shfl(x.ne, 0, 64);
                if (!in_lds) __threadfence_block();
                __syncthreads();
            }
            while (qn > 0) {
                const uint32_t k = min(qn, 64u);
                const bool has = lane < k;
                const uint32_t idx = qn - k + lane;
                uint32_t parent = 0, meta = 0;
                unsigned long long key = 0;
                if (has) {
                    if (in_lds) {
                        const uint4 e = sq[CK_(idx, SLOW_SQ, 27)];
                        parent = e.x; meta = e.y; key = ((unsigned long long)e.w << 32) | e.z;
                    } else {
                        const uint32_t ci = CK_(idx, a.s_qcap, 27);
                        parent = qpar[ci]; meta = qmeta[ci]; key = qkey[ci];
                    }
                }
                if (!in_lds) __threadfence_block();
                __syncthreads();   // every entry popped before the pushes reuse their places
                qn -= k;
                const uint32_t lc = meta & SM_LVL;
                uint32_t pw = W_PLUS;
                if (has && !(meta & SM_PLUS)) pw = w[CK_(lc - 1, d, 28)] & WID_MASK;
                Node s;
                const bool found = has && probe<CK, BIG>(a, parent, pw, s);
                Expand x; x.ne = 0; x.np = 0;
                if (found) {
                    if (!(meta & SM_DSTART)) tV += 1;
                    if (s.flags & NF_HASH) tH += 1;
                    const uint32_t fl2 = (meta & SM_SKIPE) ? M_SKIPE : 0u;
                    expand(s, lc, d, fl2, key, lc < d ? w[CK_(lc, d, 29)] : 0u, w[CK_(lc - 1, d, 28)], x);
                }
                const uint64_t b0 = __ballot(x.np >= 1), b1 = __ballot(x.np >= 2);
                const uint64_t e0 = __ballot(x.ne >= 1), e1 = __ballot(x.ne >= 2);
                const uint32_t ptot = __popcll(b0) + __popcll(b1);
                const uint32_t etot = __popcll(e0) + __popcll(e1);
                if (in_lds && qn + ptot > lcap) { spill = true; break; }
                if (qn + ptot > a.s_qcap || on + etot > a.s_ocap) { err = true; break; }
                const uint32_t pre = prefix_count(b0) + prefix_count(b1);
                const uint32_t m0 = (lc + 1) | slow_flags(x.pf0), m1 = (lc + 1) | slow_flags(x.pf1);
                if (in_lds) {
                    if (x.np >= 1) sq[qn + pre] = uint4{s.child, m0, (uint32_t)x.pk0, (uint32_t)(x.pk0 >> 32)};
                    if (x.np >= 2) sq[qn + pre + 1] = uint4{s.child, m1, (uint32_t)x.pk1, (uint32_t)(x.pk1 >> 32)};
                } else {
                    if (x.np >= 1) { const uint32_t p = qn + pre; qpar[p] = s.child; qkey[p] = x.pk0; qmeta[p] = m0; }
                    if (x.np >= 2) { const uint32_t p = qn + pre + 1; qpar[p] = s.child; qkey[p] = x.pk1; qmeta[p] = m1; }
                }
                qn += ptot;
                const uint32_t epre = prefix_count(e0) + prefix_count(e1);
                if (x.ne >= 1) { ofid[on + epre] = x.ef0; okey[on + epre] = x.ek0; }
                if (x.ne >= 2) { ofid[on + epre + 1] = x.ef1; okey[on + epre + 1] = x.ek1; }
                on += etot;
                if (!in_lds) __threadfence_block();
                __syncthreads();
            }
            if (spill) {
                in_lds = false;
                __syncthreads();
                continue;
            }
            sV += tV; sH += tH; sW += tW;
            break;
        }
        if (err) {
            if (lane == 0) atomicOr(&a.ctrl[CTRL_ERR], ERR_SLOW_SCRATCH);
            __syncthreads();
            continue;
        }
        __threadfence_block();   // this wave's emissions, read back below
        __syncthreads();
        // sort the row (path code | filter id, or filter bytes for deep /
        // irregular topics), in LDS when it fits
        uint32_t np2 = 1;
        while (np2 < on) np2 <<= 1;
        bool sorted_in_lds = false;
        uint32_t two_runs = 0;   // > 0: sorted as two runs, the second this long (merge_runs_out)
        if (on > 1) {
            if (!by_bytes && np2 > SORT_LDS && on <= 2 * SORT_LDS) {
                // run A: the first SORT_LDS entries, sorted in LDS, back to okey[]
                for (uint32_t i = lane; i < SORT_LDS; i += 64) sk[i] = okey[i] | ofid[i];
                __syncthreads();
                bitonic_lds64(sk, SORT_LDS);
                for (uint32_t i = lane; i < SORT_LDS; i += 64) okey[i] = sk[i];
                __threadfence_block();
                __syncthreads();
                // run B: the rest, sorted in LDS where it stays
                const uint32_t nb = on - SORT_LDS;
                uint32_t nb2 = 1;
                while (nb2 < nb) nb2 <<= 1;
                for (uint32_t i = lane; i < nb2; i += 64)
                    sk[i] = i < nb ? (okey[SORT_LDS + i] | ofid[SORT_LDS + i]) : ~0ull;
                __syncthreads();
                if (nb2 > 1) bitonic_lds64(sk, nb2);
                two_runs = nb;
            } else if (!by_bytes && np2 <= SORT_LDS) {
                // (path codes use bits 31..63, filter ids < 2^30: one u64
                // orders by code, then id)
                for (uint32_t i = lane; i < np2; i += 64) sk[i] = i < on ? (okey[i] | ofid[i]) : ~0ull;
                __syncthreads();
                bitonic_lds64(sk, np2);
                sorted_in_lds = true;
            } else if (by_bytes && np2 <= 2 * SORT_LDS) {
                for (uint32_t i = lane; i < np2; i += 64) sfi[i] = i < on ? ofid[i] : NONE;
                __syncthreads();
                bitonic_lds_bytes<CK>(a, sfi, np2);
                sorted_in_lds = true;
            } else if (np2 <= a.s_ocap) {
                for (uint32_t i = on + lane; i < np2; i += 64) { okey[i] = ~0ull; ofid[i] = NONE; }
                __threadfence_block();
                __syncthreads();
                bitonic<CK>(a, okey, ofid, np2, by_bytes);
            } else {
                if (lane == 0) atomicOr(&a.ctrl[CTRL_ERR], ERR_SLOW_SCRATCH);
                __syncthreads();
                continue;
            }
            __threadfence_block();
            __syncthreads();
        }
        unsigned long long base = 0;
        const uint32_t g = (blockIdx.x % TICKET_GROUPS) & a.sgmask;
        if (lane == 0 && on) base = atomicAdd(xg_top(a.xg, g), (unsigned long long)on);
        base = __shfl(base, 0, 64);
        const bool fits = base + on <= a.rcap;
        base += (uint64_t)g * a.rcap;
        if (fits && two_runs) {
            (void)CK_(base + on - 1, a.sfids_cap, 30);
            merge_runs_out(okey, sk, two_runs, a.sfids + base);
        } else if (fits) {
            for (uint32_t i = lane; i < on; i += 64) {
                const uint32_t f = !sorted_in_lds ? ofid[i] : by_bytes ? sfi[i] : (uint32_t)(sk[i] & ~KEY_MASK);
                a.sfids[CK_(base + i, a.sfids_cap, 30)] = f;
            }
        } else if (lane == 0) {
            atomicOr(&a.ctrl[CTRL_ERR], ERR_STAGING);
        }
        if (lane == 0) { a.count[t] = on; a.src[t] = base; }
        sM += (lane == 0) ? on : 0;
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) {
        sV += __shfl_xor(sV, o, 64); sH += __shfl_xor(sH, o, 64);
        sW += __shfl_xor(sW, o, 64); sM += __shfl_xor(sM, o, 64);
    }
    if (lane == 0 && sS) {
        atomicAdd(&a.stats[ST_VISITS], sV); atomicAdd(&a.stats[ST_HASH], sH);
        atomicAdd(&a.stats[ST_WORDS], sW); atomicAdd(&a.stats[ST_MATCHES], sM);
        atomicAdd(&a.stats[ST_SLOW], sS);
    }
}

// ------------------------------------------------------------ CSR build

constexpr uint32_t SCAN_BLOCK = 1024;
constexpr uint32_t SCAN_PER_THREAD = 4;
constexpr uint32_t SCAN_TILE = SCAN_BLOCK * SCAN_PER_THREAD;

uint32_t scan_block_count(uint32_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += u;
    }
    if (lane == 63) sh[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        const uint32_t nw = blockDim.x >> 6;
        const uint32_t s = lane < nw ? sh[lane] : 0;
        uint32_t si = s;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(si, o, 64);
            if (lane >= (uint32_t)o) si += u;
        }
        if (lane < nw) sh[lane] = si - s;
        if (lane == nw - 1) sh[32] = si;
    }
    __syncthreads();
    total = sh[32];
    const uint32_t r = sh[wid] + incl - v;
    __syncthreads();
    return r;
}

// Pass 1: per-block exclusive scan of count[] (slow/overflow rows included).
// A single-block scan (n <= SCAN_TILE: small batches) is final here: block
// offset 0, total -> row_off[n] and *d_total, and pass 2 is not launched.
__global__ __launch_bounds__(SCAN_BLOCK) void tm_scan_local(ScanArgs a, uint32_t* d_total) {
    __shared__ uint32_t sh[33];
    const uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER_THREAD;
    uint32_t v[SCAN_PER_THREAD];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t i = 0; i < SCAN_PER_THREAD; ++i) {
        v[i] = (base + i < a.n) ? a.count[base + i] : 0u;
        s += v[i];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan(s, sh, tot);
#pragma unroll
    for (uint32_t i = 0; i < SCAN_PER_THREAD; ++i) {
        if (base + i < a.n) a.row_off[base + i] = ex;
        ex += v[i];
    }
    if (threadIdx.x == 0) {
        if (gridDim.x == 1) {
            a.block_sums[0] = 0;
            a.row_off[a.n] = tot;
            if (d_total) *d_total = tot;
        } else {
            a.block_sums[blockIdx.x] = tot;
        }
    }
}

// Pass 2: exclusive scan of the block sums (single block), total -> row_off[n].
__global__ __launch_bounds__(SCAN_BLOCK) void tm_scan_sums(ScanArgs a, uint32_t nblocks, uint32_t* d_total) {
    __shared__ uint32_t sh[33];
    uint64_t carry = 0;   // u64: a total past u32 is flagged, never wrapped silently
    for (uint32_t b0 = 0; b0 < nblocks; b0 += SCAN_BLOCK) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < nblocks ? a.block_sums[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(v, sh, tot);
        if (i < nblocks) a.block_sums[i] = (uint32_t)(carry + ex);
        carry += tot;
    }
    if (threadIdx.x == 0) {
        a.row_off[a.n] = (uint32_t)carry;
        if (d_total) *d_total = (uint32_t)carry;
        if (carry > MAX_RESULT && a.ctrl) atomicOr(&a.ctrl[CTRL_ERR], ERR_CSR_RANGE);
    }
}

// Pass 3: one wavefront per tile of 64 topics.  Finishes the CSR offsets and
// copies the tile's sorted rows from the staging region.  A tile whose rows were
// staged as one run (no slow-path topic in it) is one contiguous copy, FIN_U
// coalesced dword loads in flight per lane; otherwise each topic is copied on
// its own.  The next tile's (count, src, offset) are loaded before this tile's
// copy, so a tile costs the copy's round trips, not one more for its header.
template <bool CK>
__global__ __launch_bounds__(64) void tm_finalize(ScanArgs a) {
    const uint32_t lane = threadIdx.x;
    const uint32_t ntiles = (a.n + TILE - 1) / TILE;
    uint32_t nc = 0, noff = 0, nbs = 0;
    uint64_t ns = 0;
    auto meta = [&](uint32_t tile) {
        const uint32_t t = tile * TILE + lane;
        if (tile < ntiles && t < a.n) {
            nc = a.count[t];
            ns = a.src[t];
            noff = a.row_off[t];
            nbs = a.block_sums[t / SCAN_TILE];
        }
    };
    meta(blockIdx.x);
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint32_t t = tile * TILE + lane;
        const bool valid = t < a.n;
        uint32_t c = 0, off = 0;
        uint64_t s = 0;
        if (valid) {
            c = nc;
            s = ns;
            off = noff + nbs;
            a.row_off[t] = off;      // finish the CSR offsets (scan pass 1 was block-local)
        }
        meta(tile + gridDim.x);
        const bool any = c > 0;
        const uint64_t m = __ballot(any);
        if (!m) continue;
        const uint64_t delta = s - (uint64_t)off;
        const uint32_t first = (uint32_t)__builtin_ctzll(m);
        const uint32_t last = 63u - (uint32_t)__builtin_clzll(m);
        const uint64_t d0 = __shfl(delta, first, 64);
        if (__ballot(any && delta != d0) == 0) {
            const uint32_t lo = __shfl(off, first, 64);
            const uint32_t hi = __shfl(off + c, last, 64);
            const uint64_t sb = (uint64_t)lo + d0;
            if ((uint64_t)hi > a.ids_cap || sb + (hi - lo) > a.sfids_cap) continue;   // rerun path
            // FIN_U loads per lane in flight before the stores: a tile's run
            // (~1,500 ids at C2) is one or two memory round trips
            constexpr uint32_t FIN_U = 16;
            for (uint32_t i = lo + lane; i < hi; i += 64 * FIN_U) {
                uint32_t v[FIN_U];
#pragma unroll
                for (uint32_t u = 0; u < FIN_U; ++u) {
                    const uint32_t iu = i + 64 * u;
                    v[u] = iu < hi ? a.sfids[CK_(sb + (iu - lo), a.sfids_cap, 30)] : 0u;
                }
#pragma unroll
                for (uint32_t u = 0; u < FIN_U; ++u) {
                    const uint32_t iu = i + 64 * u;
                    if (iu < hi) a.ids[CK_(iu, a.ids_cap, 34)] = v[u];
                }
            }
        } else if (any && s + c <= a.sfids_cap && (uint64_t)off + c <= a.ids_cap) {
            for (uint32_t i = 0; i < c; ++i) a.ids[CK_((uint64_t)off + i, a.ids_cap, 38)] = a.sfids[CK_(s + i, a.sfids_cap, 39)];
        }
    }
}

// ------------------------------------------------ routes (emqx_broker:aggre/1)

// Routes per topic = sum over its matched filters of their dest counts
// (lookup_routes/1 for every To in [Topic | Matched], src/emqx_router.erl:132;
// the topic itself is in the trie, so Matched already holds an exact route).
// Routes of a batch = for every match entry, the dests of its filter, in
// match order (emqx_router:match_routes/1 + aggre/1 per publish,
// src/emqx_router.erl:127-133, src/emqx_broker.erl:250-261): the route CSR is
// an exclusive scan of per-ENTRY dest counts, and a topic's first route is its
// first entry's offset.  One thread per entry in each kernel.
__global__ __launch_bounds__(256) void tm_route_count(RouteArgs a) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.m) return;
    const uint32_t f = a.ids[i];
    a.ecount[i] = f < a.nnodes ? a.roff[f + 1] - a.roff[f] : 0u;
}
__device__ __forceinline__ uint32_t route_eoff(const RouteArgs& a, uint32_t j) {
    return j < a.m ? a.eoff[j] + a.bsums[j / SCAN_TILE] : *a.total;
}
__global__ __launch_bounds__(256) void tm_route_rows(RouteArgs a) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t <= a.n) a.r_rowoff[t] = route_eoff(a, a.row_off[t]);
}
__global__ __launch_bounds__(256) void tm_route_fill(RouteArgs a) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.m) return;
    const uint32_t f = a.ids[i];
    if (f >= a.nnodes) return;
    uint64_t o = route_eoff(a, i);
    for (uint32_t k = a.roff[f], ke = a.roff[f + 1]; k < ke && o < a.cap; ++k, ++o) {
        a.out_fid[o] = f;
        a.out_dest[o] = a.rdest[k];
    }
}

// ------------------------------------------ fan-out (emqx_broker:dispatch/2)
//
// dispatch(To, Delivery) folds over subscribers(To) for every local route of the
// publish (src/emqx_broker.erl:243-244, 284-309).  The match CSR already lists
// the publish's filters in order, so the deliveries of a batch are the
// concatenation, over match entries j, of the subscriber run of filter ids[j]:
//   scan  moff[j] = sum of the run lengths before entry j (u64: a hot filter can
//         carry millions of subscribers), drow[i] = moff[row_off[i]];
//   fill  one thread per DELIVERY, not per publish or filter: a workgroup owns
//         4096 consecutive outputs, finds the entries covering them by binary
//         search of moff, and copies subscriber ids with coalesced loads and
//         stores -- balanced whatever the fan-out skew (1 vs 10^6 subscribers).

constexpr uint32_t FAN_BLOCK = 256;
constexpr uint32_t FAN_PER = 16;                           // entries per scan thread
constexpr uint32_t FAN_SCAN_TILE = FAN_BLOCK * FAN_PER;
#ifndef TM_FAN_FILL_PER
#define TM_FAN_FILL_PER 8
#endif
constexpr uint32_t FAN_FILL_PER = TM_FAN_FILL_PER;         // deliveries per fill thread (8 or 16)
static_assert(FAN_FILL_PER % 8 == 0 && FAN_FILL_PER >= 8, "the fill's max-scan reads its marks as uint4 words (8 per thread)");
constexpr uint32_t FAN_FILL_TILE = FAN_BLOCK * FAN_FILL_PER;
constexpr uint32_t FAN_LDS_ENTRIES = FAN_FILL_TILE * 3 / 4;  // match entries a fill tile can stage

// first delivery of match entry j: the block's offset plus the block-relative
// u32 (u64 only in scan blocks with 2^32 deliveries or more)
__device__ inline uint64_t fan_moff(const FanArgs& a, uint64_t j) {
    // the u32 offset, the block flag and the block sum are loaded together
    // (moff32 spans every entry, so the speculative read is in bounds); only a
    // block past 2^32 deliveries reads the u64 offset after the flag
    const uint64_t b = j / FAN_SCAN_TILE;
    const uint32_t m32 = a.moff32[j];
    const bool big = a.bbig[b] != 0;
    const uint64_t bs = a.bsums[b];
    return (big ? a.moff[j] : (uint64_t)m32) + bs;
}

// Rows mode: region of virtual entry j (vb[0] = 0, vb ascending)
__device__ __forceinline__ uint32_t fan_region(const FanArgs& a, uint64_t j) {
    uint32_t g = 0;
#pragma unroll
    for (uint32_t k = 1; k < TICKET_GROUPS; ++k) g += (k < a.nreg && j >= a.vb[k]) ? 1u : 0u;
    return g;
}

// filter id of entry j (rows mode: the staging entry behind it; padding ->
// nnodes, i.e. no deliveries)
__device__ __forceinline__ uint32_t fan_fid(const FanArgs& a, uint64_t j) {
    if (!a.nreg) return a.ids[j];
    const uint32_t g = fan_region(a, j);
    const uint64_t o = j - a.vb[g];
    return o < a.rtop[g] ? a.ids[g * a.rcap + o] : a.nnodes;
}

// Exclusive scan of one u64 per thread over a 256-thread block (4 waves).
__device__ inline uint64_t fan_block_scan(uint64_t v, uint64_t* lds, uint64_t& total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) lds[w] = x;
    __syncthreads();
    uint64_t base = 0;
    for (uint32_t k = 0; k < w; ++k) base += lds[k];
    total = lds[0] + lds[1] + lds[2] + lds[3];
    __syncthreads();
    return base + x - v;
}

// A block scans FAN_SCAN_TILE entries as FAN_PER striped chunks of FAN_BLOCK
// (coalesced ids loads and moff stores); all chunks' run lengths are gathered
// before the first scan so the soff loads overlap.  The block's total decides
// the width of its offsets: u32 (half the bytes every reader moves) unless the
// block delivers 2^32 or more (a hot filter with millions of subscribers).
__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_scan_local(FanArgs a) {
    __shared__ uint64_t lds[4];
    // thread t owns FAN_PER consecutive entries: a serial prefix in registers
    // and ONE block scan of the per-thread sums (striped chunks needed one
    // block scan per chunk); ids and offsets move as 16-B vectors
    const uint64_t j0 = (uint64_t)blockIdx.x * FAN_SCAN_TILE + (uint64_t)threadIdx.x * FAN_PER;
    uint32_t f[FAN_PER];
    // rows mode: the 16 entries lie in one region (its virtual base and the
    // region stride are multiples of 16), so they are one aligned chunk of
    // staging; entries past the region's top are padding
    const uint32_t* src = a.ids + j0;
    uint64_t valid = a.n_matches > j0 ? a.n_matches - j0 : 0;
    if (a.nreg && valid) {
        const uint32_t g = fan_region(a, j0);
        const uint64_t o = j0 - a.vb[g];
        src = a.ids + g * a.rcap + o;
        valid = a.rtop[g] > o ? min<uint64_t>(valid, a.rtop[g] - o) : 0;
    }
    if (j0 + FAN_PER <= a.n_matches) {
        const uint4* q = reinterpret_cast<const uint4*>(src);   // 64-B aligned
#pragma unroll
        for (uint32_t k = 0; k < FAN_PER / 4; ++k) {
            const uint4 v = q[k];
            f[4 * k] = v.x; f[4 * k + 1] = v.y; f[4 * k + 2] = v.z; f[4 * k + 3] = v.w;
        }
#pragma unroll
        for (uint32_t k = 0; k < FAN_PER; ++k)
            if (k >= valid) f[k] = a.nnodes;
    } else {
#pragma unroll
        for (uint32_t k = 0; k < FAN_PER; ++k) f[k] = k < valid ? src[k] : a.nnodes;
    }
    uint64_t c[FAN_PER], mine = 0;
#pragma unroll
    for (uint32_t k = 0; k < FAN_PER; ++k) {
        c[k] = 0;
        if (f[k] < a.nnodes) {
            const uint32_t s1 = a.scnt[f[k]];   // 1 B per node: the gather's footprint stays L2-sized
            c[k] = s1 < 255 ? s1 : a.soff[f[k] + 1] - a.soff[f[k]];
        }
        mine += c[k];
    }
    uint64_t total;
    uint64_t run = fan_block_scan(mine, lds, total);
    const bool big = total > a.big_limit;
    if (!big && j0 + FAN_PER <= a.n_matches + 1) {
        uint4* q = reinterpret_cast<uint4*>(a.moff32 + j0);
#pragma unroll
        for (uint32_t k = 0; k < FAN_PER / 4; ++k) {
            uint4 v;
            v.x = (uint32_t)run; run += c[4 * k];
            v.y = (uint32_t)run; run += c[4 * k + 1];
            v.z = (uint32_t)run; run += c[4 * k + 2];
            v.w = (uint32_t)run; run += c[4 * k + 3];
            q[k] = v;
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < FAN_PER; ++k) {
            const uint64_t j = j0 + k;
            if (j <= a.n_matches) {
                if (big) a.moff[j] = run;
                else a.moff32[j] = (uint32_t)run;
            }
            run += c[k];
        }
    }
    if (threadIdx.x == 0) {
        a.bsums[blockIdx.x] = total;
        a.bbig[blockIdx.x] = big ? 1 : 0;
    }
}

__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_scan_sums(FanArgs a, uint32_t nb) {
    // each thread owns a contiguous chunk of the block sums: a serial sum, ONE
    // block scan of the chunk sums, then a serial exclusive pass (one block
    // scan per 256 sums made this a long chain of barriers at 60k blocks)
    __shared__ uint64_t lds[4];
    const uint32_t per = (nb + FAN_BLOCK - 1) / FAN_BLOCK;
    const uint32_t lo = min(nb, threadIdx.x * per), hi = min(nb, lo + per);
    // 8 loads of a chunk in flight at a time (a dependent chain of 230 loads
    // per thread was the cost); the chunk is kept in registers for pass 2 when
    // it fits
    constexpr uint32_t U = 8;
    uint64_t mine = 0;
    for (uint32_t i0 = lo; i0 < hi; i0 += U) {
        uint64_t v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = i0 + u < hi ? a.bsums[i0 + u] : 0ull;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) mine += v[u];
    }
    uint64_t total;
    uint64_t run = fan_block_scan(mine, lds, total);
    for (uint32_t i0 = lo; i0 < hi; i0 += U) {
        uint64_t v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = i0 + u < hi ? a.bsums[i0 + u] : 0ull;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (i0 + u < hi) a.bsums[i0 + u] = run;
            run += v[u];
        }
    }
    if (threadIdx.x == 0) *a.d_total = total;
}

// After scan_local + scan_sums, moff32[j] (or moff[j] in a big block) is
// relative to its scan block and bsums[b] is the block's exclusive offset:
// rows, tiles and fill read the sum (bsums is small and cache-resident).
// tm_fan_scan_add writes the global u64 offsets into moff -- only when the
// caller asks for the match offsets, and only after the fill.
__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_scan_add(FanArgs a) {
    const uint64_t j = (uint64_t)blockIdx.x * FAN_BLOCK + threadIdx.x;
    if (j <= a.n_matches) a.moff[j] = fan_moff(a, j);   // in place for big blocks: read, then write
}

__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_rows(FanArgs a) {
    const uint32_t i = blockIdx.x * FAN_BLOCK + threadIdx.x;
    if (i <= a.n) a.drow[i] = fan_moff(a, a.row_off[i]);
}

// rows mode: the deliveries of publish i's row, read where the walk left it
// (count, first staging entry): first delivery and count
__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_rows_stg(FanArgs a) {
    const uint32_t i = blockIdx.x * FAN_BLOCK + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t c = a.rcount[i];
    uint64_t d0 = 0, dn = 0;
    if (c) {
        const uint64_t s = a.rsrc[i];
        const uint32_t g = a.nreg > 1 ? (uint32_t)(s / a.rcap) : 0u;
        const uint64_t v = a.vb[g] + (s - g * a.rcap);
        d0 = fan_moff(a, v);
        dn = fan_moff(a, v + c) - d0;
    }
    a.drow[i] = d0;
    a.dcount[i] = (uint32_t)dn;
}

// first j in [lo, hi) with moff[j] > p (hi if none)
__device__ inline uint64_t fan_upper(const FanArgs& a, uint64_t lo, uint64_t hi, uint64_t p) {
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (fan_moff(a, m) > p) hi = m;
        else lo = m + 1;
    }
    return lo;
}

// tile_j[k] = match entry of delivery k * FAN_FILL_TILE (k < ntiles), and
// tile_j[ntiles] = entry of the last delivery: one search per tile, all tiles
// at once, instead of a dependent search chain at the head of every fill block.
__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_tiles(FanArgs a, uint64_t ntiles) {
    const uint64_t k = (uint64_t)blockIdx.x * FAN_BLOCK + threadIdx.x;
    if (k > ntiles) return;
    const uint64_t p = k < ntiles ? k * FAN_FILL_TILE : a.total - 1;
    a.tile_j[k] = fan_upper(a, 0, a.n_matches + 1, p) - 1;
}

// One workgroup per 4096 consecutive deliveries.  The entries covering the
// tile (jlo..jhi) are staged in LDS: each non-empty run marks its first
// delivery in the tile with its entry index and keeps soff[f] - moff[j]; an
// inclusive max-scan over the marks gives every delivery its entry, and the
// copy is then one LDS read + one subscriber load + one coalesced store per
// delivery.  A tile covering more than FAN_LDS_ENTRIES entries (long stretches
// of filters without local subscribers) searches moff per delivery instead.
// WIDE: the batch delivers more than big_limit (some scan block may hold u64
// offsets); otherwise only the 32-bit staging path is compiled in
template <bool WIDE>
__global__ __launch_bounds__(FAN_BLOCK) void tm_fan_fill(FanArgs a) {
    __shared__ int64_t base[FAN_LDS_ENTRIES];
    __shared__ __attribute__((aligned(16))) uint16_t own[FAN_FILL_TILE];
    __shared__ uint32_t wmax[FAN_BLOCK / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t start = (uint64_t)blockIdx.x * FAN_FILL_TILE;
    const uint64_t end = min(start + FAN_FILL_TILE, a.total);
    const uint32_t len = (uint32_t)(end - start);
    const uint64_t jlo = a.tile_j[blockIdx.x];
    const uint64_t jhi = a.tile_j[blockIdx.x + 1];
    const uint64_t ne = jhi - jlo + 1;
    if (ne > FAN_LDS_ENTRIES) {
        // moff[j] <= p < moff[j + 1] for the entry of delivery p; p only grows
        // per thread, so each search starts at the previous entry
        uint64_t j = jlo;
        for (uint64_t p = start + t; p < end; p += FAN_BLOCK) {
            j = fan_upper(a, j, jhi + 1, p) - 1;
            a.out[p] = a.subs[a.soff[fan_fid(a, j)] + (p - fan_moff(a, j))];
        }
        return;
    }
    uint4* own4 = reinterpret_cast<uint4*>(own);
    for (uint32_t i = t; i < FAN_FILL_TILE / 8; i += FAN_BLOCK) own4[i] = make_uint4(0, 0, 0, 0);
    // The entries [jlo, jhi + 1] lie in at most two scan blocks (ne + 1 <=
    // FAN_LDS_ENTRIES + 1 < FAN_SCAN_TILE): their "big" flags and offsets are
    // read once, so an entry's delivery offset is one load, not a flag load
    // and then the offset load.
    const uint64_t sb0 = jlo / FAN_SCAN_TILE;
    const uint64_t nsb = a.n_matches / FAN_SCAN_TILE + 1;   // scan blocks over n_matches + 1 entries
    const bool big0 = a.bbig[sb0], big1 = sb0 + 1 < nsb ? a.bbig[sb0 + 1] != 0 : false;
    const uint64_t bs0 = a.bsums[sb0], bs1 = sb0 + 1 < nsb ? a.bsums[sb0 + 1] : 0;
    auto moff_at = [&](uint64_t j) -> uint64_t {
        const bool hi = j / FAN_SCAN_TILE != sb0;
        return ((hi ? big1 : big0) ? a.moff[j] : (uint64_t)a.moff32[j]) + (hi ? bs1 : bs0);
    };
    __syncthreads();
    // rows mode: a tile's entries usually lie in one staging region, whose
    // entries are then one offset away (padding entries have no deliveries,
    // so whatever they read is never used); a tile across regions maps each
    const bool one_reg = !a.nreg || fan_region(a, jlo) == fan_region(a, jhi + 1);
    const uint32_t* fids = a.ids;
    if (a.nreg && one_reg) {
        const uint32_t g = fan_region(a, jlo);
        fids = a.ids + g * a.rcap - a.vb[g];
    }
    // staging, FAN_STG entries per thread with every load of a step in flight
    // (the offsets and filter ids, then the dependent sone / soff gathers)
#ifndef TM_FAN_STG
#define TM_FAN_STG 8
#endif
    constexpr uint32_t FAN_STG = TM_FAN_STG;
    if (!WIDE || (!big0 && !big1)) {
        // both scan blocks of the tile's entries hold u32 offsets (the common
        // case): the loads stay 32-bit until the gathers are issued
        for (uint32_t e0 = t; e0 < (uint32_t)ne; e0 += FAN_BLOCK * FAN_STG) {
            uint32_t r0[FAN_STG], r1[FAN_STG], f[FAN_STG];
#pragma unroll
            for (uint32_t u = 0; u < FAN_STG; ++u) {
                const uint32_t e = e0 + u * FAN_BLOCK;
                r0[u] = 0; r1[u] = 0; f[u] = 0;
                if (e < (uint32_t)ne) {
                    const uint64_t j = jlo + e;
                    r0[u] = a.moff32[j];
                    r1[u] = a.moff32[j + 1];
                    f[u] = one_reg ? fids[j] : fan_fid(a, j);
                }
            }
            int64_t v[FAN_STG];
            uint32_t at[FAN_STG];   // my mark's place in own[], NONE: inactive
#pragma unroll
            for (uint32_t u = 0; u < FAN_STG; ++u) {
                const uint64_t j = jlo + e0 + u * FAN_BLOCK;
                const uint64_t m0 = r0[u] + (j / FAN_SCAN_TILE != sb0 ? bs1 : bs0);
                const uint64_t m1 = r1[u] + ((j + 1) / FAN_SCAN_TILE != sb0 ? bs1 : bs0);
                const bool act = e0 + u * FAN_BLOCK < (uint32_t)ne && m1 > m0 && m1 > start && m0 < end;
                v[u] = 0;
                at[u] = act ? (m0 > start ? (uint32_t)(m0 - start) : 0u) : NONE;
                if (act) v[u] = m1 - m0 == 1 ? INT64_MIN + (int64_t)a.sone[f[u]] : (int64_t)a.soff[f[u]] - (int64_t)m0;
            }
#pragma unroll
            for (uint32_t u = 0; u < FAN_STG; ++u) {
                if (at[u] == NONE) continue;
                const uint32_t e = e0 + u * FAN_BLOCK;
                base[e] = v[u];
                own[at[u]] = (uint16_t)(e + 1);
            }
        }
    } else
    for (uint32_t e0 = t; e0 < (uint32_t)ne; e0 += FAN_BLOCK * FAN_STG) {
        uint64_t m0[FAN_STG], m1[FAN_STG];
        uint32_t f[FAN_STG];
        bool act[FAN_STG];
#pragma unroll
        for (uint32_t u = 0; u < FAN_STG; ++u) {
            const uint32_t e = e0 + u * FAN_BLOCK;
            m0[u] = 0; m1[u] = 0; f[u] = 0;
            if (e < (uint32_t)ne) {
                const uint64_t j = jlo + e;
                m0[u] = moff_at(j);
                m1[u] = moff_at(j + 1);
                f[u] = one_reg ? fids[j] : fan_fid(a, j);
            }
        }
        int64_t v[FAN_STG];
#pragma unroll
        for (uint32_t u = 0; u < FAN_STG; ++u) {
            act[u] = m1[u] > m0[u] && m1[u] > start && m0[u] < end;
            v[u] = 0;
            // a one-delivery run keeps its subscriber inline (one 4-B gather,
            // no dependent read of subs[]): INT64_MIN + id marks it
            if (act[u]) v[u] = m1[u] - m0[u] == 1 ? INT64_MIN + (int64_t)a.sone[f[u]]
                                                  : (int64_t)a.soff[f[u]] - (int64_t)m0[u];
        }
#pragma unroll
        for (uint32_t u = 0; u < FAN_STG; ++u) {
            if (!act[u]) continue;
            const uint32_t e = e0 + u * FAN_BLOCK;
            base[e] = v[u];
            own[m0[u] > start ? (uint32_t)(m0[u] - start) : 0u] = (uint16_t)(e + 1);
        }
    }
    __syncthreads();
    // inclusive max-scan of own[] (entry starts only grow along the tile)
    constexpr uint32_t NQ = FAN_FILL_PER / 8;                // uint4 words of marks per thread
    uint32_t v[FAN_FILL_PER];
#pragma unroll
    for (uint32_t q = 0; q < NQ; ++q) {
        const uint4 u = own4[NQ * t + q];
        const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) { v[8 * q + 2 * k] = wd[k] & 0xFFFFu; v[8 * q + 2 * k + 1] = wd[k] >> 16; }
    }
    uint32_t run = 0;
#pragma unroll
    for (uint32_t k = 0; k < FAN_FILL_PER; ++k) { run = max(run, v[k]); v[k] = run; }
    uint32_t x = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x = max(x, y);
    }
    if (lane == 63) wmax[w] = x;
    uint32_t pre = __shfl_up(x, 1, 64);
    if (lane == 0) pre = 0;
    __syncthreads();
    for (uint32_t k = 0; k < w; ++k) pre = max(pre, wmax[k]);
#pragma unroll
    for (uint32_t q = 0; q < NQ; ++q) {
        uint32_t o[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            o[k] = max(v[8 * q + 2 * k], pre) | (max(v[8 * q + 2 * k + 1], pre) << 16);
        own4[NQ * t + q] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
    // the copy: every delivery's subscriber load of this thread in flight at once
    uint32_t r[FAN_FILL_PER];
#pragma unroll
    for (uint32_t u = 0; u < FAN_FILL_PER; ++u) {
        const uint32_t i = t + u * FAN_BLOCK;
        r[u] = 0;
        if (i < len) {
            const int64_t bs = base[(uint32_t)own[i] - 1u];
            r[u] = bs < INT64_MIN + (1ll << 33) ? (uint32_t)(bs - INT64_MIN)
                                                : a.subs[(uint64_t)(bs + (int64_t)(start + i))];
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < FAN_FILL_PER; ++u) {
        const uint32_t i = t + u * FAN_BLOCK;
        if (i < len) a.out[start + i] = r[u];
    }
}

// ------------------------------------------ batched predicate (emqx_topic:match/2)

// One thread per name, all rules: the word-by-word clauses of
// emqx_topic:match/2 (src/emqx_topic.erl:74-87) -- equal words or a '+' rule
// word advance, a trailing '#' matches the rest (zero words included), both
// exhausted matches -- plus the binary form's '$' rule (:68-71) when asked.
// Rule words are read by every thread at once (broadcast, L1/L2-resident).
__global__ __launch_bounds__(256) void tm_rules_match(RulesArgs a) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t nb = a.noff[t], nl = a.noff[t + 1] - nb;
    const bool dollar = a.dollar_rule && (a.nflag[t] & 1);
    for (uint32_t w0 = 0; w0 < a.r; w0 += 32) {
        uint32_t acc = 0;
        const uint32_t w1 = min(a.r, w0 + 32);
        for (uint32_t j = w0; j < w1; ++j) {
            const uint32_t rb = a.roff[j], rl = a.roff[j + 1] - rb;
            bool m = false;
            if (!(dollar && (a.rflag[j] & 1))) {
                uint32_t i = 0, k = 0;
                for (;;) {
                    if (i == nl && k == rl) { m = true; break; }
                    const uint32_t fw = k < rl ? a.rwords[rb + k] : 0u;
                    if (k + 1 == rl && fw == W_HASH) { m = true; break; }
                    if (i == nl || k == rl) break;
                    if (fw == W_PLUS || fw == a.nwords[nb + i]) { ++i; ++k; continue; }
                    break;
                }
            }
            acc |= (uint32_t)m << (j - w0);
        }
        a.bits[(uint64_t)t * a.wpr + w0 / 32] = acc;
    }
}

// ------------------------------------------------ device dedup (TM_BATCH_DEDUP)

// 8 bytes at byte offset s of a 4-aligned LDS array (any alignment of s)
__device__ __forceinline__ uint64_t lds_u64(const uint8_t* base, uint32_t s) {
    const uint32_t a = s & ~3u, sh = (s & 3u) * 8u;
    const uint32_t d0 = *reinterpret_cast<const uint32_t*>(base + a);
    const uint32_t d1 = *reinterpret_cast<const uint32_t*>(base + a + 4);
    const uint32_t d2 = *reinterpret_cast<const uint32_t*>(base + a + 8);
    const uint64_t lo = ((uint64_t)d1 << 32) | d0;
    return sh ? (lo >> sh) | ((uint64_t)d2 << (64u - sh)) : lo;
}

__device__ __forceinline__ uint64_t low_bytes(uint64_t v, uint32_t k) {   // first k (< 8) bytes of v
    return k >= 8 ? v : (v & ((1ull << (8u * k)) - 1ull));
}



// A topic's first 64 bytes as 16 little-endian u32 words, zero past len:
// the 16-B aligned loads that cover them (the batch bytes are 16-B aligned
// and padded by 16), all issued before any is used, then the topic's offset
// within the first load taken out in 32-bit ops only -- two word selects and
// one v_alignbyte per word (64-bit variable shifts cost 3-4 VALU each).
// Lanes of a wave read neighbouring topics, so a load instruction's lines are
// mostly the wave's next ones.
__device__ __forceinline__ void dd_load64(const uint8_t* bytes, uint64_t b, uint32_t len, uint32_t (&c)[16]) {
    const uint64_t a0 = b & ~15ull;
    const uint32_t sh = (uint32_t)(b & 15u);
    const uint32_t need = sh + (len < 64u ? len : 64u);
    uint32_t w[20];
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (16u * k < need) v = *reinterpret_cast<const uint4*>(bytes + a0 + 16u * k);
        w[4 * k] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    }
    // (selects as masks: written as `q ? w[i + 1] : w[i]` the compiler turns
    // them into one dynamically indexed array -- scratch memory)
    const uint32_t m1 = 0u - ((sh >> 2) & 1u), m2 = 0u - ((sh >> 3) & 1u);
    uint32_t s1[19];
#pragma unroll
    for (uint32_t i = 0; i < 19; ++i) s1[i] = w[i] ^ ((w[i] ^ w[i + 1]) & m1);
    uint32_t s2[17];
#pragma unroll
    for (uint32_t i = 0; i < 17; ++i) s2[i] = s1[i] ^ ((s1[i] ^ s1[i + 2]) & m2);
    const uint32_t r = sh & 3u;
    const uint32_t pm = (1u << ((len & 3u) * 8u)) - 1u;   // the partial last word's bytes
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t x = __builtin_amdgcn_alignbyte(s2[j + 1], s2[j], r);
        c[j] = 4u * j + 4u <= len ? x : (4u * j < len ? (x & pm) : 0u);
    }
}

// 8 bytes at any offset of the padded batch bytes: two aligned 8-B loads and a funnel shift
__device__ __forceinline__ uint64_t dd_u64(const uint8_t* bytes, uint64_t s) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(bytes + (s & ~7ull));
    const uint32_t sh = (uint32_t)(s & 7u) * 8u;
    const uint64_t lo = q[0];
    return sh ? (lo >> sh) | (q[1] << (64u - sh)) : lo;
}

__device__ __forceinline__ uint64_t dd_mix(uint64_t h, uint64_t c) {
    c *= 0x87C37B91114253D5ull;
    c = (c << 31) | (c >> 33);
    c *= 0x4CF5AD432745937Full;
    h ^= c;
    h = (h << 27) | (h >> 37);
    return h * 5u + 0x52DCE729ull;
}

// 64-bit hash of a topic.  The first 64 bytes: NH (sum over word pairs of
// (w[2i] + k[2i]) * (w[2i+1] + k[2i+1]), exact 32x32 -> 64-bit products: one
// v_mad_u64_u32 per 8 bytes, where a 64x64 multiply chain took three 64-bit
// multiplies of ~4 quarter-rate ops each); the bytes past 64 (rare) chained
// through dd_mix; then the length and a 64-bit finaliser.  Only the table's
// spread depends on it: a collision costs a probe and a byte compare.
__device__ __forceinline__ uint64_t dd_hash(const uint8_t* bytes, uint64_t b, uint32_t len, const uint32_t (&c)[16]) {
    constexpr uint32_t K[16] = {0x9E3779B1u, 0x85EBCA77u, 0xC2B2AE3Du, 0x27D4EB2Fu, 0x165667B1u, 0xD3A2646Du,
                                0xFD7046C5u, 0xB55A4F09u, 0x6C8E9CF5u, 0x7FEB352Du, 0x846CA68Bu, 0x94D049BBu,
                                0xBF58476Du, 0x1CE4E5B9u, 0x2545F491u, 0x9FB21C65u};
    uint64_t h = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) h += (uint64_t)(c[2 * j] + K[2 * j]) * (uint64_t)(c[2 * j + 1] + K[2 * j + 1]);
    for (uint32_t k = 64; k < len; k += 8)   // (topics over 64 bytes: rare, kept narrow)
        h = dd_mix(h, low_bytes(dd_u64(bytes, b + k), len - k < 8u ? len - k : 8u));
    h ^= (uint64_t)len * 0xC2B2AE3D27D4EB4Full;
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    return h ^ (h >> 33);
}

// the len bytes at b (first 64 in c) equal to the len bytes at ob?
__device__ __forceinline__ bool dd_equal(const uint8_t* bytes, const uint32_t (&c)[16], uint64_t b, uint64_t ob,
                                         uint32_t len) {
    uint32_t o[16];
    dd_load64(bytes, ob, len, o);
    uint32_t diff = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) diff |= c[j] ^ o[j];
    for (uint32_t k = 64; diff == 0 && k < len; k += 8)   // (topics over 64 bytes: rare, kept narrow)
        diff |= low_bytes(dd_u64(bytes, b + k) ^ dd_u64(bytes, ob + k), len - k < 8u ? len - k : 8u) != 0;
    return diff == 0;
}

// The global table: a slot holds ONE topic, {1 | 10 hash bits | length (13
// bits) | byte offset (40 bits)}.  A claim probes from the hash's home; an
// occupant with the same hash bits and length has its bytes compared, and
// only equal bytes join it (lowering the offset with atomicMin: the topic's
// first occurrence has the lowest offset -- offsets grow with the publish
// index, strictly for non-empty topics); anything else probes on.  So a
// slot's topic never changes once claimed, and a hash collision costs a
// probe, never a wrong row.
constexpr uint64_t DD_OFF_MASK = (1ull << DD_OFF_BITS) - 1ull;

// Slots are read with PLAIN loads (this XCD's L2, not the device-coherent
// path): a stale copy can only be 0 (then the CAS returns the slot's value)
// or an older offset of the slot's own topic (equal bytes all the same) --
// a slot's topic never changes.
__device__ __forceinline__ unsigned long long dd_want(uint64_t h, uint64_t b, uint32_t len) {
    return (1ull << 63) | (((h >> 54) & 0x3FFull) << 53) | ((uint64_t)len << DD_OFF_BITS) | b;
}

__device__ __forceinline__ uint32_t dd_claim(const DedupArgs& a, uint64_t h, uint64_t b, uint32_t len,
                                             const uint32_t (&c)[16]) {
    const unsigned long long want = dd_want(h, b, len);
    uint64_t i = h & a.mask;
    for (;;) {
        unsigned long long v = a.table[i];
        if (v == 0) {
            v = atomicCAS(&a.table[i], 0ull, want);
            if (v == 0) return (uint32_t)i;
        }
        if ((v >> DD_OFF_BITS) == (want >> DD_OFF_BITS) && dd_equal(a.bytes, c, b, v & DD_OFF_MASK, len)) {
            if (b < (v & DD_OFF_MASK)) atomicMin(&a.table[i], want);
            return (uint32_t)i;
        }
        i = (i + 1) & a.mask;
    }
}

// Pass 1 (claim), one thread per publish, its bytes in registers.  A
// publish whose topic already holds its home slot joins it at once.  C5's
// hot topics would put hundreds of thousands of claims on one slot's line
// (Zipf over 10k hot topics, the first ~9% of the publishes), so the others
// first collapse in the workgroup's LDS: equal hashes elect the lowest thread,
// whose bytes each follower compares with its own (a follower whose bytes
// differ -- a 64-bit collision -- takes part in the next round's election), and
// only the leaders claim global slots; followers take their leader's.
constexpr uint32_t DD_BLOCK = 256;
constexpr uint32_t DD_LT = 512;       // LDS election slots (load <= 1/2)

__global__ __launch_bounds__(DD_BLOCK) void tm_dedup_claim(DedupArgs a) {
    __shared__ unsigned long long lkey[DD_LT];
    __shared__ uint32_t lmin[DD_LT];
    __shared__ uint32_t lslot[DD_BLOCK];
    __shared__ uint64_t lb[DD_BLOCK];
    __shared__ uint32_t ll[DD_BLOCK];
    __shared__ uint32_t lc[16][DD_BLOCK];   // every publish's first 64 bytes: a follower checks its leader's here
    const uint32_t tid = threadIdx.x;
    const uint32_t t = blockIdx.x * DD_BLOCK + tid;
    const bool valid = t < a.n;
    uint64_t b = 0, h = 0;
    uint32_t len = 0;
    if (valid) {
        b = a.offs[t] - a.base;
        len = (uint32_t)(a.offs[t + 1] - a.base - b);
    }
    bool resolved = false;
    uint32_t rslot = 0;
    {
        uint32_t c[16];
        dd_load64(a.bytes, b, len, c);
        if (valid) {
            h = dd_hash(a.bytes, b, len, c);
            if (a.weak_hash) h = ((uint64_t)len << 40) | ((uint64_t)len << 8) | 1ull;
            // a topic already in its home slot (the common case once a hot
            // topic has been claimed: C5's 90% hot publishes) joins it here,
            // two L2 reads, no election and no atomic
            const uint64_t i = h & a.mask;
            const unsigned long long want = dd_want(h, b, len), v = a.table[i];
            if (v && (v >> DD_OFF_BITS) == (want >> DD_OFF_BITS) && dd_equal(a.bytes, c, b, v & DD_OFF_MASK, len)) {
                if (b < (v & DD_OFF_MASK)) atomicMin(&a.table[i], want);
                resolved = true;
                rslot = (uint32_t)i;
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < 16; ++q) lc[q][tid] = c[q];
    }
    lb[tid] = b;
    ll[tid] = len;
    bool pend = valid && !resolved, leader = false;
    uint32_t lead = tid, s = 0;
    while (__syncthreads_or(pend)) {
        for (uint32_t k = tid; k < DD_LT; k += DD_BLOCK) {
            lkey[k] = 0;
            lmin[k] = NONE;
        }
        __syncthreads();
        if (pend) {
            s = (uint32_t)(h >> 7) & (DD_LT - 1);
            for (;;) {
                const unsigned long long o = atomicCAS(&lkey[s], 0ull, (unsigned long long)(h | 1ull));
                if (o == 0 || o == (h | 1ull)) break;
                s = (s + 1) & (DD_LT - 1);
            }
            atomicMin(&lmin[s], tid);
        }
        __syncthreads();
        if (pend) {
            const uint32_t L = lmin[s];
            if (L == tid) {
                leader = true;
                pend = false;
            } else if (ll[L] == len) {   // the leader's first 64 bytes from LDS, the rest (long topics) from HBM
                uint32_t diff = 0;
#pragma unroll
                for (uint32_t q = 0; q < 16; ++q) diff |= lc[q][L] ^ lc[q][tid];
                bool eq = diff == 0;
                if (eq && len > 64u) {
                    uint32_t c[16];
#pragma unroll
                    for (uint32_t q = 0; q < 16; ++q) c[q] = lc[q][tid];
                    eq = dd_equal(a.bytes, c, b, lb[L], len);
                }
                if (eq) {
                    lead = L;
                    pend = false;
                }
            }
        }
    }
    if (leader) {
        uint32_t c[16];
#pragma unroll
        for (uint32_t q = 0; q < 16; ++q) c[q] = lc[q][tid];
        lslot[tid] = dd_claim(a, h, b, len, c);
    }
    __syncthreads();
    if (valid) a.slot[t] = resolved ? rslot : lslot[lead];
}

// Pass 2 (count): publish t is its topic's representative when its offset is
// the slot's (an empty topic: the first of the empty publishes at that
// offset).  Ballots -> repbits; per DD_TILE block the representatives and
// their bytes -> bcount / bbytes (scanned next).  16 independent slot ->
// table chains per thread in flight.
constexpr uint32_t DD_PT = DD_TILE / 256;

__global__ __launch_bounds__(256) void tm_dedup_count(DedupArgs a) {
    __shared__ uint32_t sc[4], sb[4];
    const uint32_t tid = threadIdx.x;
    const uint32_t t0 = blockIdx.x * DD_TILE;
    // every load of a stage issued before the next stage's: slot + offsets,
    // then the table (16 independent chains per thread)
    uint32_t sl[DD_PT];
    uint64_t o0[DD_PT], o1[DD_PT];
#pragma unroll
    for (uint32_t u = 0; u < DD_PT; ++u) {
        const uint32_t t = t0 + u * 256 + tid;
        const bool in = t < a.n;
        sl[u] = in ? a.slot[t] : 0u;
        o0[u] = in ? a.offs[t] : 0ull;
        o1[u] = in ? a.offs[t + 1] : 0ull;
    }
    unsigned long long v[DD_PT];
#pragma unroll
    for (uint32_t u = 0; u < DD_PT; ++u) v[u] = (t0 + u * 256 + tid < a.n) ? a.table[sl[u]] : 0ull;
    uint32_t cnt = 0, byt = 0;
#pragma unroll
    for (uint32_t u = 0; u < DD_PT; ++u) {
        const uint32_t t = t0 + u * 256 + tid;
        const uint32_t len = (uint32_t)(o1[u] - o0[u]);
        bool rep = t < a.n && (v[u] & DD_OFF_MASK) == o0[u] - a.base;
        if (rep && !len && t) rep = a.offs[t - 1] != o0[u];   // (empty topics: the first at that offset)
        const uint64_t bits = __ballot(rep);
        if ((tid & 63) == 0) a.repbits[(t0 + u * 256 + tid) / 64] = bits;
        cnt += rep ? 1u : 0u;
        byt += rep ? len : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_xor(cnt, o, 64);
        byt += __shfl_xor(byt, o, 64);
    }
    if ((tid & 63) == 0) {
        sc[tid >> 6] = cnt;
        sb[tid >> 6] = byt;
    }
    __syncthreads();
    if (tid == 0) {
        a.bcount[blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
        a.bbytes[blockIdx.x] = sb[0] + sb[1] + sb[2] + sb[3];
    }
}

// exclusive scan of one u64 per thread over a 256-thread block (-> the block total)
__device__ __forceinline__ uint64_t block256_excl_scan(uint64_t v, uint64_t* sh, uint64_t& total) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t incl = v;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) sh[wid] = incl;
    __syncthreads();
    uint64_t base = 0;
    for (uint32_t w = 0; w < wid; ++w) base += sh[w];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    return base + incl - v;
}

// Pass 3 (compact), same blocks, 16 consecutive publishes per thread: every
// representative's row and byte offset (block base from the scans + its rank
// in the block), its bytes copied into the tokeniser's input, and
// srow[slot] = row, rrep[row] = publish for the expansion.  A thread's
// representatives get consecutive rows and one contiguous byte range, which it
// writes as aligned dwords assembled in a shift register (byte stores only
// for the partial dwords at its two ends, shared with its neighbours): the
// first blocks hold most first occurrences (C5: ~1,900 of the first 4,096
// publishes), and byte stores made them the kernel's tail; 4 publishes per
// thread keep a thread's serial representatives few.
__device__ __forceinline__ void dd_put(uint8_t* dst, uint64_t lo, uint64_t hi, uint64_t& acc, uint32_t& bits,
                                       uint64_t& w, uint32_t v, uint32_t nb) {
    // append nb (<= 4) bytes of v at dword w's bit `bits`; full dwords inside
    // [lo, hi) are stored whole, a dword reaching outside byte by byte
    acc |= (uint64_t)v << bits;
    bits += 8u * nb;
    if (bits >= 32u) {
        const uint64_t d0 = w * 4;
        if (d0 >= lo && d0 + 4 <= hi) {
            *reinterpret_cast<uint32_t*>(dst + d0) = (uint32_t)acc;
        } else {
            for (uint32_t q = 0; q < 4; ++q)
                if (d0 + q >= lo && d0 + q < hi) dst[d0 + q] = (uint8_t)(acc >> (8 * q));
        }
        acc >>= 32;
        bits -= 32u;
        ++w;
    }
}

__global__ __launch_bounds__(256) void tm_dedup_compact(DedupArgs a) {
    __shared__ uint64_t sh[4];
    const uint32_t tid = threadIdx.x;
    const uint32_t nblk = dedup_blocks(a.n);
    const uint32_t first = blockIdx.x * DD_TILE + tid * DD_PT;
    const uint32_t row0 = a.bcount[blockIdx.x] + a.rbs[blockIdx.x / SCAN_TILE];
    const uint64_t off0 = (uint64_t)a.bbytes[blockIdx.x] + a.bbs[blockIdx.x / SCAN_TILE];
    const uint32_t mine = (uint32_t)(a.repbits[first / 64] >> (first & 63)) & ((1u << DD_PT) - 1u);
    uint32_t my_bytes = 0;
#pragma unroll
    for (uint32_t j = 0; j < DD_PT; ++j) {
        if ((mine >> j) & 1u) {
            const uint32_t t = first + j;
            my_bytes += (uint32_t)(a.offs[t + 1] - a.offs[t]);
        }
    }
    uint64_t tot;
    const uint64_t ex = block256_excl_scan(((uint64_t)my_bytes << 16) | (uint64_t)__popc(mine), sh, tot);
    uint32_t row = row0 + (uint32_t)(ex & 0xFFFFu);
    const uint64_t lo = off0 + (ex >> 16), hi = lo + my_bytes;   // this thread's bytes in cbytes
    uint64_t off = lo;
    if (blockIdx.x == 0 && tid == 0) {   // totals: the scans left them at [nblk]
        a.dd[0] = a.bcount[nblk];
        a.coffs[a.bcount[nblk]] = a.bbytes[nblk];
    }
    uint64_t acc = 0, w = lo >> 2;
    uint32_t bits = 8u * (uint32_t)(lo & 3u);
    for (uint32_t rest = mine; rest; rest &= rest - 1) {   // (representatives are few: not unrolled)
        const uint32_t t = first + (uint32_t)__ffs(rest) - 1u;
        a.srow[a.slot[t]] = row;
        a.rrep[row] = t;
        a.coffs[row] = off;
        const uint64_t b = a.offs[t] - a.base;
        const uint32_t n = (uint32_t)(a.offs[t + 1] - a.offs[t]);
        for (uint32_t k = 0; k < n; k += 64) {
            uint32_t x[16];
            dd_load64(a.bytes, b + k, n - k, x);
            const uint32_t m = n - k < 64u ? n - k : 64u;
#pragma unroll
            for (uint32_t q = 0; q < 16; ++q) {
                if (4u * q >= m) break;
                const uint32_t nb = m - 4u * q < 4u ? m - 4u * q : 4u;
                dd_put(a.cbytes, lo, hi, acc, bits, w, x[q], nb);   // (x is zero past the topic)
            }
        }
        ++row;
        off += n;
    }
    if (bits && hi > lo) {   // the last partial dword
        const uint64_t d0 = w * 4;
        for (uint32_t q = 0; q < 4; ++q)
            if (d0 + q >= lo && d0 + q < hi) a.cbytes[d0 + q] = (uint8_t)(acc >> (8 * q));
    }
}

// After the walk, per row (a grid-stride loop over the device-counted rows):
// its (count, start) go to smeta at its table slot, and the slot is cleared
// (nothing reads the table after the compaction): the next dedup pass finds it
// zero without a memset.
__global__ __launch_bounds__(256) void tm_dedup_rowmeta(DedupArgs a) {
    const uint32_t rows = *a.dd;
    for (uint32_t r = blockIdx.x * 256 + threadIdx.x; r < rows; r += gridDim.x * 256) {
        const uint32_t s = a.slot[a.rrep[r]];
        const unsigned long long sr = a.src[r];
        a.smeta[s] = uint4{a.count[r], 0u, (uint32_t)sr, (uint32_t)(sr >> 32)};
        a.table[s] = 0;
    }
}

// Then every publish gets its row's (count, start) -- the result per publish
// -- through its slot: slot[t], then smeta[slot] (the hot topics' entries
// stay in L2), and the batch's delivered matches are summed per block.
constexpr uint32_t EXPAND_PER_THREAD = DD_EXPAND_TILE / 256;
__global__ __launch_bounds__(256) void tm_dedup_expand(DedupArgs a) {
    __shared__ unsigned long long sh[4];
    const uint32_t base = blockIdx.x * 256 * EXPAND_PER_THREAD + threadIdx.x;
    // staged: every slot, then every slot's (count, start) -- each stage's
    // loads in flight together
    uint32_t sl[EXPAND_PER_THREAD];
#pragma unroll
    for (uint32_t u = 0; u < EXPAND_PER_THREAD; ++u) {
        const uint32_t t = base + u * 256;
        sl[u] = t < a.n ? a.slot[t] : 0u;
    }
    uint4 m[EXPAND_PER_THREAD];
#pragma unroll
    for (uint32_t u = 0; u < EXPAND_PER_THREAD; ++u) m[u] = base + u * 256 < a.n ? a.smeta[sl[u]] : uint4{0u, 0u, 0u, 0u};
    unsigned long long sum = 0;
#pragma unroll
    for (uint32_t u = 0; u < EXPAND_PER_THREAD; ++u) {
        const uint32_t t = base + u * 256;
        if (t < a.n) {
            a.pcount[t] = m[u].x;
            a.psrc[t] = ((unsigned long long)m[u].w << 32) | m[u].z;
            sum += m[u].x;
        }
    }
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = sum;
    __syncthreads();
    // a partial sum per block, added up by tm_dedup_sum: one same-address
    // atomic per block serialised at ~30 ns each (4,883 blocks: ~0.15 ms)
    if (threadIdx.x == 0) a.bsum[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// row_of[t] = srow[slot[t]]: the publish -> row map, built only when the host
// asks for it (tm_batch_row_map) -- the per-launch expansion skips the 40 MB
__global__ __launch_bounds__(256) void tm_dedup_rowof(DedupArgs a) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t < a.n) a.row_of[t] = a.srow[a.slot[t]];
}

// the expansion's block sums -> the batch's delivered matches; the rows for
// the host's read-back
__global__ __launch_bounds__(1024) void tm_dedup_sum(DedupArgs a, uint32_t nb) {
    __shared__ unsigned long long sh[16];
    unsigned long long s = 0;
    for (uint32_t i = threadIdx.x; i < nb; i += 1024) s += a.bsum[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < 16; ++w) t += sh[w];
        if (t) atomicAdd(&a.stats[ST_DELIVERED], t);
        a.ctrl[CTRL_NROWS] = a.dd[0];
    }
}

// ------------------------------------------------ sampled rows (tm_batch_sample)

// A few rows of a waited batch, as the walk left them (count + start into the
// staging area), gathered into a compact CSR: the multi-device self-check
// reads ~3,000 rows per slice this way instead of a whole 10M-row CSR.
__global__ __launch_bounds__(256) void tm_sample_meta(const uint32_t* count, const unsigned long long* src,
                                                       const uint32_t* rows, uint32_t k, uint32_t* out_cnt,
                                                       unsigned long long* out_src) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= k) return;
    const uint32_t r = rows[i];
    out_cnt[i] = count[r];
    out_src[i] = src[r];
}

// one wave per sampled row: its ids to out[off[i] ..)
__global__ __launch_bounds__(64) void tm_sample_ids(const uint32_t* sfids, const uint32_t* cnt,
                                                     const unsigned long long* src, const uint64_t* off,
                                                     uint32_t* out) {
    const uint32_t i = blockIdx.x;
    const uint32_t c = cnt[i];
    const unsigned long long s = src[i];
    const uint64_t o = off[i];
    for (uint32_t j = threadIdx.x; j < c; j += 64) out[o + j] = sfids[s + j];
}

// ------------------------------------------------ token batches (sharded mode)

// Row gather for the sharded exchange: 16 lanes per row (rows are short: the
// words of a topic, or one topic's match list), lanes stride over long rows.
__global__ __launch_bounds__(256) void tm_gather_rows(const uint32_t* src, const int64_t* src_off, const int64_t* idx,
                                                       uint32_t n, const int64_t* dst_off, uint32_t* dst) {
    const uint64_t g = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const uint32_t sub = threadIdx.x & 15;
    if (g >= n) return;
    const int64_t r = idx[g];
    const int64_t b = src_off[r], e = src_off[r + 1], d = dst_off[g];
    for (int64_t i = sub; i < e - b; i += 16) dst[d + i] = src[b + i];
}

// Validates a device-resident token batch before any walk reads it (toff
// monotone from 0 to nwords, deep topics flagged for the generic path) and
// compacts the generic-path topics into slow_list / *d_nslow.  Any violation
// sets *d_bad; the host refuses the batch.
__global__ __launch_bounds__(256) void tm_token_check(const uint32_t* toff, const uint8_t* tflags, uint32_t n,
                                                       uint64_t nwords, uint32_t* slow_list, uint32_t* d_nslow,
                                                       uint32_t* d_bad) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    bool slow = false;
    if (t < n) {
        const uint32_t b = toff[t], e = toff[t + 1];
        const uint8_t f = tflags[t];
        const bool ok = b <= e && (uint64_t)e <= nwords && (t > 0 || b == 0) && (t + 1 < n || (uint64_t)e == nwords) &&
                        (f & ~(TF_DOLLAR | TF_SLOW)) == 0 && (e - b <= FAST_MAX_DEPTH || (f & TF_SLOW));
        if (!ok) atomicOr(d_bad, 1u);
        slow = ok && (f & TF_SLOW);
    }
    const uint64_t m = __ballot(slow);
    if (!m) return;
    const uint32_t first = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(d_nslow, (uint32_t)__popcll(m));
    base = __shfl(base, first, 64);
    if (slow) slow_list[base + prefix_count(m)] = t;
}

// Shard of each topic (tm_filter_shard's rule on the topic side): the shard of
// its first two words when both are interned literals, else nshards (every
// shard resolves it: only replicated filters can match).
__global__ __launch_bounds__(256) void tm_tokens_shard(const uint32_t* words, const uint32_t* toff, uint32_t n,
                                                        uint32_t nshards, uint32_t* shard) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    const uint32_t b = toff[t], d = toff[t + 1] - b;
    uint32_t s = nshards;
    if (d >= 2) {
        const uint32_t i0 = words[b] & WID_MASK, i1 = words[b + 1] & WID_MASK;
        const bool lit0 = i0 != W_UNKNOWN && i0 != W_PLUS && i0 != W_HASH;
        const bool lit1 = i1 != W_UNKNOWN && i1 != W_PLUS && i1 != W_HASH;
        if (lit0 && lit1) s = prefix_shard(i0, i1, nshards);
    }
    shard[t] = s;
}

// ---------------------------------------- in-process filter-sharded group

// The publish's owner: its shard, or (G = any shard resolves it: only
// replicated filters can match) spread round-robin by publish index.
__device__ __forceinline__ uint32_t part_owner(const PartArgs& a, uint32_t t) {
    const uint32_t o = a.owner[t];
    return o < a.G ? o : t % a.G;
}

__device__ __forceinline__ uint32_t scan_at(const uint32_t* off, const uint32_t* bs, uint32_t i) {
    return off[i] + bs[i / SCAN_TILE];
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Pass 1: per block and owner, publishes and words -> cnt / wcnt (g-major, so
// one scan over them numbers each owner's publishes contiguously).
__global__ __launch_bounds__(PART_BLOCK) void tm_part_count(PartArgs a) {
    __shared__ uint32_t sc[PART_BLOCK / 64][PART_MAX_G], sw[PART_BLOCK / 64][PART_MAX_G];
    const uint32_t t = blockIdx.x * PART_BLOCK + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const bool valid = t < a.n;
    const uint32_t g_me = valid ? part_owner(a, t) : a.G;
    const uint32_t depth = valid ? a.toff[t + 1] - a.toff[t] : 0u;
    for (uint32_t g = 0; g < a.G; ++g) {
        const uint64_t m = __ballot(g_me == g);
        const uint32_t w = wave_sum(g_me == g ? depth : 0u);
        if (lane == 0) { sc[wid][g] = (uint32_t)__popcll(m); sw[wid][g] = w; }
    }
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < a.G; g += PART_BLOCK) {
        uint32_t c = 0, w = 0;
        for (uint32_t k = 0; k < PART_BLOCK / 64; ++k) { c += sc[k][g]; w += sw[k][g]; }
        a.cnt[g * a.nb + blockIdx.x] = c;
        a.wcnt[g * a.nb + blockIdx.x] = w;
    }
}

// segs[g] = first partitioned position of owner g (segs[G] = n), segs[G + 1 + g]
// = its first word (segs[2G + 1] = all words): the host sizes each shard's part.
__global__ void tm_part_segs(PartArgs a) {
    const uint32_t g = threadIdx.x;
    if (g > a.G) return;
    const uint32_t i = g * a.nb;
    a.segs[g] = g < a.G ? scan_at(a.cnt_off, a.cnt_bs, i) : a.cnt_off[a.G * a.nb];
    a.segs[a.G + 1 + g] = g < a.G ? scan_at(a.w_off, a.w_bs, i) : a.w_off[a.G * a.nb];
}

// Pass 3: every publish to its place in its owner's part, with its words; the
// part's word offsets restart at wbase[g] (where the part lands in owner g's
// token batch, after the parts of earlier slices), so part g's offsets sit at
// ptoff[segs[g] + g ..] ready to be copied.
__global__ __launch_bounds__(PART_BLOCK) void tm_part_scatter(PartArgs a) {
    __shared__ uint32_t sc[PART_BLOCK / 64][PART_MAX_G], sw[PART_BLOCK / 64][PART_MAX_G];
    const uint32_t t = blockIdx.x * PART_BLOCK + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const bool valid = t < a.n;
    const uint32_t g_me = valid ? part_owner(a, t) : a.G;
    const uint32_t depth = valid ? a.toff[t + 1] - a.toff[t] : 0u;
    uint32_t rank = 0, wpre = 0;
    for (uint32_t g = 0; g < a.G; ++g) {
        const bool mine = g_me == g;
        const uint64_t m = __ballot(mine);
        // inclusive scan of this owner's depths across the wave
        uint32_t incl = mine ? depth : 0u;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += u;
        }
        if (mine) { rank = prefix_count(m); wpre = incl - depth; }
        if (lane == 63) { sc[wid][g] = (uint32_t)__popcll(m); sw[wid][g] = incl; }
    }
    __syncthreads();
    // each part's closing offset (its word count)
    if (blockIdx.x == 0 && threadIdx.x < a.G) {
        const uint32_t g = threadIdx.x;
        const uint32_t tend = g + 1 < a.G ? scan_at(a.cnt_off, a.cnt_bs, (g + 1) * a.nb) : a.cnt_off[a.G * a.nb];
        const uint32_t wend = g + 1 < a.G ? scan_at(a.w_off, a.w_bs, (g + 1) * a.nb) : a.w_off[a.G * a.nb];
        a.ptoff[tend + g] = wend - scan_at(a.w_off, a.w_bs, g * a.nb) + a.wbase[g];
    }
    if (!valid) return;
    uint32_t bt = 0, bw = 0;   // earlier waves of the block, same owner
    for (uint32_t k = 0; k < wid; ++k) { bt += sc[k][g_me]; bw += sw[k][g_me]; }
    const uint32_t i = g_me * a.nb + blockIdx.x;
    const uint32_t p = scan_at(a.cnt_off, a.cnt_bs, i) + bt + rank;
    const uint32_t w = scan_at(a.w_off, a.w_bs, i) + bw + wpre;
    const uint32_t wseg = scan_at(a.w_off, a.w_bs, g_me * a.nb);
    a.order[p] = t + a.tbase;
    const uint32_t src = a.toff[t];
    const uint32_t woff = w - wseg + a.wbase[g_me];   // in owner g's batch
    if (a.dtoff[g_me]) {   // straight into the owner's batch (local, or a peer's HBM)
        const uint32_t tseg = scan_at(a.cnt_off, a.cnt_bs, g_me * a.nb);
        const uint32_t q = p - tseg + a.rbase[g_me];
        a.dflags[g_me][q] = a.tflags[t];
        a.dtoff[g_me][q] = woff;
        uint32_t* dw = a.dwords[g_me] + woff;
        for (uint32_t k = 0; k < depth; ++k) dw[k] = a.words[src + k];
        return;
    }
    a.ptflags[p] = a.tflags[t];
    a.ptoff[p + g_me] = woff;
    for (uint32_t k = 0; k < depth; ++k) a.pwords[w + k] = a.words[src + k];
}

__global__ __launch_bounds__(256) void tm_unpart_counts(const uint32_t* order, const uint32_t* counts_p, uint32_t n,
                                                         uint32_t* counts_o) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p < n) counts_o[order[p]] = counts_p[p];
}

// 16 lanes per row (rows are short lists of filter ids; lanes stride long ones)
__global__ __launch_bounds__(256) void tm_unpart_rows(const uint32_t* order, const uint32_t* counts_p, uint32_t n,
                                                       const uint32_t* src_off, const uint32_t* src_bs,
                                                       const uint32_t* dst_off, const uint32_t* dst_bs,
                                                       const uint32_t* ids_p, uint32_t* out, uint32_t* rowg) {
    const uint64_t p = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const uint32_t sub = threadIdx.x & 15;
    if (p > n) return;
    if (p == n) {   // the closing offset
        if (sub == 0) rowg[n] = dst_off[n];
        return;
    }
    const uint32_t t = order[p];
    const uint32_t len = counts_p[p];
    const uint32_t src = scan_at(src_off, src_bs, (uint32_t)p), dst = scan_at(dst_off, dst_bs, t);
    if (sub == 0) rowg[t] = dst;
    for (uint32_t k = sub; k < len; k += 16) out[dst + k] = ids_p[src + k];
}

// counts[t] = |row t|; gids[i] = ids[i] * mul + add (a shard's global ids).
__global__ __launch_bounds__(256) void tm_export(const uint32_t* row_off, const uint32_t* ids, uint32_t n, uint64_t total,
                                                  uint32_t* counts, uint32_t* gids, uint32_t mul, uint32_t add) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += stride) gids[i] = ids[i] * mul + add;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) counts[i] = row_off[i + 1] - row_off[i];
}

__global__ void tm_scatter_slots(Slot* slots, const uint32_t* idx, const Slot* vals, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) slots[idx[i]] = vals[i];
}

__global__ void tm_scatter_fmeta(uint64_t* foff, uint32_t* flen, const uint32_t* idx, const uint64_t* off,
                                 const uint32_t* len, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { foff[idx[i]] = off[i]; flen[idx[i]] = len[i]; }
}

// ------------------------------------------------------------ device tokeniser
// emqx_topic:words/1 (src/emqx_topic.erl:150-164: binary:split on "/", '' / '+'
// / '#' as their atoms) plus the engine's interning, on the device: the same
// word entries (class << 29 | id), flags and generic-path list as the host
// tokeniser (tm_batch.cpp tokenize_range).  One wavefront per tile of 64
// topics, whose bytes are contiguous in the batch:
//   tm_tok_count  words per tile = '/' bytes in the tile's range + topics,
//                 counted from coalesced dword loads (bit tricks, no per-byte
//                 loop); also clears the launch's control words;
//   (scan of the tile counts)
//   tm_tok_fill   the tile's bytes are staged in LDS by coalesced loads; each
//                 lane splits its own topic there (word starts / lengths into
//                 an LDS list, flags, in-tile word offsets by a wave scan);
//                 then the lanes take the tile's WORDS round-robin -- class,
//                 reserved atoms, dictionary probe with the first 8 bytes
//                 compared inline -- and the tile's words leave LDS as one
//                 coalesced run.  Tiles too long for the LDS budget take a
//                 lane-per-topic path that reads the bytes from HBM.

constexpr uint32_t TOK_LANE_BYTES = 48;                 // bytes of the window each lane splits
constexpr uint32_t TOK_BYTES = 64 * TOK_LANE_BYTES;     // LDS bytes per tile (16-B aligned window)
constexpr uint32_t TOK_WORDS = 512;                     // words per tile on the LDS path

// bytes with value v in the 4 bytes of x (SWAR): each matching byte -> 0x80
__device__ __forceinline__ uint32_t byte_eq(uint32_t x, uint32_t v) {
    const uint32_t y = x ^ (v * 0x01010101u);
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}

__device__ __forceinline__ uint32_t tok_class(uint8_t c0, uint32_t n, bool& irregular) {
    if (n == 0) return C_EMPTY;
    if (c0 == '+') {
        if (n > 1) irregular = true;
        return C_ABOVE;
    }
    if (c0 < '#') return C_BELOW;
    if (c0 < '+') return C_BETWEEN;
    return C_ABOVE;
}

// does the cuckoo key e (DictKey as uint4) hold the word of (head, n) whose
// bytes 8.. are p[8..n)?  (words over 8 bytes: the tail by id, then the arena)
template <class P>
__device__ __forceinline__ bool ck_match(const TokArgs& a, const uint4& e, uint64_t head, uint32_t n, P p) {
    if (e.z != n || e.x != (uint32_t)head || e.y != (uint32_t)(head >> 32)) return false;
    if (n <= 8) return true;
    const DictTail t = a.tails[e.w];
    uint64_t h2 = 0;
    for (uint32_t k = 8; k < 16 && k < n; ++k) h2 |= (uint64_t)p[k] << (8 * (k - 8));
    if (t.head2 != h2) return false;
    const uint8_t* q = a.arena + t.off;
    for (uint32_t k = 16; k < n; ++k)
        if (q[k] != p[k]) return false;
    return true;
}

// id of word p[0..n) in the device dictionary (W_UNKNOWN if absent); P is an
// LDS or global byte pointer
template <class P>
__device__ __forceinline__ uint32_t dict_find(const TokArgs& a, P p, uint32_t n) {
    uint32_t h32 = HW_SEED;
    for (uint32_t i = 0; i < n; i += 4) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4 && i + k < n; ++k) v |= (uint32_t)p[i + k] << (8 * k);
        h32 = hw_step(h32, v);
    }
    const uint32_t h = hw_final(h32, n), m = (uint32_t)a.dict_mask;
    uint64_t head = 0;
    for (uint32_t k = 0; k < 8 && k < n; ++k) head |= (uint64_t)p[k] << (8 * k);
    const uint4 e1 = *reinterpret_cast<const uint4*>(a.keys + (h & m));
    if (e1.w == 0) return W_UNKNOWN;   // slots never empty again once filled: absent
    if (ck_match(a, e1, head, n, p)) return e1.w;
    uint32_t g32 = HW_SEED2;
    for (uint32_t i = 0; i < n; i += 4) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4 && i + k < n; ++k) v |= (uint32_t)p[i + k] << (8 * k);
        g32 = hw_step(g32, v);
    }
    const uint4 e2 = *reinterpret_cast<const uint4*>(a.keys + (hw_final(g32, n) & m));
    if (ck_match(a, e2, head, n, p)) return e2.w;
    return W_UNKNOWN;
}

// entry of the word p[0..n): class << 29 | id
template <class P>
__device__ __forceinline__ uint32_t word_entry(const TokArgs& a, P p, uint32_t n, bool& irregular) {
    const uint8_t c0 = n ? p[0] : 0;
    const uint32_t cls = tok_class(c0, n, irregular);
    uint32_t id;
    if (n == 0) id = W_EMPTY;
    else if (n == 1 && c0 == '+') id = W_PLUS;
    else if (n == 1 && c0 == '#') id = W_HASH;
    else id = dict_find(a, p, n);
    return (cls << WID_BITS) | id;
}

__device__ __forceinline__ void tok_append_slow(const TokArgs& a, bool slow, uint32_t t) {
    const uint64_t m = __ballot(slow);
    if (!m) return;
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 0) base = atomicAdd(a.d_nslow, (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (slow) a.slow_list[base + prefix_count(m)] = t;
}

// byte_eq's 0x80 flags of one dword -> 4 bits (byte j -> bit j)
__device__ __forceinline__ uint32_t gather4(uint32_t m) { return (((m >> 7) * 0x204081u) >> 21) & 0xFu; }

// '/' bytes of 16 bytes, byte j -> bit j
__device__ __forceinline__ uint32_t slash_mask16(const uint4& x) {
    return gather4(byte_eq(x.x, '/')) | (gather4(byte_eq(x.y, '/')) << 4) | (gather4(byte_eq(x.z, '/')) << 8) |
           (gather4(byte_eq(x.w, '/')) << 12);
}

constexpr uint32_t TOK_RUN = 63;   // tiles per count run (their 64 boundaries: one per lane)

// pass 1: words per tile = '/' bytes + topics.  Each wave takes a contiguous
// run of tiles (a slice of the grid's share, TOK_RUN at a time): their
// boundaries in one vector load, then the run's bytes streamed with four
// 16-B loads per lane in flight; each lane walks a cursor over the boundaries
// and adds its chunks' '/' counts to the tiles' LDS counters.  Block 0 also
// clears the launch's control words.
__global__ __launch_bounds__(64) void tm_tok_count(TokArgs a) {
    __shared__ uint64_t bnd[TOK_RUN + 1];
    __shared__ uint32_t cnt[TOK_RUN];
    const uint32_t lane = threadIdx.x;
    if (blockIdx.x == 0) {   // the launch's control words (kernels after this one use them)
        if (lane < 2) a.d_nslow[lane] = 0;
        for (uint32_t i = lane; i < a.zero_words; i += 64) a.zero[i] = 0;
    }
    const uint32_t tt = a.tile_topics;
    if (a.d_n) {   // a device-counted batch: the tiles past its topics count 0 words (the scan covers the bound)
        const uint32_t nb = (a.n + tt - 1) / tt;
        a.n = *a.d_n;
        for (uint32_t i = (a.n + tt - 1) / tt + blockIdx.x * 64 + lane; i < nb; i += gridDim.x * 64) a.wcount[i] = 0;
    }
    const uint32_t ntiles = (a.n + tt - 1) / tt;
    const uint32_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    const uint32_t first = blockIdx.x * per, last = min(first + per, ntiles);
    for (uint32_t run = first; run < last; run += TOK_RUN) {
        const uint32_t K = min(TOK_RUN, last - run);
        if (lane <= K) bnd[lane] = a.offs[min((run + lane) * tt, a.n)] - a.base;
        if (lane < K) cnt[lane] = 0;
        __syncthreads();
        const uint64_t B0 = bnd[0], BK = bnd[K], a0 = B0 & ~15ull;
        uint32_t j = 0;   // my cursor: the tile of my current chunk
        for (uint64_t p0 = a0 + 16u * lane; p0 < BK; p0 += 4096) {
            uint4 x[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint64_t p = p0 + 1024u * u;
                x[u] = p < BK ? *reinterpret_cast<const uint4*>(a.bytes + p) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint64_t p = p0 + 1024u * u;
                if (p >= BK) break;
                uint32_t m = slash_mask16(x[u]);
                if (p < B0) m &= ~0u << (uint32_t)(B0 - p);
                if (p + 16 > BK) m &= (1u << (uint32_t)(BK - p)) - 1u;
                while (j + 1 < K && bnd[j + 1] <= p) ++j;
                while (m) {   // bits up to the next boundary belong to tile j
                    const uint64_t lim = j + 1 < K ? bnd[j + 1] - p : 16u;
                    if (lim >= 16) {
                        atomicAdd(&cnt[j], (uint32_t)__popc(m));
                        break;
                    }
                    const uint32_t below = m & ((1u << (uint32_t)lim) - 1u);
                    if (below) atomicAdd(&cnt[j], (uint32_t)__popc(below));
                    m &= ~((1u << (uint32_t)lim) - 1u);
                    ++j;
                }
            }
        }
        __syncthreads();
        if (lane < K) {
            const uint32_t t0 = (run + lane) * tt;
            a.wcount[run + lane] = cnt[lane] + (min(t0 + tt, a.n) - t0);
        }
        __syncthreads();
    }
}

struct alignas(16) TokLds {
    uint8_t bytes[TOK_BYTES + 32];      // the tile's window; + 32: 8-byte reads past a word stay inside
    uint64_t tsb[TOK_BYTES / 64 + 1];   // topic-start bitmap of the window (+1: a lane's bits may straddle)
    uint16_t wst[TOK_WORDS];            // word start | 0x8000 when it is its topic's first word
    uint8_t wtop[TOK_WORDS];            // tile-local topic of each word
    uint32_t ttoff[TILE + 1];           // tile-local first word of each topic; [cnt] = words
    uint32_t tirr[TILE];                // a word of the topic starts with '+' but is not '+'
};

#ifndef TM_TOK_WPL
#define TM_TOK_WPL 2
#endif
constexpr uint32_t TOK_WPL_FILL = TM_TOK_WPL;   // words per lane per lookup round (register budget: occupancy)

// The tile's words w = lane + 64 k, TOK_WPL per lane at a time: start from
// wst, length from the next word's start (the last word of a topic ends at
// the next topic's start, others one byte ('/') before the next word), class
// and reserved atoms, then the dictionary: hash and head from LDS, every
// word's primary cuckoo slot loaded at once; the alternate slot only when the
// primary holds another word (cuckoo slots never empty again once filled, so
// an empty primary slot means the word is absent).  Lookups are bound by L2
// requests, not instructions: one per word is the point.
// Entries (class << 29 | id) go straight to words[].
template <uint32_t TOK_WPL>
__device__ __forceinline__ void tok_lookup(const TokArgs& a, TokLds& L, uint32_t tw, uint32_t wend,
                                           uint64_t tile_base, uint32_t* lw) {
    const uint32_t lane = threadIdx.x;
    const uint32_t mask = (uint32_t)a.dict_mask;
    for (uint32_t base = 0; base < tw; base += 64 * TOK_WPL) {
        uint64_t head[TOK_WPL];
        uint32_t ent[TOK_WPL], len[TOK_WPL], st[TOK_WPL], alt[TOK_WPL], pend = 0;
        uint4 e[TOK_WPL];
#pragma unroll
        for (uint32_t k = 0; k < TOK_WPL; ++k) {
            const uint32_t w = base + lane + 64 * k;
            const bool live = w < tw;
            // word bounds: start from wst, end at the next word's start (minus
            // the '/' unless the next word starts a topic)
            const uint32_t s0 = live ? L.wst[w] & 0x7FFFu : 0u;
            const uint32_t nx = live ? (w + 1 < tw ? L.wst[w + 1] : (wend | 0x8000u)) : 0x8000u;
            const uint32_t n = live ? (nx & 0x7FFFu) - s0 - ((nx & 0x8000u) ? 0u : 1u) : 0u;
            const uint64_t c0w = live ? lds_u64(L.bytes, s0) : 0ull;
            const uint32_t c0 = n ? (uint32_t)(c0w & 0xFF) : 0u;
            // class and reserved atoms, branch-free (emqx_topic:words/1's '' / '+' / '#')
            const uint32_t cls = n == 0 ? C_EMPTY : c0 < '#' ? C_BELOW : c0 < '+' ? C_BETWEEN : C_ABOVE;
            if (live && c0 == '+' && n > 1) L.tirr[L.wtop[w]] = 1;   // "+x": irregular topic
            const bool atom = n == 0 || (n == 1 && (c0 == '+' || c0 == '#'));
            ent[k] = (cls << WID_BITS) | (n == 0 ? W_EMPTY : c0 == '+' ? W_PLUS : W_HASH);
            len[k] = n;
            st[k] = s0;
            // both cuckoo hashes in one pass over the bytes (the mixing of
            // each 4-byte chunk is shared; only the accumulators differ)
            const uint64_t hd = low_bytes(c0w, n < 8 ? n : 8);
            uint32_t d = mix_chunk((uint32_t)hd);
            uint32_t h1 = hw_acc(HW_SEED, d), h2 = hw_acc(HW_SEED2, d);
            if (n > 4) {
                d = mix_chunk((uint32_t)(hd >> 32));
                h1 = hw_acc(h1, d);
                h2 = hw_acc(h2, d);
            }
            for (uint32_t i = 8; i < n; i += 8) {   // words over 8 bytes
                const uint64_t c = low_bytes(lds_u64(L.bytes, s0 + i), n - i < 8 ? n - i : 8);
                d = mix_chunk((uint32_t)c);
                h1 = hw_acc(h1, d);
                h2 = hw_acc(h2, d);
                if (n - i > 4) {
                    d = mix_chunk((uint32_t)(c >> 32));
                    h1 = hw_acc(h1, d);
                    h2 = hw_acc(h2, d);
                }
            }
            head[k] = hd;
            alt[k] = hw_final(h2, n) & mask;
            const bool look = live && !atom;
            e[k] = look ? *reinterpret_cast<const uint4*>(a.keys + (hw_final(h1, n) & mask)) : make_uint4(0, 0, 0, 0);
            pend |= look ? 1u << k : 0u;
        }
        // primary slots: a match or an empty slot settles the word
#pragma unroll
        for (uint32_t k = 0; k < TOK_WPL; ++k) {
            if (!(pend >> k & 1u)) continue;
            if (e[k].w == 0) {
                ent[k] = (ent[k] & ~WID_MASK) | W_UNKNOWN;
                pend &= ~(1u << k);
            } else if (ck_match(a, e[k], head[k], len[k], L.bytes + st[k])) {
                ent[k] = (ent[k] & ~WID_MASK) | e[k].w;
                pend &= ~(1u << k);
            }
        }
        // alternate slots of the rest, all in flight
#pragma unroll
        for (uint32_t k = 0; k < TOK_WPL; ++k)
            if (pend >> k & 1u) e[k] = *reinterpret_cast<const uint4*>(a.keys + alt[k]);
#pragma unroll
        for (uint32_t k = 0; k < TOK_WPL; ++k) {
            if (pend >> k & 1u)
                ent[k] = (ent[k] & ~WID_MASK) | (ck_match(a, e[k], head[k], len[k], L.bytes + st[k]) ? e[k].w : W_UNKNOWN);
            const uint32_t w = base + lane + 64 * k;
            if (w < tw && tile_base + w < a.words_cap) a.words[tile_base + w] = ent[k];
            if (lw && w < tw) lw[w] = ent[k];   // (the fused walk: the tile's words stay in LDS too)
        }
    }
}

// lane-per-topic path of a tile too long for the LDS budget: bytes from HBM
__device__ __forceinline__ uint8_t tok_fill_topic_global(const TokArgs& a, uint32_t t, uint64_t o, bool& slow) {
    const uint64_t b = a.offs[t] - a.base, e = a.offs[t + 1] - a.base;
    const uint8_t* p = a.bytes;
    bool irregular = false;
    uint32_t nw = 0;
    uint64_t ws = b;
    for (uint64_t i = b;; ++i) {
        if (i == e || p[i] == '/') {
            const uint32_t w = word_entry(a, p + ws, (uint32_t)(i - ws), irregular);
            if (o < a.words_cap) a.words[o] = w;
            ++o;
            ++nw;
            if (i == e) break;
            ws = i + 1;
        }
    }
    uint8_t fl = 0;
    if (e > b && p[b] == '$') fl |= TF_DOLLAR;
    if (irregular || nw > FAST_MAX_DEPTH) fl |= TF_SLOW;
    a.tflags[t] = fl;
    slow = (fl & TF_SLOW) != 0;
    return fl;
}

// One tokeniser tile (tm_tok_fill): words, offsets and flags to HBM, the
// generic-path list.
// out: per lane, its topic's first word (tile-local), word count and flags;
// lds = the tile went the LDS path (lw, if set, then holds its words).
struct TokTile {
    bool lds;
    uint32_t w0, nw;
    uint8_t fl;
    uint64_t base;   // the tile's first word in words[]
};
// (WPL: words per lane per lookup round -- the fused walk's register budget is tighter)
template <uint32_t WPL>
__device__ __forceinline__ void tok_tile(const TokArgs& a, TokLds& L, uint32_t tile, uint32_t* lw, TokTile& out) {
    const uint32_t lane = threadIdx.x;
    const uint32_t tt = a.tile_topics;
    const uint32_t t0 = tile * tt, tend = min(t0 + tt, a.n), cnt = tend - t0;
    const uint32_t t = t0 + lane;
    const bool valid = lane < cnt;
    const uint64_t b0 = a.offs[t0] - a.base, b1 = a.offs[tend] - a.base;
    const uint64_t my_b = valid ? a.offs[t] - a.base : 0, my_e = valid ? a.offs[t + 1] - a.base : 0;
    const uint64_t a0 = b0 & ~15ull;   // bytes[] is 16-B aligned: so are the window's loads
    const uint64_t tile_base = (uint64_t)a.wcount[tile] + a.bsums[tile / SCAN_TILE];   // block-local scan + block offset
    bool slow = false;
    // the LDS path: the window fits and no topic is empty (an empty topic
    // starts where the next one does: one bit cannot mark both)
    bool lds = b1 - a0 <= TOK_BYTES && !__any(valid && my_b == my_e);
    uint32_t tw = 0, wend = 0, incl = 0, mine = 0;
    uint64_t S = 0, TS = 0;
    const uint32_t lb = lane * TOK_LANE_BYTES;   // my 48 bytes of the window
    out.base = tile_base;
    out.fl = (uint8_t)TF_SLOW;
    out.w0 = out.nw = 0;
    if (lds) {
        wend = (uint32_t)(b1 - a0);
        const uint32_t r0 = (uint32_t)(b0 - a0);
        uint4 v[TOK_LANE_BYTES / 16];
#pragma unroll
        for (uint32_t k = 0; k < TOK_LANE_BYTES / 16; ++k)
            v[k] = lb + 16 * k < wend ? *reinterpret_cast<const uint4*>(a.bytes + a0 + lb + 16 * k)
                                      : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t k = 0; k < TOK_LANE_BYTES / 16; ++k)
            *reinterpret_cast<uint4*>(L.bytes + lb + 16 * k) = v[k];
        for (uint32_t i = lane; i < 2 * (TOK_BYTES / 64 + 1); i += 64) reinterpret_cast<uint32_t*>(L.tsb)[i] = 0u;
        if (lane < TILE) L.tirr[lane] = 0;
        __syncthreads();
        if (valid) {
            const uint32_t p = (uint32_t)(my_b - a0);
            atomicOr(reinterpret_cast<unsigned long long*>(&L.tsb[p >> 6]), 1ull << (p & 63));
        }
        // '/' bytes of my 48 (inside [r0, wend)) and topic starts, as bit masks
#pragma unroll
        for (uint32_t k = 0; k < TOK_LANE_BYTES / 16; ++k) {
            S |= (uint64_t)gather4(byte_eq(v[k].x, '/')) << (16 * k);
            S |= (uint64_t)gather4(byte_eq(v[k].y, '/')) << (16 * k + 4);
            S |= (uint64_t)gather4(byte_eq(v[k].z, '/')) << (16 * k + 8);
            S |= (uint64_t)gather4(byte_eq(v[k].w, '/')) << (16 * k + 12);
        }
        const uint32_t lo = r0 > lb ? min(r0 - lb, TOK_LANE_BYTES) : 0u;
        const uint32_t hi = wend > lb ? min(wend - lb, TOK_LANE_BYTES) : 0u;
        S &= ((1ull << hi) - 1ull) & ~((1ull << lo) - 1ull);
        __syncthreads();
        const uint32_t q = lb >> 6, sh = lb & 63;
        TS = L.tsb[q] >> sh;
        if (sh) TS |= L.tsb[q + 1] << (64 - sh);
        TS &= (1ull << TOK_LANE_BYTES) - 1ull;
        // word starts = topic starts + '/' bytes; one scan numbers them
        mine = (uint32_t)(__popcll(S) + __popcll(TS)) | ((uint32_t)__popcll(TS) << 16);
        incl = mine;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += u;
        }
        tw = __shfl(incl, 63, 64) & 0xFFFFu;
        if (tw > TOK_WORDS) {
            lds = false;
            __syncthreads();
        }
    }
    uint32_t nw = 0, tincl = 0;
    if (!lds) {
        // long tile: one lane per topic, bytes from HBM; in-tile offsets by
        // a wave scan of the per-topic word counts ('/' + 1)
        if (valid) {
            nw = 1;
            for (uint64_t i = my_b; i < my_e; ++i) nw += a.bytes[i] == '/';
        }
        tincl = nw;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(tincl, o, 64);
            if (lane >= (uint32_t)o) tincl += u;
        }
        tw = __shfl(tincl, 63, 64);
    }
    if (tend == a.n && lane == 0) a.toff[a.n] = (uint32_t)(tile_base + tw);
    out.lds = lds;
    if (lds) {
        uint32_t wi = (incl - mine) & 0xFFFFu;            // my first word
        int32_t tc = (int32_t)((incl - mine) >> 16) - 1;   // the topic my first byte is in
        uint64_t m = S | TS;
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t pos = lb + b;
            if (TS >> b & 1ull) {
                ++tc;
                L.ttoff[tc] = wi;
                L.wst[wi] = (uint16_t)(pos | 0x8000u);
                L.wtop[wi++] = (uint8_t)tc;
            }
            if (S >> b & 1ull) {
                L.wst[wi] = (uint16_t)(pos + 1);
                L.wtop[wi++] = (uint8_t)tc;
            }
        }
        if (lane == 0) L.ttoff[cnt] = tw;
        __syncthreads();
        tok_lookup<WPL>(a, L, tw, wend, tile_base, lw);   // the tile's words, round-robin over lanes
        __syncthreads();
        if (valid) {
            const uint32_t w0 = L.ttoff[lane], tn = L.ttoff[lane + 1] - w0;
            uint8_t fl = 0;
            if (L.bytes[my_b - a0] == '$') fl |= TF_DOLLAR;
            if (L.tirr[lane] || tn > FAST_MAX_DEPTH) fl |= TF_SLOW;
            a.tflags[t] = fl;
            a.toff[t] = (uint32_t)(tile_base + w0);
            slow = (fl & TF_SLOW) != 0;
            out.w0 = w0;
            out.nw = tn;
            out.fl = fl;
        }
        tok_append_slow(a, slow, t);
        __syncthreads();
    } else {
        const uint64_t o = tile_base + tincl - nw;
        if (valid) {
            a.toff[t] = (uint32_t)o;
            out.fl = tok_fill_topic_global(a, t, o, slow);
            out.w0 = tincl - nw;
            out.nw = nw;
        }
        tok_append_slow(a, slow, t);
    }
}

// pass 2 (after the scan of the tile counts): word entries, offsets, flags
#ifndef TM_TOK_WPE
#define TM_TOK_WPE 5
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(TM_TOK_WPE, 8))) void tm_tok_fill(TokArgs a) {
    __shared__ TokLds L;
    if (a.d_n) a.n = *a.d_n;   // a device-counted batch (its bound sized the grid and the scan)
    const uint32_t tt = a.tile_topics;
    const uint32_t ntiles = (a.n + tt - 1) / tt;
    TokTile out;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) tok_tile<TOK_WPL_FILL>(a, L, tile, nullptr, out);
}


// Read-back of an async batch in ONE kernel, written straight into pinned host
// memory: the header block's first hdr_words (ctrl + stats + src), the counts,
// and exactly the staging entries the walk reserved (ctrl's u64 ticket; the
// host checks it against rows_cap) -- instead of three DMA copies, one of them
// sized by a guess.
__global__ __launch_bounds__(256) void tm_export_host(ExportArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (a.d_n) {   // a bounded batch: the layout follows its count
        a.n = *a.d_n;
        a.hdr_words = a.fixed_words + 2 * a.n;
        a.h_count = a.h_hdr + a.hdr_words;
    }
    for (uint64_t i = i0; i < a.hdr_words; i += stride) a.h_hdr[i] = a.hdr[i];
    for (uint64_t i = i0; i < a.n; i += stride) a.h_count[i] = a.count[i];
    for (uint32_t g = 0; g < TICKET_GROUPS; ++g) {   // each group region's reserved entries
        const uint64_t top = xg_top_read(a.hdr, g);
        const uint64_t lo = g * a.rcap, hi = lo + (top < a.rcap ? top : a.rcap);
        for (uint64_t i = lo + i0; i < hi && i < a.rows_cap; i += stride) a.h_rows[i] = a.rows[i];
    }
}

__global__ __launch_bounds__(256) void tm_csr_to_host(const uint32_t* row_off, const uint32_t* ids, uint32_t n,
                                                       const uint32_t* d_total, uint64_t cap, uint32_t* h_row,
                                                       uint32_t* h_ids) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint64_t i0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t total = min((uint64_t)*d_total, cap);
    for (uint64_t i = i0; i <= n; i += stride) h_row[i] = row_off[i];
    for (uint64_t i = i0; i < total; i += stride) h_ids[i] = ids[i];
}

hipError_t launch_csr_to_host(const uint32_t* row_off, const uint32_t* ids, uint32_t n, const uint32_t* d_total,
                              uint64_t cap, uint32_t* h_row, uint32_t* h_ids, hipStream_t s) {
    const uint64_t work = std::max<uint64_t>(cap, (uint64_t)n + 1);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((work / 8 + 255) / 256, 1), 1024);
    hipLaunchKernelGGL(tm_csr_to_host, dim3(grid), dim3(256), 0, s, row_off, ids, n, d_total, cap, h_row, h_ids);
    return hipGetLastError();
}

// 4 ids -> 12 bytes (three aligned dword stores) per thread; the last
// partial group byte by byte
__global__ __launch_bounds__(256) void tm_pack_ids(const uint32_t* ids, uint64_t n, uint8_t* out) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x, j = 4 * g;
    if (j >= n) return;
    if (j + 4 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(ids + j);
        uint32_t* o = reinterpret_cast<uint32_t*>(out + 12 * g);
        o[0] = (v.x & 0xFFFFFFu) | (v.y << 24);
        o[1] = ((v.y >> 8) & 0xFFFFu) | (v.z << 16);
        o[2] = ((v.z >> 16) & 0xFFu) | (v.w << 8);
        return;
    }
    for (uint64_t q = j; q < n; ++q)
        for (uint32_t b = 0; b < 3; ++b) out[3 * q + b] = (uint8_t)(ids[q] >> (8 * b));
}

hipError_t launch_pack_ids(const uint32_t* ids, uint64_t n, uint8_t* out, hipStream_t s) {
    const uint64_t groups = (n + 3) / 4;
    if (groups) hipLaunchKernelGGL(tm_pack_ids, dim3((uint32_t)((groups + 255) / 256)), dim3(256), 0, s, ids, n, out);
    return hipGetLastError();
}

hipError_t launch_export_host(const ExportArgs& a, hipStream_t s) {
    const uint64_t work = a.hdr_words + a.n + a.rows_cap;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((work / 4 + 255) / 256, 1), 512);
    hipLaunchKernelGGL(tm_export_host, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

__global__ void tm_scatter_keys(DictKey* keys, const uint32_t* idx, const DictKey* vals, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[idx[i]] = vals[i];
}

// ------------------------------------------------------------ launchers

// Topics per tile: 64 (one per lane) for large batches; small batches use
// fewer per wave so that they spread over >= ~2048 waves -- a tile's latency
// is its probe count / 64 iterations, so one topic per wave walks in about
// depth dependent rounds instead of the 64 topics' combined frontier.
#ifndef TM_MIN_TILES
#define TM_MIN_TILES 256    // small batches: tiles shrink until there are this many (4,096-topic batch p50: 2048 / 1024 / 512 / 256 / 128 -> 0.16 / 0.10 / 0.07 / 0.063 / 0.082 ms)
#endif
uint32_t tile_topics(uint32_t n) {
    uint32_t tt = 64;
    while (tt > 1 && (n + tt - 1) / tt < TM_MIN_TILES) tt >>= 1;
    return tt;
}

uint32_t match_waves(uint32_t n, int device, uint32_t qcap) {
    static uint32_t cap[64][2] = {};
    const int qi = qcap <= 384 ? 0 : 1;
    const uint32_t tt = tile_topics(n);
    const uint32_t ntiles = (n + tt - 1) / tt;
    uint32_t c = (device >= 0 && device < 64) ? cap[device][qi] : 0u;
    if (!c) {
        int per_cu = 0, cus = 0;
        // the four instances of one stack size share its LDS footprint, which bounds residency
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, qi == 0 ? tm_match_tiles<false, false, 384> : tm_match_tiles<false, false, 512>, 64, 0) !=
                hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
            per_cu <= 0 || cus <= 0) {
            (void)hipGetLastError();
            per_cu = qi == 0 ? 16 : 14;
            cus = 256;
        }
        // TM_WAVES_PER_CU: fewer resident waves (occupancy sweeps in tools/; never more than fit)
        if (const char* w = getenv("TM_WAVES_PER_CU")) per_cu = std::min(per_cu, std::max(1, atoi(w)));
        c = (uint32_t)per_cu * (uint32_t)cus;
        if (device >= 0 && device < 64) cap[device][qi] = c;
    }
    return ntiles < c ? ntiles : c;
}

template <bool CK, bool BIG>
static hipError_t launch_match_t(const MatchArgs& a, hipStream_t s, hipEvent_t ev_a, hipEvent_t ev_b,
                                 unsigned ev_flags) {
    const uint32_t ntiles = (a.n + a.tile_topics - 1) / a.tile_topics;
    hipError_t e;
    if (ev_a && (e = hipEventRecordWithFlags(ev_a, s, ev_flags)) != hipSuccess) return e;
    if (ntiles) {
        const uint32_t grid = a.grid;
        if (a.qcap <= 384) hipLaunchKernelGGL((tm_match_tiles<CK, BIG, 384>), dim3(grid), dim3(64), 0, s, a);
        else hipLaunchKernelGGL((tm_match_tiles<CK, BIG, 512>), dim3(grid), dim3(64), 0, s, a);
    }
    if (ev_b && (e = hipEventRecordWithFlags(ev_b, s, ev_flags)) != hipSuccess) return e;
    if (ntiles && a.wstats) hipLaunchKernelGGL(tm_stats_reduce, dim3(1), dim3(256), 0, s, a.wstats, a.grid, a.stats);
    hipLaunchKernelGGL((tm_match_slow<CK, BIG>), dim3(a.s_waves), dim3(64), 0, s, a);
    return hipSuccess;
}

// ev_flags: hipEventRecordExternal while the stream is being captured into a
// graph, so that every replay re-records the timing events (a plain record in
// a capture only adds a dependency, and the events would keep the times of the
// last direct launch)
hipError_t launch_match(const MatchArgs& a, hipStream_t s, hipEvent_t ev_a, hipEvent_t ev_b, bool checked,
                        unsigned ev_flags) {
    // the edge hash is read with 32-bit-offset buffer loads unless it exceeds 4 GiB
    const bool big = (uint64_t)a.nslots * sizeof(Slot) > 0xFFFFFFFFull;
    hipError_t e;
    if (checked) e = big ? launch_match_t<true, true>(a, s, ev_a, ev_b, ev_flags)
                         : launch_match_t<true, false>(a, s, ev_a, ev_b, ev_flags);
    else e = big ? launch_match_t<false, true>(a, s, ev_a, ev_b, ev_flags)
                 : launch_match_t<false, false>(a, s, ev_a, ev_b, ev_flags);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_scan(const ScanArgs& a, hipStream_t s, uint32_t* d_total) {
    const uint32_t nb = scan_block_count(a.n);
    if (nb <= 1) {
        hipLaunchKernelGGL(tm_scan_local, dim3(1), dim3(SCAN_BLOCK), 0, s, a, d_total);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(tm_scan_local, dim3(nb), dim3(SCAN_BLOCK), 0, s, a, (uint32_t*)nullptr);
    hipLaunchKernelGGL(tm_scan_sums, dim3(1), dim3(SCAN_BLOCK), 0, s, a, nb, d_total);
    return hipGetLastError();
}

hipError_t launch_finalize(const ScanArgs& a, hipStream_t s, bool checked) {
    const uint32_t ntiles = (a.n + TILE - 1) / TILE;
    if (!ntiles) return hipGetLastError();
    const uint32_t grid = min(ntiles, 256u * 32u);   // 8 waves per SIMD
    if (checked) hipLaunchKernelGGL(tm_finalize<true>, dim3(grid), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(tm_finalize<false>, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_route_count(const RouteArgs& a, hipStream_t s) {
    if (a.m) hipLaunchKernelGGL(tm_route_count, dim3((a.m + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_route_rows(const RouteArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(tm_route_rows, dim3((a.n + 1 + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_route_fill(const RouteArgs& a, hipStream_t s) {
    if (a.m) hipLaunchKernelGGL(tm_route_fill, dim3((a.m + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fan_scan(const FanArgs& a, hipStream_t s) {
    const uint64_t ne = a.n_matches + 1;
    const uint32_t nb = (uint32_t)((ne + FAN_SCAN_TILE - 1) / FAN_SCAN_TILE);
    hipLaunchKernelGGL(tm_fan_scan_local, dim3(nb), dim3(FAN_BLOCK), 0, s, a);
    hipLaunchKernelGGL(tm_fan_scan_sums, dim3(1), dim3(FAN_BLOCK), 0, s, a, nb);
    if (a.nreg) {
        if (a.n) hipLaunchKernelGGL(tm_fan_rows_stg, dim3((a.n + FAN_BLOCK - 1) / FAN_BLOCK), dim3(FAN_BLOCK), 0, s, a);
    } else {
        hipLaunchKernelGGL(tm_fan_rows, dim3((a.n + 1 + FAN_BLOCK - 1) / FAN_BLOCK), dim3(FAN_BLOCK), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_fan_globalize(const FanArgs& a, hipStream_t s) {
    const uint64_t ne = a.n_matches + 1;
    hipLaunchKernelGGL(tm_fan_scan_add, dim3((uint32_t)((ne + FAN_BLOCK - 1) / FAN_BLOCK)), dim3(FAN_BLOCK), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fan_fill(const FanArgs& a, hipStream_t s) {
    if (a.total) {
        const uint64_t nt = (a.total + FAN_FILL_TILE - 1) / FAN_FILL_TILE;
        hipLaunchKernelGGL(tm_fan_tiles, dim3((uint32_t)((nt + 1 + FAN_BLOCK - 1) / FAN_BLOCK)), dim3(FAN_BLOCK), 0, s,
                           a, nt);
        if (a.total > a.big_limit) hipLaunchKernelGGL(tm_fan_fill<true>, dim3((uint32_t)nt), dim3(FAN_BLOCK), 0, s, a);
        else hipLaunchKernelGGL(tm_fan_fill<false>, dim3((uint32_t)nt), dim3(FAN_BLOCK), 0, s, a);
    }
    return hipGetLastError();
}

uint32_t fan_scan_tile() { return FAN_SCAN_TILE; }
uint32_t fan_fill_tile() { return FAN_FILL_TILE; }

hipError_t launch_rules_match(const RulesArgs& a, hipStream_t s) {
    if (a.n) hipLaunchKernelGGL(tm_rules_match, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gather_rows(const uint32_t* src, const int64_t* src_off, const int64_t* idx, uint32_t n,
                              const int64_t* dst_off, uint32_t* dst, hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_gather_rows, dim3((uint32_t)(((uint64_t)n * 16 + 255) / 256)), dim3(256), 0, s, src,
                              src_off, idx, n, dst_off, dst);
    return hipGetLastError();
}

hipError_t launch_dedup(const DedupArgs& a, ScanArgs rows_scan, ScanArgs bytes_scan, hipStream_t s) {
    if (!a.n) return hipGetLastError();
    const uint32_t nblk = dedup_blocks(a.n);
    hipLaunchKernelGGL(tm_dedup_claim, dim3((a.n + DD_BLOCK - 1) / DD_BLOCK), dim3(DD_BLOCK), 0, s, a);
    hipLaunchKernelGGL(tm_dedup_count, dim3(nblk), dim3(256), 0, s, a);
    hipError_t e;
    if ((e = launch_scan(rows_scan, s, nullptr)) != hipSuccess) return e;
    if ((e = launch_scan(bytes_scan, s, nullptr)) != hipSuccess) return e;
    hipLaunchKernelGGL(tm_dedup_compact, dim3(nblk), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dedup_rowof(const DedupArgs& a, hipStream_t s) {
    if (a.n) hipLaunchKernelGGL(tm_dedup_rowof, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dedup_expand(const DedupArgs& a, hipStream_t s) {
    const uint32_t g = (a.n + 256 * EXPAND_PER_THREAD - 1) / (256 * EXPAND_PER_THREAD);
    // (the rows are counted on the device: a grid for the bound, strided)
    const uint32_t gr = std::min<uint32_t>(2048, (a.n + 255) / 256);
    if (gr) hipLaunchKernelGGL(tm_dedup_rowmeta, dim3(gr), dim3(256), 0, s, a);
    if (g) hipLaunchKernelGGL(tm_dedup_expand, dim3(g), dim3(256), 0, s, a);
    hipLaunchKernelGGL(tm_dedup_sum, dim3(1), dim3(1024), 0, s, a, g);   // (also reports the rows)
    return hipGetLastError();
}

hipError_t launch_sample_meta(const uint32_t* count, const unsigned long long* src, const uint32_t* rows, uint32_t k,
                              uint32_t* out_cnt, unsigned long long* out_src, hipStream_t s) {
    if (k) hipLaunchKernelGGL(tm_sample_meta, dim3((k + 255) / 256), dim3(256), 0, s, count, src, rows, k, out_cnt, out_src);
    return hipGetLastError();
}

hipError_t launch_sample_ids(const uint32_t* sfids, const uint32_t* cnt, const unsigned long long* src,
                             const uint64_t* off, uint32_t k, uint32_t* out, hipStream_t s) {
    if (k) hipLaunchKernelGGL(tm_sample_ids, dim3(k), dim3(64), 0, s, sfids, cnt, src, off, out);
    return hipGetLastError();
}

hipError_t launch_token_check(const uint32_t* toff, const uint8_t* tflags, uint32_t n, uint64_t nwords,
                              uint32_t* slow_list, uint32_t* d_nslow, uint32_t* d_bad, hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_token_check, dim3((n + 255) / 256), dim3(256), 0, s, toff, tflags, n, nwords,
                              slow_list, d_nslow, d_bad);
    return hipGetLastError();
}

hipError_t launch_tokens_shard(const uint32_t* words, const uint32_t* toff, uint32_t n, uint32_t nshards,
                               uint32_t* shard, hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_tokens_shard, dim3((n + 255) / 256), dim3(256), 0, s, words, toff, n, nshards, shard);
    return hipGetLastError();
}

hipError_t launch_part_count(const PartArgs& a, hipStream_t s) {
    if (a.n) hipLaunchKernelGGL(tm_part_count, dim3(a.nb), dim3(PART_BLOCK), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_part_segs(const PartArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(tm_part_segs, dim3(1), dim3(PART_MAX_G + 1), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_part_scatter(const PartArgs& a, hipStream_t s) {
    if (a.n) hipLaunchKernelGGL(tm_part_scatter, dim3(a.nb), dim3(PART_BLOCK), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_unpart_counts(const uint32_t* order, const uint32_t* counts_p, uint32_t n, uint32_t* counts_o,
                                hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_unpart_counts, dim3((n + 255) / 256), dim3(256), 0, s, order, counts_p, n, counts_o);
    return hipGetLastError();
}
hipError_t launch_unpart_rows(const uint32_t* order, const uint32_t* counts_p, uint32_t n, const uint32_t* src_off,
                              const uint32_t* src_bs, const uint32_t* dst_off, const uint32_t* dst_bs,
                              const uint32_t* ids_p, uint32_t* out, uint32_t* rowg, hipStream_t s) {
    const uint64_t threads = ((uint64_t)n + 1) * 16;
    hipLaunchKernelGGL(tm_unpart_rows, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, order, counts_p, n,
                       src_off, src_bs, dst_off, dst_bs, ids_p, out, rowg);
    return hipGetLastError();
}

hipError_t launch_export(const uint32_t* row_off, const uint32_t* ids, uint32_t n, uint64_t total,
                         uint32_t* counts, uint32_t* gids, uint32_t mul, uint32_t add, hipStream_t s) {
    const uint64_t work = total > n ? total : n;
    if (!work) return hipGetLastError();
    const uint64_t blocks = (work + 255) / 256;
    const uint32_t grid = (uint32_t)(blocks < 4096u ? blocks : 4096u);
    hipLaunchKernelGGL(tm_export, dim3(grid), dim3(256), 0, s, row_off, ids, n, total, counts, gids, mul, add);
    return hipGetLastError();
}

hipError_t launch_scatter_slots(Slot* slots, const uint32_t* idx, const Slot* vals, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_scatter_slots, dim3((n + 255) / 256), dim3(256), 0, s, slots, idx, vals, n);
    return hipGetLastError();
}

hipError_t launch_scatter_fmeta(uint64_t* foff, uint32_t* flen, const uint32_t* idx, const uint64_t* off,
                                const uint32_t* len, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_scatter_fmeta, dim3((n + 255) / 256), dim3(256), 0, s, foff, flen, idx, off, len, n);
    return hipGetLastError();
}

uint32_t tok_tile_topics(uint32_t n, uint64_t nbytes) {
    // the most topics (64 at most) whose average bytes fill ~3/4 of the LDS window
    uint32_t tt = TILE;
    while (tt > 1 && (uint64_t)tt * nbytes > (uint64_t)(TOK_BYTES * 3 / 4) * (n ? n : 1)) tt >>= 1;
    // small batches (per-publish calls): at least 32 tiles down to 4 topics a
    // tile -- one wave walking a whole 64-topic tile's lookups is a chain of
    // dependent rounds; several short tiles run them side by side
    while (tt > 4 && (n + tt - 1) / tt < 32) tt >>= 1;
    return tt;
}

// blocks of `kernel` (block threads, no dynamic LDS) the device holds at once:
// a grid of that size runs in one round (no tail of late blocks)
template <class K>
static uint32_t resident_blocks(K kernel, int block) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess || cus <= 0 || per <= 0)
        return 256u * 32u;
    return (uint32_t)(cus * per);
}

// tokeniser passes 1 and 2: words per tile, their scan (f: the fill's arguments)
static hipError_t launch_tok_count_scan(const TokArgs& a, ScanArgs scan, uint32_t* d_nwords, hipStream_t s,
                                        TokArgs& f) {
    static const uint32_t cap_count = resident_blocks(tm_tok_count, 64);
    const uint32_t ntiles = (a.n + a.tile_topics - 1) / a.tile_topics;
    hipLaunchKernelGGL(tm_tok_count, dim3(ntiles ? min(ntiles, cap_count) : 1u), dim3(64), 0, s, a);   // also clears d_nslow + zero[]
    f = a;
    if (!a.n) return hipGetLastError();
    scan.count = a.wcount;
    scan.row_off = a.wcount;   // in place: tile counts -> block-local tile offsets
    scan.n = ntiles;
    const hipError_t e = launch_scan(scan, s, d_nwords);
    f.bsums = scan.block_sums;
    return e;
}

hipError_t launch_tokenize(const TokArgs& a, ScanArgs scan, uint32_t* d_nwords, hipStream_t s) {
    static const uint32_t cap_fill = resident_blocks(tm_tok_fill, 64);
    TokArgs f;
    const hipError_t e = launch_tok_count_scan(a, scan, d_nwords, s, f);
    if (e != hipSuccess || !a.n) return e != hipSuccess ? e : hipGetLastError();
    const uint32_t ntiles = (a.n + a.tile_topics - 1) / a.tile_topics;
    hipLaunchKernelGGL(tm_tok_fill, dim3(min(ntiles, cap_fill)), dim3(64), 0, s, f);
    return hipGetLastError();
}

hipError_t launch_scatter_keys(DictKey* keys, const uint32_t* idx, const DictKey* vals, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(tm_scatter_keys, dim3((n + 255) / 256), dim3(256), 0, s, keys, idx, vals, n);
    return hipGetLastError();
}

}  // namespace etm
