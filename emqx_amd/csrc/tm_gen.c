/*
 * tm_gen.c -- seeded synthetic subscription/publish workloads.
 *
 * Bench/test tooling, not on the match path.  Mirrored bit-for-bit by
 * emqx_amd/gen.py (tests check the two agree), so small fixtures generated in
 * Python reproduce on the GPU box from the seed alone.
 *
 * RNG: splitmix64.  Vocabulary word k of level l is "w<l>_<k>" except 5 % that
 * are random words of length 1..16 over a 64-symbol alphabet (alnum + '!' '%',
 * so all three byte classes relative to '#' and '+' occur).  Word choice is
 * Zipf(s) over the V-word vocabulary of each level.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

typedef struct {
    uint64_t seed;
    uint64_t n_filters;
    uint32_t vocab;
    uint32_t max_depth;
    double   zipf_s;
    double   p_plus;        /* '+' at a non-final level */
    double   p_hash;        /* '#' at the final level */
    double   p_final_plus;  /* '+' at the final level */
    double   exact_frac;    /* fraction of exact (wildcard-free) filters */
    int32_t  require_wildcard;
    double   p_dollar;      /* filter rooted at $SYS */
    double   p_empty;       /* filter has one empty level */
    double   p_topic_dollar;
    double   p_topic_inst;  /* topic instantiates a random filter */
    double   p_unseen;      /* literal topic word not in any vocabulary */
} tm_gen_params;

static inline uint64_t sm_next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline double sm_u01(uint64_t* s) { return (double)(sm_next(s) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint64_t sm_below(uint64_t* s, uint64_t n) { return sm_next(s) % n; }

static const char ALPH[65] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789!%";

typedef struct { char* b; size_t n, cap; } sbuf;
static void sb_put(sbuf* s, const char* p, size_t n) {
    if (s->n + n > s->cap) { s->cap = (s->n + n) * 2 + 256; s->b = (char*)realloc(s->b, s->cap); }
    memcpy(s->b + s->n, p, n); s->n += n;
}

/* vocabulary word (l, k) written into out (<= 24 bytes); returns length */
static int vocab_word(uint64_t seed, uint32_t l, uint32_t k, char* out) {
    uint64_t st = seed * 0x9E3779B97F4A7C15ull + (((uint64_t)l << 32) | k) + 1;
    if (sm_u01(&st) < 0.05) {
        int len = 1 + (int)sm_below(&st, 16);
        for (int i = 0; i < len; i++) out[i] = ALPH[sm_below(&st, 64)];
        return len;
    }
    return snprintf(out, 24, "w%u_%u", l, k);
}

typedef struct {
    const tm_gen_params* p;
    double* cdf;
} zipf_t;

static void zipf_init(zipf_t* z, const tm_gen_params* p) {
    z->p = p;
    z->cdf = (double*)malloc(sizeof(double) * p->vocab);
    double acc = 0;
    for (uint32_t k = 0; k < p->vocab; k++) { acc += pow((double)(k + 1), -p->zipf_s); z->cdf[k] = acc; }
    for (uint32_t k = 0; k < p->vocab; k++) z->cdf[k] /= acc;
}

static uint32_t zipf_draw(const zipf_t* z, uint64_t* s) {
    double u = sm_u01(s);
    uint32_t lo = 0, hi = z->p->vocab - 1;
    while (lo < hi) { uint32_t mid = (lo + hi) / 2; if (u < z->cdf[mid]) hi = mid; else lo = mid + 1; }
    return lo;
}

static void put_vocab(sbuf* o, const tm_gen_params* p, const zipf_t* z, uint64_t* s, uint32_t l) {
    char w[32];
    int n = vocab_word(p->seed, l, zipf_draw(z, s), w);
    sb_put(o, w, (size_t)n);
}

/* one filter into o (no trailing separator); returns 1 if it has a wildcard */
static int gen_filter(sbuf* o, const tm_gen_params* p, const zipf_t* z, uint64_t* s, int exact) {
    uint32_t depth = 1 + (uint32_t)sm_below(s, p->max_depth);
    int dollar = sm_u01(s) < p->p_dollar;
    int64_t empty_at = sm_u01(s) < p->p_empty ? (int64_t)sm_below(s, depth) : -1;
    int wild = 0;
    for (uint32_t l = 0; l < depth; l++) {
        if (l) sb_put(o, "/", 1);
        if (l == 0 && dollar) { sb_put(o, "$SYS", 4); continue; }
        if ((int64_t)l == empty_at) continue;
        if (exact) { put_vocab(o, p, z, s, l); continue; }
        if (l + 1 < depth) {
            if (sm_u01(s) < p->p_plus) { sb_put(o, "+", 1); wild = 1; }
            else put_vocab(o, p, z, s, l);
        } else {
            double r = sm_u01(s);
            if (r < p->p_hash) { sb_put(o, "#", 1); wild = 1; }
            else if (r < p->p_hash + p->p_final_plus) { sb_put(o, "+", 1); wild = 1; }
            else put_vocab(o, p, z, s, l);
        }
    }
    return wild;
}

/* string set for dedup */
typedef struct { uint64_t* h; uint64_t* off; uint32_t* len; size_t cap, n; } sset;
static uint64_t fnv(const char* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) { h ^= (uint8_t)p[i]; h *= 1099511628211ull; }
    return h | 1;
}
static void sset_init(sset* s, size_t cap) {
    size_t c = 1024; while (c < cap * 2) c <<= 1;
    s->cap = c; s->n = 0;
    s->h = (uint64_t*)calloc(c, 8); s->off = (uint64_t*)calloc(c, 8); s->len = (uint32_t*)calloc(c, 4);
}
/* returns 1 if inserted (new) */
static int sset_add(sset* s, const char* base, uint64_t off, uint32_t len) {
    uint64_t h = fnv(base + off, len);
    size_t i = h & (s->cap - 1);
    while (s->h[i]) {
        if (s->h[i] == h && s->len[i] == len && memcmp(base + s->off[i], base + off, len) == 0) return 0;
        i = (i + 1) & (s->cap - 1);
    }
    s->h[i] = h; s->off[i] = off; s->len[i] = len; s->n++;
    return 1;
}

typedef struct {
    char* buf; uint64_t* offs; uint64_t n;
} tm_strs;

EXPORT void tm_gen_free(tm_strs* s) { if (s) { free(s->buf); free(s->offs); s->buf = NULL; s->offs = NULL; } }

/* Generates p->n_filters distinct filters. */
EXPORT int tm_gen_filters(const tm_gen_params* p, tm_strs* out) {
    zipf_t z; zipf_init(&z, p);
    uint64_t s = p->seed;
    sbuf o = {0};
    sset set; sset_init(&set, p->n_filters);
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (p->n_filters + 1));
    uint64_t n = 0;
    offs[0] = 0;
    uint64_t guard = 0;
    while (n < p->n_filters) {
        if (++guard > p->n_filters * 1000 + 100000) { free(z.cdf); free(o.b); free(offs); return -1; }
        int exact = sm_u01(&s) < p->exact_frac;
        size_t start = o.n;
        int wild = gen_filter(&o, p, &z, &s, exact);
        if (!exact && p->require_wildcard && !wild) { o.n = start; continue; }
        if (!sset_add(&set, o.b, start, (uint32_t)(o.n - start))) { o.n = start; continue; }
        offs[++n] = o.n;
    }
    free(set.h); free(set.off); free(set.len); free(z.cdf);
    out->buf = o.b ? o.b : (char*)malloc(1); out->offs = offs; out->n = n;
    return 0;
}

static void put_unseen(sbuf* o, uint64_t* s) {
    char w[16];
    int n = snprintf(w, sizeof(w), "u%08x", (unsigned)(sm_next(s) & 0xffffffffu));
    sb_put(o, w, (size_t)n);
}

/* instantiate filter f into o; returns number of words written */
static uint32_t instantiate(sbuf* o, const tm_gen_params* p, const zipf_t* z, uint64_t* s,
                            const char* f, uint32_t fl) {
    uint32_t nw = 0, l = 0, i = 0;
    while (1) {
        uint32_t j = i;
        while (j < fl && f[j] != '/') j++;
        const char* w = f + i; uint32_t wl = j - i;
        if (wl == 1 && w[0] == '#') {
            uint32_t extra = (uint32_t)sm_below(s, 4);
            for (uint32_t e = 0; e < extra; e++, l++, nw++) {
                if (nw) sb_put(o, "/", 1);
                put_vocab(o, p, z, s, l);
            }
        } else {
            if (nw) sb_put(o, "/", 1);
            if (wl == 1 && w[0] == '+') {
                if (sm_u01(s) < 0.9) put_vocab(o, p, z, s, l); else put_unseen(o, s);
            } else sb_put(o, w, wl);
            nw++; l++;
        }
        if (j >= fl) break;
        i = j + 1;
    }
    return nw;
}

/* Generates n topics against the given filter set with topic seed `tseed`. */
EXPORT int tm_gen_topics(const tm_gen_params* p, const tm_strs* filters, uint64_t tseed,
                         uint64_t n, tm_strs* out) {
    zipf_t z; zipf_init(&z, p);
    uint64_t s = tseed;
    sbuf o = {0};
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    offs[0] = 0;
    for (uint64_t t = 0; t < n; t++) {
        double r = sm_u01(&s);
        size_t start = o.n;
        if (filters->n && r < p->p_topic_dollar + p->p_topic_inst) {
            int dollar = r < p->p_topic_dollar;
            uint64_t fi = sm_below(&s, filters->n);
            const char* f = filters->buf + filters->offs[fi];
            uint32_t fl = (uint32_t)(filters->offs[fi + 1] - filters->offs[fi]);
            uint32_t nw = instantiate(&o, p, &z, &s, f, fl);
            (void)nw;
            if (o.n == start) put_vocab(&o, p, &z, &s, 0);
            if (dollar) {
                /* replace the first word with "$SYS" */
                size_t k = start;
                while (k < o.n && o.b[k] != '/') k++;
                size_t rest = o.n - k;
                char* tmp = (char*)malloc(rest + 1);
                memcpy(tmp, o.b + k, rest);
                o.n = start;
                sb_put(&o, "$SYS", 4);
                sb_put(&o, tmp, rest);
                free(tmp);
            }
        } else {
            uint32_t depth = 1 + (uint32_t)sm_below(&s, p->max_depth);
            for (uint32_t l = 0; l < depth; l++) {
                if (l) sb_put(&o, "/", 1);
                if (sm_u01(&s) < p->p_unseen) put_unseen(&o, &s);
                else put_vocab(&o, p, &z, &s, l);
            }
        }
        offs[t + 1] = o.n;
    }
    free(z.cdf);
    out->buf = o.b ? o.b : (char*)malloc(1); out->offs = offs; out->n = n;
    return 0;
}

/* ---- C4: IoT filters and publishes ------------------------
 *
 * Filter i of n_filters is a pure function of (seed, i), so any index range can
 * be generated on its own, and the filters are distinct by construction:
 *   i <  0.7 F : device/d<id>/sensor/s<s>/#     (id, s) = perm(i) over ids x sensors
 *   i <  0.9 F : device/d<id>/+/m<m>            (id, m) = perm(i - 0.7F) over ids x metrics
 *   otherwise  : +/d<id>/sensor/+/#             id = perm(i - 0.9F) over ids   (replicated)
 * Publishes: device/d<id>/sensor/s<s>/m<m>, or device/d<id>/status/m<m> with
 * probability p_status; id ~ Zipf(zipf_s) over the ids.
 */
typedef struct {
    uint64_t seed;
    uint64_t n_filters;
    uint32_t n_ids;
    uint32_t n_sensors;
    uint32_t n_metrics;
    uint32_t pad;
    double   zipf_s;
    double   p_status;
} tm_iot_params;

/* bijection of [0, space) (cycle-walking a bijective mixer of [0, 2^k)) */
static uint64_t iot_perm(uint64_t j, uint64_t space, uint64_t seed) {
    uint32_t k = 1;
    while ((1ull << k) < space) k++;
    const uint64_t mask = (1ull << k) - 1;
    const uint64_t c = (seed * 2 + 1) & mask;
    uint64_t x = j;
    do {
        x = (x * 0x9E3779B97F4A7C15ull + c) & mask;
        x ^= x >> (k / 2 + 1);
        x = (x * 0xBF58476D1CE4E5B9ull) & mask;
        x ^= x >> (k / 2 + 1);
    } while (x >= space);
    return x;
}

EXPORT int tm_gen_iot_vocab(const tm_iot_params* p, tm_strs* out) {
    sbuf o = {0};
    uint64_t n = 3ull + p->n_ids + p->n_sensors + p->n_metrics;
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    uint64_t k = 0;
    char w[32];
    offs[0] = 0;
    sb_put(&o, "device", 6); offs[++k] = o.n;
    sb_put(&o, "sensor", 6); offs[++k] = o.n;
    sb_put(&o, "status", 6); offs[++k] = o.n;
    for (uint32_t i = 0; i < p->n_ids; i++) { int l = snprintf(w, sizeof(w), "d%u", i); sb_put(&o, w, (size_t)l); offs[++k] = o.n; }
    for (uint32_t i = 0; i < p->n_sensors; i++) { int l = snprintf(w, sizeof(w), "s%u", i); sb_put(&o, w, (size_t)l); offs[++k] = o.n; }
    for (uint32_t i = 0; i < p->n_metrics; i++) { int l = snprintf(w, sizeof(w), "m%u", i); sb_put(&o, w, (size_t)l); offs[++k] = o.n; }
    out->buf = o.b ? o.b : (char*)malloc(1); out->offs = offs; out->n = n;
    return 0;
}

EXPORT int tm_gen_iot_filters(const tm_iot_params* p, uint64_t lo, uint64_t hi, tm_strs* out) {
    const uint64_t F = p->n_filters;
    const uint64_t fa = F * 7 / 10, fb = F * 9 / 10;
    if (hi > F || lo > hi) return -1;
    if (fa > (uint64_t)p->n_ids * p->n_sensors || fb - fa > (uint64_t)p->n_ids * p->n_metrics || F - fb > p->n_ids)
        return -1;
    sbuf o = {0};
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (hi - lo + 1));
    offs[0] = 0;
    char w[96];
    for (uint64_t i = lo; i < hi; i++) {
        int l;
        if (i < fa) {
            const uint64_t key = iot_perm(i, (uint64_t)p->n_ids * p->n_sensors, p->seed);
            l = snprintf(w, sizeof(w), "device/d%u/sensor/s%u/#", (unsigned)(key / p->n_sensors), (unsigned)(key % p->n_sensors));
        } else if (i < fb) {
            const uint64_t key = iot_perm(i - fa, (uint64_t)p->n_ids * p->n_metrics, p->seed + 1);
            l = snprintf(w, sizeof(w), "device/d%u/+/m%u", (unsigned)(key / p->n_metrics), (unsigned)(key % p->n_metrics));
        } else {
            const uint64_t id = iot_perm(i - fb, p->n_ids, p->seed + 2);
            l = snprintf(w, sizeof(w), "+/d%u/sensor/+/#", (unsigned)id);
        }
        sb_put(&o, w, (size_t)l);
        offs[i - lo + 1] = o.n;
    }
    out->buf = o.b ? o.b : (char*)malloc(1); out->offs = offs; out->n = hi - lo;
    return 0;
}

EXPORT int tm_gen_iot_topics(const tm_iot_params* p, uint64_t tseed, uint64_t n, tm_strs* out) {
    /* Zipf over the ids: CDF table, binary search per draw */
    double* cdf = (double*)malloc(sizeof(double) * p->n_ids);
    double acc = 0;
    for (uint32_t k = 0; k < p->n_ids; k++) { acc += pow((double)(k + 1), -p->zipf_s); cdf[k] = acc; }
    for (uint32_t k = 0; k < p->n_ids; k++) cdf[k] /= acc;
    uint64_t s = tseed;
    sbuf o = {0};
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    offs[0] = 0;
    char w[96];
    for (uint64_t t = 0; t < n; t++) {
        const double u = sm_u01(&s);
        uint32_t lo = 0, hi = p->n_ids - 1;
        while (lo < hi) { uint32_t mid = (lo + hi) / 2; if (u < cdf[mid]) hi = mid; else lo = mid + 1; }
        const uint32_t id = lo;
        int l;
        if (sm_u01(&s) < p->p_status)
            l = snprintf(w, sizeof(w), "device/d%u/status/m%u", id, (unsigned)sm_below(&s, p->n_metrics));
        else {
            const unsigned sn = (unsigned)sm_below(&s, p->n_sensors);
            l = snprintf(w, sizeof(w), "device/d%u/sensor/s%u/m%u", id, sn, (unsigned)sm_below(&s, p->n_metrics));
        }
        sb_put(&o, w, (size_t)l);
        offs[t + 1] = o.n;
    }
    free(cdf);
    out->buf = o.b ? o.b : (char*)malloc(1); out->offs = offs; out->n = n;
    return 0;
}

/* ---- C5: high-fanout skew ---------------------------------
 *
 * n_hot distinct hot topics of hot_depth levels ("h<l>_<k>", k < vocab), and
 * per hot topic k_per_hot distinct filters derived from it: each level becomes
 * '+' with probability 0.3, and with probability 0.3 the filter is cut at a
 * random level by '#'; at least 3 literal levels are kept, so filters of
 * different hot topics rarely coincide (global duplicates are skipped).
 * derive_one() makes one more such filter for the churn deltas.
 */
typedef struct {
    uint64_t seed;
    uint32_t n_hot;
    uint32_t hot_depth;
    uint32_t vocab;
    uint32_t k_per_hot;
} tm_skew_params;

static uint32_t derive(sbuf* o, const char* t, uint32_t tl, uint32_t depth, uint64_t* s) {
    /* word boundaries of t */
    uint32_t st[64], en[64], nw = 0, i = 0;
    while (nw < 64) {
        uint32_t j = i;
        while (j < tl && t[j] != '/') j++;
        st[nw] = i; en[nw] = j; nw++;
        if (j >= tl) break;
        i = j + 1;
    }
    (void)depth;
    for (int attempt = 0; attempt < 64; attempt++) {
        uint32_t cut = nw;
        if (sm_u01(s) < 0.3) cut = (uint32_t)sm_below(s, nw);    /* '#' replaces levels >= cut */
        uint64_t plus = 0;
        uint32_t lit = 0;
        for (uint32_t l = 0; l < cut; l++) {
            if (sm_u01(s) < 0.3) plus |= 1ull << l; else lit++;
        }
        if (lit < 3) continue;
        size_t start = o->n;
        for (uint32_t l = 0; l < cut; l++) {
            if (l) sb_put(o, "/", 1);
            if (plus >> l & 1) sb_put(o, "+", 1); else sb_put(o, t + st[l], en[l] - st[l]);
        }
        if (cut < nw) { if (cut) sb_put(o, "/", 1); sb_put(o, "#", 1); }
        return (uint32_t)(o->n - start);
    }
    return 0;
}

EXPORT int tm_gen_skew(const tm_skew_params* p, tm_strs* hot, tm_strs* filters) {
    uint64_t s = p->seed;
    sbuf ho = {0}, fo = {0};
    uint64_t* hoffs = (uint64_t*)malloc(sizeof(uint64_t) * (p->n_hot + 1));
    uint64_t nf_cap = (uint64_t)p->n_hot * p->k_per_hot;
    uint64_t* foffs = (uint64_t*)malloc(sizeof(uint64_t) * (nf_cap + 1));
    sset hs; sset_init(&hs, p->n_hot);
    sset fs; sset_init(&fs, nf_cap + 1);
    char w[32];
    hoffs[0] = 0; foffs[0] = 0;
    uint64_t nh = 0, nf = 0, guard = 0;
    while (nh < p->n_hot) {
        if (++guard > (uint64_t)p->n_hot * 100) break;
        size_t start = ho.n;
        for (uint32_t l = 0; l < p->hot_depth; l++) {
            if (l) sb_put(&ho, "/", 1);
            int n = snprintf(w, sizeof(w), "h%u_%u", l, (unsigned)sm_below(&s, p->vocab));
            sb_put(&ho, w, (size_t)n);
        }
        if (!sset_add(&hs, ho.b, start, (uint32_t)(ho.n - start))) { ho.n = start; continue; }
        hoffs[++nh] = ho.n;
    }
    for (uint64_t h = 0; h < nh; h++) {
        uint32_t got = 0, tries = 0;
        while (got < p->k_per_hot && tries++ < p->k_per_hot * 40) {
            size_t start = fo.n;
            /* derive() reads the hot topic while appending to fo: copy it first (ho is not fo) */
            uint32_t len = derive(&fo, ho.b + hoffs[h], (uint32_t)(hoffs[h + 1] - hoffs[h]), p->hot_depth, &s);
            if (!len || !sset_add(&fs, fo.b, start, len)) { fo.n = start; continue; }
            foffs[++nf] = fo.n;
            got++;
        }
    }
    free(hs.h); free(hs.off); free(hs.len); free(fs.h); free(fs.off); free(fs.len);
    hot->buf = ho.b ? ho.b : (char*)malloc(1); hot->offs = hoffs; hot->n = nh;
    filters->buf = fo.b ? fo.b : (char*)malloc(1); filters->offs = foffs; filters->n = nf;
    return nh == p->n_hot ? 0 : -1;
}

/* One more derived filter of hot topic t (churn deltas), seeded. */
EXPORT int tm_gen_derive_one(const char* t, uint32_t tl, uint64_t seed, char* out, uint32_t cap) {
    sbuf o = {0};
    uint64_t s = seed;
    uint32_t len = derive(&o, t, tl, 0, &s);
    int r = -1;
    if (len && len <= cap) { memcpy(out, o.b, len); r = (int)len; }
    free(o.b);
    return r;
}

/* n publishes: with probability p_a a Zipf(zipf_s)-chosen element of A (rank 0
 * hottest), otherwise a uniformly chosen element of B. */
EXPORT int tm_gen_pick(const tm_strs* A, const tm_strs* B, uint64_t seed, uint64_t n, double p_a, double zipf_s,
                       tm_strs* out) {
    double* cdf = (double*)malloc(sizeof(double) * (A->n ? A->n : 1));
    double acc = 0;
    for (uint64_t k = 0; k < A->n; k++) { acc += pow((double)(k + 1), -zipf_s); cdf[k] = acc; }
    for (uint64_t k = 0; k < A->n; k++) cdf[k] /= acc;
    uint64_t s = seed;
    sbuf o = {0};
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    offs[0] = 0;
    for (uint64_t t = 0; t < n; t++) {
        const tm_strs* S;
        uint64_t i;
        if (A->n && (B->n == 0 || sm_u01(&s) < p_a)) {
            const double u = sm_u01(&s);
            uint64_t lo = 0, hi = A->n - 1;
            while (lo < hi) { uint64_t mid = (lo + hi) / 2; if (u < cdf[mid]) hi = mid; else lo = mid + 1; }
            S = A; i = lo;
        } else {
            S = B; i = sm_below(&s, B->n);
        }
        sb_put(&o, S->buf + S->offs[i], S->offs[i + 1] - S->offs[i]);
        offs[t + 1] = o.n;
    }
    free(cdf);
    out->buf = o.b ? o.b : (char*)malloc(1); out->offs = offs; out->n = n;
    return 0;
}
