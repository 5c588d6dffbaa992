/*
 * tm_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A faithful CPU restatement of the reference's publish-time matching path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library; the product (emqx_amd/) never links or calls it.
 *
 * What it restates (reference = /root/reference, EMQ X 4.2.x, Erlang):
 *   emqx_topic:words/1, word/1      src/emqx_topic.erl:150-164
 *   emqx_topic:match/2              src/emqx_topic.erl:65-87
 *   emqx_topic:wildcard/1           src/emqx_topic.erl:52-62
 *   emqx_trie:insert/1              src/emqx_trie.erl:81-93, add_path/1 :145-158
 *   emqx_trie:match/1               src/emqx_trie.erl:96-99
 *   match_node/2,3, 'match_#'/2     src/emqx_trie.erl:162-186
 *   emqx_trie:delete/1, delete_path src/emqx_trie.erl:107-116, :190-204
 *   emqx_trie:lookup/1, empty/0     src/emqx_trie.erl:102-104, :119-121
 *   emqx_router:match_routes/1      src/emqx_router.erl:127-145
 *
 * Data layout deliberately mirrors the reference's ETS tables
 * (src/emqx_trie.erl:53-68, include/emqx.hrl:96-113):
 *   - trie node ids are the filter PREFIX strings (atom `root` for the root);
 *   - the edge table is a hash set keyed by (node_id, word) -> child node id,
 *     so every lookup hashes the whole prefix, like ets:lookup on
 *     {trie_edge, PrefixBinary, Word};
 *   - the node table is keyed by node id -> {edge_count, topic}.
 * match/1 returns the reference's DFS order (prepend/foldl semantics kept);
 * the batch entry points return per-topic lists sorted by Erlang binary order
 * (unsigned bytewise, shorter prefix first), which is the build's contract.
 *
 * Brute force: tmo_brute_batch applies emqx_topic:match/2 to every (t, f)
 * pair -- an independent formulation used to cross-check the trie walk.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* hashing + a byte-string keyed open-addressing map (ETS `set` analog) */
/* ------------------------------------------------------------------ */

static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

static uint64_t hash_bytes(const uint8_t* p, size_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
    while (n >= 8) {
        h ^= rd64(p) * 0xBF58476D1CE4E5B9ull;
        h = (h << 27 | h >> 37) * 0x94D049BB133111EBull;
        p += 8; n -= 8;
    }
    uint64_t t = 0;
    for (size_t i = 0; i < n; i++) t |= (uint64_t)p[i] << (8 * i);
    h ^= t * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31; h *= 0x94D049BB133111EBull; h ^= h >> 29;
    return h;
}

typedef struct {
    uint8_t* key;   /* NULL = empty, TOMB = deleted */
    uint32_t klen;
    uint64_t h;
    void*    val;
} mslot_t;

static uint8_t tomb_sentinel;
#define TOMB (&tomb_sentinel)

typedef struct {
    mslot_t* s;
    size_t   cap;   /* power of two */
    size_t   live;
    size_t   used;  /* live + tombstones */
} bmap_t;

static void bmap_init(bmap_t* m, size_t cap) {
    size_t c = 16;
    while (c < cap) c <<= 1;
    m->s = (mslot_t*)calloc(c, sizeof(mslot_t));
    m->cap = c; m->live = 0; m->used = 0;
}

static void bmap_free(bmap_t* m, int free_vals) {
    for (size_t i = 0; i < m->cap; i++) {
        if (m->s[i].key && m->s[i].key != TOMB) {
            free(m->s[i].key);
            if (free_vals) free(m->s[i].val);
        }
    }
    free(m->s);
    m->s = NULL;
}

static mslot_t* bmap_find(const bmap_t* m, const uint8_t* k, uint32_t kl, uint64_t h) {
    size_t mask = m->cap - 1, i = h & mask;
    for (;;) {
        mslot_t* s = &m->s[i];
        if (!s->key) return NULL;
        if (s->key != TOMB && s->h == h && s->klen == kl && memcmp(s->key, k, kl) == 0) return s;
        i = (i + 1) & mask;
    }
}

static void bmap_grow(bmap_t* m) {
    bmap_t n;
    bmap_init(&n, m->cap * 2);
    for (size_t i = 0; i < m->cap; i++) {
        mslot_t* s = &m->s[i];
        if (s->key && s->key != TOMB) {
            size_t j = s->h & (n.cap - 1);
            while (n.s[j].key) j = (j + 1) & (n.cap - 1);
            n.s[j] = *s;
            n.live++; n.used++;
        }
    }
    free(m->s);
    *m = n;
}

/* insert or overwrite; returns slot */
static mslot_t* bmap_put(bmap_t* m, const uint8_t* k, uint32_t kl, uint64_t h, void* val) {
    mslot_t* s = bmap_find(m, k, kl, h);
    if (s) { s->val = val; return s; }
    if ((m->used + 1) * 10 > m->cap * 7) bmap_grow(m);
    size_t mask = m->cap - 1, i = h & mask;
    while (m->s[i].key && m->s[i].key != TOMB) i = (i + 1) & mask;
    s = &m->s[i];
    if (!s->key) m->used++;
    s->key = (uint8_t*)malloc(kl ? kl : 1);
    memcpy(s->key, k, kl);
    s->klen = kl; s->h = h; s->val = val;
    m->live++;
    return s;
}

static void bmap_del_slot(bmap_t* m, mslot_t* s) {
    free(s->key);
    s->key = TOMB;
    s->val = NULL;
    m->live--;
}

/* ------------------------------------------------------------------ */
/* words/1 (src/emqx_topic.erl:150-164)                                */
/* ------------------------------------------------------------------ */

enum { W_BIN = 0, W_EMPTY = 1, W_PLUS = 2, W_HASH = 3 };

typedef struct { const uint8_t* p; uint32_t n; uint8_t kind; } word_t;

typedef struct { word_t* w; size_t n, cap; } words_t;

static void words_of(const uint8_t* t, size_t len, words_t* out) {
    out->n = 0;
    size_t start = 0;
    for (size_t i = 0; i <= len; i++) {
        if (i == len || t[i] == '/') {
            if (out->n == out->cap) {
                out->cap = out->cap ? out->cap * 2 : 16;
                out->w = (word_t*)realloc(out->w, out->cap * sizeof(word_t));
            }
            word_t* w = &out->w[out->n++];
            w->p = t + start; w->n = (uint32_t)(i - start);
            if (w->n == 0) w->kind = W_EMPTY;
            else if (w->n == 1 && w->p[0] == '+') w->kind = W_PLUS;
            else if (w->n == 1 && w->p[0] == '#') w->kind = W_HASH;
            else w->kind = W_BIN;
            start = i + 1;
        }
    }
}

static int word_eq(const word_t* a, const word_t* b) {
    if (a->kind != b->kind) return 0;
    if (a->kind != W_BIN) return 1;
    return a->n == b->n && memcmp(a->p, b->p, a->n) == 0;
}

/* emqx_topic:match/2 on word lists (src/emqx_topic.erl:74-87) */
static int match_words(const word_t* n, size_t nn, const word_t* f, size_t fn) {
    size_t i = 0, j = 0;
    for (;;) {
        if (i == nn && j == fn) return 1;                       /* match([], []) */
        if (i < nn && j < fn && word_eq(&n[i], &f[j])) { i++; j++; continue; }
        if (i < nn && j < fn && f[j].kind == W_PLUS) { i++; j++; continue; }
        if (j + 1 == fn && f[j].kind == W_HASH) return 1;        /* match(_, ['#']) */
        return 0;
    }
}

/* emqx_topic:match/2 on binaries (src/emqx_topic.erl:68-73) */
static int topic_match_bin(const uint8_t* name, size_t nl, const uint8_t* flt, size_t fl,
                           words_t* wn, words_t* wf) {
    if (nl > 0 && name[0] == '$' && fl > 0 && (flt[0] == '+' || flt[0] == '#')) return 0;
    words_of(name, nl, wn);
    words_of(flt, fl, wf);
    return match_words(wn->w, wn->n, wf->w, wf->n);
}

EXPORT int tmo_topic_match(const uint8_t* name, size_t nl, const uint8_t* flt, size_t fl) {
    words_t a = {0}, b = {0};
    int r = topic_match_bin(name, nl, flt, fl, &a, &b);
    free(a.w); free(b.w);
    return r;
}

/* emqx_topic:wildcard/1 (src/emqx_topic.erl:52-62) */
EXPORT int tmo_wildcard(const uint8_t* t, size_t len) {
    words_t w = {0};
    words_of(t, len, &w);
    int r = 0;
    for (size_t i = 0; i < w.n; i++) if (w.w[i].kind == W_PLUS || w.w[i].kind == W_HASH) { r = 1; break; }
    free(w.w);
    return r;
}

/* ------------------------------------------------------------------ */
/* the trie (src/emqx_trie.erl) over two ETS-like tables               */
/* ------------------------------------------------------------------ */

/* node id encoding: root -> {0x01}; binary B -> {0x02, B...} */
/* edge key: u32 len(node_enc) | node_enc | word_enc;
 * word_enc: 0x10 '' | 0x11 '+' | 0x12 '#' | 0x13 bytes */

typedef struct {
    uint32_t edge_count;
    int64_t  topic;   /* index into the filter registry, -1 = undefined */
} trie_node_t;

typedef struct {
    uint8_t* id;      /* encoded child node id */
    uint32_t idlen;
} trie_edge_val_t;

typedef struct {
    uint8_t* p;
    uint32_t n;
} fstr_t;

typedef struct tmo {
    bmap_t   nodes;   /* emqx_trie_node */
    bmap_t   edges;   /* emqx_trie */
    bmap_t   freg;    /* filter bytes -> registry index (uintptr) */
    fstr_t*  fstr;
    size_t   nf, fcap;
    bmap_t   routes;  /* emqx_route bag: topic bytes -> (uintptr) route count */
} tmo_t;

typedef struct {
    uint64_t topics, visits, hash_hits, ets_probes, words, matches, routes;
} tmo_stats_t;

EXPORT tmo_t* tmo_create(void) {
    tmo_t* o = (tmo_t*)calloc(1, sizeof(tmo_t));
    bmap_init(&o->nodes, 1024);
    bmap_init(&o->edges, 1024);
    bmap_init(&o->freg, 1024);
    bmap_init(&o->routes, 1024);
    return o;
}

EXPORT void tmo_destroy(tmo_t* o) {
    if (!o) return;
    bmap_free(&o->nodes, 1);
    for (size_t i = 0; i < o->edges.cap; i++) {
        mslot_t* s = &o->edges.s[i];
        if (s->key && s->key != TOMB) { trie_edge_val_t* v = (trie_edge_val_t*)s->val; free(v->id); free(v); }
    }
    bmap_free(&o->edges, 0);
    bmap_free(&o->freg, 0);
    bmap_free(&o->routes, 0);
    for (size_t i = 0; i < o->nf; i++) free(o->fstr[i].p);
    free(o->fstr);
    free(o);
}

/* registry: interned filter strings (what the trie_node `topic` field holds) */
EXPORT int64_t tmo_register(tmo_t* o, const uint8_t* f, size_t fl) {
    uint64_t h = hash_bytes(f, fl);
    mslot_t* s = bmap_find(&o->freg, f, (uint32_t)fl, h);
    if (s) return (int64_t)(uintptr_t)s->val;
    if (o->nf == o->fcap) {
        o->fcap = o->fcap ? o->fcap * 2 : 1024;
        o->fstr = (fstr_t*)realloc(o->fstr, o->fcap * sizeof(fstr_t));
    }
    int64_t idx = (int64_t)o->nf++;
    o->fstr[idx].p = (uint8_t*)malloc(fl ? fl : 1);
    memcpy(o->fstr[idx].p, f, fl);
    o->fstr[idx].n = (uint32_t)fl;
    bmap_put(&o->freg, f, (uint32_t)fl, h, (void*)(uintptr_t)idx);
    return idx;
}

typedef struct { uint8_t* b; size_t n, cap; } buf_t;

static void buf_res(buf_t* b, size_t n) {
    if (n > b->cap) { b->cap = n * 2 + 64; b->b = (uint8_t*)realloc(b->b, b->cap); }
}

static void enc_word(buf_t* b, const word_t* w) {
    buf_res(b, b->n + 1 + w->n);
    b->b[b->n++] = (uint8_t)(0x10 + (w->kind == W_EMPTY ? 0 : w->kind == W_PLUS ? 1 : w->kind == W_HASH ? 2 : 3));
    if (w->kind == W_BIN) { memcpy(b->b + b->n, w->p, w->n); b->n += w->n; }
}

static void edge_key(buf_t* b, const uint8_t* nid, uint32_t nl, const word_t* w) {
    b->n = 0;
    buf_res(b, 4 + nl + 1 + w->n);
    memcpy(b->b, &nl, 4); b->n = 4;
    memcpy(b->b + 4, nid, nl); b->n += nl;
    enc_word(b, w);
}

/* join/2 (src/emqx_trie.erl:138-141): root -> bin(W); else Parent/W */
static void join_child(buf_t* out, const uint8_t* nid, uint32_t nl, const word_t* w) {
    out->n = 0;
    buf_res(out, nl + 2 + w->n);
    out->b[out->n++] = 0x02;
    if (nid[0] == 0x02) {
        memcpy(out->b + out->n, nid + 1, nl - 1); out->n += nl - 1;
        out->b[out->n++] = '/';
    }
    const uint8_t* wp; uint32_t wn;
    static const uint8_t plus = '+', hash = '#';
    if (w->kind == W_PLUS) { wp = &plus; wn = 1; }
    else if (w->kind == W_HASH) { wp = &hash; wn = 1; }
    else if (w->kind == W_EMPTY) { wp = NULL; wn = 0; }
    else { wp = w->p; wn = w->n; }
    if (wn) { memcpy(out->b + out->n, wp, wn); out->n += wn; }
}

static trie_node_t* node_read(tmo_t* o, const uint8_t* id, uint32_t n) {
    mslot_t* s = bmap_find(&o->nodes, id, n, hash_bytes(id, n));
    return s ? (trie_node_t*)s->val : NULL;
}

static void node_write(tmo_t* o, const uint8_t* id, uint32_t n, uint32_t ec, int64_t topic) {
    uint64_t h = hash_bytes(id, n);
    mslot_t* s = bmap_find(&o->nodes, id, n, h);
    if (s) { trie_node_t* t = (trie_node_t*)s->val; t->edge_count = ec; t->topic = topic; return; }
    trie_node_t* t = (trie_node_t*)malloc(sizeof(trie_node_t));
    t->edge_count = ec; t->topic = topic;
    bmap_put(&o->nodes, id, n, h, t);
}

static void node_delete(tmo_t* o, const uint8_t* id, uint32_t n) {
    mslot_t* s = bmap_find(&o->nodes, id, n, hash_bytes(id, n));
    if (s) { free(s->val); bmap_del_slot(&o->nodes, s); }
}

static trie_edge_val_t* edge_read(tmo_t* o, const buf_t* k) {
    mslot_t* s = bmap_find(&o->edges, k->b, (uint32_t)k->n, hash_bytes(k->b, k->n));
    return s ? (trie_edge_val_t*)s->val : NULL;
}

static const uint8_t ROOT_ID[1] = {0x01};

/* emqx_trie:insert/1 (src/emqx_trie.erl:81-93) with add_path/1 (:145-158) */
EXPORT int tmo_insert(tmo_t* o, const uint8_t* t, size_t len) {
    int64_t fidx = tmo_register(o, t, len);
    buf_t nid = {0};
    buf_res(&nid, len + 1);
    nid.b[0] = 0x02; memcpy(nid.b + 1, t, len); nid.n = len + 1;
    trie_node_t* tn = node_read(o, nid.b, (uint32_t)nid.n);
    if (tn) {
        if (tn->topic < 0) tn->topic = fidx;   /* topic = undefined -> Topic */
        free(nid.b);
        return 0;
    }
    words_t w = {0};
    words_of(t, len, &w);
    buf_t parent = {0}, child = {0}, key = {0};
    buf_res(&parent, 1); parent.b[0] = 0x01; parent.n = 1;
    for (size_t i = 0; i < w.n; i++) {           /* triples/1 :128-136 */
        join_child(&child, parent.b, (uint32_t)parent.n, &w.w[i]);
        edge_key(&key, parent.b, (uint32_t)parent.n, &w.w[i]);
        trie_node_t* pn = node_read(o, parent.b, (uint32_t)parent.n);
        int write_edge = 0;
        if (pn) {
            if (!edge_read(o, &key)) { pn->edge_count++; write_edge = 1; }
        } else {
            node_write(o, parent.b, (uint32_t)parent.n, 1, -1);
            write_edge = 1;
        }
        if (write_edge) {
            trie_edge_val_t* v = (trie_edge_val_t*)malloc(sizeof(*v));
            v->id = (uint8_t*)malloc(child.n); memcpy(v->id, child.b, child.n); v->idlen = (uint32_t)child.n;
            bmap_put(&o->edges, key.b, (uint32_t)key.n, hash_bytes(key.b, key.n), v);
        }
        buf_t tmp = parent; parent = child; child = tmp;
    }
    /* write_trie_node(#trie_node{node_id = Topic, topic = Topic}) -- edge_count = 0 */
    node_write(o, nid.b, (uint32_t)nid.n, 0, fidx);
    free(w.w); free(parent.b); free(child.b); free(key.b); free(nid.b);
    return 0;
}

/* emqx_trie:delete/1 (src/emqx_trie.erl:107-116), delete_path/1 (:190-204).
 * Returns 0, or -1 for the reference's mnesia:abort({node_not_found, _})
 * (unreachable on a trie built only through insert/delete). */
EXPORT int tmo_delete(tmo_t* o, const uint8_t* t, size_t len) {
    buf_t nid = {0};
    buf_res(&nid, len + 1);
    nid.b[0] = 0x02; memcpy(nid.b + 1, t, len); nid.n = len + 1;
    trie_node_t* tn = node_read(o, nid.b, (uint32_t)nid.n);
    int rc = 0;
    if (!tn) { free(nid.b); return 0; }
    if (tn->edge_count != 0) { tn->topic = -1; free(nid.b); return 0; }
    node_delete(o, nid.b, (uint32_t)nid.n);
    words_t w = {0};
    words_of(t, len, &w);
    /* build the triples, then walk them in reverse */
    buf_t* ids = (buf_t*)calloc(w.n + 1, sizeof(buf_t));
    buf_res(&ids[0], 1); ids[0].b[0] = 0x01; ids[0].n = 1;
    for (size_t i = 0; i < w.n; i++) join_child(&ids[i + 1], ids[i].b, (uint32_t)ids[i].n, &w.w[i]);
    buf_t key = {0};
    for (size_t k = w.n; k-- > 0;) {
        edge_key(&key, ids[k].b, (uint32_t)ids[k].n, &w.w[k]);
        mslot_t* es = bmap_find(&o->edges, key.b, (uint32_t)key.n, hash_bytes(key.b, key.n));
        if (es) { trie_edge_val_t* v = (trie_edge_val_t*)es->val; free(v->id); free(v); bmap_del_slot(&o->edges, es); }
        trie_node_t* pn = node_read(o, ids[k].b, (uint32_t)ids[k].n);
        if (!pn) { rc = -1; break; }
        if (pn->edge_count == 1 && pn->topic < 0) { node_delete(o, ids[k].b, (uint32_t)ids[k].n); continue; }
        if (pn->edge_count == 1) { pn->edge_count = 0; break; }
        pn->edge_count--;
        break;
    }
    for (size_t i = 0; i <= w.n; i++) free(ids[i].b);
    free(ids); free(key.b); free(w.w); free(nid.b);
    return rc;
}

/* emqx_trie:lookup/1: node_id = NULL -> root. Returns 1 if found. */
EXPORT int tmo_lookup(tmo_t* o, const uint8_t* id, size_t len, int is_root,
                      uint32_t* edge_count, int64_t* topic) {
    buf_t nid = {0};
    if (is_root) { buf_res(&nid, 1); nid.b[0] = 0x01; nid.n = 1; }
    else { buf_res(&nid, len + 1); nid.b[0] = 0x02; memcpy(nid.b + 1, id, len); nid.n = len + 1; }
    trie_node_t* tn = node_read(o, nid.b, (uint32_t)nid.n);
    free(nid.b);
    if (!tn) return 0;
    *edge_count = tn->edge_count;
    *topic = tn->topic;
    return 1;
}

/* emqx_trie:empty/0: ets:info(emqx_trie, size) == 0 */
EXPORT int tmo_empty(tmo_t* o) { return o->edges.live == 0; }
EXPORT uint64_t tmo_edge_count_total(tmo_t* o) { return o->edges.live; }
EXPORT uint64_t tmo_node_count_total(tmo_t* o) { return o->nodes.live; }

EXPORT const uint8_t* tmo_filter_bytes(tmo_t* o, int64_t idx, uint32_t* len) {
    if (idx < 0 || (size_t)idx >= o->nf) return NULL;
    *len = o->fstr[idx].n;
    return o->fstr[idx].p;
}

/* ---- match/1 --------------------------------------------------------- */

typedef struct {
    words_t  w;
    buf_t    key;
    buf_t    nid;
    int64_t* acc;     /* reversed result list (prepend == push) */
    size_t   nacc, cacc;
    tmo_stats_t st;
} mctx_t;

static void acc_push(mctx_t* c, int64_t topic) {
    if (c->nacc == c->cacc) {
        c->cacc = c->cacc ? c->cacc * 2 : 64;
        c->acc = (int64_t*)realloc(c->acc, c->cacc * sizeof(int64_t));
    }
    c->acc[c->nacc++] = topic;
}

static const word_t WORD_HASH_ATOM = {NULL, 0, W_HASH};
static const word_t WORD_PLUS_ATOM = {NULL, 0, W_PLUS};

/* 'match_#'/2 (src/emqx_trie.erl:181-186) */
static void match_hash(tmo_t* o, mctx_t* c, const uint8_t* nid, uint32_t nl) {
    edge_key(&c->key, nid, nl, &WORD_HASH_ATOM);
    c->st.ets_probes++;
    trie_edge_val_t* e = edge_read(o, &c->key);
    if (e) {
        c->st.hash_hits++;
        c->st.ets_probes++;
        trie_node_t* tn = node_read(o, e->id, e->idlen);
        if (tn) acc_push(c, tn->topic);
    }
}

/* match_node/3 (src/emqx_trie.erl:168-177) */
static void match_node(tmo_t* o, mctx_t* c, const uint8_t* nid, uint32_t nl, size_t wi) {
    c->st.visits++;
    if (wi == c->w.n) {
        /* mnesia:read(?TRIE_NODE_TAB, NodeId) ++ 'match_#'(NodeId, ResAcc) */
        match_hash(o, c, nid, nl);
        c->st.ets_probes++;
        trie_node_t* tn = node_read(o, nid, nl);
        if (tn) acc_push(c, tn->topic);
        return;
    }
    match_hash(o, c, nid, nl);
    /* lists:foldl over [W, '+'] */
    const word_t* args[2] = {&c->w.w[wi], &WORD_PLUS_ATOM};
    for (int a = 0; a < 2; a++) {
        edge_key(&c->key, nid, nl, args[a]);
        c->st.ets_probes++;
        trie_edge_val_t* e = edge_read(o, &c->key);
        if (e) {
            /* the child id lives in the edge table; copy it since key buf is reused */
            uint8_t stackid[256];
            uint8_t* cid = e->idlen <= sizeof(stackid) ? stackid : (uint8_t*)malloc(e->idlen);
            memcpy(cid, e->id, e->idlen);
            match_node(o, c, cid, e->idlen, wi + 1);
            if (cid != stackid) free(cid);
        }
    }
}

/* emqx_trie:match/1 (src/emqx_trie.erl:96-99) incl. the `$` root rule (:162-163) */
static void trie_match(tmo_t* o, mctx_t* c, const uint8_t* t, size_t len) {
    c->nacc = 0;
    words_of(t, len, &c->w);
    c->st.topics++;
    c->st.words += c->w.n;
    if (o->edges.live == 0) return;    /* emqx_router:match_trie/1 empty() short-cut */
    if (c->w.n > 0 && c->w.w[0].kind == W_BIN && c->w.w[0].p[0] == '$') {
        buf_res(&c->nid, c->w.w[0].n + 1);
        c->nid.b[0] = 0x02; memcpy(c->nid.b + 1, c->w.w[0].p, c->w.w[0].n);
        uint32_t nl = c->w.w[0].n + 1;
        uint8_t* cid = (uint8_t*)malloc(nl);
        memcpy(cid, c->nid.b, nl);
        match_node(o, c, cid, nl, 1);
        free(cid);
    } else {
        match_node(o, c, ROOT_ID, 1, 0);
    }
}

static void ctx_free(mctx_t* c) { free(c->w.w); free(c->key.b); free(c->nid.b); free(c->acc); }

/* Single-topic match in the reference's DFS order, topic==undefined removed.
 * Writes up to cap registry indices; returns the full count. */
EXPORT size_t tmo_match(tmo_t* o, const uint8_t* t, size_t len, int64_t* out, size_t cap,
                        tmo_stats_t* st) {
    mctx_t c; memset(&c, 0, sizeof(c));
    trie_match(o, &c, t, len);
    size_t n = 0;
    for (size_t i = c.nacc; i-- > 0;) {
        if (c.acc[i] < 0) continue;
        if (n < cap) out[n] = c.acc[i];
        n++;
    }
    if (st) *st = c.st;
    ctx_free(&c);
    return n;
}

/* ---- batches (sorted by Erlang binary order) ------------------------- */

static int cmp_bin(const fstr_t* a, const fstr_t* b) {
    uint32_t m = a->n < b->n ? a->n : b->n;
    int r = memcmp(a->p, b->p, m);
    if (r) return r;
    return (a->n > b->n) - (a->n < b->n);
}

typedef struct {
    const fstr_t* tab;
} sort_ctx_t;

static int cmp_idx_r(const void* x, const void* y, void* arg) {
    const fstr_t* tab = ((sort_ctx_t*)arg)->tab;
    int64_t a = *(const int64_t*)x, b = *(const int64_t*)y;
    return cmp_bin(&tab[a], &tab[b]);
}

typedef struct {
    uint32_t* counts;
    int64_t*  idx;
    uint64_t  total;
    tmo_stats_t st;
} tmo_batch_t;

typedef struct {
    tmo_t* o;
    const uint8_t* topics; const uint64_t* offs;
    uint64_t lo, hi;
    int sorted, mode;                 /* mode 0 = trie, 1 = brute, 2 = match_routes */
    const fstr_t* flist; uint64_t nfl; /* brute force filter list */
    uint32_t* counts;                 /* global array, slice [lo,hi) */
    int64_t* out; uint64_t nout, cout;
    tmo_stats_t st;
} job_t;

static void job_push(job_t* j, int64_t v) {
    if (j->nout == j->cout) {
        j->cout = j->cout ? j->cout * 2 : 4096;
        j->out = (int64_t*)realloc(j->out, j->cout * sizeof(int64_t));
    }
    j->out[j->nout++] = v;
}

static uint64_t route_count(tmo_t* o, const uint8_t* t, uint32_t n) {
    mslot_t* s = bmap_find(&o->routes, t, n, hash_bytes(t, n));
    return s ? (uint64_t)(uintptr_t)s->val : 0;
}

static void* job_run(void* arg) {
    job_t* j = (job_t*)arg;
    mctx_t c; memset(&c, 0, sizeof(c));
    words_t wn = {0}, wf = {0};
    sort_ctx_t sc = { j->mode == 1 ? j->flist : (j->o ? j->o->fstr : NULL) };
    for (uint64_t t = j->lo; t < j->hi; t++) {
        const uint8_t* tp = j->topics + j->offs[t];
        size_t tl = j->offs[t + 1] - j->offs[t];
        uint64_t start = j->nout;
        if (j->mode == 1) {
            for (uint64_t f = 0; f < j->nfl; f++)
                if (topic_match_bin(tp, tl, j->flist[f].p, j->flist[f].n, &wn, &wf)) job_push(j, (int64_t)f);
        } else {
            trie_match(j->o, &c, tp, tl);
            for (size_t i = c.nacc; i-- > 0;) if (c.acc[i] >= 0) job_push(j, c.acc[i]);
            if (j->mode == 2) {
                /* emqx_router:match_routes/1 (src/emqx_router.erl:127-133):
                 * Matched == [] -> lookup_routes(Topic);
                 * else append([lookup_routes(To) || To <- [Topic | Matched]]) */
                uint64_t r = route_count(j->o, tp, (uint32_t)tl);
                for (uint64_t k = start; k < j->nout; k++) {
                    const fstr_t* f = &j->o->fstr[j->out[k]];
                    r += route_count(j->o, f->p, f->n);
                }
                j->st.routes += r;
                j->st.matches += j->nout - start;
                j->nout = start;          /* routes are counted, not materialised */
                j->counts[t] = (uint32_t)r;
                continue;
            }
        }
        if (j->sorted && j->nout - start > 1) {
            qsort_r(j->out + start, j->nout - start, sizeof(int64_t), cmp_idx_r, &sc);
            /* the contract is the deduplicated set: the reference walk lists a
             * filter twice only for topic names containing '+'/'#' words */
            uint64_t w = start + 1;
            for (uint64_t r = start + 1; r < j->nout; r++)
                if (j->out[r] != j->out[w - 1]) j->out[w++] = j->out[r];
            j->nout = w;
        }
        j->counts[t] = (uint32_t)(j->nout - start);
        j->st.matches += j->nout - start;
    }
    j->st.topics += c.st.topics; j->st.visits += c.st.visits; j->st.hash_hits += c.st.hash_hits;
    j->st.ets_probes += c.st.ets_probes; j->st.words += c.st.words;
    ctx_free(&c); free(wn.w); free(wf.w);
    return NULL;
}

static tmo_batch_t* run_jobs(tmo_t* o, const uint8_t* topics, const uint64_t* offs, uint64_t n,
                             int nthreads, int sorted, int mode, const fstr_t* fl, uint64_t nfl) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n && n > 0) nthreads = (int)n;
    tmo_batch_t* b = (tmo_batch_t*)calloc(1, sizeof(tmo_batch_t));
    b->counts = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; i < nthreads; i++) {
        job_t* j = &jobs[i];
        j->o = o; j->topics = topics; j->offs = offs;
        j->lo = n * (uint64_t)i / (uint64_t)nthreads;
        j->hi = n * (uint64_t)(i + 1) / (uint64_t)nthreads;
        j->sorted = sorted; j->mode = mode; j->flist = fl; j->nfl = nfl;
        j->counts = b->counts;
    }
    if (nthreads == 1) job_run(&jobs[0]);
    else {
        for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, job_run, &jobs[i]);
        for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    }
    uint64_t total = 0;
    for (int i = 0; i < nthreads; i++) total += jobs[i].nout;
    b->idx = (int64_t*)malloc((total ? total : 1) * sizeof(int64_t));
    uint64_t p = 0;
    for (int i = 0; i < nthreads; i++) {
        if (jobs[i].nout) memcpy(b->idx + p, jobs[i].out, jobs[i].nout * sizeof(int64_t));
        p += jobs[i].nout;
        free(jobs[i].out);
        tmo_stats_t* s = &jobs[i].st;
        b->st.topics += s->topics; b->st.visits += s->visits; b->st.hash_hits += s->hash_hits;
        b->st.ets_probes += s->ets_probes; b->st.words += s->words; b->st.matches += s->matches;
        b->st.routes += s->routes;
    }
    b->total = total;
    free(jobs); free(th);
    return b;
}

/* trie-walk batch: per-topic lists of registry indices, sorted by bytes when `sorted` */
EXPORT tmo_batch_t* tmo_match_batch(tmo_t* o, const uint8_t* topics, const uint64_t* offs,
                                    uint64_t n, int nthreads, int sorted) {
    return run_jobs(o, topics, offs, n, nthreads, sorted, 0, NULL, 0);
}

/* emqx_router:match_routes/1 batch: per-topic route counts only (CPU baseline) */
EXPORT tmo_batch_t* tmo_match_routes_batch(tmo_t* o, const uint8_t* topics, const uint64_t* offs,
                                           uint64_t n, int nthreads) {
    return run_jobs(o, topics, offs, n, nthreads, 0, 2, NULL, 0);
}

/* brute force emqx_topic:match/2 over an explicit filter list; indices are into that list */
EXPORT tmo_batch_t* tmo_brute_batch(const uint8_t* fbytes, const uint64_t* foffs, uint64_t nf,
                                    const uint8_t* topics, const uint64_t* offs, uint64_t n,
                                    int nthreads) {
    fstr_t* fl = (fstr_t*)malloc((nf ? nf : 1) * sizeof(fstr_t));
    for (uint64_t i = 0; i < nf; i++) { fl[i].p = (uint8_t*)fbytes + foffs[i]; fl[i].n = (uint32_t)(foffs[i + 1] - foffs[i]); }
    tmo_batch_t* b = run_jobs(NULL, topics, offs, n, nthreads, 1, 1, fl, nf);
    free(fl);
    return b;
}

EXPORT void tmo_batch_get(tmo_batch_t* b, uint32_t** counts, int64_t** idx, uint64_t* total,
                          tmo_stats_t* st) {
    *counts = b->counts; *idx = b->idx; *total = b->total;
    if (st) *st = b->st;
}

EXPORT void tmo_batch_free(tmo_batch_t* b) {
    if (!b) return;
    free(b->counts); free(b->idx); free(b);
}

/* route bag (emqx_route, include/emqx.hrl:87-90): only the per-topic route
 * count matters to the baseline's work (one ets:lookup per [Topic|Matched]). */
EXPORT void tmo_route_add(tmo_t* o, const uint8_t* t, size_t len) {
    uint64_t h = hash_bytes(t, len);
    mslot_t* s = bmap_find(&o->routes, t, (uint32_t)len, h);
    if (s) s->val = (void*)((uintptr_t)s->val + 1);
    else bmap_put(&o->routes, t, (uint32_t)len, h, (void*)(uintptr_t)1);
}

/* emqx_router:do_add_route/1 minus the gen_server: wildcard -> trie + route,
 * exact -> route only (src/emqx_router.erl:113-124, 226-234) */
EXPORT void tmo_add_route(tmo_t* o, const uint8_t* t, size_t len) {
    if (tmo_wildcard(t, len)) {
        if (route_count(o, t, (uint32_t)len) == 0) tmo_insert(o, t, len);
    } else {
        tmo_register(o, t, len);
    }
    tmo_route_add(o, t, len);
}
