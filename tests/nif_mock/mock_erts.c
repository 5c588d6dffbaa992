/*
 * mock_erts.c -- test stand-in for the Erlang runtime under the emqx_tm NIF
 * (see erl_nif.h next to it).  Linked with emqx_tm_nif.c into
 * libemqx_nif_mock.so, which tests/test_nif.py drives through ctypes: build
 * argument terms, call a NIF by name as a given "process", read the reply
 * terms back as Python literals, and read what the engine's completion
 * threads sent to a process's mailbox.
 */
#include <pthread.h>
#include <stdarg.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "erl_nif.h"

#define API __attribute__((visibility("default")))

enum { T_ATOM, T_INT, T_BIN, T_TUPLE, T_CONS, T_NIL, T_REF, T_RES, T_BADARG };

typedef struct node {
    int tag;
    size_t n;                 /* binary size / tuple arity */
    int64_t v;                /* integer / ref id */
    unsigned char* data;      /* binary bytes */
    char* name;               /* atom */
    const struct node** el;   /* tuple elements; cons: el[0] head, el[1] tail */
    void* obj;                /* resource */
} node;

struct mock_env { int pid; };
struct mock_rt { ErlNifResourceDtor* dtor; };
typedef struct {
    ErlNifResourceType* type;
    atomic_int refs;
    int pad;
    long long align[1];
} res_hdr;

static atomic_int live_resources;
static atomic_long next_ref = 1;

static node* mk(int tag) {
    node* x = calloc(1, sizeof(node));
    if (!x) abort();
    x->tag = tag;
    return x;
}
#define T(x) ((ERL_NIF_TERM)(x))
#define N(t) ((const node*)(t))

void* enif_alloc(size_t size) { return malloc(size ? size : 1); }
void enif_free(void* p) { free(p); }

ErlNifEnv* enif_alloc_env(void) {
    ErlNifEnv* e = calloc(1, sizeof(ErlNifEnv));
    e->pid = -1;
    return e;
}
void enif_free_env(ErlNifEnv* env) { free(env); }   /* terms live on */

ErlNifPid* enif_self(ErlNifEnv* env, ErlNifPid* pid) {
    pid->id = env->pid;
    return pid;
}

/* ---- mailboxes ---- */
typedef struct msg { int pid; ERL_NIF_TERM t; struct msg* next; } msg;
static msg *mb_head, *mb_tail;
static pthread_mutex_t mb_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t mb_cv = PTHREAD_COND_INITIALIZER;

int enif_send(ErlNifEnv* caller_env, const ErlNifPid* to, ErlNifEnv* msg_env, ERL_NIF_TERM t) {
    (void)caller_env; (void)msg_env;
    msg* m = calloc(1, sizeof(msg));
    m->pid = to->id;
    m->t = t;
    pthread_mutex_lock(&mb_mu);
    if (mb_tail) mb_tail->next = m; else mb_head = m;
    mb_tail = m;
    pthread_cond_broadcast(&mb_cv);
    pthread_mutex_unlock(&mb_mu);
    return 1;
}

ERL_NIF_TERM enif_make_copy(ErlNifEnv* dst, ERL_NIF_TERM t) { (void)dst; return t; }

/* ---- resources ---- */
ErlNifResourceType* enif_open_resource_type(ErlNifEnv* env, const char* module, const char* name,
                                            ErlNifResourceDtor* dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags* tried) {
    (void)env; (void)module; (void)name; (void)flags; (void)tried;
    ErlNifResourceType* t = calloc(1, sizeof(ErlNifResourceType));
    t->dtor = dtor;
    return t;
}

static res_hdr* hdr_of(void* obj) { return (res_hdr*)((char*)obj - offsetof(res_hdr, align)); }

void* enif_alloc_resource(ErlNifResourceType* type, size_t size) {
    res_hdr* h = calloc(1, sizeof(res_hdr) + size);
    h->type = type;
    atomic_store(&h->refs, 1);
    atomic_fetch_add(&live_resources, 1);
    return (void*)h->align;
}
void enif_keep_resource(void* obj) { atomic_fetch_add(&hdr_of(obj)->refs, 1); }
void enif_release_resource(void* obj) {
    res_hdr* h = hdr_of(obj);
    if (atomic_fetch_sub(&h->refs, 1) == 1) {
        if (h->type->dtor) h->type->dtor(NULL, obj);
        atomic_fetch_sub(&live_resources, 1);
        free(h);
    }
}
ERL_NIF_TERM enif_make_resource(ErlNifEnv* env, void* obj) {
    (void)env;
    node* x = mk(T_RES);
    x->obj = obj;
    enif_keep_resource(obj);   /* the term's reference: mock_drop_resource_term */
    return T(x);
}
int enif_get_resource(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifResourceType* type, void** objp) {
    (void)env;
    if (N(t)->tag != T_RES || hdr_of(N(t)->obj)->type != type) return 0;
    *objp = N(t)->obj;
    return 1;
}

/* ---- term construction ---- */
ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name) {
    (void)env;
    node* x = mk(T_ATOM);
    x->name = strdup(name);
    return T(x);
}
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env) { (void)env; return T(mk(T_BADARG)); }
ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, uint64_t v) {
    (void)env;
    node* x = mk(T_INT);
    x->v = (int64_t)v;
    return T(x);
}
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned v) { return enif_make_uint64(env, v); }
static ERL_NIF_TERM tuple(unsigned n, const ERL_NIF_TERM* e) {
    node* x = mk(T_TUPLE);
    x->n = n;
    x->el = calloc(n ? n : 1, sizeof(node*));
    for (unsigned i = 0; i < n; ++i) x->el[i] = N(e[i]);
    return T(x);
}
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b) {
    (void)env;
    ERL_NIF_TERM e[2] = {a, b};
    return tuple(2, e);
}
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c) {
    (void)env;
    ERL_NIF_TERM e[3] = {a, b, c};
    return tuple(3, e);
}
ERL_NIF_TERM enif_make_tuple5(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c, ERL_NIF_TERM d,
                              ERL_NIF_TERM f) {
    (void)env;
    ERL_NIF_TERM e[5] = {a, b, c, d, f};
    return tuple(5, e);
}
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv* env, ERL_NIF_TERM head, ERL_NIF_TERM tail) {
    (void)env;
    node* x = mk(T_CONS);
    x->el = calloc(2, sizeof(node*));
    x->el[0] = N(head);
    x->el[1] = N(tail);
    return T(x);
}
ERL_NIF_TERM enif_make_list(ErlNifEnv* env, unsigned cnt, ...) {
    ERL_NIF_TERM* e = calloc(cnt ? cnt : 1, sizeof(ERL_NIF_TERM));
    va_list ap;
    va_start(ap, cnt);
    for (unsigned i = 0; i < cnt; ++i) e[i] = va_arg(ap, ERL_NIF_TERM);
    va_end(ap);
    ERL_NIF_TERM l = T(mk(T_NIL));
    for (unsigned i = cnt; i-- > 0;) l = enif_make_list_cell(env, e[i], l);
    free(e);
    return l;
}
ERL_NIF_TERM enif_make_list1(ErlNifEnv* env, ERL_NIF_TERM e1) { return enif_make_list(env, 1, e1); }
unsigned char* enif_make_new_binary(ErlNifEnv* env, size_t size, ERL_NIF_TERM* termp) {
    (void)env;
    node* x = mk(T_BIN);
    x->n = size;
    x->data = malloc(size ? size : 1);
    *termp = T(x);
    return x->data;
}

/* ---- term inspection ---- */
int enif_get_int(ErlNifEnv* env, ERL_NIF_TERM t, int* ip) {
    (void)env;
    if (N(t)->tag != T_INT || N(t)->v < -2147483648LL || N(t)->v > 2147483647LL) return 0;
    *ip = (int)N(t)->v;
    return 1;
}
int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM t, unsigned* ip) {
    (void)env;
    if (N(t)->tag != T_INT || N(t)->v < 0 || N(t)->v > 4294967295LL) return 0;
    *ip = (unsigned)N(t)->v;
    return 1;
}
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM t, ErlNifBinary* bin) {
    (void)env;
    if (N(t)->tag != T_BIN) return 0;
    bin->size = N(t)->n;
    bin->data = N(t)->data;
    return 1;
}
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM t, unsigned* len) {
    (void)env;
    unsigned n = 0;
    const node* x = N(t);
    while (x->tag == T_CONS) { ++n; x = x->el[1]; }
    if (x->tag != T_NIL) return 0;
    *len = n;
    return 1;
}
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM list, ERL_NIF_TERM* head, ERL_NIF_TERM* tail) {
    (void)env;
    if (N(list)->tag != T_CONS) return 0;
    *head = T(N(list)->el[0]);
    *tail = T(N(list)->el[1]);
    return 1;
}
int enif_get_tuple(ErlNifEnv* env, ERL_NIF_TERM t, int* arity, const ERL_NIF_TERM** array) {
    (void)env;
    if (N(t)->tag != T_TUPLE) return 0;
    *arity = (int)N(t)->n;
    *array = (const ERL_NIF_TERM*)N(t)->el;
    return 1;
}
static int same(const node* a, const node* b) {
    if (a == b) return 1;
    if (a->tag != b->tag) return 0;
    switch (a->tag) {
        case T_ATOM: return strcmp(a->name, b->name) == 0;
        case T_INT: case T_REF: return a->v == b->v;
        case T_BIN: return a->n == b->n && (!a->n || memcmp(a->data, b->data, a->n) == 0);
        case T_NIL: return 1;
        case T_RES: return a->obj == b->obj;
        case T_CONS: return same(a->el[0], b->el[0]) && same(a->el[1], b->el[1]);
        case T_TUPLE:
            if (a->n != b->n) return 0;
            for (size_t i = 0; i < a->n; ++i)
                if (!same(a->el[i], b->el[i])) return 0;
            return 1;
        default: return 0;
    }
}
int enif_is_identical(ERL_NIF_TERM a, ERL_NIF_TERM b) { return same(N(a), N(b)); }
int enif_compare(ERL_NIF_TERM a, ERL_NIF_TERM b) { return same(N(a), N(b)) ? 0 : 1; }   /* equality only */
int enif_is_ref(ErlNifEnv* env, ERL_NIF_TERM t) { (void)env; return N(t)->tag == T_REF; }

/* ---- test API ---- */
API ERL_NIF_TERM mock_atom(const char* name) { return enif_make_atom(NULL, name); }
API ERL_NIF_TERM mock_int(int64_t v) { return enif_make_uint64(NULL, (uint64_t)v); }
API ERL_NIF_TERM mock_bin(const void* p, size_t n) {
    ERL_NIF_TERM t;
    unsigned char* d = enif_make_new_binary(NULL, n, &t);
    if (n) memcpy(d, p, n);
    return t;
}
API ERL_NIF_TERM mock_list(const ERL_NIF_TERM* e, unsigned n) {
    ERL_NIF_TERM l = T(mk(T_NIL));
    for (unsigned i = n; i-- > 0;) l = enif_make_list_cell(NULL, e[i], l);
    return l;
}
API ERL_NIF_TERM mock_tuple(const ERL_NIF_TERM* e, unsigned n) { return tuple(n, e); }
API ERL_NIF_TERM mock_ref(void) {
    node* x = mk(T_REF);
    x->v = atomic_fetch_add(&next_ref, 1);
    return T(x);
}
API ErlNifEnv* mock_process(int pid) {
    ErlNifEnv* e = enif_alloc_env();
    e->pid = pid;
    return e;
}

extern ErlNifEntry* nif_init(void);

API int mock_load(void) {
    ErlNifEnv* env = mock_process(0);
    ErlNifEntry* en = nif_init();
    int rc = en->load ? en->load(env, NULL, T(mk(T_NIL))) : 0;
    enif_free_env(env);
    return rc;
}

API void mock_unload(void) {
    ErlNifEntry* en = nif_init();
    if (en->unload) en->unload(NULL, NULL);
}

/* flags of the NIF (its scheduler class), -1 if absent */
API int mock_nif_flags(const char* name, unsigned arity) {
    ErlNifEntry* en = nif_init();
    for (int i = 0; i < en->num_of_funcs; ++i)
        if (strcmp(en->funcs[i].name, name) == 0 && en->funcs[i].arity == arity) return (int)en->funcs[i].flags;
    return -1;
}

API ERL_NIF_TERM mock_call(const char* name, unsigned arity, ErlNifEnv* env, const ERL_NIF_TERM* argv) {
    ErlNifEntry* en = nif_init();
    for (int i = 0; i < en->num_of_funcs; ++i)
        if (strcmp(en->funcs[i].name, name) == 0 && en->funcs[i].arity == arity)
            return en->funcs[i].fptr(env, (int)arity, argv);
    return 0;
}

/* next message for pid, waiting up to timeout_ms; 0 if none */
API ERL_NIF_TERM mock_recv(int pid, int timeout_ms) {
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    dl.tv_sec += timeout_ms / 1000;
    dl.tv_nsec += (long)(timeout_ms % 1000) * 1000000L;
    if (dl.tv_nsec >= 1000000000L) { dl.tv_sec++; dl.tv_nsec -= 1000000000L; }
    ERL_NIF_TERM out = 0;
    pthread_mutex_lock(&mb_mu);
    for (;;) {
        msg *prev = NULL, *m = mb_head;
        while (m && m->pid != pid) { prev = m; m = m->next; }
        if (m) {
            if (prev) prev->next = m->next; else mb_head = m->next;
            if (mb_tail == m) mb_tail = prev;
            out = m->t;
            free(m);
            break;
        }
        if (pthread_cond_timedwait(&mb_cv, &mb_mu, &dl)) break;
    }
    pthread_mutex_unlock(&mb_mu);
    return out;
}

API ERL_NIF_TERM mock_tuple_elem(ERL_NIF_TERM t, unsigned i) {
    return (N(t)->tag == T_TUPLE && i < N(t)->n) ? T(N(t)->el[i]) : 0;
}

API void mock_drop_resource_term(ERL_NIF_TERM t) {
    if (N(t)->tag == T_RES) enif_release_resource(N(t)->obj);
}
API int mock_live_resources(void) { return atomic_load(&live_resources); }

/* The term as a Python literal: atom -> 'name', binary -> b'\x..', integer,
 * tuple, list, ref -> ('#ref', id), resource -> ('#res',), badarg ->
 * ('#badarg',).  Returns the length needed (writes at most cap bytes). */
typedef struct { char* p; size_t cap, len; } sbuf;
static void put(sbuf* s, const char* fmt, ...) {
    char tmp[64];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(tmp, sizeof tmp, fmt, ap);
    va_end(ap);
    for (int i = 0; i < n; ++i, ++s->len)
        if (s->len < s->cap) s->p[s->len] = tmp[i];
}
static void fmt(sbuf* s, const node* x) {
    switch (x->tag) {
        case T_ATOM: put(s, "'"); for (const char* c = x->name; *c; ++c) put(s, "%c", *c); put(s, "'"); break;
        case T_INT: put(s, "%lld", (long long)x->v); break;
        case T_BIN: put(s, "b'"); for (size_t i = 0; i < x->n; ++i) put(s, "\\x%02x", x->data[i]); put(s, "'"); break;
        case T_NIL: put(s, "[]"); break;
        case T_REF: put(s, "('#ref', %lld)", (long long)x->v); break;
        case T_RES: put(s, "('#res',)"); break;
        case T_BADARG: put(s, "('#badarg',)"); break;
        case T_TUPLE:
            put(s, "(");
            for (size_t i = 0; i < x->n; ++i) { fmt(s, x->el[i]); put(s, ","); }
            put(s, ")");
            break;
        case T_CONS:
            put(s, "[");
            while (x->tag == T_CONS) { fmt(s, x->el[0]); put(s, ","); x = x->el[1]; }
            put(s, "]");
            break;
    }
}
API size_t mock_format(ERL_NIF_TERM t, char* buf, size_t cap) {
    sbuf s = {buf, cap, 0};
    fmt(&s, N(t));
    if (s.len < cap) buf[s.len] = 0;
    return s.len + 1;
}
