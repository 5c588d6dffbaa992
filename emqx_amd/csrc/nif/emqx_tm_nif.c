/*
 * emqx_tm_nif.c -- erl_nif shim binding include/emqx_tm.h to the Erlang module
 * `emqx_tm` (emqx_amd/erlang/emqx_tm.erl).  It is the reference-side binding of
 * the C ABI: EMQ X's emqx_trie / emqx_router call these instead of walking the
 * mnesia trie tables.
 *
 * Build (needs OTP headers, absent from this image):
 *   gcc -O2 -fPIC -shared -I$(erl -noshell -eval 'io:format("~s",[code:root_dir()])' \
 *       -s init stop)/usr/include -I../../../include emqx_tm_nif.c \
 *       -L../.. -lemqx_tm -Wl,-rpath,'$ORIGIN' -o priv/emqx_tm_nif.so
 *
 * Scheduling: trie mutations and lookups are host-only and short, but they
 * share the engine mutex with device batches, so every call that takes the
 * engine runs on a dirty I/O scheduler.  match_async/3 only queues the topic
 * (tm_match_async) and runs on a normal scheduler; the engine's completion
 * thread builds the reply in a process-independent environment and sends it.
 * The pairwise predicate is pure and runs on a normal scheduler.
 *
 * Results never alias engine scratch: batch calls run on a tm_batch of their
 * own (freed before the NIF returns), and filter ids become binaries through
 * tm_filters_copy, which copies under the engine lock and skips ids whose
 * filter is gone -- so concurrent callers and writers cannot free or rewrite
 * what a reply is being built from.
 *
 * Errors: a non-binary topic raises badarg (the reference's function_clause
 * class, src/emqx_trie.erl:82,97,108); engine errors return {error, Reason}.
 */
#include <erl_nif.h>
#include <pthread.h>
#include <string.h>

#include "emqx_tm.h"

static ErlNifResourceType* ENGINE_RT;

typedef struct {
    tm_engine* e;
} engine_res;

static ERL_NIF_TERM ATOM_OK, ATOM_ERROR, ATOM_TRUE, ATOM_FALSE, ATOM_UNDEFINED, ATOM_ROOT,
    ATOM_TRIE_NODE, ATOM_NODE_NOT_FOUND, ATOM_ENOMEM, ATOM_EIO, ATOM_EINVAL, ATOM_ENODEV,
    ATOM_EOVERFLOW, ATOM_NOT_FOUND, ATOM_WRITE, ATOM_DELETE_OBJECT, ATOM_EMQX_TM_MATCH;

/* set while a match callback runs on the engine's completion thread */
static __thread int in_engine_callback;

/* Engines whose last reference went away inside a match callback cannot be
 * destroyed there (tm_destroy joins the completion thread that runs the
 * callback): they go to the library's reaper thread, started by load/3 and
 * joined by unload/2, so no engine outlives the module and none leaks. */
typedef struct reap_node {
    tm_engine* e;
    struct reap_node* next;
} reap_node;
static pthread_mutex_t reap_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t reap_cv = PTHREAD_COND_INITIALIZER;
static reap_node* reap_head;
static int reap_stop, reap_running;
static pthread_t reap_thread;

static void* reaper(void* arg) {
    (void)arg;
    pthread_mutex_lock(&reap_mu);
    for (;;) {
        while (!reap_head && !reap_stop) pthread_cond_wait(&reap_cv, &reap_mu);
        if (!reap_head) break;   /* stopping and drained */
        reap_node* n = reap_head;
        reap_head = n->next;
        pthread_mutex_unlock(&reap_mu);
        tm_destroy(n->e);
        enif_free(n);
        pthread_mutex_lock(&reap_mu);
    }
    pthread_mutex_unlock(&reap_mu);
    return NULL;
}

static void engine_dtor(ErlNifEnv* env, void* obj) {
    (void)env;
    engine_res* r = (engine_res*)obj;
    if (r->e && in_engine_callback) {
        reap_node* n = enif_alloc(sizeof(reap_node));
        if (n) {
            n->e = r->e;
            pthread_mutex_lock(&reap_mu);
            n->next = reap_head;
            reap_head = n;
            pthread_cond_signal(&reap_cv);
            pthread_mutex_unlock(&reap_mu);
        }
        /* (allocation failure: the engine leaks rather than deadlocking here) */
    } else if (r->e) {
        tm_destroy(r->e);
    }
    r->e = NULL;
}

static ERL_NIF_TERM err(ErlNifEnv* env, int rc) {
    ERL_NIF_TERM why;
    switch (rc) {
        case TM_ENOMEM: why = ATOM_ENOMEM; break;
        case TM_ENODEV: why = ATOM_ENODEV; break;
        case TM_EINVAL: why = ATOM_EINVAL; break;
        case TM_EOVERFLOW: why = ATOM_EOVERFLOW; break;
        default: why = ATOM_EIO; break;
    }
    return enif_make_tuple2(env, ATOM_ERROR, why);
}

static int get_engine(ErlNifEnv* env, ERL_NIF_TERM t, engine_res** out) {
    return enif_get_resource(env, t, ENGINE_RT, (void**)out) && (*out)->e;
}

static ERL_NIF_TERM make_bin(ErlNifEnv* env, const uint8_t* p, size_t n) {
    ERL_NIF_TERM t;
    unsigned char* d = enif_make_new_binary(env, n, &t);
    if (n) memcpy(d, p, n);
    return t;
}

/* new(Device | [Device]) -> {ok, Engine} | {error, Reason}
 * A list makes one engine over those GPUs (tm_create_replicated): one host
 * trie, an HBM replica per device, per-publish matches dealt over them and
 * batch calls spread over them -- a broker node uses every GPU through the
 * same Engine term.  The async pipeline starts here (a dirty scheduler), so
 * match_async/3 on a normal scheduler never pays its setup. */
#define MAX_DEVICES 64
static ERL_NIF_TERM nif_new(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    int32_t devs[MAX_DEVICES];
    unsigned ndev = 0;
    int dev;
    (void)argc;
    if (enif_get_int(env, argv[0], &dev)) {
        devs[0] = dev;
        ndev = dev >= 0 ? 1 : 0;   /* -1: host-only engine (trie ops, no match) */
    } else {
        ERL_NIF_TERM head, tail = argv[0];
        if (!enif_get_list_length(env, tail, &ndev) || ndev == 0 || ndev > MAX_DEVICES) return enif_make_badarg(env);
        for (unsigned i = 0; i < ndev; i++)
            if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_int(env, head, &dev))
                return enif_make_badarg(env);
            else
                devs[i] = dev;
    }
    tm_config cfg = {devs[0], 0, 0, 0};
    tm_engine* e = NULL;
    int rc = tm_create_replicated(&cfg, devs, ndev, &e);
    if (rc) return err(env, rc);
    if (tm_replica_count(e) && (rc = tm_async_start(e))) {   /* (device -1: host-only engine, no pipeline) */
        tm_destroy(e);
        return err(env, rc);
    }
    engine_res* r = enif_alloc_resource(ENGINE_RT, sizeof(engine_res));
    r->e = e;
    ERL_NIF_TERM t = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, ATOM_OK, t);
}

/* insert(Engine, Topic) -> ok  (emqx_trie:insert/1, src/emqx_trie.erl:81-93) */
static ERL_NIF_TERM nif_insert(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b)) return enif_make_badarg(env);
    int rc = tm_trie_insert(r->e, b.data, b.size);
    return rc ? err(env, rc) : ATOM_OK;
}

/* delete(Engine, Topic) -> ok | {error, {node_not_found, Topic}}  (:107-116, :203) */
static ERL_NIF_TERM nif_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b)) return enif_make_badarg(env);
    int rc = tm_trie_delete(r->e, b.data, b.size);
    if (rc == TM_EABORT)
        return enif_make_tuple2(env, ATOM_ERROR, enif_make_tuple2(env, ATOM_NODE_NOT_FOUND, argv[1]));
    return rc ? err(env, rc) : ATOM_OK;
}

/* lookup(Engine, NodeId | root) -> [] | [{trie_node, NodeId, EdgeCount, Topic | undefined, undefined}] */
static ERL_NIF_TERM nif_lookup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    tm_trie_node n;
    int is_root = 0, rc;
    (void)argc;
    if (!get_engine(env, argv[0], &r)) return enif_make_badarg(env);
    if (enif_is_identical(argv[1], ATOM_ROOT)) { is_root = 1; b.data = NULL; b.size = 0; }
    else if (!enif_inspect_binary(env, argv[1], &b)) return enif_make_badarg(env);
    rc = tm_trie_lookup(r->e, b.data, b.size, is_root, &n);
    if (rc < 0) return err(env, rc);
    if (rc == 0) return enif_make_list(env, 0);
    ERL_NIF_TERM topic = ATOM_UNDEFINED;
    if (n.has_topic) {
        uint8_t tmp[TM_MAX_TOPIC_LEN];
        size_t len = 0;
        if (tm_filter_copy(r->e, n.filter_id, tmp, sizeof tmp, &len) == TM_OK && len <= sizeof tmp)
            topic = make_bin(env, tmp, len);
    }
    ERL_NIF_TERM rec = enif_make_tuple5(env, ATOM_TRIE_NODE, argv[1], enif_make_uint(env, n.edge_count), topic,
                                        ATOM_UNDEFINED);
    return enif_make_list1(env, rec);
}

/* empty(Engine) -> boolean()  (:119-121) */
static ERL_NIF_TERM nif_empty(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    (void)argc;
    if (!get_engine(env, argv[0], &r)) return enif_make_badarg(env);
    return tm_trie_empty(r->e) ? ATOM_TRUE : ATOM_FALSE;
}

/* Filter ids -> their bytes, packed under one engine lock (tm_filters_copy):
 * filter k = buf[offs[k], offs[k+1]) for ids[keep[k]]; ids whose filter was
 * deleted and its id reused are skipped.  enif_alloc'ed; packed_free. */
typedef struct {
    uint8_t* buf;
    uint64_t* offs;
    uint32_t* keep;
    uint32_t n;
} packed;

static void packed_free(packed* p) {
    enif_free(p->buf); enif_free(p->offs); enif_free(p->keep);
    p->buf = NULL; p->offs = NULL; p->keep = NULL;
}

/* ids are uint32 (id_bytes 0) or packed id_bytes each (tm_batch_result_packed) */
static int pack_filters_w(tm_engine* e, const void* ids, uint32_t id_bytes, uint64_t n, packed* p) {
    if (n > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    size_t cap = 32 * (size_t)n + 64;
    uint64_t need = 0;
    p->offs = enif_alloc(sizeof(uint64_t) * (n + 1));
    p->keep = enif_alloc(sizeof(uint32_t) * (n ? n : 1));
    p->buf = NULL;
    for (;;) {
        p->buf = enif_alloc(cap);
        if (!p->offs || !p->keep || !p->buf) { packed_free(p); return TM_ENOMEM; }
        int rc = id_bytes
                     ? tm_filters_copy_packed(e, (const uint8_t*)ids, id_bytes, (uint32_t)n, p->buf, cap, p->offs,
                                              p->keep, &p->n, &need)
                     : tm_filters_copy(e, (const uint32_t*)ids, (uint32_t)n, p->buf, cap, p->offs, p->keep, &p->n,
                                       &need);
        if (rc) { packed_free(p); return rc; }
        if (need <= cap) return TM_OK;
        enif_free(p->buf);
        cap = (size_t)need;
    }
}

static int pack_filters(tm_engine* e, const uint32_t* ids, uint64_t n, packed* p) {
    return pack_filters_w(e, ids, 0, n, p);
}

/* The list of the packed filters k with lo <= keep[k] < hi, for *k counting
 * down from the end (rows are built back to front: lists come out in order). */
static ERL_NIF_TERM packed_row(ErlNifEnv* env, const packed* p, uint32_t* k, uint64_t lo) {
    ERL_NIF_TERM list = enif_make_list(env, 0);
    while (*k > 0 && p->keep[*k - 1] >= lo) {
        --*k;
        list = enif_make_list_cell(env, make_bin(env, p->buf + p->offs[*k], p->offs[*k + 1] - p->offs[*k]), list);
    }
    return list;
}

static ERL_NIF_TERM ids_to_filters(ErlNifEnv* env, tm_engine* e, const uint32_t* ids, uint32_t n) {
    packed p;
    int rc = pack_filters(e, ids, n, &p);
    if (rc) return err(env, rc);
    uint32_t k = p.n;
    ERL_NIF_TERM list = packed_row(env, &p, &k, 0);
    packed_free(&p);
    return list;
}

typedef struct {
    ErlNifPid pid;
    ErlNifEnv* env;       /* process-independent: the reply is built here */
    ERL_NIF_TERM ref;     /* the caller's reference, copied into env */
    engine_res* res;      /* kept until the reply is sent */
} match_call;

static void match_done(void* ctx, int rc, const uint32_t* ids, uint32_t n) {
    match_call* c = (match_call*)ctx;
    in_engine_callback = 1;
    ERL_NIF_TERM reply = rc ? err(c->env, rc) : ids_to_filters(c->env, c->res->e, ids, n);
    enif_send(NULL, &c->pid, c->env, enif_make_tuple3(c->env, ATOM_EMQX_TM_MATCH, c->ref, reply));
    enif_free_env(c->env);
    enif_release_resource(c->res);
    enif_free(c);
    in_engine_callback = 0;
}

/* match_async(Engine, Topic, Ref) -> ok | {error, Reason}
 * emqx_trie:match/1 (:96-99) for one publish, answered by the message
 * {emqx_tm_match, Ref, [Filter] | {error, Reason}} (sorted set of filters).
 * Every publishing process can have its match in flight: the engine forms
 * device batches from everything queued (tm_match_async). */
static ERL_NIF_TERM nif_match_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b) || !enif_is_ref(env, argv[2]))
        return enif_make_badarg(env);
    match_call* c = enif_alloc(sizeof(match_call));
    if (!c) return err(env, TM_ENOMEM);
    c->env = enif_alloc_env();
    if (!c->env) { enif_free(c); return err(env, TM_ENOMEM); }
    enif_self(env, &c->pid);
    c->ref = enif_make_copy(c->env, argv[2]);
    c->res = r;
    enif_keep_resource(r);
    int rc = tm_match_async(r->e, b.size ? b.data : (const uint8_t*)"", b.size, match_done, c);
    if (rc) {   /* not queued: no callback will run */
        enif_release_resource(r);
        enif_free_env(c->env);
        enif_free(c);
        return err(env, rc);
    }
    return ATOM_OK;
}

/* Concatenates a list of binaries: buf/offs are enif_alloc'ed (caller frees). */
static int pack_binaries(ErlNifEnv* env, ERL_NIF_TERM list, unsigned* n_out, uint8_t** buf_out, uint64_t** offs_out) {
    unsigned n;
    if (!enif_get_list_length(env, list, &n)) return 0;
    uint64_t* offs = enif_alloc(sizeof(uint64_t) * (n + 1));
    ErlNifBinary* bins = enif_alloc(sizeof(ErlNifBinary) * (n ? n : 1));
    ERL_NIF_TERM head, tail = list;
    uint64_t total = 0;
    offs[0] = 0;
    for (unsigned i = 0; i < n; i++) {
        if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_inspect_binary(env, head, &bins[i])) {
            enif_free(offs); enif_free(bins);
            return 0;
        }
        total += bins[i].size;
        offs[i + 1] = total;
    }
    uint8_t* buf = enif_alloc(total ? total : 1);
    for (unsigned i = 0; i < n; i++) memcpy(buf + offs[i], bins[i].data, bins[i].size);
    enif_free(bins);
    *n_out = n; *buf_out = buf; *offs_out = offs;
    return 1;
}

/* Runs the device pipeline for the packed topics on a batch of this call's
 * own (its pinned result buffers belong to no other caller). */
static int run_batch(tm_engine* e, uint8_t* buf, uint64_t* offs, unsigned n, tm_batch** out) {
    tm_batch* b = NULL;
    int rc = tm_batch_prepare(e, buf, offs, n, &b);
    if (!rc) rc = tm_batch_launch(e, b);
    if (!rc) rc = tm_batch_wait(e, b);
    if (rc && b) { tm_batch_free(e, b); b = NULL; }
    *out = b;
    return rc;
}

/* match_batch(Engine, [Topic]) -> [[Filter]]  (one device pipeline per call) */
static ERL_NIF_TERM nif_match_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned n;
    uint8_t* buf;
    uint64_t* offs;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !pack_binaries(env, argv[1], &n, &buf, &offs)) return enif_make_badarg(env);
    tm_batch* b;
    tm_result_packed res;
    packed p;
    int rc = run_batch(r->e, buf, offs, n, &b);
    enif_free(buf); enif_free(offs);
    /* ids 3 bytes each off the device, read in place by the filter copy */
    if (!rc) rc = tm_batch_result_packed(r->e, b, &res);
    if (!rc) rc = pack_filters_w(r->e, res.ids, res.id_bytes, res.n_matches, &p);
    if (rc) {
        if (b) tm_batch_free(r->e, b);
        return err(env, rc);
    }
    ERL_NIF_TERM out = enif_make_list(env, 0);
    uint32_t k = p.n;
    for (unsigned i = n; i-- > 0;) out = enif_make_list_cell(env, packed_row(env, &p, &k, res.row_offsets[i]), out);
    packed_free(&p);
    tm_batch_free(r->e, b);
    return out;
}

/* route_add(Engine, Topic, DestId) -> ok  (emqx_router:do_add_route/2 after the
 * mnesia transaction committed; DestId = the aggre/1 destination's id: the node,
 * or the share group, src/emqx_broker.erl:250-261) */
static ERL_NIF_TERM nif_route_add(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    unsigned dest;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b) || !enif_get_uint(env, argv[2], &dest))
        return enif_make_badarg(env);
    int rc = tm_route_add(r->e, b.data, b.size, dest);
    return rc ? err(env, rc) : ATOM_OK;
}

/* route_delete(Engine, Topic, DestId) -> ok | {error, not_found}  (do_delete_route/2) */
static ERL_NIF_TERM nif_route_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    unsigned dest;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b) || !enif_get_uint(env, argv[2], &dest))
        return enif_make_badarg(env);
    int rc = tm_route_delete(r->e, b.data, b.size, dest);
    if (rc == TM_ENOENT) return enif_make_tuple2(env, ATOM_ERROR, ATOM_NOT_FOUND);
    return rc ? err(env, rc) : ATOM_OK;
}

/* route_apply(Engine, [{write | delete_object, Topic, DestId}]) -> {ok, NChanged}
 * The cluster route delta feed: emqx_route table events (mnesia replication,
 * cleanup_routes/1 on nodedown, shared-subscription group routes) applied in
 * order in one call; an absent delete_object is a no-op. */
static ERL_NIF_TERM nif_route_apply(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned n;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_get_list_length(env, argv[1], &n)) return enif_make_badarg(env);
    uint64_t* offs = enif_alloc(sizeof(uint64_t) * (n + 1));
    uint32_t* dests = enif_alloc(sizeof(uint32_t) * (n ? n : 1));
    uint8_t* ops = enif_alloc(n ? n : 1);
    ErlNifBinary* bins = enif_alloc(sizeof(ErlNifBinary) * (n ? n : 1));
    ERL_NIF_TERM l = argv[1], h;
    size_t total = 0;
    offs[0] = 0;
    for (unsigned i = 0; i < n; ++i) {
        const ERL_NIF_TERM* el;
        int arity;
        unsigned d;
        if (!enif_get_list_cell(env, l, &h, &l) || !enif_get_tuple(env, h, &arity, &el) || arity != 3 ||
            !enif_inspect_binary(env, el[1], &bins[i]) || !enif_get_uint(env, el[2], &d) ||
            (enif_compare(el[0], ATOM_WRITE) != 0 && enif_compare(el[0], ATOM_DELETE_OBJECT) != 0)) {
            enif_free(offs); enif_free(dests); enif_free(ops); enif_free(bins);
            return enif_make_badarg(env);
        }
        ops[i] = enif_compare(el[0], ATOM_WRITE) == 0 ? TM_ROUTE_WRITE : TM_ROUTE_DELETE;
        dests[i] = d;
        total += bins[i].size;
        offs[i + 1] = total;
    }
    uint8_t* buf = enif_alloc(total ? total : 1);
    for (unsigned i = 0; i < n; ++i) memcpy(buf + offs[i], bins[i].data, bins[i].size);
    uint64_t changed = 0;
    int rc = tm_route_apply(r->e, buf, offs, dests, ops, n, &changed);
    enif_free(buf); enif_free(offs); enif_free(dests); enif_free(ops); enif_free(bins);
    return rc ? err(env, rc) : enif_make_tuple2(env, ATOM_OK, enif_make_uint64(env, changed));
}

/* subscribe(Engine, Topic, SubId, NodeDestId) -> ok
 * emqx_broker:do_subscribe/4, non-shared (src/emqx_broker.erl:150-158): the
 * topic's first local subscriber also adds the (Topic, node()) route. */
static ERL_NIF_TERM nif_subscribe(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    unsigned sub, dest;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b) || !enif_get_uint(env, argv[2], &sub) ||
        !enif_get_uint(env, argv[3], &dest))
        return enif_make_badarg(env);
    int rc = tm_subscribe(r->e, b.data, b.size, sub, dest);
    return rc ? err(env, rc) : ATOM_OK;
}

/* unsubscribe(Engine, Topic, SubId, NodeDestId) -> ok  (do_unsubscribe/4, :179-191;
 * not subscribed -> ok, as unsubscribe/1's `[] -> ok`) */
static ERL_NIF_TERM nif_unsubscribe(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    unsigned sub, dest;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b) || !enif_get_uint(env, argv[2], &sub) ||
        !enif_get_uint(env, argv[3], &dest))
        return enif_make_badarg(env);
    int rc = tm_unsubscribe(r->e, b.data, b.size, sub, dest);
    return (rc && rc != TM_ENOENT) ? err(env, rc) : ATOM_OK;
}

/* subscriber_down(Engine, SubId, NodeDestId) -> {ok, NRemoved}  (subscriber_down/1, :332-347) */
static ERL_NIF_TERM nif_subscriber_down(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned sub, dest;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !enif_get_uint(env, argv[1], &sub) || !enif_get_uint(env, argv[2], &dest))
        return enif_make_badarg(env);
    uint64_t n = 0;
    int rc = tm_subscriber_down(r->e, sub, dest, &n);
    return rc ? err(env, rc) : enif_make_tuple2(env, ATOM_OK, enif_make_uint64(env, n));
}

/* dispatch_batch(Engine, [Topic]) -> [[SubId]]
 * Per publish, the local deliveries dispatch/2 makes (src/emqx_broker.erl:284-309):
 * the subscribers of every matched filter, filters in Erlang binary order, each
 * filter's subscribers in subscription order; [] = {error, no_subscribers}. */
static ERL_NIF_TERM nif_dispatch_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned n;
    uint8_t* buf;
    uint64_t* offs;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !pack_binaries(env, argv[1], &n, &buf, &offs)) return enif_make_badarg(env);
    tm_batch* b;
    tm_deliveries d;
    int rc = run_batch(r->e, buf, offs, n, &b);
    enif_free(buf); enif_free(offs);
    if (!rc) rc = tm_batch_dispatch(r->e, b, 0, &d);
    if (rc) {
        if (b) tm_batch_free(r->e, b);
        return err(env, rc);
    }
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (unsigned i = n; i-- > 0;) {
        ERL_NIF_TERM row = enif_make_list(env, 0);
        for (uint64_t k = d.row_offsets[i + 1]; k-- > d.row_offsets[i];)
            row = enif_make_list_cell(env, enif_make_uint(env, d.subscribers[k]), row);
        out = enif_make_list_cell(env, row, out);
    }
    tm_batch_free(r->e, b);
    return out;
}

/* match_routes_batch(Engine, [Topic]) -> [[{Filter, DestId}]]
 * (aggre(emqx_router:match_routes(T)) per publish, resolved on the device) */
static ERL_NIF_TERM nif_match_routes_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned n;
    uint8_t* buf;
    uint64_t* offs;
    (void)argc;
    if (!get_engine(env, argv[0], &r) || !pack_binaries(env, argv[1], &n, &buf, &offs)) return enif_make_badarg(env);
    tm_batch* b;
    tm_routes res;
    packed p;
    int rc = run_batch(r->e, buf, offs, n, &b);
    enif_free(buf); enif_free(offs);
    if (!rc) rc = tm_batch_routes(r->e, b, &res);
    if (!rc) rc = pack_filters(r->e, res.filter_ids, res.n_routes, &p);
    if (rc) {
        if (b) tm_batch_free(r->e, b);
        return err(env, rc);
    }
    ERL_NIF_TERM out = enif_make_list(env, 0);
    uint32_t k = p.n;
    for (unsigned i = n; i-- > 0;) {
        ERL_NIF_TERM row = enif_make_list(env, 0);
        while (k > 0 && p.keep[k - 1] >= res.row_offsets[i]) {
            --k;
            ERL_NIF_TERM f = make_bin(env, p.buf + p.offs[k], p.offs[k + 1] - p.offs[k]);
            row = enif_make_list_cell(env, enif_make_tuple2(env, f, enif_make_uint(env, res.dests[p.keep[k]])), row);
        }
        out = enif_make_list_cell(env, row, out);
    }
    packed_free(&p);
    tm_batch_free(r->e, b);
    return out;
}

/* rules_match(Engine, [Name], [Rule], DollarRule) -> [[RuleIndex]]
 * emqx_topic:match/2 of every name against every rule on the device (ACL rules
 * with DollarRule = false, rewrite / tracer filters with true); per name the
 * 0-based indices of the matching rules in rule order, so an ACL caller takes
 * the first whose `who` also matches (src/emqx_access_rule.erl:91-99). */
static ERL_NIF_TERM nif_rules_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned n, nr;
    uint8_t *nb, *rb;
    uint64_t *no, *ro;
    (void)argc;
    if (!get_engine(env, argv[0], &r)) return enif_make_badarg(env);
    int dollar = enif_is_identical(argv[3], ATOM_TRUE);
    if (!dollar && !enif_is_identical(argv[3], ATOM_FALSE)) return enif_make_badarg(env);
    if (!pack_binaries(env, argv[1], &n, &nb, &no)) return enif_make_badarg(env);
    if (!pack_binaries(env, argv[2], &nr, &rb, &ro)) { enif_free(nb); enif_free(no); return enif_make_badarg(env); }
    const unsigned wpr = (nr + 31) / 32;
    uint32_t* bits = enif_alloc(sizeof(uint32_t) * ((size_t)n * wpr + 1));
    int rc = tm_rules_match(r->e, nb, no, n, rb, ro, nr, dollar, bits);
    enif_free(nb); enif_free(no); enif_free(rb); enif_free(ro);
    if (rc) { enif_free(bits); return err(env, rc); }
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (unsigned i = n; i-- > 0;) {
        ERL_NIF_TERM row = enif_make_list(env, 0);
        for (unsigned j = nr; j-- > 0;)
            if (bits[(size_t)i * wpr + j / 32] >> (j % 32) & 1u) row = enif_make_list_cell(env, enif_make_uint(env, j), row);
        out = enif_make_list_cell(env, row, out);
    }
    enif_free(bits);
    return out;
}

/* topic_match(Name, Filter) -> boolean()  (emqx_topic:match/2, src/emqx_topic.erl:65-87) */
static ERL_NIF_TERM nif_topic_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    ErlNifBinary a, f;
    (void)argc;
    if (!enif_inspect_binary(env, argv[0], &a) || !enif_inspect_binary(env, argv[1], &f)) return enif_make_badarg(env);
    return tm_topic_match(a.data, a.size, f.data, f.size) ? ATOM_TRUE : ATOM_FALSE;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
    (void)priv; (void)info;
    ENGINE_RT = enif_open_resource_type(env, NULL, "tm_engine", engine_dtor, ERL_NIF_RT_CREATE, NULL);
    if (!ENGINE_RT) return -1;
    reap_stop = 0;
    if (pthread_create(&reap_thread, NULL, reaper, NULL) != 0) return -1;
    reap_running = 1;
    ATOM_OK = enif_make_atom(env, "ok");
    ATOM_ERROR = enif_make_atom(env, "error");
    ATOM_TRUE = enif_make_atom(env, "true");
    ATOM_FALSE = enif_make_atom(env, "false");
    ATOM_UNDEFINED = enif_make_atom(env, "undefined");
    ATOM_ROOT = enif_make_atom(env, "root");
    ATOM_TRIE_NODE = enif_make_atom(env, "trie_node");
    ATOM_NODE_NOT_FOUND = enif_make_atom(env, "node_not_found");
    ATOM_ENOMEM = enif_make_atom(env, "enomem");
    ATOM_EIO = enif_make_atom(env, "eio");
    ATOM_EINVAL = enif_make_atom(env, "einval");
    ATOM_ENODEV = enif_make_atom(env, "enodev");
    ATOM_EOVERFLOW = enif_make_atom(env, "eoverflow");
    ATOM_NOT_FOUND = enif_make_atom(env, "not_found");
    ATOM_WRITE = enif_make_atom(env, "write");
    ATOM_DELETE_OBJECT = enif_make_atom(env, "delete_object");
    ATOM_EMQX_TM_MATCH = enif_make_atom(env, "emqx_tm_match");
    return 0;
}

static ErlNifFunc funcs[] = {
    {"new", 1, nif_new, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"insert", 2, nif_insert, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"delete", 2, nif_delete, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"lookup", 2, nif_lookup, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"empty", 1, nif_empty, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"match_async", 3, nif_match_async, 0},
    {"match_batch", 2, nif_match_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"route_add", 3, nif_route_add, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"route_delete", 3, nif_route_delete, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"route_apply", 2, nif_route_apply, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"subscribe", 4, nif_subscribe, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"unsubscribe", 4, nif_unsubscribe, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"subscriber_down", 3, nif_subscriber_down, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"dispatch_batch", 2, nif_dispatch_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"match_routes_batch", 2, nif_match_routes_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"rules_match", 4, nif_rules_match, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"topic_match", 2, nif_topic_match, 0},
};

/* the reaper destroys what is queued, then exits */
static void unload(ErlNifEnv* env, void* priv) {
    (void)env; (void)priv;
    if (!reap_running) return;
    pthread_mutex_lock(&reap_mu);
    reap_stop = 1;
    pthread_cond_signal(&reap_cv);
    pthread_mutex_unlock(&reap_mu);
    pthread_join(reap_thread, NULL);
    reap_running = 0;
}

ERL_NIF_INIT(emqx_tm, funcs, load, NULL, NULL, unload)
