/*
 * emqx_tm.h -- C ABI of the MI355X topic-matching engine (libemqx_tm.so).
 *
 * Drop-in boundary for EMQ X's publish-time matching path.  The reference is
 * pure Erlang and has no FFI of its own; each entry point below names the
 * reference function it replaces (paths relative to the reference tree).  An
 * erl_nif shim (emqx_amd/csrc/nif/emqx_tm_nif.c) binds these
 * 1:1 to the Erlang module API.
 *
 * Conventions
 *   - plain pointers + sizes; caller-owned inputs are borrowed for the call;
 *   - return codes: 0 = ok, negative errno-style values (TM_E*) on error;
 *     predicates return 0/1; no C++ exceptions cross this boundary;
 *   - one engine = one host trie mirrored into one HBM replica per device it
 *     was created on (tm_create: one device; tm_create_replicated: a list).
 *     Calls on one engine are serialised by an internal mutex (readers and the
 *     single writer of the reference's mnesia tables become ordered operations
 *     on each replica's HIP stream, so a match issued after tm_trie_insert
 *     returns always sees the filter on every device: read-your-writes,
 *     src/emqx_broker.erl:150-158).
 */
#ifndef EMQX_TM_H
#define EMQX_TM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TM_OK          0
#define TM_ENOENT     (-2)
#define TM_EIO        (-5)
#define TM_ENOMEM     (-12)
#define TM_ENODEV     (-19)
#define TM_EINVAL     (-22)
#define TM_EOVERFLOW  (-75)
#define TM_EABORT     (-125)   /* mnesia:abort({node_not_found, _}), src/emqx_trie.erl:203 */

#if defined(__GNUC__)
#define TM_API __attribute__((visibility("default")))
#else
#define TM_API
#endif

#define TM_NONE        0xFFFFFFFFu
#define TM_MAX_TOPIC_LEN 4096  /* ?MAX_TOPIC_LEN, src/emqx_topic.erl:45 */

typedef struct tm_engine tm_engine;
typedef struct tm_batch  tm_batch;

typedef struct {
    int32_t  device;        /* HIP device ordinal; -1 = host-only engine (trie ops, no match) */
    uint32_t init_slots;    /* initial edge-hash capacity in 32-B slots (0 = default) */
    uint32_t host_threads;  /* threads for host tokenise+intern (0 = auto) */
    uint32_t flags;         /* TM_CFG_* bits; unknown bits are rejected */
} tm_config;

/* Filter-sharded mode: the word dictionary is shared by every shard engine and
 * grows only through tm_dict_load (called identically on every shard), so the
 * u32 word ids of a tokenised topic mean the same on every GPU and tokenised
 * publish batches can be exchanged between devices.  tm_trie_insert of a filter
 * with a word outside the dictionary fails with TM_ENOENT. */
#define TM_CFG_FROZEN_DICT 1u
/* Tokenise + intern publish batches on the host (emqx_topic:words/1 on the
 * CPU, then the word ids are copied to HBM) instead of the default device
 * tokeniser, which copies the topic bytes and tokenises them in HBM against
 * the device mirror of the word dictionary.  Results are identical. */
#define TM_CFG_HOST_TOKENIZE 2u

/* #trie_node{} view (include/emqx.hrl:98-103) */
typedef struct {
    uint32_t edge_count;
    uint32_t has_topic;     /* topic =/= undefined */
    uint32_t filter_id;     /* id of `topic` when has_topic, else TM_NONE */
} tm_trie_node;

/* CSR result: row i = sorted (Erlang binary order), deduplicated filter ids
 * matching topic i.  Memory is engine-owned, valid until the next match call on
 * the same engine (or tm_batch_free for batch results). */
typedef struct {
    uint32_t        n_topics;
    uint64_t        n_matches;
    const uint32_t* row_offsets;  /* n_topics + 1 entries */
    const uint32_t* filter_ids;   /* n_matches entries */
} tm_result;

typedef struct {
    uint64_t topics;        /* topics matched */
    uint64_t visits;        /* V: match_node invocations (src/emqx_trie.erl:165-177) */
    uint64_t hash_hits;     /* H: 'match_#' hits (src/emqx_trie.erl:181-186) */
    uint64_t words;         /* sum of topic depths d */
    uint64_t matches;       /* sum |M(t)| */
    uint64_t slow_topics;   /* topics served by the generic (deep/irregular/overflow) kernel */
    uint64_t overflow_tiles;
    float    ms_match;      /* device time of the frontier kernel (last launch) */
    float    ms_total;      /* device time of the whole batch pipeline (last launch) */
    float    ms_tokenize;   /* device tokeniser time of the last launch (0: tokens reused) */
    uint64_t probes;        /* 64-B edge-hash bucket reads of the tile walk (hits + misses) */
    float    ms_csr;        /* device time of the last dense-CSR build (scan + copy; 0: not built) */
    float    ms_queue;      /* device time from the last launch call to its pipeline's start (work queued ahead) */
    uint64_t iterations;    /* frontier iterations of the tile walk (each pops <= 64 probes) */
    uint64_t publishes;     /* publishes of the batch (TM_BATCH_DEDUP: >= topics, the rows) */
    uint64_t delivered;     /* sum over the publishes of their rows' lengths (= matches without dedup) */
    float    ms_dedup;      /* device time of the last device dedup pass (0: none) */
    float    ms_expand;     /* device time of the per-publish row expansion (TM_BATCH_DEDUP) */
} tm_batch_stats;

typedef struct {
    uint64_t version;       /* bumped on every trie mutation */
    uint64_t nodes;         /* live trie nodes incl. root */
    uint64_t edges;         /* live edges (ets:info(emqx_trie, size)) */
    uint64_t filters;       /* nodes with topic =/= undefined */
    uint64_t words;         /* interned words */
    uint64_t slots;         /* edge-hash capacity (32-B slots) */
    uint64_t device_bytes;  /* HBM held by the trie replica */
    uint64_t uploads_full;  /* full trie uploads */
    uint64_t uploads_delta; /* incremental delta uploads */
    uint64_t delta_slots;   /* slots written by delta uploads */
    uint64_t graph_launches;   /* batch launches replayed as a captured HIP graph (repeated or fresh deduplicated batches) */
} tm_engine_stats;

/* ---- engine ---------------------------------------------------------- */
TM_API int  tm_create(const tm_config* cfg, tm_engine** out);
/* One engine over several devices (a node's GPUs): every node of the
 * reference cluster holds the whole emqx_trie (src/emqx_trie.erl:53-74), so
 * the engine keeps ONE host trie and an HBM replica of it on each listed
 * device (a device may be listed twice); cfg->device is ignored.  A mutation
 * is made once and its delta uploaded to every replica, so filter ids are the
 * same everywhere.  Per-publish calls (tm_match_async / tm_match_coalesced)
 * are dealt over the replicas; whole-batch calls (tm_match_batch,
 * tm_match_routes_batch, tm_rules_match) of 65,536+ publishes are split into
 * one contiguous slice per replica and their results concatenated (no
 * collective); a fresh tm_batch goes to the next replica round-robin, or to
 * the one named by tm_batch_prepare_on.  n_devices = 0: host-only engine. */
TM_API int  tm_create_replicated(const tm_config* cfg, const int32_t* devices, uint32_t n_devices,
                                 tm_engine** out);
/* Number of device replicas (0 for a host-only engine). */
TM_API uint32_t tm_replica_count(tm_engine* e);
/* Starts the async pipeline (tm_match_async) of every replica now instead of
 * at the first call -- a NIF calls it from new/1, which runs on a dirty
 * scheduler, so the first match_async/3 never pays thread and stream setup. */
TM_API int  tm_async_start(tm_engine* e);
TM_API void tm_destroy(tm_engine* e);
TM_API uint64_t tm_version(tm_engine* e);
TM_API int  tm_stats(tm_engine* e, tm_engine_stats* out);
/* Applies pending trie deltas to the device replica (also done implicitly by
 * every match call). */
TM_API int  tm_sync(tm_engine* e);
/* tm_sync without the wait: the pending deltas are gathered now and their
 * upload is queued on every replica's stream, behind the work already there
 * (a walk in flight keeps its snapshot) and ahead of the next launch. */
TM_API int  tm_sync_async(tm_engine* e);

/* ---- emqx_trie (src/emqx_trie.erl) ----------------------------------- */
/* emqx_trie:insert/1 (:81-93): idempotent; add_path/1 (:145-158) semantics. */
TM_API int  tm_trie_insert(tm_engine* e, const uint8_t* topic, size_t len);
/* emqx_trie:delete/1 (:107-116) + delete_path/1 (:190-204). */
TM_API int  tm_trie_delete(tm_engine* e, const uint8_t* topic, size_t len);
/* emqx_trie:lookup/1 (:102-104): returns 1 found, 0 not found.  is_root
 * selects the atom `root` node id. */
TM_API int  tm_trie_lookup(tm_engine* e, const uint8_t* node_id, size_t len, int is_root,
                    tm_trie_node* out);
/* emqx_trie:empty/0 (:119-121): 1 if the edge table is empty. */
TM_API int  tm_trie_empty(tm_engine* e);
/* emqx_trie:match/1 (:96-99) for one topic: writes up to cap ids (sorted by
 * filter bytes), *n_out = full count.  Runs on the device. */
TM_API int  tm_trie_match(tm_engine* e, const uint8_t* topic, size_t len,
                   uint32_t* ids, uint32_t cap, uint32_t* n_out);

/* emqx_trie:match/1 for one topic, blocking, for callers on many threads:
 * tm_match_async below plus a futex wait for the caller's own row, so
 * concurrent callers share device batches formed by the engine's launcher
 * (see tm_match_async / tm_coalesce_config for the batching policy and
 * INTEGRATION.md for how it relates to emqx_batch, src/emqx_batch.erl:56-82).
 * Results and errors as tm_trie_match, per caller (len > TM_MAX_TOPIC_LEN ->
 * TM_EINVAL). */
TM_API int  tm_match_coalesced(tm_engine* e, const uint8_t* topic, size_t len,
                               uint32_t* ids, uint32_t cap, uint32_t* n_out);
/* Sets max_batch (0 = keep; default 16384) and linger_us (TM_NONE = keep;
 * default 0: a batch is whatever queued while the pipeline was busy) of the
 * async pipeline below, which tm_match_coalesced rides on; *batches /
 * *requests (may be NULL) = device batches run and requests served so far. */
TM_API int  tm_coalesce_config(tm_engine* e, uint32_t max_batch, uint32_t linger_us,
                               uint64_t* batches, uint64_t* requests);

/* Asynchronous emqx_trie:match/1 for one topic -- the form the NIF uses:
 * the caller (an Erlang process) returns at once and receives its row later
 * (enif_send), so every publishing process can have a match in flight, as
 * every publisher runs match_routes/1 concurrently in the reference
 * (src/emqx_broker.erl:201-210).  Calls are queued; an engine thread forms
 * device batches from the queue (emqx_batch's size + linger policy,
 * src/emqx_batch.erl:49-90) and keeps up to `depth` of them in flight, each on
 * a HIP stream of its own: H2D of the topics, device tokeniser, trie walk,
 * read-back of the rows.  cb(ctx, rc, ids, n) runs once per call on the
 * engine's completion thread: rc 0 and the topic's sorted filter ids
 * (engine memory, valid during the callback only), or a TM_E* code with no
 * ids.  A match submitted after tm_trie_insert returned sees the filter.
 * Returns TM_EINVAL (no callback) for len > TM_MAX_TOPIC_LEN; callbacks must
 * not destroy the engine. */
typedef void (*tm_match_cb)(void* ctx, int rc, const uint32_t* ids, uint32_t n);
TM_API int  tm_match_async(tm_engine* e, const uint8_t* topic, size_t len, tm_match_cb cb, void* ctx);
typedef struct {
    uint64_t batches;       /* device batches completed */
    uint64_t requests;      /* calls completed */
    uint64_t recoveries;    /* batches re-run through the CSR path (capacity misses) */
    uint64_t max_batch;     /* largest batch formed */
    uint32_t depth;         /* batches in flight at most (TM_ASYNC_DEPTH, default 4) */
    uint32_t queued;        /* calls waiting for a batch now */
    double   us_launch;     /* host time forming + enqueueing batches (launcher thread) */
    double   us_wait;       /* completer time blocked on device batches */
    double   us_deliver;    /* completer time running callbacks */
    uint64_t inline_launches; /* batches a submitting caller launched itself (pipeline idle) */
} tm_async_stats;
TM_API int  tm_async_stats_get(tm_engine* e, tm_async_stats* out);

/* ---- batched publish matching: emqx_router:match_routes/1 hot path ---- */
/* (src/emqx_router.erl:127-141 applied to a batch of publishes,
 *  src/emqx_broker.erl:201-210).  topics = concatenated topic bytes,
 *  offsets[n+1] byte offsets.  Result as tm_result above. */
TM_API int  tm_match_batch(tm_engine* e, const uint8_t* topics, const uint64_t* offsets,
                    uint32_t n, tm_result* out);

/* tm_match_batch for consumers that read the ids in place (the NIF turning
 * them into filter binaries through tm_filters_copy_packed): filter id j of
 * the result is ids[j * id_bytes ..] little-endian, id_bytes = 3 while every
 * node id of the engine fits 24 bits (~16.7M trie nodes), else 4.  The ids
 * cross PCIe packed -- 3/4 of the bytes -- and nobody unpacks them.  Rows
 * (row_offsets, u32) as in tm_result; the buffers live until the next call. */
typedef struct {
    uint32_t        n_topics;
    uint32_t        id_bytes;
    uint64_t        n_matches;
    const uint32_t* row_offsets;
    const uint8_t*  ids;
} tm_result_packed;
TM_API int  tm_match_batch_packed(tm_engine* e, const uint8_t* topics, const uint64_t* offsets,
                    uint32_t n, tm_result_packed* out);

/* Split form for pipelining / device-resident benchmarking:
 * prepare = H2D of the topic bytes and offsets (default), or host tokenise +
 *           intern + H2D of the word ids with TM_CFG_HOST_TOKENIZE
 *           (emqx_topic:words/1, src/emqx_topic.erl:158-164);
 * launch  = enqueue the device pipeline (async): with device tokenisation the
 *           first launch tokenises the bytes in HBM against the dictionary
 *           mirror, after the pending deltas; later launches reuse the tokens
 *           unless the dictionary grew in between;
 * wait    = block until done; result = D2H of the CSR.
 * *out must be NULL (a new batch) or a batch of this engine, which is then
 * re-prepared in place: its device and pinned buffers are reused and only
 * grow, so a caller cycling a few batches allocates nothing in steady state. */
TM_API int  tm_batch_prepare(tm_engine* e, const uint8_t* topics, const uint64_t* offsets,
                      uint32_t n, tm_batch** out);
/* tm_batch_prepare with flags.  TM_BATCH_DEDUP: identical topics of the batch
 * are matched once (hot-topic skew, BASELINE config C5); the result then has
 * one row per DISTINCT topic (tm_result.n_topics = distinct count, rows in
 * first-occurrence order) and tm_batch_row_map gives the row of every
 * publish.  With the device tokeniser (the default) the dedup runs on the
 * device at launch, behind the tokeniser, on every fresh pass over the batch
 * (prepare / tm_batch_retokenize): the row count and row_of exist once the
 * batch has been waited, and tm_batch_publish_rows gives every publish its
 * row in HBM. */
#define TM_BATCH_DEDUP 1u
/* TM_BATCH_STREAM: the batch runs on a HIP stream of its own, so launches of
 * different batches overlap on the device (one batch's CSR pass with the
 * next batch's walk); trie updates still reach a launch that follows them
 * (read-your-writes) and wait for the batch's walk before changing the
 * tables.  Every call on the batch stays synchronous for the caller. */
#define TM_BATCH_STREAM 2u
TM_API int  tm_batch_prepare_ex(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                                uint32_t flags, tm_batch** out);
/* tm_batch_prepare_ex on replica `replica` (< tm_replica_count) of the engine.
 * A batch stays on the replica it was created on (re-preparing it on another
 * is TM_EINVAL); tm_batch_replica names it. */
TM_API int  tm_batch_prepare_on(tm_engine* e, uint32_t replica, const uint8_t* topics, const uint64_t* offsets,
                                uint32_t n, uint32_t flags, tm_batch** out);
TM_API uint32_t tm_batch_replica(tm_engine* e, tm_batch* b);
/* row_of[i] = result row of publish i (identity for batches without
 * TM_BATCH_DEDUP); *n_rows = number of result rows.  Engine-owned memory,
 * valid until the batch is re-prepared or freed. */
TM_API int  tm_batch_row_map(tm_engine* e, tm_batch* b, const uint32_t** row_of, uint32_t* n_rows);
TM_API int  tm_batch_launch(tm_engine* e, tm_batch* b);
TM_API int  tm_batch_wait(tm_engine* e, tm_batch* b);
TM_API int  tm_batch_result(tm_engine* e, tm_batch* b, tm_result* out);
/* tm_batch_result with the ids packed on the device as in tm_match_batch_packed
 * (3 bytes while node ids fit 24 bits, else 4), into the batch's own pinned
 * buffers: valid until the batch is re-prepared or freed, so concurrent
 * callers on their own batches (the NIF's match_batch) do not share them. */
TM_API int  tm_batch_result_packed(tm_engine* e, tm_batch* b, tm_result_packed* out);
/* Rows rows[0..k) of a waited batch (each < the batch's row count) as a host
 * CSR: n_topics = k, row i = filter_ids[row_offsets[i] .. row_offsets[i+1]),
 * sorted and deduplicated like tm_batch_result's.  Gathered on the device from
 * where the walk wrote them -- no dense CSR, no whole-batch copy: a self-check
 * of a 10M-publish batch reads ~3,000 rows this way.  Batch-owned memory,
 * valid until the next tm_batch_sample, re-prepare or free of the batch.
 * Replaces nothing in the reference (a diagnostic of the device result). */
TM_API int  tm_batch_sample(tm_engine* e, tm_batch* b, const uint32_t* rows, uint32_t k, tm_result* out);
TM_API int  tm_batch_stats_get(tm_engine* e, tm_batch* b, tm_batch_stats* out);
/* A waited batch's result is the rows as the walk wrote them to HBM: row i
 * (one per topic, or per distinct topic with TM_BATCH_DEDUP) is
 * d_ids[d_start[i] .. d_start[i] + d_count[i]), sorted (Erlang binary order)
 * and deduplicated; rows of different topics are not adjacent.  Device
 * pointers of the batch, valid until its next launch or re-prepare; no copy,
 * no extra pass.  *n_matches = sum of the counts. */
TM_API int  tm_batch_rows(tm_engine* e, tm_batch* b, const uint32_t** d_count, const uint64_t** d_start,
                          const uint32_t** d_ids, uint64_t* n_matches);
/* The result per PUBLISH of a waited batch, on the device: publish i's
 * sorted, deduplicated filter ids are d_ids[d_start[i] .. d_start[i] +
 * d_count[i]).  For a TM_BATCH_DEDUP batch deduplicated on the device this is
 * every publish's row (expanded behind the walk: publishes of one topic share
 * the ids), and *n_delivered = the sum of the counts -- the (publish, filter)
 * matches delivered (emqx_broker:publish/1 matches every message,
 * src/emqx_broker.erl:201-210); without TM_BATCH_DEDUP it is tm_batch_rows.
 * TM_EINVAL for a batch deduplicated on the host. */
TM_API int  tm_batch_publish_rows(tm_engine* e, tm_batch* b, const uint32_t** d_count, const uint64_t** d_start,
                                  const uint32_t** d_ids, uint64_t* n_delivered);
/* Device pointers of the batch's dense CSR: row_offsets[n + 1], ids[total]
 * in topic order.  Built from the rows on first request after a launch
 * (scan + one copy, on the batch's stream; tm_batch_result, routes, dispatch
 * and export build it too); valid until the next launch. */
TM_API int  tm_batch_device_csr(tm_engine* e, tm_batch* b, const uint32_t** d_row_offsets,
                         const uint32_t** d_ids, uint64_t* n_matches);
TM_API void tm_batch_free(tm_engine* e, tm_batch* b);
/* Drops the tokens of a device-tokenised batch: its next launch tokenises the
 * resident bytes again -- a never-seen batch's full device pipeline without a
 * new H2D (bench: pipeline_fresh_ms).  TM_EINVAL for host-tokenised batches. */
TM_API int  tm_batch_retokenize(tm_engine* e, tm_batch* b);

/* ---- routes: emqx_router + emqx_broker:aggre/1 on the device ----------- */
/* One route of `topic` to an aggregated destination id chosen by the caller
 * (emqx_broker:aggre/1, src/emqx_broker.erl:250-261: a node() dest aggregates
 * to the node, a shared-subscription dest {Group, Node} to the Group, so the
 * routes {G, n1} and {G, n2} share one id).  emqx_router:do_add_route/2
 * (src/emqx_router.erl:113-124, 229-234): the first route of a topic puts it
 * into the trie (exact topics too, so one walk returns exact + wildcard
 * matches); a repeated (topic, dest) only counts. */
TM_API int  tm_route_add(tm_engine* e, const uint8_t* topic, size_t len, uint32_t dest);
/* do_delete_route/2 (:163-169, 239-247): TM_ENOENT if (topic, dest) has no
 * route; removing the last route of a topic deletes it from the trie. */
TM_API int  tm_route_delete(tm_engine* e, const uint8_t* topic, size_t len, uint32_t dest);

/* Cluster route delta feed: n route-table events applied
 * in order under one engine lock.  The emqx_route bag and the trie tables are
 * mnesia ram_copies replicated to every node (src/emqx_router.erl:77-86,
 * src/emqx_trie.erl:53-74), so a node sees remote route writes as table
 * events ({write, #route{}} / {delete_object, #route{}}); the feed also carries
 * the deletes of cleanup_routes(Node) on nodedown
 * (src/emqx_router_helper.erl:135-141, 173-177) and the
 * {Group, node()} routes of shared subscriptions (src/emqx_shared_sub.erl:
 * 297-313).  ops[i] = TM_ROUTE_WRITE -> tm_route_add(topic i, dests[i]);
 * TM_ROUTE_DELETE -> tm_route_delete, where a missing (topic, dest) is a no-op
 * (mnesia:delete_object of an absent record).  *n_changed (may be NULL) counts
 * the events that changed the table.  Stops at the first other error. */
#define TM_ROUTE_DELETE 0u
#define TM_ROUTE_WRITE  1u
TM_API int  tm_route_apply(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, const uint32_t* dests,
                           const uint8_t* ops, uint32_t n, uint64_t* n_changed);

/* aggre(match_routes(T)) per topic: row i lists (filter id, dest) pairs,
 * filters in Erlang binary order, each filter's dests in first-added order,
 * no (filter, dest) twice.  Engine-owned memory, valid like tm_result. */
typedef struct {
    uint32_t        n_topics;
    uint64_t        n_routes;
    const uint32_t* row_offsets;  /* n_topics + 1 */
    const uint32_t* filter_ids;   /* n_routes */
    const uint32_t* dests;        /* n_routes */
} tm_routes;

/* Device route resolution of a waited batch (its match CSR stays in HBM). */
TM_API int  tm_batch_routes(tm_engine* e, tm_batch* b, tm_routes* out);
/* tm_match_batch + tm_batch_routes in one call (emqx_router:match_routes/1 +
 * emqx_broker:aggre/1 over a batch of publishes). */
TM_API int  tm_match_routes_batch(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                                  tm_routes* out);

/* ---- subscribers + fan-out: emqx_broker dispatch on the device --------- */
/* The local node's subscriber bag (?SUBSCRIBER / ?SUBSCRIPTION,
 * src/emqx_broker.erl:145-196), non-shared subscriptions; subscriber ids are
 * the caller's (one per subscriber pid).  node_dest = the aggregated dest id
 * the caller uses for node() in tm_route_add.
 * tm_subscribe: do_subscribe/4 (:150-158); idempotent per (topic, subscriber)
 * (:127-139); the topic's first subscriber adds route (topic, node_dest)
 * (handle_call({subscribe, Topic}), :438-440 -> emqx_router:do_add_route/1).
 * Topics with > 1024 subscribers are sharded into {shard, Topic, I} keys by the
 * reference (src/emqx_broker_helper.erl:82-87): a storage split of the same
 * set, so a topic keeps one run here, in subscription order. */
TM_API int  tm_subscribe(tm_engine* e, const uint8_t* topic, size_t len, uint32_t subscriber, uint32_t node_dest);
/* do_unsubscribe/4 (:179-191): TM_ENOENT if not subscribed (unsubscribe/1's
 * `[] -> ok`, :170-177); the last subscriber of a topic deletes its route
 * (handle_cast({unsubscribed, Topic}), :463-469). */
TM_API int  tm_unsubscribe(tm_engine* e, const uint8_t* topic, size_t len, uint32_t subscriber, uint32_t node_dest);
/* subscriber_down/1 (:332-347): drops every subscription of the subscriber;
 * *n_removed (may be NULL) = how many. */
TM_API int  tm_subscriber_down(tm_engine* e, uint32_t subscriber, uint32_t node_dest, uint64_t* n_removed);

/* Deliveries of a waited batch: dispatch(To, Delivery) (:284-309) for every
 * filter To matched by publish i (its local route, do_route/2 :243-244):
 * deliveries of row i = subscribers[row_offsets[i] .. row_offsets[i+1]), the
 * runs of its matched filters in match (Erlang binary) order, each run in
 * subscription order; row_offsets[i+1] - row_offsets[i] = DispN (0 =
 * {error, no_subscribers}).  match_offsets[j] (TM_DISPATCH_MATCH_OFFSETS) =
 * first delivery of match entry j, i.e. of filter ids[j] of tm_batch_result.
 * TM_DISPATCH_COUNT_ONLY: counts only, subscribers = NULL.
 * TM_DISPATCH_DEVICE: no copy back; the pointers are device memory of the
 * batch, valid until its next dispatch or re-prepare (match_offsets only with
 * TM_DISPATCH_MATCH_OFFSETS too: without it the engine skips making them
 * global).  Otherwise engine-owned
 * pinned memory valid likewise.  fill_ms = device time of the copy kernel.
 * TM_DISPATCH_ROWS (device only, implies TM_DISPATCH_DEVICE, excludes
 * MATCH_OFFSETS): the fan-out reads the walk's rows where it wrote them
 * (tm_batch_rows) instead of a dense CSR built first; the deliveries of row i
 * are then subscribers[row_offsets[i] .. row_offsets[i] + row_counts[i]) --
 * the same runs in the same order, rows no longer adjacent in publish order
 * (row_offsets has n_topics entries). */
typedef struct {
    uint32_t        n_topics;
    uint64_t        n_matches;
    uint64_t        n_deliveries;
    const uint64_t* row_offsets;    /* n_topics + 1 (TM_DISPATCH_ROWS: n_topics row starts) */
    const uint64_t* match_offsets;  /* n_matches + 1, or NULL */
    const uint32_t* subscribers;    /* n_deliveries, or NULL */
    float           fill_ms;
    const uint32_t* row_counts;     /* TM_DISPATCH_ROWS: deliveries of each row; otherwise NULL */
} tm_deliveries;
#define TM_DISPATCH_COUNT_ONLY    1u
#define TM_DISPATCH_MATCH_OFFSETS 2u
#define TM_DISPATCH_DEVICE        4u
#define TM_DISPATCH_ROWS          8u
TM_API int  tm_batch_dispatch(tm_engine* e, tm_batch* b, uint32_t flags, tm_deliveries* out);

/* ---- bulk load + filter-sharded mode ------------------ */
/* emqx_trie:insert/1 over n filters (filters = concatenated bytes, offsets[n+1]).
 * nshards <= 1: every filter.  Otherwise only the filters whose
 * tm_filter_shard() is `shard` or nshards (replicated); *n_inserted (may be
 * NULL) counts them.  Stops at the first error.  A batch of >= 2,048
 * filters on a big trie is applied by parallel workers: after an error the
 * filters applied are each worker's finished ones (every filter is applied
 * whole or not at all, the trie stays consistent), so a subset of the batch
 * that need not be a prefix; *n_inserted counts them and re-applying the
 * batch is idempotent (emqx_trie:insert/1 is). */
TM_API int  tm_trie_insert_many(tm_engine* e, const uint8_t* filters, const uint64_t* offsets,
                                uint32_t n, uint32_t shard, uint32_t nshards, uint64_t* n_inserted);
/* emqx_trie:delete/1 over n filters; *n_deleted (may be NULL) counts the calls
 * made.  Stops at the first error (subset semantics of a parallel batch as
 * for tm_trie_insert_many). */
TM_API int  tm_trie_delete_many(tm_engine* e, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                                uint64_t* n_deleted);
/* One subscription delta: tm_trie_delete_many(del...) then
 * tm_trie_insert_many(ins..., 0, 1), with the two lists planned together (one
 * pass of the workers over both; an insert whose planned node a delete of the
 * same call removed walks again).  The result equals the two calls in that
 * order, filter for filter: emqx_trie:delete/1 then insert/1
 * (src/emqx_trie.erl:81-116) as a session's unsubscribe + subscribe batch
 * reaches the router (src/emqx_router.erl:113-124, 163-169).  A delete error
 * returns before any insert; *n_deleted / *n_inserted (may be NULL) count as
 * the two calls do. */
TM_API int  tm_trie_apply_many(tm_engine* e, const uint8_t* del_filters, const uint64_t* del_offsets, uint32_t n_del,
                               const uint8_t* ins_filters, const uint64_t* ins_offsets, uint32_t n_ins,
                               uint64_t* n_deleted, uint64_t* n_inserted);
/* Interns n words in order (the shared dictionary of the sharded mode).  Words
 * must not contain '/'; '', "+" and "#" have fixed ids and are skipped. */
TM_API int  tm_dict_load(tm_engine* e, const uint8_t* words, const uint64_t* offsets, uint32_t n);
/* Shard of a filter among nshards: filters of >= 2 levels whose first two
 * levels are literal words live on shard hash(id(w0), id(w1)) mod nshards; all
 * others return nshards (replicated on every shard).  A publish whose first two
 * words are known literals can only be matched by filters of its own shard or
 * replicated ones, so one shard resolves it completely. */
TM_API int  tm_filter_shard(tm_engine* e, const uint8_t* filter, size_t len, uint32_t nshards);
/* Host tokenisation (emqx_topic:words/1 + interning): words[] = (class << 29 |
 * word id) per level, toff[n+1] word offsets, tflags[n] (bit 0: '$' topic, bit
 * 1: generic path).  *nwords_out = total words; TM_EOVERFLOW if > words_cap. */
TM_API int  tm_tokenize(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                        uint32_t* words, uint64_t words_cap, uint32_t* toff, uint8_t* tflags,
                        uint64_t* nwords_out);
/* tm_tokenize on the device (the tokeniser tm_match_batch uses by default):
 * the host topic bytes are copied to HBM and tokenised against the device
 * mirror of the word dictionary into caller DEVICE buffers words[words_cap],
 * toff[n+1], tflags[n] -- the same values tm_tokenize writes.  *nwords_out =
 * total words; TM_EOVERFLOW (nothing past words_cap written) if > words_cap.
 * Returns when done.  Replaces emqx_topic:words/1 (src/emqx_topic.erl:150-164)
 * for a whole batch. */
TM_API int  tm_tokenize_device(tm_engine* e, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                               uint32_t* d_words, uint64_t words_cap, uint32_t* d_toff, uint8_t* d_tflags,
                               uint64_t* nwords_out);
/* A batch from tokenised arrays (tm_tokenize layout).  on_device = 1: the
 * pointers are device memory of this engine's GPU (e.g. received from another
 * shard); they are copied (and validated on the device: TM_EINVAL for offsets
 * that are not monotone from 0 to nwords or unflagged deep topics), so the
 * caller may reuse them once this returns.  A non-NULL *out is re-prepared in
 * place (its buffers only grow); NULL allocates a new batch. */
TM_API int  tm_batch_prepare_tokens(tm_engine* e, const uint32_t* words, const uint32_t* toff,
                                    const uint8_t* tflags, uint32_t n, uint64_t nwords, int on_device,
                                    tm_batch** out);
/* Device kernel: shard[t] = the shard owning tokenised topic t (tm_filter_shard's
 * rule applied to its first two words), or nshards when any shard resolves it
 * (only replicated filters can match).  Device pointers; returns when done. */
TM_API int  tm_tokens_shard(tm_engine* e, const uint32_t* d_words, const uint32_t* d_toff, uint32_t n,
                            uint32_t nshards, uint32_t* d_shard);
/* Writes the batch's per-topic match counts and its filter ids mapped to
 * id * mul + add (global ids of a shard) into caller device buffers
 * (counts[n], ids[n_matches]) on the engine stream; returns when done. */
TM_API int  tm_batch_export(tm_engine* e, tm_batch* b, uint32_t* d_counts, uint32_t* d_ids,
                            uint32_t mul, uint32_t add);

/* Device row gather (the exchange's reorder step): for i < n, copies the u32
 * row src[src_off[idx[i]] .. src_off[idx[i] + 1]) to dst[dst_off[i] ..).  All
 * pointers are device memory; offsets and indices are int64.  Returns when done. */
TM_API int  tm_gather_rows(tm_engine* e, const uint32_t* d_src, const int64_t* d_src_off, const int64_t* d_idx,
                           uint32_t n, const int64_t* d_dst_off, uint32_t* d_dst);

/* ---- filters ---------------------------------------------------------- */
/* Bytes of a filter id returned by a match (the #trie_node.topic binary).
 * A matched id keeps naming its filter while the result that holds it is
 * valid, even if the filter is deleted meanwhile: ids freed by deletes are
 * reused only after every batch launched before the delete has been
 * re-launched or freed.  The pointer is into engine memory that a later
 * insert may move: callers racing with writers use tm_filter_copy. */
TM_API const uint8_t* tm_filter_bytes(tm_engine* e, uint32_t id, size_t* len);
/* Copies the bytes of filter `id` into buf[cap] under the engine lock; *len =
 * its length (copied only if <= cap).  TM_ENOENT if the id never named a
 * filter or was reused for a node without one. */
TM_API int  tm_filter_copy(tm_engine* e, uint32_t id, uint8_t* buf, size_t cap, size_t* len);
/* Bulk tm_filter_copy under one acquisition of the engine lock (a result row
 * turned into filter binaries).  *need = the bytes of every id still naming a
 * filter; if *need > cap nothing is copied (grow buf and call again).
 * Otherwise the live filters are packed into buf in id order: filter k is
 * buf[offs[k], offs[k+1]), *n_out = count (offs holds n+1 entries); ids no
 * longer naming a filter are skipped, and keep[k] (may be NULL) = the index
 * in ids of filter k. */
TM_API int  tm_filters_copy(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, size_t cap,
                            uint64_t* offs, uint32_t* keep, uint32_t* n_out, uint64_t* need);
/* tm_filters_copy over ids packed id_bytes (3 or 4) bytes each, as
 * tm_match_batch_packed returns them (no unpack pass). */
TM_API int  tm_filters_copy_packed(tm_engine* e, const uint8_t* ids, uint32_t id_bytes, uint32_t n, uint8_t* buf,
                            size_t cap, uint64_t* offs, uint32_t* keep, uint32_t* n_out, uint64_t* need);
/* Id of an inserted filter, TM_ENOENT if absent. */
TM_API int  tm_filter_id(tm_engine* e, const uint8_t* filter, size_t len, uint32_t* id);

/* ---- emqx_topic (src/emqx_topic.erl), host predicates ----------------- */
/* emqx_topic:match/2 (:65-87) on binaries: 1 match, 0 no match. */
TM_API int  tm_topic_match(const uint8_t* name, size_t name_len, const uint8_t* filter, size_t filter_len);
/* emqx_topic:wildcard/1 (:52-62). */
TM_API int  tm_topic_wildcard(const uint8_t* topic, size_t len);
/* emqx_topic:validate/2 (:96-127): 0 ok, TM_EINVAL otherwise; *reason set to
 * one of "empty_topic", "topic_too_long", "topic_invalid_#",
 * "topic_invalid_char", "topic_name_error". */
TM_API int  tm_topic_validate(int is_name, const uint8_t* topic, size_t len, const char** reason);

/* Batched predicate on the device: emqx_topic:match(Name_i, Rule_j) for n
 * names x r rule filters -- the pairwise callers that do not use the trie:
 * ACL rules (src/emqx_access_rule.erl:124-139, word-list form: dollar_rule = 0),
 * rewrite rules (src/emqx_mod_rewrite.erl:86-90) and topic tracers
 * (src/emqx_tracer.erl:142-151), both binary form: dollar_rule = 1 (a name
 * starting with '$' never matches a filter starting with '+' or '#',
 * src/emqx_topic.erl:68-71).  bits (host memory, n * ceil(r/32) u32): bit j%32
 * of word i*ceil(r/32) + j/32 = match(name i, rule j). */
TM_API int  tm_rules_match(tm_engine* e, const uint8_t* names, const uint64_t* name_offsets, uint32_t n,
                           const uint8_t* rules, const uint64_t* rule_offsets, uint32_t r, int dollar_rule,
                           uint32_t* bits);

/* ---- replicated multi-device group (BASELINE config C3) --------------- */
/* A view of one tm_create_replicated engine (tm_group_engine(g, i) returns it
 * for every i < tm_group_size): one host trie, one HBM replica per listed
 * device (a device may be listed twice: two replicas on one GPU), so node /
 * filter ids are identical everywhere (the reference replicates emqx_trie to
 * every node, src/emqx_trie.erl:53-74).  The split form keeps one slice per
 * replica explicit: a publish batch is split into contiguous slices matched
 * concurrently with no collective, and the slices' CSRs concatenate into the
 * batch's CSR. */
typedef struct tm_group tm_group;
typedef struct tm_group_batch tm_group_batch;
TM_API int  tm_group_create(const int32_t* devices, uint32_t n_devices, const tm_config* cfg, tm_group** out);
TM_API void tm_group_destroy(tm_group* g);
TM_API uint32_t tm_group_size(tm_group* g);
/* Replica i (read-only use: stats, filter bytes; mutate only through tm_group_*). */
TM_API tm_engine* tm_group_engine(tm_group* g, uint32_t i);
TM_API int  tm_group_trie_insert(tm_group* g, const uint8_t* topic, size_t len);
TM_API int  tm_group_trie_delete(tm_group* g, const uint8_t* topic, size_t len);
TM_API int  tm_group_insert_many(tm_group* g, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                                 uint64_t* n_inserted);
TM_API int  tm_group_route_apply(tm_group* g, const uint8_t* topics, const uint64_t* offsets, const uint32_t* dests,
                                 const uint8_t* ops, uint32_t n, uint64_t* n_changed);
TM_API int  tm_group_sync(tm_group* g);
/* Split form: prepare slices (H2D on every device), launch all (async), wait
 * all, merged CSR (group-owned pinned memory, valid until the batch is
 * re-prepared or freed).  A non-NULL *out is re-prepared in place. */
TM_API int  tm_group_prepare(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                             tm_group_batch** out);
TM_API int  tm_group_launch(tm_group* g, tm_group_batch* b);
TM_API int  tm_group_wait(tm_group* g, tm_group_batch* b);
TM_API int  tm_group_result(tm_group* g, tm_group_batch* b, tm_result* out);
/* tm_batch_sample over a group batch: publishes[0..k) (indices into the whole
 * batch, any order) -> their rows as a host CSR in that order, each gathered
 * on the device of the slice that holds it (group-owned memory, valid until
 * the next tm_group_sample or free of the batch). */
TM_API int  tm_group_sample(tm_group* g, tm_group_batch* b, const uint32_t* publishes, uint32_t k, tm_result* out);
/* Counters summed over the slices; ms_match / ms_total = the slowest slice. */
TM_API int  tm_group_batch_stats(tm_group* g, tm_group_batch* b, tm_batch_stats* out);
TM_API void tm_group_batch_free(tm_group* g, tm_group_batch* b);
/* prepare + launch + wait + result in one call. */
TM_API int  tm_group_match_batch(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                                 tm_result* out);
/* Deliveries of a waited group batch (tm_batch_dispatch per slice, merged in
 * publish order into group-owned memory valid like tm_group_result's). */
TM_API int  tm_group_dispatch(tm_group* g, tm_group_batch* b, tm_deliveries* out);
/* The per-publish and whole-batch calls of the group's engine (each spans the
 * replicas, see tm_create_replicated): tm_match_async, tm_match_coalesced,
 * tm_match_routes_batch, tm_rules_match. */
TM_API int  tm_group_match_async(tm_group* g, const uint8_t* topic, size_t len, tm_match_cb cb, void* ctx);
TM_API int  tm_group_match_coalesced(tm_group* g, const uint8_t* topic, size_t len, uint32_t* ids, uint32_t cap,
                                     uint32_t* n_out);
TM_API int  tm_group_match_routes_batch(tm_group* g, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                                        tm_routes* out);
TM_API int  tm_group_rules_match(tm_group* g, const uint8_t* names, const uint64_t* name_offsets, uint32_t n,
                                 const uint8_t* rules, const uint64_t* rule_offsets, uint32_t r, int dollar_rule,
                                 uint32_t* bits);

/* ---- filter-sharded group in one process (BASELINE config C4) -------- */
/* Subscription sets too large to replicate, partitioned over G shard engines
 * (one per listed device; a device may repeat), no collective: a filter whose
 * first two levels are literal lives on shard tm_filter_shard(); all others
 * are replicated on every shard.  A publish is matched completely by its
 * owner shard (the shard of its first two words, or any shard when only
 * replicated filters can match it), so rows stay bit-exact.  A batch is cut
 * into G contiguous slices, slice i tokenised on shard i's device at prepare.
 * One step: every slice partitioned by owner on its own device, every shard
 * receiving its parts (D2D, xGMI peer copies, or staged through pinned host
 * memory) and walking them -- all queued, then ONE host wait.  The rows stay
 * where each shard's walk wrote them; the publish-order CSR with global
 * filter ids (local id * G + shard) is built on request (tm_sharded_result /
 * tm_sharded_device_csr).  The shards' dictionaries grow only by the deltas of
 * tm_sharded_insert_many, so word ids agree everywhere.  Reference: the
 * replicated emqx_trie (src/emqx_trie.erl:53-74) matched in full by
 * match_routes/1 (src/emqx_router.erl:127-141); sharding it is new. */
typedef struct tm_sharded tm_sharded;
typedef struct tm_sharded_batch tm_sharded_batch;
typedef struct {
    tm_batch_stats match;     /* summed over the parts; ms_* = the slowest part */
    float ms_partition;       /* device time: owner + partition of a slice (the slowest) */
    float ms_exchange;        /* device time: a shard receiving its parts (the slowest) */
    float ms_step;            /* host wall time of the last tm_sharded_run */
    float ms_unpartition;     /* host wall time: the publish-order CSR (on request) */
    uint32_t host_waits;      /* blocking host waits in the last step: 1, + 1 per capacity relaunch */
    uint32_t part_topics[64]; /* publishes each shard matched */
    float ms_stage;           /* host wall time of the last prepare's copy of the publishes into pinned memory */
    float ms_plan;            /* host wall time of the last prepare's plan (uploads, device tokenisers, counts);
                                 the uploads start while the copy runs, so the two overlap */
} tm_sharded_stats;
/* how shard i's memory reaches shard j's device */
#define TM_LINK_SAME   0      /* same device: D2D copies */
#define TM_LINK_PEER   1      /* peer access enabled both ways (xGMI): peer copies */
#define TM_LINK_STAGED 2      /* no peer access: copies staged through pinned host memory */
TM_API int  tm_sharded_create(const int32_t* devices, uint32_t n_shards, const tm_config* cfg, tm_sharded** out);
TM_API void tm_sharded_destroy(tm_sharded* s);
TM_API uint32_t tm_sharded_size(tm_sharded* s);
/* TM_LINK_* between shards i and j (TM_EINVAL out of range). */
TM_API int  tm_sharded_link(tm_sharded* s, uint32_t i, uint32_t j);
/* Shard g's engine (read-only use: stats, filter bytes of its local ids). */
TM_API tm_engine* tm_sharded_engine(tm_sharded* s, uint32_t shard);
/* Interns n words in order on every shard (tm_dict_load). */
TM_API int  tm_sharded_dict_load(tm_sharded* s, const uint8_t* words, const uint64_t* offsets, uint32_t n);
/* emqx_trie:insert/1 of a subscribe batch: the batch's literal words no shard
 * knows are appended to every shard's dictionary in first-appearance order,
 * then every shard inserts its filters and the replicated ones.
 * *n_inserted = insertions summed over the shards. */
TM_API int  tm_sharded_insert_many(tm_sharded* s, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                                   uint64_t* n_inserted);
/* emqx_trie:delete/1 of an unsubscribe batch on every shard (absent: no-op).
 * *n_deleted = deletions summed over the shards each filter lives on (its
 * owner, or all G for a replicated filter), as tm_sharded_insert_many counts. */
TM_API int  tm_sharded_delete_many(tm_sharded* s, const uint8_t* filters, const uint64_t* offsets, uint32_t n,
                                   uint64_t* n_deleted);
/* A publish batch: bytes copied (into pinned memory, by several threads),
 * slice i tokenised on shard i's device and its parts counted (the plan of
 * the exchange).  A non-NULL *out is re-prepared in place. */
TM_API int  tm_sharded_prepare(tm_sharded* s, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                               tm_sharded_batch** out);
/* One step (returns with every shard's rows in its HBM; one host wait). */
TM_API int  tm_sharded_run(tm_sharded* s, tm_sharded_batch* b);
/* D2H of the step's CSR of global filter ids (memory valid like tm_result). */
TM_API int  tm_sharded_result(tm_sharded* s, tm_sharded_batch* b, tm_result* out);
TM_API int  tm_sharded_device_csr(tm_sharded* s, tm_sharded_batch* b, const uint32_t** d_row_offsets,
                                  const uint32_t** d_ids, uint64_t* n_matches);
TM_API int  tm_sharded_batch_stats(tm_sharded* s, tm_sharded_batch* b, tm_sharded_stats* out);
TM_API void tm_sharded_batch_free(tm_sharded* s, tm_sharded_batch* b);
/* prepare + run + result in one call. */
TM_API int  tm_sharded_match_batch(tm_sharded* s, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                                   tm_result* out);
/* Bytes of global filter id gid (tm_filter_copy on its shard). */
TM_API int  tm_sharded_filter_copy(tm_sharded* s, uint32_t gid, uint8_t* buf, size_t cap, size_t* len);

/* ---- diagnostics ------------------------------------------------------ */
/* Consistency check of the host edge hash (tests): slots of a bucket filled
 * in order, every key's probe run unbroken and within max_disp, every key
 * found by the lookup the kernels mirror.  TM_EIO + tm_last_error() on the
 * first violation; *max_disp_out (may be NULL) = the largest displacement. */
TM_API int  tm_debug_check(tm_engine* e, uint64_t* max_disp_out);
/* Text of the last TM_EIO on this thread (HIP error string + call site). */
TM_API const char* tm_last_error(void);
TM_API const char* tm_build_info(void);
/* Number of visible HIP devices (0 when there is no driver or device). */
TM_API int  tm_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* EMQX_TM_H */
