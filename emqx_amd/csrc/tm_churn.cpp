// tm_churn.cpp -- trie mutations (emqx_trie insert/1, delete/1 and their batched
// parallel pass: plan, node records, edge phase, summaries).  Semantics follow
// src/emqx_trie.erl:81-116, 145-158, 190-204.
#include "tm_engine_impl.hpp"

int tm_engine::trie_insert_ids(const uint8_t* t, size_t len, const uint32_t* ids_p, uint32_t nids, uint32_t from,
                    uint32_t k0, uint32_t sd) {
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
                if (!M && nd.size() + need >= MAX_NODES && free_nodes.size() + pending_n < need)
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

int tm_engine::trie_delete(const uint8_t* t, size_t len) {
    std::vector<uint32_t> ids;
    if (!filter_words(t, len, false, ids)) return TM_OK;
    const uint32_t n = walk(ids);
    if (n == NONE) return TM_OK;
    return trie_delete_at(n, ids.data(), (uint32_t)ids.size());
}

int tm_engine::trie_delete_at(uint32_t n, const uint32_t* ids_p, uint32_t nids, uint32_t sd) {
    struct { const uint32_t* d; uint32_t n; size_t size() const { return n; } uint32_t operator[](size_t i) const { return d[i]; } } ids{ids_p, nids};
    Mut* const M = tl_mut;
    std::unique_lock<std::recursive_mutex> nl;
    if (M && ids.size() < sd) nl = std::unique_lock<std::recursive_mutex>(shared_mu(n));
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
        // (a parallel batch: the nodes of depth < sd are shared by workers)
        std::unique_lock<std::recursive_mutex> rl;
        if (M && k < sd) rl = std::unique_lock<std::recursive_mutex>(shared_mu(p));
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

void tm_engine::plan_range(const uint8_t* buf, const uint64_t* offs, uint32_t lo, uint32_t hi, bool del, uint32_t part,
                uint32_t pbase, bool append) {
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
    const bool ptrace = kn.par_trace;
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
            const uint32_t* w = W.data() + pe.woff;
            pe.pkey = mix_word(pe.nw ? w[0] : 0) ^ (pe.nw > 1 ? mix_word(w[1] * 0x85EBCA6Bu + 1) : 0u);
            pe.sub = (uint8_t)(pe.nw > 2 ? mix_word(w[2] * 0xC2B2AE35u + 7) % PART_SPLIT : 0);
            pe.unk = !known[q];
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

void tm_engine::make_plan(const uint8_t* buf, const uint64_t* offs, uint32_t n, bool del) {
    plan.resize(n);
    // (PLAN_PARTS parts per worker, taken by whichever worker is free: a
    // worker the box's scheduler preempts holds up a part, not the run)
    const unsigned nt = std::max(1u, std::min<unsigned>(PLAN_PARTS * threads, n / 256));
    if (plan_words.size() < nt) plan_words.resize(nt);
    if (plan_tw.size() < nt) plan_tw.resize(nt);
    if (nt == 1) { plan_range(buf, offs, 0, n, del, 0); return; }
    ensure_pool();   // the engine's workers (no thread start-up per batch)
    std::atomic<unsigned> next{0};
    pool.run([&](unsigned) {
        for (unsigned j; (j = next.fetch_add(1, std::memory_order_relaxed)) < nt;) {
            const uint32_t lo = (uint32_t)((uint64_t)n * j / nt), hi = (uint32_t)((uint64_t)n * (j + 1) / nt);
            plan_range(buf, offs, lo, hi, del, j);
        }
    });
}

void tm_engine::make_plan_pair(const uint8_t* dbuf, const uint64_t* doffs, uint32_t ndel, const uint8_t* ibuf,
                    const uint64_t* ioffs, uint32_t nins) {
    plan.resize((size_t)ndel + nins);
    const unsigned nt = std::max(1u, std::min<unsigned>(PLAN_PARTS * threads, (ndel + nins) / 256));
    if (plan_words.size() < nt) plan_words.resize(nt);
    if (plan_tw.size() < nt) plan_tw.resize(nt);
    auto part = [&](unsigned j) {
        plan_range(dbuf, doffs, (uint32_t)((uint64_t)ndel * j / nt), (uint32_t)((uint64_t)ndel * (j + 1) / nt), true, j);
        plan_range(ibuf, ioffs, (uint32_t)((uint64_t)nins * j / nt), (uint32_t)((uint64_t)nins * (j + 1) / nt), false, j,
                   ndel, true);
    };
    if (nt == 1) { part(0); return; }
    ensure_pool();
    std::atomic<unsigned> next{0};
    pool.run([&](unsigned) {
        for (unsigned j; (j = next.fetch_add(1, std::memory_order_relaxed)) < nt;) part(j);
    });
}

uint32_t tm_engine::replan_dead_inserts(uint32_t n) {
    const unsigned nt = std::max(1u, std::min<unsigned>(threads, n / 1024));
    if (replan_buf.size() < nt) replan_buf.resize(nt);
    if (nt == 1) {
        replan_range(0, n, replan_buf[0]);
        return (uint32_t)replan_buf[0].size();
    }
    ensure_pool();
    std::atomic<uint32_t> total{0};
    pool.run([&](unsigned i) {   // (read-only on the trie; each worker's own plan entries)
        for (unsigned j = i; j < nt; j += pool.n) {
            replan_range((uint32_t)((uint64_t)n * j / nt), (uint32_t)((uint64_t)n * (j + 1) / nt), replan_buf[j]);
            total.fetch_add((uint32_t)replan_buf[j].size(), std::memory_order_relaxed);
        }
    });
    return total.load();
}

void tm_engine::replan_range(uint32_t lo, uint32_t hi, std::vector<uint32_t>& redo) {
    redo.clear();
    for (uint32_t i = lo; i < hi; ++i) {
        if (i + 16 < hi && plan[i + 16].node != ROOT) __builtin_prefetch(&nd[plan[i + 16].node]);
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
}

void tm_engine::prefetch_insert(uint32_t i, uint32_t n) {
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

void tm_engine::prefetch_delete(uint32_t i, uint32_t n) {
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

int tm_engine::insert_planned(const uint8_t* buf, const uint64_t* offs, uint32_t i) {
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

void tm_engine::ensure_pool() {
    if (!pool_started) {
        cpu_set_t cpus;
        pool.trace = kn.par_trace;
        pool.start(threads, device_node_cpus(device, threads, kn.pool_pin, cpus) ? &cpus : nullptr);
        pool_started = true;
    }
}

void tm_engine::prefetch_edge_of(const std::vector<uint32_t>& v, size_t q) const {
    if (q + 16 < v.size()) {
        __builtin_prefetch(&nd[v[q + 16]]);
        __builtin_prefetch(&n_lext[v[q + 16]]);
    }
    if (q + 8 < v.size()) {
        const uint32_t s = nd[v[q + 8]].inslot;
        if (s != NONE && s < slots.size()) {
            __builtin_prefetch(&slots[s], 1);
            if ((s >> 6) < dirty_mark.size()) __builtin_prefetch(&dirty_mark[s >> 6], 1);
        }
    }
}

void tm_engine::edge_phase(const std::vector<std::vector<Mut>*>& Ws) {
    const unsigned T = std::max(1u, threads);
    std::vector<Mut*> ms;   // every phase-1 state
    for (std::vector<Mut>* W : Ws)
        for (Mut& m : *W) {
            m.defer = false;
            ms.push_back(&m);
        }
    auto merge_edges = [&](std::vector<Mut>& X) {
        for (Mut& m : X) {
            live_edges += m.live_edges; used_slots += m.used_slots; max_disp = std::max(max_disp, m.max_disp);
            dirty.insert(dirty.end(), m.dirty.begin(), m.dirty.end());
            m.live_edges = m.used_slots = 0; m.max_disp = 0; m.dirty.clear();
        }
    };
    // T2 range pairs (EDGE_PAIRS per worker, each pass's ranges taken by
    // whichever worker is free)
    auto ranges = [&](unsigned& T2, uint32_t& RS, uint32_t& R) {
        const uint32_t nb = nbuckets();
        T2 = std::min<unsigned>(EDGE_PAIRS * T, nb / (2 * PAR_RANGE_MIN));
        if (T2 < 2) { T2 = 0; return; }
        RS = ((nb + 2 * T2 - 1) / (2 * T2) + 15) / 16 * 16;   // whole 16-bucket groups: dirty-mark words stay per range
        R = (nb + RS - 1) / RS;
    };
    const bool trace = kn.par_trace;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto msd = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto e0 = now();
    size_t ndel = 0, nins = 0;
    for (Mut* m : ms) {
        ndel += m->del.size();
        nins += m->ins.size();
    }
    // Whether the inserts need a rehash first (the serial insert_edge's rule,
    // for the whole batch) is known now: the deletes free exactly ndel slots
    // and leave max_disp as it is.  Without one, the inserts' ranges are the
    // deletes' and everything is bucketed in one run below.
    const auto need_rehash = [&](uint64_t used) { return (used + nins) * 4 > slots.size() * 3 || max_disp > 48; };
    const bool rehash_ahead = need_rehash(used_slots - ndel);
    unsigned T2 = 0;
    uint32_t RS = 0, R = 0;
    ranges(T2, RS, R);
    const unsigned TS = (unsigned)std::min<size_t>(T, std::max<size_t>(1, slots.size() / 4096));   // summary workers
    // ---- bucketing, each worker over the phase-1 states it owns: deletes
    // by the slot recorded in phase 1 (nothing has moved since), inserts by
    // home bucket, summaries by node.  Range tail = the last range when R is
    // odd (it wraps onto range 0: run serially), or everything without T2.
    const uint32_t nb = nbuckets(), tail = 2 * T2;
    const unsigned NB = pool.n;
    if (edge_bins.size() < NB) edge_bins.resize(NB);
    auto bin_of = [&](uint32_t bucket) { const uint32_t r = bucket / RS; return (R % 2 && r == R - 1) ? tail : r; };
    pool.run([&](unsigned t) {
        EdgeBins& B = edge_bins[t];
        B.del.resize(tail + 1);
        B.ins.resize(tail + 1);
        B.sum.resize(TS);
        for (auto& v : B.del) v.clear();
        for (auto& v : B.ins) v.clear();
        for (auto& v : B.sum) v.clear();
        for (size_t j = t; j < ms.size(); j += NB) {
            const Mut& m = *ms[j];
            for (const auto& d : m.del) B.del[T2 ? bin_of(d.second / BUCKET) : tail].push_back(d);
            if (!rehash_ahead)
                for (const auto& e : m.ins) B.ins[T2 ? bin_of(home_bucket(e[0], e[1], nb)) : tail].push_back(e);
            for (uint32_t c : m.sum) B.sum[mix_word(c) % TS].push_back(c);
        }
    });
    tr_mark("e.bucket");
    // ---- deletes: even ranges in parallel, then odd ones
    if (ndel && T2) {
        std::vector<Mut>& X = edge_states(NB);
        std::vector<std::vector<uint32_t>> late(NB);
        for (uint32_t par = 0; par < 2; ++par) {
            std::atomic<unsigned> next{0};
            pool.run([&](unsigned t) {
                tl_mut = &X[t];
                for (unsigned pr; (pr = next.fetch_add(1, std::memory_order_relaxed)) < T2;) {
                    const uint32_t r = 2 * pr + par;
                    for (unsigned w = 0; w < NB; ++w) {
                        const auto& v = edge_bins[w].del[r];
                        for (size_t q = 0; q < v.size(); ++q) {
                            if (q + 16 < v.size()) {   // the record 16 ahead, the slot (as recorded) 8 ahead
                                __builtin_prefetch(&nd[v[q + 16].first]);
                                __builtin_prefetch(&n_lext[v[q + 16].first]);
                            }
                            if (q + 8 < v.size() && v[q + 8].second < slots.size()) {   // (and its dirty-mark word)
                                __builtin_prefetch(&slots[v[q + 8].second], 1);
                                if ((v[q + 8].second >> 6) < dirty_mark.size()) __builtin_prefetch(&dirty_mark[v[q + 8].second >> 6], 1);
                            }
                            const uint32_t c = v[q].first;
                            // an odd range's slot may have been pulled back into the even range before it
                            if (nd[c].inslot / BUCKET / RS != r) { late[t].push_back(c); continue; }
                            delete_edge_of(c);
                        }
                    }
                }
                tl_mut = nullptr;
            });
        }
        tr_mark("e.druns");
        merge_edges(X);
        for (auto& l : late)
            for (uint32_t c : l) delete_edge_of(c);   // serially, global counters
    }
    for (unsigned w = 0; w < NB && ndel; ++w)
        for (const auto& d : edge_bins[w].del[tail]) delete_edge_of(d.first);
    tr_mark("e.dtail");
    // ---- inserts: room first, then by range as the deletes
    const auto e1 = now();
    bool rehashed = false;
    if (need_rehash(used_slots)) {
        rehash(std::max<size_t>((size_t)((live_edges + nins) / 0.55), slots.size() * (max_disp > 48 ? 2 : 1)));
        rehashed = true;
    }
    const auto e2 = now();
    if (rehashed || rehash_ahead) {   // (rare) inserts bucketed for the table as it is now, by one worker
        ranges(T2, RS, R);
        const uint32_t nb2 = nbuckets(), tail2 = 2 * T2;
        for (unsigned w = 0; w < NB; ++w)
            for (auto& v : edge_bins[w].ins) v.clear();
        EdgeBins& B = edge_bins[0];
        B.ins.resize(tail2 + 1);
        for (const Mut* m : ms)
            for (const auto& e : m->ins) {
                const uint32_t r = T2 ? home_bucket(e[0], e[1], nb2) / RS : tail2;
                B.ins[T2 && R % 2 && r == R - 1 ? tail2 : r].push_back(e);
            }
    }
    const uint32_t itail = 2 * T2;
    if (nins && T2) {
        const uint32_t nbi = nbuckets();
        std::vector<Mut>& X = edge_states(NB);
        for (uint32_t par = 0; par < 2; ++par) {
            std::atomic<unsigned> next{0};
            pool.run([&](unsigned t) {
                tl_mut = &X[t];
                for (unsigned pr; (pr = next.fetch_add(1, std::memory_order_relaxed)) < T2;) {
                    const uint32_t r = 2 * pr + par;
                    for (unsigned w = 0; w < NB; ++w) {
                        if (r >= edge_bins[w].ins.size()) continue;
                        const auto& v = edge_bins[w].ins[r];
                        for (size_t q = 0; q < v.size(); ++q) {
                            if (q + 8 < v.size()) {   // the home bucket and the child's record, a few edges ahead
                                const size_t hs = (size_t)home_bucket(v[q + 8][0], v[q + 8][1], nbi) * BUCKET;
                                __builtin_prefetch(&slots[hs], 1);
                                if ((hs >> 6) < dirty_mark.size()) __builtin_prefetch(&dirty_mark[hs >> 6], 1);
                                __builtin_prefetch(&nd[v[q + 8][2]], 1);
                                __builtin_prefetch(&n_lext[v[q + 8][2]]);   // (its summary is written)
                            }
                            insert_edge(v[q][0], v[q][1], v[q][2]);
                        }
                    }
                }
                tl_mut = nullptr;
            });
        }
        tr_mark("e.iruns");
        merge_edges(X);
    }
    for (unsigned w = 0; w < NB && nins; ++w)
        if (itail < edge_bins[w].ins.size())
            for (const auto& e : edge_bins[w].ins[itail]) insert_edge(e[0], e[1], e[2]);
    if (max_disp > 48) rehash(std::max<size_t>((size_t)(live_edges / 0.55), slots.size() * 2));
    tr_mark("e.itail");
    const auto e3 = now();
    // ---- summaries of the nodes whose record changed: by node (a node's
    // records are rewritten by one worker; dirty marks set atomically)
    const unsigned TS2 = (unsigned)std::min<size_t>(T, std::max<size_t>(1, slots.size() / 4096));
    if (TS2 != TS) {   // (the table grew: rebucketed by one worker)
        std::vector<uint32_t> all;
        for (unsigned w = 0; w < NB; ++w)
            for (auto& v : edge_bins[w].sum) {
                all.insert(all.end(), v.begin(), v.end());
                v.clear();
            }
        edge_bins[0].sum.assign(TS2, {});
        for (uint32_t c : all) edge_bins[0].sum[mix_word(c) % TS2].push_back(c);
    }
    std::vector<Mut>& X = edge_states(TS2);
    pool.run([&](unsigned t) {
        if (t >= TS2) return;
        std::vector<uint32_t>& v = X[t].sum;   // (a fresh state's list: scratch)
        v.clear();
        for (unsigned w = 0; w < NB; ++w)
            if (t < edge_bins[w].sum.size()) v.insert(v.end(), edge_bins[w].sum[t].begin(), edge_bins[w].sum[t].end());
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (size_t q = 0; q < v.size(); ++q) {
            prefetch_edge_of(v, q);
            const uint32_t c = v[q];
            if (!nd[c].live || nd[c].inslot == NONE) continue;
            write_summary_at(c, X[t].dirty);
        }
        v.clear();
    });
    tr_mark("e.srun");
    merge_edges(X);
    tr_mark("e.smerge");
    if (trace)
        fprintf(stderr, "[par edges T2=%u nb=%u] del %.2f rehash %d %.2f ins %.2f sum %.2f ms\n", T2, nbuckets(),
                msd(e0, e1), (int)rehashed, msd(e1, e2), msd(e2, e3), msd(e3, now()));
}

void tm_engine::write_summary_at(uint32_t c, std::vector<uint32_t>& dl) {
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

std::vector<Mut> mut_w2;   // the insert states of tm_trie_apply_many (its deletes use mut_w)

// tm_trie_insert_many / delete_many of n >= PAR_MIN planned filters (make_plan ran).
// Returns 1 when the batch must run serially instead (nothing changed then).
int tm_engine::mutate_parallel(bool del, const uint8_t* buf, const uint64_t* offs, uint32_t n, uint64_t* done_out,
                    int* rc_out) {
    ParRun R;
    if (par_begin(del, buf, offs, n, mut_w, R)) return 1;
    ParRun* runs[1] = {&R};
    par_finish(runs, 1);
    *done_out = R.done;
    *rc_out = R.rc;
    return 0;
}

int tm_engine::par_begin(bool del, const uint8_t* buf, const uint64_t* offs, uint32_t n, std::vector<Mut>& W, ParRun& R) {
    const unsigned T = std::max(1u, threads);
    if (T < 2 || (uint64_t)n * 4 > n_filters) return 1;   // bulk builds stay serial: churn on a big trie only
    if (!del) {
        // new words are interned first, serially (the dictionary is not thread-safe)
        for (uint32_t i = 0; i < n; ++i) {
            PlanEnt& pe = plan[i];
            if (!pe.unk) continue;
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
    tr_mark(del ? "d.intern" : "i.intern");
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
    // (the keys come from the plan: filters with the same first two words
    // -- a new word counting as one word -- land in the same part)
    for (uint32_t i = 0; i < n; ++i) parts[mix_word(plan[i].pkey) % P].push_back(i);
    // A part far above a worker's share (a hot first-two-words prefix, e.g.
    // 10% of C5's churn under "+/+") is split by its third word: its filters
    // then share the depth-2 nodes too, under the same striped locks (and,
    // for inserts, the shared made map); parts split_from.. are those.
    const uint32_t split_from = P;
    {
        const size_t big = std::max<size_t>(64, n / (2 * T));
        for (uint32_t q = 0; q < split_from; ++q) {
            if (parts[q].size() <= big) continue;
            std::vector<uint32_t> whole;
            whole.swap(parts[q]);
            const size_t first = parts.size();
            parts.resize(first + PART_SPLIT);
            for (uint32_t i : whole) parts[first + plan[i].sub].push_back(i);
        }
    }
    tr_mark(del ? "d.parts" : "i.parts");
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
        tr_mark("i.sort");
        release_pending_ids();
        tr_mark("i.release");
        uint64_t total = 0;
        for (uint32_t i = 0; i < n; ++i) total += plan[i].nw - plan[i].depth;
        // (+ slack: ids are taken a chunk per worker)
        const size_t need = total + (size_t)T * Mut::ID_CHUNK;
        const size_t take = std::min<size_t>(need, free_nodes.size());
        fresh = need - take;
        if (base + fresh >= MAX_NODES) return 1;
        // Transactional: every allocation first (a bad_alloc here leaves
        // the engine as it was: the caller may still finish other work on
        // it), then the commit below, which allocates nothing.  (Growth
        // is geometric: an exact reserve would copy the arrays every batch.)
        auto grow = [&](auto& v) {
            if (v.capacity() < base + fresh) v.reserve(std::max(base + fresh, v.capacity() + v.capacity() / 2));
        };
        ids.reserve(take);
        if (fresh) {
            grow(nd);
            grow(n_flen);
            grow(n_lext);
            grow(n_foff);
        }
        if (!full_f_dirty) grow(dirty_f_mark);
        ids.assign(free_nodes.end() - (long)take, free_nodes.end());
        free_nodes.resize(free_nodes.size() - take);
        if (fresh) {
            nd.resize(base + fresh);   // dead records until handed out; the unused ones join the free list after
            n_flen.resize(base + fresh, 0);
            n_lext.resize(base + fresh, 0);
            n_foff.resize(base + fresh, 0);
        }
        if (!full_f_dirty && dirty_f_mark.size() < nd.size()) dirty_f_mark.resize(nd.size(), 0);
    }
    // (shared_made was cleared at the end of the previous batch)
    tr_mark(del ? "d.alloc" : "i.alloc");
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
                    // a few filters ahead: their plan entries and byte offsets
                    // first (written by other workers' plans: other cores'
                    // caches), then from those the record the walk starts
                    // from, the filter's word ids and its bytes
                    if (q + 16 < ni) {
                        __builtin_prefetch(&plan[items[q + 16]]);
                        if (!del) __builtin_prefetch(&offs[items[q + 16]]);
                    }
                    if (q + 8 < ni) {
                        const PlanEnt& pf = plan[items[q + 8]];
                        if (pf.node != NONE) {
                            __builtin_prefetch(&nd[pf.node]);
                            __builtin_prefetch(&n_lext[pf.node]);   // (a new literal child sets a bit there)
                        }
                        __builtin_prefetch(plan_words[pf.part].data() + pf.woff + (del ? 0 : pf.depth));
                        if (!del) __builtin_prefetch(buf + offs[items[q + 8]]);
                    }
                    const PlanEnt& pe = plan[i];
                    int rc;
                    if (del) {
                        rc = delete_planned(i, sd);
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
    tr_mark(del ? "d.phase1" : "i.phase1");
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

void tm_engine::par_finish(ParRun* const* runs, size_t nr) {
    const unsigned T = std::max(1u, threads);
    std::vector<std::vector<Mut>*> Ws;
    for (size_t r = 0; r < nr; ++r) Ws.push_back(runs[r]->W);
    edge_phase(Ws);
    const auto tp2 = std::chrono::steady_clock::now();
    // the workers' filter bytes and dirty filter ids go to the end of the
    // engine's arrays: places first, copies in parallel below
    size_t fb_end = fbytes.size(), df_end = dirty_f.size();
    std::vector<size_t> df_at;
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
            m.fresh_base = fb_end;   // (reused: this worker's bytes start here)
            fb_end += m.fb.size();
            df_at.push_back(df_end);
            df_end += m.dirty_f.size();
            pend_ids(launch_seq, m.pend.data(), m.pend.size());
        }
    }
    fbytes.resize(fb_end);
    dirty_f.resize(df_end);
    tr_mark("f.merge");
    pool.run([&](unsigned t) {   // bytes, dirty ids and filter byte offsets: distinct nodes per worker
        size_t k = 0;
        for (size_t r = 0; r < nr; ++r) {
            const std::vector<Mut>& W = *runs[r]->W;
            for (size_t j = 0; j < W.size(); ++j, ++k) {
                if (j % pool.n != t) continue;
                const Mut& m = W[j];
                if (!m.fb.empty()) memcpy(fbytes.data() + m.fresh_base, m.fb.data(), m.fb.size());
                if (!m.dirty_f.empty()) memcpy(dirty_f.data() + df_at[k], m.dirty_f.data(), m.dirty_f.size() * sizeof(uint32_t));
                for (const auto& f : m.foff) n_foff[f.first] = m.fresh_base + f.second;
            }
        }
        for (unsigned j = t; j < 64; j += pool.n) shared_made[j].clear();   // for the next batch
    });
    tr_mark("f.foff");
    for (size_t r = 0; r < nr; ++r) {
        ParRun& R = *runs[r];
        if (R.del) continue;
        std::vector<Mut>& W = *R.W;
        const std::vector<uint32_t>& ids = R.ids;
        const size_t fresh = R.fresh, base = R.base;
        // ids not handed out go (back) to the free list: the rest of each
        // worker's last chunk, the free-list ids past the highest one handed
        // out, and the fresh records past it
        size_t used = 0;
        for (const Mut& m : W) used = std::max(used, m.id_lo);   // highest id index handed out + 1
        const size_t avail = ids.size() + fresh;
        if (used > avail) used = avail;
        for (const Mut& m : W)
            for (size_t k = m.id_lo; k < std::min(m.id_hi, used); ++k)
                free_nodes.push_back(k < ids.size() ? ids[k] : (uint32_t)(base + (k - ids.size())));
        for (size_t k = used; k < ids.size(); ++k) free_nodes.push_back(ids[k]);
        // fresh records not handed out stay, as free dead records (cutting
        // them re-initialised the arrays' tails every batch)
        const size_t fresh_used = used > ids.size() ? used - ids.size() : 0;
        for (size_t k = fresh; k-- > fresh_used;) free_nodes.push_back((uint32_t)(base + k));
    }
    tr_mark("f.ids");
    if (kn.par_trace) {
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
