// tm_fanout.cpp -- routes (emqx_router), subscriptions and the fan-out dispatch
// (emqx_broker:publish -> subscribers), rule predicates.
#include "tm_engine_impl.hpp"

int tm_engine::route_add(const uint8_t* t, size_t len, uint32_t dest) {
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

int tm_engine::route_delete(const uint8_t* t, size_t len, uint32_t dest) {
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

int tm_engine::sync_routes(Replica& R) {
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

int tm_engine::batch_routes(tm_batch* b, tm_routes* out) {
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

int tm_engine::subscribe(const uint8_t* t, size_t len, uint32_t sub, uint32_t node_dest) {
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

int tm_engine::unsubscribe(const uint8_t* t, size_t len, uint32_t sub, uint32_t node_dest) {
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

int tm_engine::subscriber_down(uint32_t sub, uint32_t node_dest, uint64_t* n_removed) {
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

int tm_engine::sync_subs(Replica& R) {
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

int tm_engine::batch_dispatch(tm_batch* b, uint32_t flags, tm_deliveries* out) {
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
    const bool counts_only = flags & TM_DISPATCH_COUNT_ONLY;
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

int tm_engine::rules_match(Replica& R, const uint8_t* names, const uint64_t* noffs, uint32_t n, const uint8_t* rules,
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
