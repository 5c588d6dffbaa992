// tm_pipeline.cpp -- engine setup / teardown, batches split over replicas, and
// the chunked host-to-host pipeline of tm_match_batch.
#include "tm_engine_impl.hpp"

int tm_engine::init(const tm_config* cfg, const int32_t* devices, uint32_t ndev) {
    frozen = cfg && (cfg->flags & TM_CFG_FROZEN_DICT);
    kn = Knobs::read();
    checked = kn.checked;
    if (kn.row_cap) row_cap = (uint32_t)kn.row_cap;
    if (kn.fan_big) fan_big_limit = kn.fan_big;
    if (kn.result_limit) result_limit = std::min<uint64_t>(MAX_RESULT, kn.result_limit);
    if (kn.staging_min) staging_min = kn.staging_min;
    threads = (cfg && cfg->host_threads) ? cfg->host_threads : default_threads(kn);
    dev_tok = !(cfg && (cfg->flags & TM_CFG_HOST_TOKENIZE));
    use_graphs = !kn.no_graph;
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

void tm_engine::destroy() {
    for (Replica* R : reps) async_stop(*R);
    for (Replica* R : reps) {
        (void)hipSetDevice(R->device);
        if (R->stream) (void)hipStreamSynchronize(R->stream);
        pipe_teardown(*R);
        R->scratch.release();
        R->tokb.release();
        dev_free(R->d_slots); dev_free(R->d_foff); dev_free(R->d_flen); dev_free(R->d_fbytes);
        dev_free(R->d_dkey); dev_free(R->d_tail); dev_free(R->d_arena); dev_free(R->d_dxidx); dev_free(R->d_dxval);
        dev_free(R->d_dblob);
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
    for (void* h : {(void*)h_dxidx, (void*)h_dxval, (void*)h_dblob})
        if (h) (void)hipHostFree(h);
    h_dxidx = nullptr; h_dxval = nullptr; h_dblob = nullptr;
    h_didx = nullptr; h_dval = nullptr; h_fidx = nullptr; h_foffv = nullptr; h_flenv = nullptr;
}

int tm_engine::run_slices(const uint8_t* topics, const uint64_t* offsets, uint32_t n) {
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

int tm_engine::pipe_setup(Replica& R) {
    if (R.pipe_ready) return TM_OK;
    for (int k = 0; k < 2; ++k) {
        tm_batch& b = R.pipe[k];
        b.rep = &R;
        HIP_OK(hipStreamCreateWithFlags(&b.own, hipStreamNonBlocking));
        b.own_user = true;   // (kept out of async_stop's sweep of slot batches)
        R.readers.push_back(&b);
        HIP_OK(hipEventCreateWithFlags(&R.pipe_h2d[k], hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&R.pipe_cp[k], hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&R.pipe_pk[k], hipEventDisableTiming));
    }
    HIP_OK(hipStreamCreateWithFlags(&R.pipe_copy, hipStreamNonBlocking));
    R.pipe_ready = true;
    return TM_OK;
}

void tm_engine::pipe_teardown(Replica& R) {
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
        if (R.pipe_pk[k]) (void)hipEventDestroy(R.pipe_pk[k]);
        R.pipe_h2d[k] = R.pipe_cp[k] = R.pipe_pk[k] = nullptr;
        if (R.h_stage[k]) (void)hipHostFree(R.h_stage[k]);
        R.h_stage[k] = nullptr;
        R.ch_stage[k] = 0;
    }
    if (R.pipe_copy) (void)hipStreamDestroy(R.pipe_copy);
    R.pipe_copy = nullptr;
    if (R.h_prow) (void)hipHostFree(R.h_prow);
    if (R.h_pids) (void)hipHostFree(R.h_pids);
    if (R.h_pids8) (void)hipHostFree(R.h_pids8);
    R.h_prow = R.h_pids = nullptr;
    R.h_pids8 = nullptr;
    R.ch_prow = R.ch_pids = R.ch_pids8 = 0;
    R.pipe_ready = false;
}

int tm_engine::match_batch_pipelined(Replica& R, const uint8_t* topics, const uint64_t* offsets, uint32_t n,
                          tm_result* out, uint32_t pack) {
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
            if (pack == 3) {   // ids packed to 3 bytes on the device, copied packed (h_pids8)
                if (base + total > R.ch_pids8 / 3) {
                    HIP_OK(hipStreamSynchronize(R.pipe_copy));
                    const size_t want = (size_t)(base + total) +
                                        (size_t)((double)(total + 1) / cnt * (n - lo - cnt) * 1.25) + 1024;
                    uint8_t* np = nullptr;
                    HIP_OK(hipHostMalloc((void**)&np, want * 3 + 16, hipHostMallocDefault));
                    if (base) memcpy(np, R.h_pids8, base * 3);
                    if (R.h_pids8) (void)hipHostFree(R.h_pids8);
                    R.h_pids8 = np;
                    R.ch_pids8 = want * 3 + 16;
                }
                if (total) {
                    if ((rc = dev_reserve(Y->d_pack, Y->c_pack, total * 3 + 16))) return rc;
                    HIP_OK(launch_pack_ids(Y->d_ids, total, Y->d_pack, Y->own));
                }
                HIP_OK(hipEventRecord(R.pipe_pk[k], Y->own));
                HIP_OK(hipStreamWaitEvent(R.pipe_copy, R.pipe_pk[k], 0));
                if (total)
                    HIP_OK(hipMemcpyAsync(R.h_pids8 + base * 3, Y->d_pack, total * 3, hipMemcpyDeviceToHost,
                                          R.pipe_copy));
                HIP_OK(hipMemcpyAsync(R.h_prow + lo, Y->d_rowoff, (size_t)cnt * 4, hipMemcpyDeviceToHost,
                                      R.pipe_copy));
                HIP_OK(hipEventRecord(R.pipe_cp[k], R.pipe_copy));
                cp_pending[k] = true;
                cbase[j] = base + total;
                continue;
            }
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

int tm_engine::match_batch_split(const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_result* out) {
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

int tm_engine::match_routes_split(const uint8_t* topics, const uint64_t* offsets, uint32_t n, tm_routes* out) {
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

int tm_engine::rules_match_split(const uint8_t* names, const uint64_t* noffs, uint32_t n, const uint8_t* rules,
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
