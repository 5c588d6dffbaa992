// tm_upload.cpp -- delta uploads: the host trie's dirty nodes, edge slots and
// dictionary entries copied to every HBM replica before the next walk.
#include "tm_engine_impl.hpp"

bool tm_engine::upload_pending(const Replica& R) {
    if (full_dirty || !dirty.empty() || R.d_nslots != slots.size() || needs_repack()) return true;
    if (full_f_dirty || !dirty_f.empty() || fbytes.size() > R.fbytes_uploaded) return true;
    if (R.c_foff < nd.size() || R.c_flen < nd.size() || R.c_fbytes < fbytes.size() + 1) return true;
    if (dev_tok && (R.d_dict_n != dict.keys().size() || R.d_dict_gen != dict.gen() || !dict.dirty().empty() ||
                    dict.tails().size() > R.tails_uploaded || dict.arena().size() > R.arena_uploaded ||
                    R.c_arena < dict.arena().size() + 1))
        return true;
    return false;
}

int tm_engine::ensure_delta_idle() {
    for (Replica* R : reps)
        if (R->delta_inflight) {
            HIP_OK(hipSetDevice(R->device));
            HIP_OK(hipEventSynchronize(R->ev_delta));
            R->delta_inflight = false;
        }
    return TM_OK;
}

int tm_engine::sync_device(const Replica* back) {
    if (reps.empty()) return TM_ENODEV;
    bool any = false;
    for (Replica* R : reps) any = any || upload_pending(*R);
    if (!any) {   // (an upload in flight is ordered before later work on the device: no host wait)
        HIP_OK(hipSetDevice(back ? back->device : device));
        return TM_OK;
    }
    // the last async upload still reads the pinned staging this one rewrites
    int rc = ensure_delta_idle();
    if (rc) return rc;
    // after a bulk build or heavy churn, re-pack the host table to the
    // target load so the walk's working set stays small (a full upload)
    if (needs_repack()) {
        rehash((size_t)(live_edges / target_load));
        rebuild_lext();   // (a full upload follows the re-pack anyway)
    }
    const size_t nn = nd.size();
    // gather the deltas once
    const bool slots_full = full_dirty || dirty.size() > slots.size() / 8;
    {   // the blob's layout: the slot deltas, then the filter-metadata deltas
        const size_t k1 = (!slots_full && !dirty.empty()) ? dirty.size() : 0;
        const size_t k2 = (!full_f_dirty && !dirty_f.empty()) ? dirty_f.size() : 0;
        auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
        blob_off[0] = 0;
        blob_off[1] = al(k1 * sizeof(uint32_t));
        blob_off[2] = blob_off[1] + al(k1 * sizeof(Slot));
        blob_off[3] = blob_off[2] + al(k2 * sizeof(uint32_t));
        blob_off[4] = blob_off[3] + al(k2 * sizeof(uint64_t));
        blob_bytes = blob_off[4] + al(k2 * sizeof(uint32_t));
        if (blob_bytes && (rc = host_reserve(h_dblob, ch_dblob, blob_bytes))) return rc;
        h_didx = reinterpret_cast<uint32_t*>(h_dblob + blob_off[0]);
        h_dval = reinterpret_cast<Slot*>(h_dblob + blob_off[1]);
        h_fidx = reinterpret_cast<uint32_t*>(h_dblob + blob_off[2]);
        h_foffv = reinterpret_cast<uint64_t*>(h_dblob + blob_off[3]);
        h_flenv = reinterpret_cast<uint32_t*>(h_dblob + blob_off[4]);
    }
    if (!slots_full && !dirty.empty()) {
        const size_t k = dirty.size();
        par_chunks(k, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i) {
                if (i + 16 < i1) __builtin_prefetch(&slots[dirty[i + 16]]);
                const uint32_t d = dirty[i];
                h_didx[i] = d;
                h_dval[i] = slots[d];
                // the set is consumed here (every set bit is in `dirty`; words
                // shared by two entries are cleared twice, to the same 0)
                __atomic_store_n(&dirty_mark[d >> 6], 0ull, __ATOMIC_RELAXED);
            }
        });
    }
    if (!full_f_dirty && !dirty_f.empty()) {
        const size_t k = dirty_f.size();
        par_chunks(k, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; ++i) {
                const uint32_t c = dirty_f[i];
                h_fidx[i] = c; h_foffv[i] = n_foff[c]; h_flenv[i] = n_flen[c];
                dirty_f_mark[c] = 0;   // (each node is listed once)
            }
        });
    }
    std::vector<uint32_t>& dx = dict.dirty();
    const bool keys_full = dx.size() > dict.keys().size() / 8;
    if (dev_tok && !keys_full && !dx.empty()) {
        std::sort(dx.begin(), dx.end());
        dx.erase(std::unique(dx.begin(), dx.end()), dx.end());   // a slot may move twice: scatter it once
        const size_t k = dx.size();
        if ((rc = host_reserve(h_dxidx, ch_dxidx, k))) return rc;
        if ((rc = host_reserve(h_dxval, ch_dxval, k))) return rc;
        for (size_t i = 0; i < k; ++i) {
            h_dxidx[i] = dx[i];
            h_dxval[i] = dict.keys()[dx[i]];
        }
    }
    // apply to every replica (different devices run their copies concurrently)
    std::vector<uint8_t> pageable(reps.size(), 0), async(reps.size(), 0);
    for (size_t r = 0; r < reps.size(); ++r) {
        Replica& R = *reps[r];
        bool pg = false, as = false;
        if ((rc = upload_to(R, slots_full, keys_full, nn, pg, as))) return rc;
        pageable[r] = pg;
        async[r] = as;
    }
    // the dirty sets are consumed: every replica has them now
    // (the delta gathers above cleared their marks on the workers)
    if (slots_full) {
        full_dirty = false;
        for (uint32_t i : dirty) dirty_mark[i >> 6] = 0;   // every set bit is in `dirty`
        if (dirty_mark.size() != (slots.size() + 63) / 64) dirty_mark.assign((slots.size() + 63) / 64, 0);
    }
    dirty.clear();
    if (full_f_dirty) {
        full_f_dirty = false;
        dirty_f_mark.assign(nn, 0);
    }
    dirty_f.clear();
    if (dev_tok) dx.clear();
    for (size_t r = 0; r < reps.size(); ++r) {
        Replica& R = *reps[r];
        HIP_OK(hipSetDevice(R.device));
        if (pageable[r]) {
            // host vectors may be mutated / reallocated right after we return
            HIP_OK(hipStreamSynchronize(R.stream));
        } else if (async[r]) {
            HIP_OK(hipEventRecord(R.ev_delta, R.stream));
            R.delta_inflight = true;
            if (!R.readers.empty()) {   // own-stream batches launched from now on wait for this upload
                HIP_OK(hipEventRecord(R.ev_sync, R.stream));
                ++R.upload_seq;
            }
        }
    }
    HIP_OK(hipSetDevice(back ? back->device : device));
    return TM_OK;
}

int tm_engine::upload_to(Replica& R, bool slots_full, bool keys_full, size_t nn, bool& pageable_used, bool& async_used) {
    int rc;
    HIP_OK(hipSetDevice(R.device));
    const hipStream_t stream = R.stream;
    // tables change under the walks of this replica's own-stream batches in
    // flight: the uploads wait for them on the device, or on the host when
    // a table is reallocated (its old buffer is freed here)
    const bool realloc = R.d_nslots != slots.size() || R.c_foff < nn || R.c_flen < nn ||
                         R.c_fbytes < fbytes.size() + 1 ||
                         (dev_tok && (R.d_dict_n != dict.keys().size() || R.c_tail < dict.tails().size() + 1 ||
                                      R.c_arena < dict.arena().size() + 1));
    for (tm_batch* r : R.readers)
        if (r->launched && !r->done) {   // (a waited batch has finished reading them)
            if (realloc) {
                HIP_OK(hipStreamSynchronize(r->own));
                continue;
            }
            if (!r->ev_read) HIP_OK(hipEventCreateWithFlags(&r->ev_read, hipEventDisableTiming));
            HIP_OK(hipEventRecord(r->ev_read, r->own));
            HIP_OK(hipStreamWaitEvent(stream, r->ev_read, 0));
        }
    // the delta blob, in one copy (the scatters below read their parts)
    if (blob_bytes) {
        if ((rc = dev_reserve(R.d_dblob, R.cd_dblob, blob_bytes))) return rc;
        HIP_OK(hipMemcpyAsync(R.d_dblob, h_dblob, blob_bytes, hipMemcpyHostToDevice, stream));
        async_used = true;
    }
    // edge hash
    bool full = slots_full;
    if (R.d_nslots != slots.size()) {
        dev_free(R.d_slots);
        HIP_OK(hipMalloc((void**)&R.d_slots, slots.size() * sizeof(Slot)));
        R.d_nslots = slots.size();
        full = true;
    }
    if (full) {
        pageable_used = true;
        HIP_OK(hipMemcpyAsync(R.d_slots, slots.data(), slots.size() * sizeof(Slot), hipMemcpyHostToDevice, stream));
        ++uploads_full;
    } else if (!dirty.empty()) {
        const size_t k = dirty.size();
        HIP_OK(launch_scatter_slots(R.d_slots, reinterpret_cast<const uint32_t*>(R.d_dblob + blob_off[0]),
                                    reinterpret_cast<const Slot*>(R.d_dblob + blob_off[1]), (uint32_t)k, stream));
        ++uploads_delta;
        delta_slots += k;
        async_used = true;
    }
    // appended tails up to APP_MAX bytes in all go through the replica's
    // pinned staging (reserved once here: copies queued below read it until
    // the upload's event, and ensure_delta_idle waits for that before the
    // next upload reuses it)
    size_t app_need = 0, app_used = 0;
    {
        const uint64_t fb_from = R.c_fbytes < fbytes.size() + 1 ? 0 : R.fbytes_uploaded;
        app_need += fbytes.size() > fb_from ? fbytes.size() - fb_from : 0;
        if (dev_tok) {
            const size_t t_from = R.c_tail < dict.tails().size() + 1 ? 0 : R.tails_uploaded;
            const size_t a_from = R.c_arena < dict.arena().size() + 1 ? 0 : R.arena_uploaded;
            if (dict.tails().size() > t_from) app_need += (dict.tails().size() - t_from) * sizeof(DictTail) + 16;
            if (dict.arena().size() > a_from) app_need += dict.arena().size() - a_from + 16;
        }
    }
    const bool app_pinned = app_need > 0 && app_need <= APP_MAX;
    if (app_pinned && (rc = host_reserve(R.h_app, R.ch_app, app_need))) return rc;
    // a host range -> device, through the pinned staging when it fits
    auto h2d_tail = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        if (app_pinned && app_used + bytes <= R.ch_app) {
            uint8_t* stg = R.h_app + app_used;
            memcpy(stg, src, bytes);
            app_used = (app_used + bytes + 15) & ~(size_t)15;
            async_used = true;
            return hipMemcpyAsync(dst, stg, bytes, hipMemcpyHostToDevice, stream);
        }
        pageable_used = true;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream);
    };
    // filter bytes (slow-path sort): arena + per-node (off, len)
    bool f_full = full_f_dirty;
    // (grown 2x: churn appends to these every step, and a new buffer
    // costs a full copy, a host wait for the batches reading the old one
    // and a new capture of every batch's launch graph -- its address is an
    // argument)
    if (R.c_foff < nn || R.c_flen < nn) {
        if ((rc = dev_reserve(R.d_foff, R.c_foff, 2 * nn))) return rc;
        if ((rc = dev_reserve(R.d_flen, R.c_flen, 2 * nn))) return rc;
        f_full = true;
    }
    if (R.c_fbytes < fbytes.size() + 1) {
        if ((rc = dev_reserve(R.d_fbytes, R.c_fbytes, 2 * (fbytes.size() + 1)))) return rc;
        R.fbytes_uploaded = 0;
    }
    if (fbytes.size() > R.fbytes_uploaded) {
        HIP_OK(h2d_tail(R.d_fbytes + R.fbytes_uploaded, fbytes.data() + R.fbytes_uploaded,
                        fbytes.size() - R.fbytes_uploaded));
        R.fbytes_uploaded = fbytes.size();
    }
    if (f_full) {
        pageable_used = true;
        HIP_OK(hipMemcpyAsync(R.d_foff, n_foff.data(), nn * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(R.d_flen, n_flen.data(), nn * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    } else if (!dirty_f.empty()) {
        const size_t k = dirty_f.size();
        HIP_OK(launch_scatter_fmeta(R.d_foff, R.d_flen, reinterpret_cast<const uint32_t*>(R.d_dblob + blob_off[2]),
                                    reinterpret_cast<const uint64_t*>(R.d_dblob + blob_off[3]),
                                    reinterpret_cast<const uint32_t*>(R.d_dblob + blob_off[4]), (uint32_t)k, stream));
        async_used = true;
    }
    if (dev_tok && (rc = sync_dict(R, keys_full, pageable_used, async_used, h2d_tail))) return rc;
    return TM_OK;
}
