// tm_async.cpp -- the per-publish async pipeline (tm_match_async): queued calls
// batched onto the device by a launcher thread, rows delivered in chunks by
// completer threads.  src/emqx_broker.erl:201-210 is the caller it replaces.
#include "tm_engine_impl.hpp"

int tm_engine::async_start(Replica& R) {
    if (R.a_started) return TM_OK;
    if (reps.empty()) return TM_ENODEV;
    if (kn.async_depth) R.a_depth = (uint32_t)kn.async_depth;
    if (kn.async_completers) R.a_ncompleters = (uint32_t)kn.async_completers;
    if (kn.async_spin_us >= 0) R.a_spin_us = (uint32_t)kn.async_spin_us;
    {
        std::lock_guard<std::recursive_mutex> g(mu);
        HIP_OK(hipSetDevice(R.device));
        for (uint32_t i = 0; i < R.a_depth; ++i) {
            AsyncSlot* sl = new AsyncSlot();
            R.a_slots.push_back(sl);
            sl->b.rep = &R;
            HIP_OK(hipStreamCreateWithFlags(&sl->b.own, hipStreamNonBlocking));
            HIP_OK(hipEventCreateWithFlags(&sl->ev_done, hipEventDisableTiming));
            R.a_free.push_back(sl);
            R.readers.push_back(&sl->b);
        }
    }
    R.a_stop = false;
    R.a_launcher_done = false;
    R.a_launcher = std::thread([this, &R] { launcher_loop(R); });
    for (uint32_t i = 0; i < R.a_ncompleters; ++i) R.a_completers.emplace_back([this, &R] { completer_loop(R); });
    R.a_started = true;
    R.a_live.store(true, std::memory_order_release);
    return TM_OK;
}

void tm_engine::async_stop(Replica& R) {
    {
        std::lock_guard<std::mutex> lk(R.amu);
        if (!R.a_started && R.a_slots.empty()) return;
        R.a_stop = true;
        R.a_live.store(false, std::memory_order_release);
    }
    R.a_work.notify_all();
    R.a_done.notify_all();
    if (R.a_launcher.joinable()) R.a_launcher.join();
    for (auto& t : R.a_completers)
        if (t.joinable()) t.join();
    R.a_completers.clear();
    std::lock_guard<std::recursive_mutex> g(mu);
    (void)hipSetDevice(R.device);
    for (AsyncSlot* sl : R.a_slots) {
        if (sl->b.own) (void)hipStreamSynchronize(sl->b.own);
        forget_launch(&sl->b);
        sl->b.release();
        if (sl->b.own) (void)hipStreamDestroy(sl->b.own);
        if (sl->ev_done) (void)hipEventDestroy(sl->ev_done);
        if (sl->h_in) (void)hipHostFree(sl->h_in);
        if (sl->h_bin) (void)hipHostFree(sl->h_bin);
        for (AsyncSlot::GraphCache& gc : sl->gc)
            if (gc.exec) (void)hipGraphExecDestroy(gc.exec);
        if (sl->h_rows) (void)hipHostFree(sl->h_rows);
        if (sl->h_out) (void)hipHostFree(sl->h_out);
        if (sl->h_flag) (void)hipHostFree(sl->h_flag);
        delete sl;
    }
    R.a_slots.clear();
    R.a_free.clear();
    R.readers.erase(std::remove_if(R.readers.begin(), R.readers.end(), [](tm_batch* r) { return !r->own_user; }),
                    R.readers.end());
    R.a_started = false;
}

int tm_engine::match_async(const uint8_t* t, size_t len, tm_match_cb cb, void* ctx) {
    if (reps.empty()) return TM_ENODEV;
    static std::atomic<uint32_t> next_sub{0};
    static thread_local uint32_t my_sub = next_sub.fetch_add(1);
    static thread_local uint32_t my_calls = 0;
    Replica& R = *reps[(my_sub + my_calls++) % reps.size()];
    return match_async(R, t, len, cb, ctx);
}

int tm_engine::match_async(Replica& R, const uint8_t* t, size_t len, tm_match_cb cb, void* ctx) {
    if (!R.a_live.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lk(R.amu);
        if (R.a_stop) return TM_ENODEV;
        if (!R.a_started) {
            int rc = async_start(R);
            if (rc) return rc;
        }
    }
    static std::atomic<uint32_t> next_shard{0};
    static thread_local uint32_t my_shard = next_shard.fetch_add(1) % Replica::QSHARDS;
    Replica::QShard& sh = R.qs[my_shard];
    {
        std::lock_guard<std::mutex> g(sh.mu);
        if (len) sh.bytes.insert(sh.bytes.end(), t, t + len);
        sh.lens.push_back((uint32_t)len);
        sh.calls.push_back(AsyncCall{cb, ctx});
    }
    const uint64_t q = R.q_count.fetch_add(1, std::memory_order_acq_rel) + 1;
    if (q == 1 && R.a_inline) {   // the queue was empty: launch it here if the pipeline is idle
        std::unique_lock<std::mutex> lk(R.amu, std::try_to_lock);
        if (lk.owns_lock() && R.a_started && !R.a_stop && !R.a_free.empty() &&
            R.a_free.size() == R.a_slots.size() && R.q_count.load(std::memory_order_acquire) > 0) {
            ++R.a_inline_launches;
            launch_locked(R, lk);
            return TM_OK;
        }
    }
    if (q == 1 || q == R.a_gather_at.load() || q == R.a_max) {   // the launcher may be waiting for this
        std::lock_guard<std::mutex> lk(R.amu);
        R.a_work.notify_one();
    }
    return TM_OK;
}

void tm_engine::drain_queue(Replica& R, AsyncSlot* sl, size_t take) {
    constexpr uint32_t QSHARDS = Replica::QSHARDS;
    sl->calls.clear();
    sl->bytes.clear();
    sl->offs.assign(1, 0);
    static thread_local uint32_t start = 0;
    for (uint32_t k = 0; sl->calls.size() < take; ++k) {
        if (k && k % QSHARDS == 0) std::this_thread::yield();   // another drainer is mid-shard

        Replica::QShard& sh = R.qs[(start + k) % QSHARDS];
        std::lock_guard<std::mutex> g(sh.mu);
        size_t h = sh.head, hb = sh.head_bytes;
        while (h < sh.calls.size() && sl->calls.size() < take) {
            const uint32_t len = sh.lens[h];
            sl->calls.push_back(sh.calls[h]);
            sl->bytes.insert(sl->bytes.end(), sh.bytes.begin() + (long)hb, sh.bytes.begin() + (long)(hb + len));
            sl->offs.push_back(sl->bytes.size());
            hb += len;
            ++h;
        }
        if (h == sh.calls.size()) {   // shard emptied: reset, keep the capacity
            sh.calls.clear();
            sh.lens.clear();
            sh.bytes.clear();
            sh.head = sh.head_bytes = 0;
        } else {
            sh.head = h;
            sh.head_bytes = hb;
        }
    }
    start = (start + 1) % QSHARDS;   // no shard is always last
}

void tm_engine::launch_locked(Replica& R, std::unique_lock<std::mutex>& lk) {
    AsyncSlot* sl = R.a_free.back();
    R.a_free.pop_back();
    const size_t take =
        std::min<uint64_t>(R.q_count.load(std::memory_order_acquire), std::max<uint32_t>(R.a_max, 1));
    R.q_count.fetch_sub(take, std::memory_order_acq_rel);   // reserved: no other drainer counts on them
    R.a_inflight_calls += take;
    lk.unlock();
    drain_queue(R, sl, take);
    const auto t0 = std::chrono::steady_clock::now();
    try {
        sl->rc = slot_launch(sl);
    } catch (...) {
        sl->rc = TM_ENOMEM;
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    lk.lock();
    R.a_max_seen = std::max<uint64_t>(R.a_max_seen, sl->calls.size());
    R.a_us_launch += us;
    R.a_inflight.push_back(sl);
    R.a_done.notify_all();
}

void tm_engine::launcher_loop(Replica& R) {
    (void)hipSetDevice(R.device);
    std::unique_lock<std::mutex> lk(R.amu);
    auto queued = [&] { return R.q_count.load(std::memory_order_acquire); };
    for (;;) {
        R.a_work.wait(lk, [&] {
            if (R.a_stop) return queued() == 0 || !R.a_free.empty();
            return queued() && !R.a_free.empty();
        });
        if (queued() == 0) {
            if (R.a_stop) break;   // stopping, queue drained
            continue;              // an inline launch took the calls
        }
        // Batches in flight and few calls queued: gather more for a while.
        // "Few" scales with the calls the pipeline holds: a share of them per
        // slot, at most a_busy_min.  Under load (thousands of calls in flight)
        // batches stay large; with a few dozen blocking callers their calls
        // spread over the slots instead of queueing behind one batch, so the
        // device runs several small batches at once.
        // (A/B, 64 blocking callers: 0.47 M calls/s with a fixed 128, 0.62 M
        // calls/s scaled; the 2,048 / 4,096-in-flight legs unchanged)
        auto need = [&] {
            return std::min<uint64_t>(R.a_busy_min, std::max<uint64_t>(1, (R.a_inflight_calls + queued()) / R.a_depth));
        };
        if (!R.a_stop && R.a_free.size() != R.a_slots.size() && queued() < need()) {
            auto enough = [&] {
                const uint64_t k = need();
                R.a_gather_at.store(k);   // (seq_cst: a caller that reaches k after this sees it)
                return R.a_stop || R.a_free.size() == R.a_slots.size() || queued() >= k;
            };
            R.a_work.wait(lk, enough);
            R.a_gather_at.store(~0ull);
            if (R.a_free.empty() || queued() == 0) continue;
        }
        if (R.a_linger_us && !R.a_stop && queued() < R.a_max)
            R.a_work.wait_for(lk, std::chrono::microseconds(R.a_linger_us),
                              [&] { return R.a_stop || queued() >= R.a_max; });
        if (R.a_free.empty() || queued() == 0) continue;
        launch_locked(R, lk);
    }
    R.a_launcher_done = true;
    R.a_done.notify_all();
}

int tm_engine::slot_launch(AsyncSlot* sl) {
    const uint32_t n = (uint32_t)sl->calls.size();
    const size_t nb = sl->bytes.size(), head = packed_head(n);
    int rc;
    Replica& R = *sl->b.rep;
    // The bounded form (tm_batch::bounded): the batch is sized for max_batch
    // calls once, its input written into mapped pinned memory, and from the
    // second launch on the device work and the export replay one captured
    // graph.  Topics the size doesn't fit (more bytes than the slot holds)
    // take the packed H2D form below.
    const bool bounded = dev_tok && use_graphs && !checked && n <= R.a_max;
    if (bounded) {
        // size class: 1/512, 1/64, 1/8 of max_batch (at least 32 calls), or all of it
        uint32_t cls = 0, bound = R.a_max;
        for (; cls + 1 < AsyncSlot::NCLASS; ++cls) {
            const uint32_t c = std::max<uint32_t>(32, R.a_max >> (9 - 3 * cls));
            if (n <= c && c < R.a_max) { bound = c; break; }
        }
        sl->bound = bound;
        if (nb > sl->bytes_cap || sl->bytes_cap < (uint64_t)R.a_max * 64)
            sl->bytes_cap = std::max<uint64_t>({sl->bytes_cap, (uint64_t)R.a_max * 64, (uint64_t)nb + nb / 2});
        const size_t o_offs = 64, o_bytes = (o_offs + ((size_t)sl->bound + 1) * 8 + 15) & ~(size_t)15;
        if ((rc = host_reserve_coherent(sl->h_bin, sl->c_bin, o_bytes + sl->bytes_cap + 32))) return rc;
        *reinterpret_cast<volatile uint32_t*>(sl->h_bin) = n;
        memcpy(sl->h_bin + o_offs, sl->offs.data(), ((size_t)n + 1) * 8);
        if (nb) memcpy(sl->h_bin + o_bytes, sl->bytes.data(), nb);
        std::lock_guard<std::recursive_mutex> g(mu);
        HIP_OK(hipSetDevice(R.device));
        tm_batch* b = &sl->b;
        const hipStream_t S = b->own;
        uint8_t* d_bin = nullptr;
        HIP_OK(hipHostGetDevicePointer((void**)&d_bin, sl->h_bin, 0));
        if ((rc = prepare_bounded(b, sl->bound, sl->bytes_cap, reinterpret_cast<const uint64_t*>(d_bin + o_offs),
                                  d_bin + o_bytes, reinterpret_cast<uint32_t*>(d_bin))))
            return rc;
        ExportArgs x{};
        if ((rc = slot_export_args(sl, x, sl->bound))) return rc;
        x.d_n = reinterpret_cast<const uint32_t*>(d_bin);
        x.fixed_words = tm_batch::HDR_FIXED / 4;
        b->tail_key.assign(sizeof x + sizeof(uint32_t*), 0);
        memcpy(b->tail_key.data(), &x, sizeof x);
        memcpy(b->tail_key.data() + sizeof x, &sl->d_flag, sizeof(uint32_t*));
        b->tail = [this, sl, x](hipStream_t st) { return slot_tail(sl, x, st); };
        AsyncSlot::GraphCache& gc = sl->gc[cls];
        std::swap(b->gexec, gc.exec);
        std::swap(b->gkey, gc.key);
        rc = launch(b, false);
        std::swap(b->gexec, gc.exec);
        std::swap(b->gkey, gc.key);
        if (rc) return rc;
        if (!b->tail_done) HIP_OK(slot_tail(sl, x, S));
        HIP_OK(hipEventRecord(sl->ev_done, S));
        return TM_OK;
    }
    if ((rc = host_reserve(sl->h_in, sl->c_in, head + nb))) return rc;
    memcpy(sl->h_in, sl->offs.data(), ((size_t)n + 1) * 8);
    if (nb) memcpy(sl->h_in + head, sl->bytes.data(), nb);
    std::lock_guard<std::recursive_mutex> g(mu);
    HIP_OK(hipSetDevice(R.device));
    tm_batch* b = &sl->b;
    const hipStream_t S = b->own;
    rc = dev_tok ? upload_packed(b, sl->h_in, n, nb)
                 : prepare(b, sl->h_in + head, reinterpret_cast<const uint64_t*>(sl->h_in), n);
    if (rc) return rc;
    b->tail = nullptr;
    if ((rc = launch(b, false))) return rc;
    ExportArgs x{};
    if ((rc = slot_export_args(sl, x, n))) return rc;
    HIP_OK(slot_tail(sl, x, S));
    HIP_OK(hipEventRecord(sl->ev_done, S));
    return TM_OK;
}

// the export of a slot's batch of n (or, bounded, at most n) calls into its
// pinned buffers: [ctrl | stats | src n u64 | count n u32] and the rows
int tm_engine::slot_export_args(AsyncSlot* sl, ExportArgs& x, uint32_t n) {
    int rc;
    tm_batch* b = &sl->b;
    const size_t hdr_bytes = tm_batch::HDR_FIXED + (size_t)n * 8;
    if ((rc = host_reserve_coherent(sl->h_out, sl->c_out, hdr_bytes + (size_t)n * 4 + 8))) return rc;
    uint8_t* rows8 = reinterpret_cast<uint8_t*>(sl->h_rows);
    if ((rc = host_reserve_coherent(rows8, sl->c_rows, std::max<size_t>(b->c_sfids, 1) * 4))) return rc;
    sl->h_rows = reinterpret_cast<uint32_t*>(rows8);
    void *d_out = nullptr, *d_rows = nullptr;
    HIP_OK(hipHostGetDevicePointer(&d_out, sl->h_out, 0));
    HIP_OK(hipHostGetDevicePointer(&d_rows, sl->h_rows, 0));
    x.hdr = reinterpret_cast<const uint32_t*>(b->d_hdr);
    x.hdr_words = hdr_bytes / 4;
    x.h_hdr = reinterpret_cast<uint32_t*>(d_out);
    x.count = b->d_count;
    x.h_count = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_out) + hdr_bytes);
    x.n = n;
    x.rows = b->d_sfids;
    x.h_rows = reinterpret_cast<uint32_t*>(d_rows);
    x.rows_cap = std::min<uint64_t>(b->c_sfids, sl->c_rows / 4);
    x.rcap = region_cap(std::min<uint64_t>(b->c_sfids, MAX_RESULT), b->one_region);
    if (b->rep->a_spin_us && !sl->h_flag) {
        HIP_OK(hipHostMalloc((void**)&sl->h_flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
        *sl->h_flag = 0;
        HIP_OK(hipHostGetDevicePointer((void**)&sl->d_flag, sl->h_flag, 0));
    }
    return TM_OK;
}

// the export kernel, and the completion flag when completers poll it
hipError_t tm_engine::slot_tail(AsyncSlot* sl, const ExportArgs& x, hipStream_t S) {
    hipError_t e = launch_export_host(x, S);
    if (e == hipSuccess && sl->b.rep->a_spin_us && sl->d_flag) e = hipStreamWriteValue32(S, sl->d_flag, ++sl->seq, 0);
    return e;
}

void tm_engine::completer_loop(Replica& R) {
    (void)hipSetDevice(R.device);
    std::unique_lock<std::mutex> lk(R.amu);
    for (;;) {
        AsyncSlot* sl = nullptr;
        bool head = false;
        R.a_done.wait(lk, [&] {
            for (AsyncSlot* x : R.a_inflight)
                if (x->ready && x->next_chunk < x->nchunks) {
                    sl = x;
                    return true;
                }
            for (AsyncSlot* x : R.a_inflight)
                if (!x->claimed) {
                    sl = x;
                    head = true;
                    return true;
                }
            return R.a_launcher_done && R.a_inflight.empty();
        });
        if (!sl) break;
        if (head) {
            sl->claimed = true;
            lk.unlock();
            bool whole = true, recovered = false;
            double us_wait = 0;
            try {
                whole = slot_wait(sl, us_wait, recovered);
            } catch (...) {
            }
            lk.lock();
            R.a_us_wait += us_wait;
            R.a_recoveries += recovered ? 1 : 0;
            if (whole) {
                slot_finish(R, sl);
            } else {
                sl->nchunks = std::max<uint32_t>(
                    1, (uint32_t)((sl->calls.size() + AsyncSlot::DELIVER_CHUNK - 1) / AsyncSlot::DELIVER_CHUNK));
                sl->next_chunk = sl->chunks_done = 0;
                sl->ready = true;
                R.a_done.notify_all();
            }
            continue;
        }
        const uint32_t c = sl->next_chunk++;
        lk.unlock();
        const auto t0 = std::chrono::steady_clock::now();
        const uint32_t n = (uint32_t)sl->calls.size();
        const uint32_t lo = std::min(n, c * AsyncSlot::DELIVER_CHUNK);
        const uint32_t hi = std::min(n, lo + AsyncSlot::DELIVER_CHUNK);
        syncwake::in_batch = true;
        for (uint32_t i = lo; i < hi; ++i) {
            const uint32_t k = sl->d_count[i];
            sl->calls[i].cb(sl->calls[i].ctx, TM_OK, k ? sl->h_rows + sl->d_src[i] : sl->h_rows, k);
        }
        syncwake::in_batch = false;
        syncwake::flush();
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        lk.lock();
        R.a_us_deliver += us;
        if (++sl->chunks_done == sl->nchunks) slot_finish(R, sl);
    }
}

void tm_engine::slot_finish(Replica& R, AsyncSlot* sl) {
    R.a_inflight.erase(std::find(R.a_inflight.begin(), R.a_inflight.end(), sl));
    R.a_inflight_calls -= sl->calls.size();
    ++R.a_batches;
    R.a_requests += sl->calls.size();
    sl->calls.clear();
    sl->claimed = sl->ready = false;
    sl->nchunks = sl->next_chunk = sl->chunks_done = 0;
    R.a_free.push_back(sl);
    R.a_work.notify_all();
    R.a_done.notify_all();
}

bool tm_engine::slot_wait(AsyncSlot* sl, double& us_wait, bool& recovered) {
    tm_batch* b = &sl->b;
    const uint32_t n = (uint32_t)sl->calls.size();
    auto fail_all = [&](int rc) {
        syncwake::in_batch = true;
        for (const AsyncCall& c : sl->calls) c.cb(c.ctx, rc, nullptr, 0);
        syncwake::in_batch = false;
        syncwake::flush();
    };
    if (sl->rc) {
        (void)hipStreamSynchronize(b->own);   // whatever was enqueued before the failure
        fail_all(sl->rc);
        return true;
    }
    const auto tw = std::chrono::steady_clock::now();
    if (sl->h_flag && b->rep->a_spin_us) {   // poll the pinned flag first (no interrupt wake-up)
        const volatile uint32_t* f = sl->h_flag;
        const auto lim = tw + std::chrono::microseconds(b->rep->a_spin_us);
        for (uint32_t it = 0; *f != sl->seq; ++it) {
            __builtin_ia32_pause();
            if ((it & 255) == 0 && std::chrono::steady_clock::now() > lim) break;
        }
        // the flag follows the export in stream order; the event right after it
        if (*f == sl->seq)
            while (hipEventQuery(sl->ev_done) == hipErrorNotReady && std::chrono::steady_clock::now() < lim)
                __builtin_ia32_pause();
    }
    if (hipEventSynchronize(sl->ev_done) != hipSuccess) {
        fail_all(TM_EIO);
        return true;
    }
    us_wait = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw).count();
    const size_t hdr_bytes = tm_batch::HDR_FIXED + (size_t)n * 8;
    const uint32_t* ctrl = reinterpret_cast<const uint32_t*>(sl->h_out);
    const unsigned long long* stats = reinterpret_cast<const unsigned long long*>(sl->h_out + CTRL_WORDS * 4);
    uint32_t err = 0;
    uint64_t need = 0, staged = 0;
    int rc = check_ctrl(ctrl, stats, &err, &need, &staged);
    if (rc) {
        fail_all(rc);
        return true;
    }
    if (b->one_region) need = staged;
    if (!err && need > sl->c_rows / 4) err = ERR_STAGING;   // (cannot happen: rows hold the staging area)
    if (err) {
        // capacity miss (staging, generic-path scratch): the CSR path grows
        // and re-runs, then the rows come from the CSR
        recovered = true;
        tm_result r{};
        {
            std::lock_guard<std::recursive_mutex> g(mu);
            (void)hipSetDevice(b->rep->device);
            if (b->bounded) {   // sized for its bound: re-run as a packed batch of exactly these calls
                const size_t nb = sl->bytes.size(), head = packed_head(n);
                rc = host_reserve(sl->h_in, sl->c_in, head + nb);
                if (!rc) {
                    memcpy(sl->h_in, sl->offs.data(), ((size_t)n + 1) * 8);
                    if (nb) memcpy(sl->h_in + head, sl->bytes.data(), nb);
                    rc = upload_packed(b, sl->h_in, n, nb);
                }
                if (!rc) rc = grow_for(b, err, need, staged);
                if (!rc) rc = launch(b);
            } else {
                rc = grow_for(b, err, need, staged);
            }
            if (!rc) rc = wait(b);
            if (!rc) rc = result(b, &r);
        }
        if (rc) {
            fail_all(rc);
            return true;
        }
        syncwake::in_batch = true;
        for (uint32_t i = 0; i < n; ++i)
            sl->calls[i].cb(sl->calls[i].ctx, TM_OK, r.filter_ids + r.row_offsets[i],
                            r.row_offsets[i + 1] - r.row_offsets[i]);
        syncwake::in_batch = false;
        syncwake::flush();
        return true;
    }
    sl->d_src = reinterpret_cast<const unsigned long long*>(sl->h_out + tm_batch::HDR_FIXED);
    sl->d_count = reinterpret_cast<const uint32_t*>(sl->h_out + hdr_bytes);
    return false;
}
