// tm_load.cpp -- load generator for the per-publish path (bench.py --workload
// coalesce, tests/test_gpu_coalesce.py).  Not part of the engine: it plays the
// broker's publishing processes against the C ABI.
//
// The reference calls emqx_router:match_routes/1 once per message from every
// publishing client's own process (src/emqx_broker.erl:201-210), so a node has
// as many matches in flight as it has publishers.  Two caller models:
//   mode 0  `threads` OS threads, each calling tm_match_coalesced (blocking)
//           one topic at a time -- a NIF on dirty schedulers;
//   mode 1  `threads` submitter threads each keeping up to `window` calls of
//           tm_match_async outstanding -- threads x window publishing
//           processes blocked in `receive` while the NIF replies by enif_send.
// Every topic i is matched exactly once; per-topic row length and an FNV-1a
// hash of the row (ids in order) are written for verification, and per-call
// latency (submit -> row delivered) is collected.
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/emqx_tm.h"

extern "C" {
typedef struct {
    double seconds;       // wall time of the whole run
    uint64_t calls;       // calls completed
    uint64_t errors;      // calls that returned an error
    double mean_us, p50_us, p99_us, max_us;   // per-call latency
    double max_at_s;      // when the slowest call was submitted, seconds into the run (async mode; -1 otherwise)
} tml_result;
}

namespace {

using clk = std::chrono::steady_clock;

inline uint64_t row_hash(const uint32_t* ids, uint32_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t v = ids[i];
        for (int k = 0; k < 4; ++k) {
            h ^= (v >> (8 * k)) & 0xFF;
            h *= 0x100000001b3ull;
        }
    }
    return h;
}

struct Submitter;

struct Call {
    Submitter* who;
    uint32_t topic;
    clk::time_point t0;
};

// A submitter that found its window full sleeps until it has drained to
// `resume` calls in flight (a scheduler wakes for a run of replies, not one
// futex round trip per reply).
// (a cache line each: completers touch the submitters of the calls they deliver)
struct alignas(64) Submitter {
    std::atomic<int> outstanding{0};
    std::atomic<int> sleeping{0};
    std::atomic<int> resume{0};
    std::atomic<int> active{0};   // its callbacks running: tml_run returns only once none is
};

struct Shared {
    uint32_t* counts;
    uint64_t* hashes;
    float* lat_us;
    std::atomic<uint64_t> errors{0};
};
Shared* g_shared = nullptr;

void futex_wake(std::atomic<int>* a) { syscall(SYS_futex, reinterpret_cast<int*>(a), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0); }

void on_done(void* ctx, int rc, const uint32_t* ids, uint32_t n) {
    Call* c = static_cast<Call*>(ctx);
    Shared* s = g_shared;
    Submitter* w = c->who;
    w->active.fetch_add(1, std::memory_order_acq_rel);
    const double us = std::chrono::duration<double, std::micro>(clk::now() - c->t0).count();
    s->lat_us[c->topic] = (float)us;
    if (rc) {
        s->errors.fetch_add(1, std::memory_order_relaxed);
        s->counts[c->topic] = 0xFFFFFFFFu;
    } else {
        s->counts[c->topic] = n;
        if (s->hashes) s->hashes[c->topic] = row_hash(ids, n);
    }
    const int left = w->outstanding.fetch_sub(1, std::memory_order_acq_rel) - 1;
    if (left <= w->resume && w->sleeping.load(std::memory_order_acquire)) {
        w->sleeping.store(0, std::memory_order_release);
        futex_wake(&w->sleeping);
    }
    w->active.fetch_sub(1, std::memory_order_acq_rel);   // last touch of shared state
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) int tml_run(tm_engine* e, const uint8_t* topics, const uint64_t* offs,
                                                   uint32_t n, int mode, uint32_t threads, uint32_t window,
                                                   uint32_t* counts, uint64_t* hashes, tml_result* out) {
    if (!e || !offs || !counts || !out || !threads || (mode == 1 && !window)) return TM_EINVAL;
    std::vector<float> lat(std::max<uint32_t>(n, 1), 0.f);
    Shared sh;
    sh.counts = counts;
    sh.hashes = hashes;
    sh.lat_us = lat.data();
    g_shared = &sh;
    std::vector<Call> calls(std::max<uint32_t>(n, 1));
    std::vector<Submitter> subs(threads);
    std::atomic<int> first_rc{0};
    const auto t0 = clk::now();
    std::vector<std::thread> th;
    for (uint32_t k = 0; k < threads; ++k) {
        th.emplace_back([&, k] {
            if (mode == 0) {
                std::vector<uint32_t> ids(4096);
                for (uint32_t i = k; i < n; i += threads) {
                    const uint8_t* t = topics + offs[i];
                    const size_t len = offs[i + 1] - offs[i];
                    uint32_t m = 0;
                    const auto c0 = clk::now();
                    int rc = tm_match_coalesced(e, t, len, ids.data(), (uint32_t)ids.size(), &m);
                    if (rc == TM_OK && m > ids.size()) {   // longer row: ask again with room
                        ids.resize(m);
                        rc = tm_match_coalesced(e, t, len, ids.data(), (uint32_t)ids.size(), &m);
                    }
                    lat[i] = (float)std::chrono::duration<double, std::micro>(clk::now() - c0).count();
                    if (rc) {
                        sh.errors.fetch_add(1);
                        counts[i] = 0xFFFFFFFFu;
                    } else {
                        counts[i] = m;
                        if (hashes) hashes[i] = row_hash(ids.data(), m);
                    }
                }
                return;
            }
            Submitter& me = subs[k];
            me.resume = (int)window - std::max<int>(1, (int)window / 4);
            for (uint32_t i = k; i < n; i += threads) {
                if (me.outstanding.load(std::memory_order_acquire) >= (int)window) {
                    while (me.outstanding.load(std::memory_order_acquire) > me.resume) {
                        me.sleeping.store(1, std::memory_order_release);
                        if (me.outstanding.load(std::memory_order_acquire) > me.resume) {
                            struct timespec ts = {0, 1000000};   // re-check at least every ms
                            syscall(SYS_futex, reinterpret_cast<int*>(&me.sleeping), FUTEX_WAIT_PRIVATE, 1, &ts,
                                    nullptr, 0);
                        }
                        me.sleeping.store(0, std::memory_order_release);
                    }
                }
                Call& c = calls[i];
                c.who = &me;
                c.topic = i;
                c.t0 = clk::now();
                me.outstanding.fetch_add(1, std::memory_order_acq_rel);
                int rc = tm_match_async(e, topics + offs[i], offs[i + 1] - offs[i], on_done, &c);
                if (rc) {
                    me.outstanding.fetch_sub(1);
                    sh.errors.fetch_add(1);
                    counts[i] = 0xFFFFFFFFu;
                    int z = 0;
                    first_rc.compare_exchange_strong(z, rc);
                }
            }
            me.resume = 0;
            while (me.outstanding.load(std::memory_order_acquire) > 0) {   // drain
                me.sleeping.store(1, std::memory_order_release);
                if (me.outstanding.load(std::memory_order_acquire) > 0) {
                    struct timespec ts = {0, 200000};
                    syscall(SYS_futex, reinterpret_cast<int*>(&me.sleeping), FUTEX_WAIT_PRIVATE, 1, &ts, nullptr, 0);
                }
                me.sleeping.store(0, std::memory_order_release);
            }
        });
    }
    for (auto& t : th) t.join();
    for (Submitter& w : subs)
        while (w.active.load(std::memory_order_acquire)) std::this_thread::yield();
    out->seconds = std::chrono::duration<double>(clk::now() - t0).count();
    out->calls = n;
    out->errors = sh.errors.load();
    out->max_at_s = -1;
    if (n && mode == 1) {
        const size_t im = (size_t)(std::max_element(lat.begin(), lat.begin() + n) - lat.begin());
        out->max_at_s = std::chrono::duration<double>(calls[im].t0 - t0).count();
    }
    std::vector<float> s(lat.begin(), lat.begin() + n);
    double sum = 0;
    for (float v : s) sum += v;
    std::sort(s.begin(), s.end());
    out->mean_us = n ? sum / n : 0;
    out->p50_us = n ? s[(size_t)(0.50 * (n - 1))] : 0;
    out->p99_us = n ? s[(size_t)(0.99 * (n - 1))] : 0;
    out->max_us = n ? s[n - 1] : 0;
    g_shared = nullptr;
    return first_rc.load();
}

// FNV-1a of every row of a CSR (the expected hashes of tml_run's rows).
__attribute__((visibility("default"))) void tml_row_hashes(const uint32_t* row_offsets, const uint32_t* ids, uint32_t n,
                                                           uint64_t* out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = row_hash(ids + row_offsets[i], row_offsets[i + 1] - row_offsets[i]);
}

}  // extern "C"
