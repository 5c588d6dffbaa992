// tm_batch.cpp -- batches: tokenise (host or device), byte-level dedup, upload,
// launch of the walk, wait / capacity relaunch, the dense CSR and samples.
// The device side is tm_kernels.hip; the path is src/emqx_router.erl:127-133.
#include "tm_engine_impl.hpp"

int tm_engine::ensure_slow_scratch(tm_batch* b) {
    int rc;
    if (!b->s_waves) {
        // one wave per generic-path topic at a time, latency-bound: a
        // skewed batch (C5: ~28k rows of ~1,000 matches) needs several
        // waves per CU; idle waves exit at once (scratch ~350 KB each)
        uint32_t w = b->n < 65536 ? 64u : std::min<uint32_t>(TM_SLOW_WAVES_MAX, b->n / 32);
        b->s_waves = w;
    }
    const size_t q = (size_t)b->s_waves * b->s_qcap, o = (size_t)b->s_waves * b->s_ocap;
    if ((rc = dev_reserve(b->d_sqpar, b->c_sq, q))) return rc;
    if ((rc = dev_reserve(b->d_sqpw, b->c_sq2, q))) return rc;
    if ((rc = dev_reserve(b->d_sqmeta, b->c_sq3, q))) return rc;
    if ((rc = dev_reserve(b->d_sqkey, b->c_sq4, q))) return rc;
    if ((rc = dev_reserve(b->d_sofid, b->c_so, o))) return rc;
    if ((rc = dev_reserve(b->d_sokey, b->c_so2, o))) return rc;
    return TM_OK;
}

void tm_engine::tokenize_range(const TokView& v, uint32_t lo, uint32_t hi, std::vector<uint32_t>& slow_out) const {
    std::vector<TWord> ws;
    for (uint32_t t = lo; t < hi; ++t) {
        const uint8_t* p = v.bytes + v.offs[t];
        const size_t len = v.offs[t + 1] - v.offs[t];
        split_words(p, len, ws);
        uint32_t* out = v.words + v.toff[t];
        bool irregular = false;
        for (size_t i = 0; i < ws.size(); ++i) {
            const TWord& w = ws[i];
            const uint32_t cls = word_class(w, irregular);
            uint32_t id;
            if (w.n == 0) id = W_EMPTY;
            else if (is_plus(w)) id = W_PLUS;
            else if (is_hash(w)) id = W_HASH;
            else id = dict.find(w.p, w.n);
            out[i] = (cls << WID_BITS) | id;
        }
        uint8_t fl = 0;
        if (len > 0 && p[0] == '$') fl |= TF_DOLLAR;
        if (irregular || ws.size() > FAST_MAX_DEPTH) fl |= TF_SLOW;
        v.tflags[t] = fl;
        if (fl & TF_SLOW) slow_out.push_back(t);
    }
}

int tm_engine::count_words(const uint8_t* bytes, const uint64_t* offs, uint32_t n, uint32_t* toff, uint64_t* total) {
    uint64_t acc = 0;
    for (uint32_t t = 0; t < n; ++t) {
        toff[t] = (uint32_t)acc;
        const uint8_t* p = bytes + offs[t];
        const size_t len = offs[t + 1] - offs[t];
        acc += 1 + (uint64_t)std::count(p, p + len, (uint8_t)'/');
        if (acc > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    }
    toff[n] = (uint32_t)acc;
    *total = acc;
    return TM_OK;
}

void tm_engine::tokenize_view(const TokView& v, uint32_t n, std::vector<uint32_t>& slow_all) const {
    slow_all.clear();
    const unsigned nt = (n >= 65536) ? threads : 1;
    if (nt <= 1) {
        tokenize_range(v, 0, n, slow_all);
        return;
    }
    std::vector<std::vector<uint32_t>> slow(nt);
    std::vector<std::thread> th;
    for (unsigned i = 0; i < nt; ++i) {
        const uint32_t lo = (uint32_t)((uint64_t)n * i / nt), hi = (uint32_t)((uint64_t)n * (i + 1) / nt);
        th.emplace_back([this, &v, lo, hi, &slow, i] { tokenize_range(v, lo, hi, slow[i]); });
    }
    for (auto& x : th) x.join();
    for (auto& s : slow) slow_all.insert(slow_all.end(), s.begin(), s.end());
}

int tm_engine::tokenize(tm_batch* b) {
    const uint32_t n = b->n;
    b->h_toff.resize((size_t)n + 1);
    b->h_tflags.resize(n);
    uint64_t acc = 0;
    int rc = count_words(b->bytes.data(), b->offs.data(), n, b->h_toff.data(), &acc);
    if (rc) return rc;
    b->nwords = acc;
    b->h_words.resize(acc ? acc : 1);
    TokView v{b->bytes.data(), b->offs.data(), b->h_words.data(), b->h_toff.data(), b->h_tflags.data()};
    tokenize_view(v, n, b->h_slow);
    b->dict_size = dict.size();
    return TM_OK;
}

int tm_engine::tokenize_into(const uint8_t* bytes, const uint64_t* offs, uint32_t n, uint32_t* words, uint64_t cap,
                  uint32_t* toff, uint8_t* tflags, uint64_t* nwords) {
    uint64_t acc = 0;
    int rc = count_words(bytes, offs, n, toff, &acc);
    if (rc) return rc;
    *nwords = acc;
    if (acc > cap) return TM_EOVERFLOW;
    std::vector<uint32_t> slow;
    TokView v{bytes, offs, words, toff, tflags};
    tokenize_view(v, n, slow);
    return TM_OK;
}

int tm_engine::upload_batch(tm_batch* b) {
    int rc;
    const uint32_t n = b->n;
    if ((rc = dev_reserve(b->d_words, b->c_words, b->h_words.size()))) return rc;
    if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
    if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(b->h_slow.size(), 1)))) return rc;
    const hipStream_t S = st(b);
    HIP_OK(hipMemcpyAsync(b->d_words, b->h_words.data(), b->h_words.size() * 4, hipMemcpyHostToDevice, S));
    HIP_OK(hipMemcpyAsync(b->d_toff, b->h_toff.data(), ((size_t)n + 1) * 4, hipMemcpyHostToDevice, S));
    if (n) HIP_OK(hipMemcpyAsync(b->d_tflags, b->h_tflags.data(), n, hipMemcpyHostToDevice, S));
    if (!b->h_slow.empty())
        HIP_OK(hipMemcpyAsync(b->d_slow, b->h_slow.data(), b->h_slow.size() * 4, hipMemcpyHostToDevice, S));
    b->dev_slow = false;
    return reserve_outputs(b);
}

int tm_engine::tokenize_device(const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t* d_words, uint64_t cap,
                    uint32_t* d_toff, uint8_t* d_tflags, uint64_t* nwords, const TokStaged* st,
                    uint64_t st_base, uint64_t st_nbytes, uint64_t off_item0) {
    if (reps.empty()) return TM_ENODEV;
    int rc;
    Replica& R = *reps[0];   // the caller's device buffers are on the first replica's device
    const hipStream_t stream = R.stream;
    tm_batch* b = &R.tokb;
    const uint64_t base = st ? st_base : offsets[0], nbytes = st ? st_nbytes : offsets[n] - base;
    if (nbytes + n + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    if ((rc = sync_device(&R))) return rc;
    if ((rc = dev_reserve(b->d_bytes, b->c_bytes, nbytes + 16))) return rc;
    if ((rc = dev_reserve(b->d_boffs, b->c_boffs, (size_t)n + 1))) return rc;
    if ((rc = dev_reserve(b->d_wcount, b->c_wcount, (size_t)n + 2))) return rc;   // per tile + total
    if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
    if ((rc = dev_reserve(b->d_bsums, b->c_bsums, (size_t)scan_block_count(n) + 1))) return rc;
    if ((rc = host_reserve(b->h_total, b->ch_total, 4))) return rc;
    if (st) {
        // each staged chunk crosses as soon as it is in place; the chunks
        // are cut at the staging's own item bounds, so a chunk never waits
        // for more than the items it covers
        auto wait_item = [&](uint64_t item) {
            while (!__atomic_load_n(st->ready + item, __ATOMIC_ACQUIRE)) std::this_thread::yield();
        };
        for (uint64_t lo = base; lo < base + nbytes;) {
            const uint64_t item = lo / st->chunk_bytes, hi = std::min(base + nbytes, (item + 1) * st->chunk_bytes);
            wait_item(item);
            HIP_OK(hipMemcpyAsync(b->d_bytes + (lo - base), topics + lo, hi - lo, hipMemcpyHostToDevice, stream));
            lo = hi;
        }
        for (uint64_t lo = 0; lo <= n;) {
            const uint64_t g = off_item0 + lo, item = g / st->chunk_offs;
            const uint64_t hi = std::min<uint64_t>((uint64_t)n + 1, (item + 1) * st->chunk_offs - off_item0);
            wait_item(st->nbyte_items + item);
            HIP_OK(hipMemcpyAsync(b->d_boffs + lo, offsets + lo, (hi - lo) * 8, hipMemcpyHostToDevice, stream));
            lo = hi;
        }
        if (__atomic_load_n(st->bad, __ATOMIC_ACQUIRE)) {   // (checked before any kernel reads the offsets)
            HIP_OK(hipStreamSynchronize(stream));
            return TM_EINVAL;
        }
    } else {
        if (nbytes) HIP_OK(hipMemcpyAsync(b->d_bytes, topics + base, nbytes, hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(b->d_boffs, offsets, ((size_t)n + 1) * 8, hipMemcpyHostToDevice, stream));
    }
    if (!n) HIP_OK(hipMemsetAsync(d_toff, 0, 4, stream));
    TokArgs t{};
    t.bytes = b->d_bytes; t.offs = b->d_boffs; t.base = base; t.n = n;
    t.keys = R.d_dkey; t.tails = R.d_tail; t.dict_mask = R.d_dict_n - 1; t.arena = R.d_arena;
    t.wcount = b->d_wcount; t.tflags = d_tflags; t.toff = d_toff; t.words = d_words; t.words_cap = cap;
    t.slow_list = b->d_slow; t.d_nslow = b->d_nslow;
    t.tile_topics = tok_tile_topics(n, nbytes);
    ScanArgs ts{};
    ts.block_sums = b->d_bsums;
    HIP_OK(launch_tokenize(t, ts, b->d_nslow + 1, stream));
    HIP_OK(hipMemcpyAsync(b->h_total, b->d_nslow + 1, 4, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    *nwords = n ? b->h_total[0] : 0;
    return *nwords > cap ? TM_EOVERFLOW : TM_OK;
}

int tm_engine::prepare_tokens(tm_batch* b, const uint32_t* words, const uint32_t* toff, const uint8_t* tflags, uint32_t n,
                   uint64_t nwords, bool on_device) {
    if (nwords > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    const hipStream_t stream = b->rep ? st(b) : nullptr;   // (host-only engine: none)
    b->n = n;
    b->nwords = nwords;
    b->tokens_only = true;
    b->dev_tok = false;
    b->launched = b->done = false;
    b->bytes.clear();
    b->offs.clear();
    int rc;
    if (!on_device) {
        if (toff[0] != 0 || toff[n] != nwords) return TM_EINVAL;
        b->h_slow.clear();
        for (uint32_t t = 0; t < n; ++t) {
            const uint8_t f = tflags[t];
            if (toff[t + 1] < toff[t] || (f & ~(TF_DOLLAR | TF_SLOW))) return TM_EINVAL;
            if (toff[t + 1] - toff[t] > FAST_MAX_DEPTH && !(f & TF_SLOW)) return TM_EINVAL;
            if (f & TF_SLOW) b->h_slow.push_back(t);
        }
        b->h_words.assign(words, words + nwords);
        if (b->h_words.empty()) b->h_words.push_back(0);
        b->h_toff.assign(toff, toff + (size_t)n + 1);
        b->h_tflags.assign(tflags, tflags + n);
        if (device < 0) return TM_OK;
        return upload_batch(b);
    }
    if (device < 0) return TM_ENODEV;
    b->h_words.clear(); b->h_toff.clear(); b->h_tflags.clear(); b->h_slow.clear();
    if ((rc = dev_reserve(b->d_words, b->c_words, std::max<uint64_t>(nwords, 1)))) return rc;
    if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
    if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
    if ((rc = host_reserve(b->h_bad, b->ch_bad, 2))) return rc;
    if (nwords) HIP_OK(hipMemcpyAsync(b->d_words, words, nwords * 4, hipMemcpyDeviceToDevice, stream));
    HIP_OK(hipMemcpyAsync(b->d_toff, toff, ((size_t)n + 1) * 4, hipMemcpyDeviceToDevice, stream));
    if (n) HIP_OK(hipMemcpyAsync(b->d_tflags, tflags, n, hipMemcpyDeviceToDevice, stream));
    HIP_OK(hipMemsetAsync(b->d_nslow, 0, 2 * 4, stream));
    // toff[0] and toff[n] checked with the rest: a walk must never read past words[]
    HIP_OK(launch_token_check(b->d_toff, b->d_tflags, n, nwords, b->d_slow, b->d_nslow, b->d_nslow + 1, stream));
    HIP_OK(hipMemcpyAsync(b->h_bad, b->d_nslow, 2 * 4, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    if (b->h_bad[1] || (n == 0 && nwords != 0)) return TM_EINVAL;
    if (n == 0) {   // no thread checked toff[0] == nwords == 0
        uint32_t t0 = 0;
        HIP_OK(hipMemcpy(&t0, b->d_toff, 4, hipMemcpyDeviceToHost));
        if (t0 != 0) return TM_EINVAL;
    }
    b->dev_slow = true;
    return reserve_outputs(b);
}

int tm_engine::part_buffers(tm_batch* b, uint32_t n, uint64_t nwords, PartBuffers* out) {
    if (nwords > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    int rc;
    b->n = n;
    b->nwords = nwords;
    b->tokens_only = true;
    b->dev_tok = false;
    b->check_tokens = true;
    b->gbad = true;   // launched directly: the token check belongs to every launch
    b->launched = b->done = false;
    b->bytes.clear(); b->offs.clear();
    b->h_words.clear(); b->h_toff.clear(); b->h_tflags.clear(); b->h_slow.clear();
    if ((rc = dev_reserve(b->d_words, b->c_words, std::max<uint64_t>(nwords, 1)))) return rc;
    if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
    if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
    if ((rc = host_reserve(b->h_bad, b->ch_bad, 2))) return rc;
    b->h_bad[0] = b->h_bad[1] = 0;
    b->dev_slow = true;
    if ((rc = reserve_outputs(b))) return rc;
    out->words = b->d_words;
    out->toff = b->d_toff;
    out->tflags = b->d_tflags;
    out->words_cap = b->c_words;
    out->stream = st(b);
    out->device = b->rep->device;
    return TM_OK;
}

int tm_engine::export_batch(tm_batch* b, uint32_t* d_counts, uint32_t* d_ids, uint32_t mul, uint32_t add) {
    if (!b->done) return TM_EINVAL;
    if (int rc = ensure_dense(b)) return rc;
    const uint64_t top = (uint64_t)(nd.size() ? nd.size() - 1 : 0) * mul + add;
    if (top > 0xFFFFFFFFull) return TM_EOVERFLOW;
    HIP_OK(launch_export(b->d_rowoff, b->d_ids, b->n, b->total, d_counts, d_ids, mul, add, st(b)));
    HIP_OK(hipStreamSynchronize(st(b)));
    return TM_OK;
}

int tm_engine::reserve_hdr(tm_batch* b, size_t cap) {
    if (b->d_hdr && b->hdr_cap >= cap) return TM_OK;
    cap = std::max<size_t>(cap + cap / 4, 1024);
    uint8_t *d = nullptr, *h = nullptr;
    HIP_OK(hipMalloc((void**)&d, tm_batch::hdr_bytes(cap)));
    if (hipHostMalloc((void**)&h, tm_batch::hdr_bytes(cap), hipHostMallocDefault) != hipSuccess) {
        (void)hipFree(d);
        snprintf(last_error(), 512, "hipHostMalloc of %zu bytes failed", tm_batch::hdr_bytes(cap));
        return TM_ENOMEM;
    }
    dev_free(b->d_hdr);
    if (b->h_hdr) (void)hipHostFree(b->h_hdr);
    b->d_hdr = d;
    b->h_hdr = h;
    b->hdr_cap = cap;
    const size_t o_stats = CTRL_WORDS * 4, o_src = tm_batch::HDR_FIXED, o_count = o_src + cap * 8;
    b->d_ctrl = (uint32_t*)d; b->h_ctrl = (uint32_t*)h;
    b->d_stats = (unsigned long long*)(d + o_stats); b->h_stats = (unsigned long long*)(h + o_stats);
    b->d_src = (unsigned long long*)(d + o_src); b->h_src = (unsigned long long*)(h + o_src);
    b->d_count = (uint32_t*)(d + o_count); b->h_count = (uint32_t*)(h + o_count);
    return TM_OK;
}

int tm_engine::reserve_outputs(tm_batch* b) {
    int rc;
    const uint32_t n = b->n;
    const size_t nn = std::max<size_t>(n, 1);
    if ((rc = reserve_hdr(b, nn))) return rc;
    if ((rc = dev_reserve(b->d_rowoff, b->c_rowoff, nn + 1))) return rc;
    if ((rc = dev_reserve(b->d_bsums, b->c_bsums, (size_t)scan_block_count(n) + 1))) return rc;
    if ((rc = dev_reserve(b->d_ovf, b->c_ovf, nn))) return rc;
    if ((rc = dev_reserve(b->d_total, b->c_total, 1))) return rc;
    if ((rc = reserve_rows(b))) return rc;
    if (!b->ev0) {
        HIP_OK(hipEventCreate(&b->ev0));
        HIP_OK(hipEventCreate(&b->ev1));
        HIP_OK(hipEventCreate(&b->ev2));
        HIP_OK(hipEventCreate(&b->evt));
        HIP_OK(hipEventCreate(&b->evc0));
        HIP_OK(hipEventCreate(&b->evc1));
        HIP_OK(hipEventCreateWithFlags(&b->ev_end, hipEventDisableTiming));
        HIP_OK(hipEventCreate(&b->evq));
    }
    return TM_OK;
}

int tm_engine::reserve_rows(tm_batch* b) {
    int rc;
    const uint64_t fast =
        std::max<uint64_t>((uint64_t)match_waves(b->n, b->rep->device, qcap) * tile_topics(b->n) * row_cap, 1);
    // + a byte per entry past the rows: the emission-log variant's lanes (TM_EMIT_LOG)
    if ((rc = dev_reserve(b->d_rows, b->c_rows, fast + fast / 8 + 8))) return rc;
    if ((rc = dev_reserve(b->d_sfids, b->c_sfids, std::max<uint64_t>((uint64_t)b->n * 32, staging_min)))) return rc;
    if ((rc = dev_reserve(b->d_ids, b->c_ids, std::max<uint64_t>((uint64_t)b->n * 32, 1u << 16)))) return rc;
    if ((rc = host_reserve(b->h_total, b->ch_total, 4))) return rc;
    return TM_OK;
}

void tm_engine::dedup_topics(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n) {
    std::vector<uint64_t> h(n);
    const unsigned nt = (n >= 65536) ? threads : 1;
    auto hash_range = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t t = lo; t < hi; ++t) h[t] = hash_bytes(topics + offsets[t], offsets[t + 1] - offsets[t]);
    };
    if (nt <= 1) hash_range(0, n);
    else {
        std::vector<std::thread> th;
        for (unsigned i = 0; i < nt; ++i)
            th.emplace_back(hash_range, (uint32_t)((uint64_t)n * i / nt), (uint32_t)((uint64_t)n * (i + 1) / nt));
        for (auto& x : th) x.join();
    }
    size_t cap = 1024;
    while (cap < (size_t)n * 2) cap <<= 1;
    std::vector<uint32_t> tab(cap, 0);          // distinct index + 1
    std::vector<uint32_t> first;                 // publish index of each distinct topic
    b->row_of.resize(n);
    for (uint32_t t = 0; t < n; ++t) {
        const uint8_t* p = topics + offsets[t];
        const size_t len = offsets[t + 1] - offsets[t];
        size_t i = h[t] & (cap - 1);
        for (;;) {
            const uint32_t u = tab[i];
            if (u == 0) {
                first.push_back(t);
                tab[i] = (uint32_t)first.size();
                b->row_of[t] = (uint32_t)first.size() - 1;
                break;
            }
            const uint32_t f = first[u - 1];
            const size_t fl = offsets[f + 1] - offsets[f];
            if (h[f] == h[t] && fl == len && memcmp(topics + offsets[f], p, len) == 0) {
                b->row_of[t] = u - 1;
                break;
            }
            i = (i + 1) & (cap - 1);
        }
    }
    const uint32_t nu = (uint32_t)first.size();
    b->offs.assign((size_t)nu + 1, 0);
    uint64_t tot = 0;
    for (uint32_t u = 0; u < nu; ++u) tot += offsets[first[u] + 1] - offsets[first[u]];
    b->bytes.resize(tot);
    uint64_t o = 0;
    for (uint32_t u = 0; u < nu; ++u) {
        const uint32_t f = first[u];
        const size_t len = offsets[f + 1] - offsets[f];
        if (len) memcpy(b->bytes.data() + o, topics + offsets[f], len);
        o += len;
        b->offs[u + 1] = o;
    }
    b->n = nu;
}

int tm_engine::prepare(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n, uint32_t flags) {
    if (int rc = check_topics(offsets, n)) return rc;
    forget_launch(b);   // its previous results are gone
    b->dedup = (flags & TM_BATCH_DEDUP) != 0;
    b->n_pub = n;
    b->row_of.clear();
    b->dev_tok = false;
    b->dedup_dev = b->dedup_stale = b->rowof_host = false;
    if (device >= 0 && dev_tok) {
        b->launched = b->done = false;
        b->tokens_only = false;
        b->n = n;
        b->bytes.clear();
        b->offs.clear();
        int rc = upload_bytes(b, topics, offsets, n);
        if (rc || !b->dedup) return rc;
        // deduplicated on the device at launch, ahead of the tokeniser
        b->dedup_dev = b->dedup_stale = true;
        return reserve_dedup(b, offsets[n] - offsets[0]);
    }
    if (b->dedup) {
        dedup_topics(b, topics, offsets, n);
    } else {
        b->n = n;
        b->offs.assign(offsets, offsets + (size_t)n + 1);
        const uint64_t base = offsets[0];
        for (auto& o : b->offs) o -= base;
        b->bytes.assign(topics + base, topics + base + b->offs[n]);
    }
    b->launched = b->done = false;
    b->tokens_only = false;
    int rc = tokenize(b);
    if (rc) return rc;
    if (device < 0) return TM_OK;
    return upload_batch(b);
}

void tm_engine::drop_user_stream(tm_batch* b) {
    auto& rd = b->rep->readers;
    rd.erase(std::remove(rd.begin(), rd.end(), b), rd.end());
    if (b->own) (void)hipStreamDestroy(b->own);
    b->own = nullptr;
    b->own_user = false;
}

int tm_engine::upload_bytes(tm_batch* b, const uint8_t* topics, const uint64_t* offsets, uint32_t n) {
    int rc;
    const hipStream_t S = st(b);
    const uint64_t base = offsets[0], nbytes = offsets[n] - base;
    if (nbytes + n + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;   // u32 word offsets
    b->tok_base = base;
    if ((rc = dev_reserve(b->d_bytes, b->c_bytes, nbytes + 16))) return rc;   // +16: no tail reads past
    if ((rc = dev_reserve(b->d_boffs, b->c_boffs, (size_t)n + 1))) return rc;
    if ((rc = reserve_tokens(b, n, nbytes))) return rc;
    if (nbytes) HIP_OK(hipMemcpyAsync(b->d_bytes, topics + base, nbytes, hipMemcpyHostToDevice, S));
    HIP_OK(hipMemcpyAsync(b->d_boffs, offsets, ((size_t)n + 1) * 8, hipMemcpyHostToDevice, S));
    // the caller's buffers are only borrowed for the call; tm_match_batch
    // (and the async slots, whose inputs are their own pinned buffers)
    // wait for the whole pipeline later, so they skip this sync
    if (!upload_nosync && !b->own) HIP_OK(hipStreamSynchronize(S));
    b->in_bytes = b->d_bytes;
    b->in_offs = b->d_boffs;
    return tokens_pending(b);
}

int tm_engine::reserve_tokens(tm_batch* b, uint32_t n, uint64_t nbytes) {
    int rc;
    b->nwords = nbytes + n;                  // bound: one word per byte + 1 per topic
    if ((rc = dev_reserve(b->d_wcount, b->c_wcount, (size_t)n + 2))) return rc;   // per tile + total
    if ((rc = dev_reserve(b->d_words, b->c_words, std::max<uint64_t>(b->nwords, 1)))) return rc;
    if ((rc = dev_reserve(b->d_toff, b->c_toff, (size_t)n + 1))) return rc;
    if ((rc = dev_reserve(b->d_tflags, b->c_tflags, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_slow, b->c_slow, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_nslow, b->c_nslow, 2))) return rc;
    return TM_OK;
}

int tm_engine::reserve_dedup(tm_batch* b, uint64_t nbytes) {
    int rc;
    const size_t n = b->n;
    if (nbytes >> DD_OFF_BITS) {   // (a table slot holds a 40-bit byte offset)
        snprintf(last_error(), 512, "device dedup: batch of %llu bytes over 2^40", (unsigned long long)nbytes);
        return TM_EINVAL;
    }
    uint64_t cap = 1024;
    while (cap < (uint64_t)n + n / 2) cap <<= 1;   // load <= 2/3 when every publish is distinct
    const uint64_t old_mask = b->dtab_mask;
    b->dtab_mask = cap - 1;
    b->dd_bytes = nbytes;
    const size_t nblk = dedup_blocks((uint32_t)n);
    const size_t nb = scan_block_count((uint32_t)nblk) + 1;
    void* old_tab = b->d_dtab;
    if ((rc = dev_reserve(b->d_dtab, b->c_dtab, cap))) return rc;
    if (b->d_dtab != old_tab || old_mask != b->dtab_mask) b->dtab_dirty = true;
    if ((rc = dev_reserve(b->d_dsrow, b->c_dsrow, cap))) return rc;
    if ((rc = dev_reserve(b->d_dsmeta, b->c_dsmeta, cap))) return rc;
    if ((rc = dev_reserve(b->d_drrep, b->c_drrep, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_dbsum, b->c_dbsum, n / DD_EXPAND_TILE + 2))) return rc;   // (expansion blocks)
    if ((rc = dev_reserve(b->d_dslot, b->c_dslot, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_dbits, b->c_dbits, std::max<size_t>(nblk, 1) * (DD_TILE / 64)))) return rc;
    if ((rc = dev_reserve(b->d_dbc, b->c_dbc, nblk + 1))) return rc;
    if ((rc = dev_reserve(b->d_dbb, b->c_dbb, nblk + 1))) return rc;
    if ((rc = dev_reserve(b->d_drbs, b->c_drbs, nb))) return rc;
    if ((rc = dev_reserve(b->d_dbbs, b->c_dbbs, nb))) return rc;
    if ((rc = dev_reserve(b->d_rowof, b->c_rowof, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_cbytes, b->c_cbytes, nbytes + 32))) return rc;   // (the tokeniser's 16-B windows)
    if ((rc = dev_reserve(b->d_coffs, b->c_coffs, n + 1))) return rc;
    if ((rc = dev_reserve(b->d_dd, b->c_dd, 2))) return rc;
    if ((rc = dev_reserve(b->d_pcount, b->c_pcount, std::max<size_t>(n, 1)))) return rc;
    if ((rc = dev_reserve(b->d_psrc, b->c_psrc, std::max<size_t>(n, 1)))) return rc;
    if (!b->evd) {
        HIP_OK(hipEventCreate(&b->evd));
        HIP_OK(hipEventCreate(&b->evx0));
        HIP_OK(hipEventCreate(&b->evx1));
    }
    return TM_OK;
}

DedupArgs tm_engine::dedup_args(tm_batch* b) const {
    DedupArgs d{};
    d.bytes = b->in_bytes; d.offs = b->in_offs; d.base = b->tok_base; d.n = b->n_pub;
    d.table = b->d_dtab; d.mask = b->dtab_mask;
    d.slot = b->d_dslot; d.repbits = b->d_dbits; d.bcount = b->d_dbc; d.bbytes = b->d_dbb;
    d.rbs = b->d_drbs; d.bbs = b->d_dbbs; d.srow = b->d_dsrow; d.rrep = b->d_drrep;
    d.smeta = b->d_dsmeta;
    d.row_of = b->d_rowof; d.cbytes = b->d_cbytes; d.coffs = b->d_coffs; d.dd = b->d_dd;
    d.ctrl = b->d_ctrl; d.count = b->d_count; d.src = b->d_src; d.pcount = b->d_pcount; d.psrc = b->d_psrc;
    d.stats = b->d_stats;
    d.bsum = b->d_dbsum;
    d.weak_hash = kn.dedup_weak_hash ? 1u : 0u;
    return d;
}

// the dedup passes (no table clear: clear_dedup_table, outside any capture)
int tm_engine::enqueue_dedup(tm_batch* b, hipStream_t S) {
    const DedupArgs d = dedup_args(b);
    if (!d.n) HIP_OK(hipMemsetAsync(b->d_dd, 0, 8, S));   // (no compact kernel: zero rows)
    const uint32_t nblk = dedup_blocks(d.n);
    ScanArgs rs{}, bs{};
    rs.count = d.bcount; rs.row_off = d.bcount; rs.block_sums = b->d_drbs; rs.n = nblk;   // (in place)
    bs.count = d.bbytes; bs.row_off = d.bbytes; bs.block_sums = b->d_dbbs; bs.n = nblk;
    HIP_OK(launch_dedup(d, rs, bs, S));
    return TM_OK;
}

// a dirty table (new, or a pass whose expansion was not waited for) is
// cleared before the next pass; a clean one is zero already
int tm_engine::clear_dedup_table(tm_batch* b, hipStream_t S) {
    if (b->dtab_dirty) HIP_OK(hipMemsetAsync(b->d_dtab, 0, (b->dtab_mask + 1) * 8, S));
    b->dtab_dirty = true;   // until this pass's expansion has been waited for
    return TM_OK;
}

int tm_engine::tokens_pending(tm_batch* b) {
    b->h_words.clear(); b->h_toff.clear(); b->h_tflags.clear(); b->h_slow.clear();
    b->dev_tok = true;
    b->tok_dict = ~0ull;
    b->dev_slow = true;
    return reserve_outputs(b);
}

int tm_engine::upload_packed(tm_batch* b, const uint8_t* blk, uint32_t n, uint64_t nbytes) {
    int rc;
    const size_t head = packed_head(n);
    if (nbytes + n + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    b->dedup = false;
    b->bounded = false;
    b->n_pub = n;
    b->row_of.clear();
    b->launched = b->done = false;
    b->tokens_only = false;
    b->n = n;
    b->bytes.clear();
    b->offs.clear();
    b->tok_base = 0;
    if ((rc = reserve_tokens(b, n, nbytes))) return rc;
    if ((rc = dev_reserve(b->d_in, b->c_in, head + nbytes + 16))) return rc;   // +16: no tail reads past
    HIP_OK(hipMemcpyAsync(b->d_in, blk, head + nbytes, hipMemcpyHostToDevice, b->own));
    b->in_offs = reinterpret_cast<const uint64_t*>(b->d_in);
    b->in_bytes = b->d_in + head;
    return tokens_pending(b);
}

// An async slot's bounded batch (see tm_batch::bounded): sized for `bound`
// topics and `bytes_cap` bytes; its offsets, bytes and count live in mapped
// pinned memory (d_offs / d_bytes / d_n, device pointers), written by the
// slot before every launch.  Called before every launch (cheap once sized):
// the tokens are made fresh each time.
int tm_engine::prepare_bounded(tm_batch* b, uint32_t bound, uint64_t bytes_cap, const uint64_t* d_offs,
                               const uint8_t* d_bytes, uint32_t* d_n) {
    int rc;
    if (bytes_cap + bound + 1 > 0xFFFFFFF0ull) return TM_EOVERFLOW;
    b->dedup = b->dedup_dev = false;
    b->n_pub = bound;
    b->n = bound;
    b->row_of.clear();
    b->launched = b->done = false;
    b->tokens_only = false;
    b->bytes.clear();
    b->offs.clear();
    b->tok_base = 0;
    if ((rc = reserve_tokens(b, bound, bytes_cap))) return rc;
    b->in_offs = d_offs;
    b->in_bytes = d_bytes;
    b->d_nb = d_n;
    b->bounded = true;
    return tokens_pending(b);
}

// A captured deduplicated batch replayed: its timing events are recorded on
// the stream around the graph (an event record inside that capture is refused
// by the runtime), so the replay's whole span is its walk time.
hipError_t tm_engine::graph_replay(tm_batch* b, hipStream_t S) {
    hipError_t e;
    if (b->dedup_timed && (e = hipEventRecord(b->evd, S)) != hipSuccess) return e;
    if ((e = hipEventRecord(b->ev0, S)) != hipSuccess) return e;
    if ((e = hipGraphLaunch(b->gexec, S)) != hipSuccess) return e;
    if ((e = hipEventRecord(b->ev1, S)) != hipSuccess) return e;
    if ((e = hipEventRecord(b->ev2, S)) != hipSuccess) return e;
    ++graph_launches;
    return hipSuccess;
}

int tm_engine::launch(tm_batch* b, bool csr) {
    if (reps.empty()) return TM_ENODEV;
    int rc;
    Replica& R = *b->rep;
    const hipStream_t S = st(b);
    if (!b->tokens_only && !b->dev_tok && b->dict_size != dict.size()) {   // new words since tokenisation
        if ((rc = tokenize(b))) return rc;
        if ((rc = upload_batch(b))) return rc;
    }
    if (csr) HIP_OK(hipEventRecord(b->evq, S));   // (before the delta upload and the waits below)
    if ((rc = sync_device(&R))) return rc;
    if (b->own && b->seen_upload != R.upload_seq) {   // trie deltas still in flight on the replica stream land first
        HIP_OK(hipStreamWaitEvent(S, R.ev_sync, 0));
        b->seen_upload = R.upload_seq;
    }
    if ((rc = ensure_slow_scratch(b))) return rc;
    if (checked) {
        if ((rc = dev_reserve(R.d_dbg, R.c_dbg, 8))) return rc;
        if ((rc = host_reserve(R.h_dbg, R.ch_dbg, 8))) return rc;
        HIP_OK(hipMemsetAsync(R.d_dbg, 0, 8 * 4, S));
    }
    // A device-deduplicated batch: fresh bytes are deduplicated first, and
    // only the rows are tokenised (again when the dictionary grew) and
    // walked.  The rows are counted on the device, so the tokeniser and
    // the walk are sized for every publish (the bound) and read the count
    // there; wait() sets n to the rows.
    const bool dedup_now = b->dedup_dev && b->dedup_stale;
    const bool tokenize_now = b->dev_tok && (b->tok_dict != dict.size() || dedup_now);
    if (b->dedup_dev) b->n = b->n_pub;
    b->dedup_timed = dedup_now && csr;
    const bool graph = csr && !checked && !tokenize_now && use_graphs && !b->gbad && b->n <= GRAPH_MAX &&
                       !b->dedup_dev;
    // a fresh device-deduplicated batch (C5: every launch) replays its whole
    // sequence -- dedup, tokeniser, walk, expand, read-back -- as one captured
    // graph: ~25 enqueues cost ~0.2 ms of host time per launch otherwise
    const bool dgraph = csr && !checked && use_graphs && !b->gbad && b->dedup_dev && dedup_now && tokenize_now &&
                        !b->check_tokens;
    b->tok_timed = tokenize_now && csr;
    TokArgs t{};
    ScanArgs ts{};
    if (tokenize_now) {
        b->tok_dict = dict.size();
        t.zero = reinterpret_cast<uint32_t*>(b->d_hdr);   // the tokeniser's first kernel clears ctrl + stats
        t.zero_words = tm_batch::HDR_FIXED / 4;
        t.bytes = b->in_bytes; t.offs = b->in_offs; t.base = b->tok_base; t.n = b->n;
        t.keys = R.d_dkey; t.tails = R.d_tail; t.dict_mask = R.d_dict_n - 1; t.arena = R.d_arena;
        t.wcount = b->d_wcount; t.tflags = b->d_tflags; t.toff = b->d_toff; t.words = b->d_words;
        t.words_cap = b->c_words;
        t.slow_list = b->d_slow; t.d_nslow = b->d_nslow;
        t.tile_topics = tok_tile_topics(b->n, b->nwords - b->n);   // nwords = bytes + topics (reserve_tokens)
        t.d_n = nullptr;
        if (b->dedup_dev) {   // the rows' bytes, compacted by the dedup pass
            t.bytes = b->d_cbytes; t.offs = b->d_coffs; t.base = 0; t.d_n = b->d_dd;
        }
        if (b->bounded) t.d_n = b->d_nb;   // (sized for the bound, counted in pinned memory)
        ts.block_sums = b->d_bsums;
    }
    MatchArgs a{};
    a.slots = R.d_slots;
    a.nbuckets = nbuckets();
    // (a bound on the probe run, not the exact max_disp: a longer run stops
    // at its first bucket with a free last slot all the same, and a value
    // that changes only at these steps keeps the captured launch graphs of
    // churned batches valid)
    a.max_probe = max_disp <= 4 ? 4 : max_disp <= 8 ? 8 : max_disp <= 16 ? 16 : max_disp <= 48 ? 48 : max_disp;
    a.root = root_rec();
    a.foff = R.d_foff; a.flen = R.d_flen; a.fbytes = R.d_fbytes;
    a.words = b->d_words; a.toff = b->d_toff; a.tflags = b->d_tflags; a.n = b->n;
    a.slow_list = b->d_slow; a.n_slow = b->dev_slow ? 0u : (uint32_t)b->h_slow.size();
    a.d_nslow = b->dev_slow ? b->d_nslow : nullptr;
    a.d_n = b->dedup_dev ? b->d_dd : b->bounded ? b->d_nb : nullptr;   // the rows, counted by the dedup pass
    a.count = b->d_count; a.src = b->d_src; a.rows = b->d_rows; a.row_cap = row_cap;
    a.grid = match_waves(b->n, R.device, qcap);
    a.tile_topics = tile_topics(b->n);
    a.qcap = qcap;
    {   // the first static_frac of the tiles round-robin, the tail by per-XCD tickets
        const uint64_t ntiles = ((uint64_t)b->n + a.tile_topics - 1) / a.tile_topics;
        a.static_rounds = std::max<uint32_t>(1, (uint32_t)(static_frac * (double)ntiles / std::max(a.grid, 1u)));
    }
    if ((uint64_t)a.grid * a.tile_topics * row_cap > b->c_rows) {
        snprintf(last_error(), 512, "emission rows sized for fewer waves than the launch");
        return TM_EIO;
    }
    a.sfids = b->d_sfids; a.sfids_cap = std::min<uint64_t>(b->c_sfids, MAX_RESULT);
    a.rcap = region_cap(a.sfids_cap, b->one_region);
    a.sgmask = b->one_region ? 0u : TICKET_GROUPS - 1;
    a.xg = b->d_ctrl + XG_WORD;
    a.ctrl = b->d_ctrl; a.ovf_list = b->d_ovf; a.ovf_cap = (uint32_t)std::min<size_t>(b->c_ovf, 0xFFFFFFF0ull);
    a.stats = b->d_stats;
    // a walk of many waves writes per-wave sums (one reduce kernel after it);
    // a small one adds them atomically -- a few dozen same-line atomics cost
    // less than one more launch on the per-publish path
    if (a.grid >= WSTATS_MIN_WAVES) {
        if ((rc = dev_reserve(b->d_wstats, b->c_wstats, (size_t)a.grid * WSTATS))) return rc;
        a.wstats = b->d_wstats;
    }
    a.s_qparent = b->d_sqpar; a.s_qpw = b->d_sqpw; a.s_qmeta = b->d_sqmeta; a.s_qkey = b->d_sqkey;
    a.s_ofid = b->d_sofid; a.s_okey = b->d_sokey;
    a.s_qcap = b->s_qcap; a.s_ocap = b->s_ocap; a.s_waves = b->s_waves; a.s_lcap = kn.slow_lds;
    a.nwords = (uint32_t)std::max<uint64_t>(b->nwords, 1);
    a.nslots = (uint32_t)slots.size();
    // (bounds of the checked build only: left 0 otherwise, so churn does not
    // change the launch's arguments and a captured graph stays valid)
    a.nnodes = checked ? (uint32_t)nd.size() : 0u;
    a.nfbytes = checked ? fbytes.size() : 0u;
    a.dbg = checked ? R.d_dbg : nullptr;
    ScanArgs s{};
    s.count = b->d_count; s.src = b->d_src;
    s.sfids = b->d_sfids; s.sfids_cap = std::min<uint64_t>(b->c_sfids, MAX_RESULT);
    s.row_off = b->d_rowoff; s.ids = b->d_ids; s.block_sums = b->d_bsums;
    s.n = b->n; s.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull); s.ctrl = b->d_ctrl;
    s.dbg = checked ? R.d_dbg : nullptr;
    b->end_recorded = false;
    b->graphed = false;
    b->dense_enq = false;
    // Everything the launch puts on the stream (cap: captured into a graph,
    // without the timing events -- the runtime refuses event records inside this
    // capture, so graph_replay records them around the whole graph; csr_too:
    // the read-back of ctrl + stats as well)
    auto enqueue = [&](bool cap, bool csr_too) -> hipError_t {
        hipError_t e;
        if (!tokenize_now && (e = hipMemsetAsync(b->d_hdr, 0, tm_batch::HDR_FIXED, S)) != hipSuccess) return e;
        if (dedup_now) {
            if (b->dedup_timed && !cap && (e = hipEventRecord(b->evd, S)) != hipSuccess) return e;
            if (enqueue_dedup(b, S) != TM_OK) return hipErrorUnknown;
        }
        if (b->tok_timed && !cap && (e = hipEventRecord(b->evt, S)) != hipSuccess) return e;
        if (tokenize_now && (e = launch_tokenize(t, ts, b->d_nslow + 1, S)) != hipSuccess) return e;
        if (b->check_tokens && b->n) {
            if ((e = hipMemsetAsync(b->d_nslow, 0, 2 * 4, S)) != hipSuccess) return e;
            if ((e = launch_token_check(b->d_toff, b->d_tflags, b->n, b->nwords, b->d_slow, b->d_nslow,
                                        b->d_nslow + 1, S)) != hipSuccess)
                return e;
        }
        e = launch_match(a, S, csr && !cap ? b->ev0 : nullptr, csr && !cap ? b->ev1 : nullptr, checked, 0u);
        if (e != hipSuccess) return e;
        if (b->dedup_dev) {   // every publish's row (count, start) + the delivered matches
            if (!cap && (e = hipEventRecord(b->evx0, S)) != hipSuccess) return e;
            if ((e = launch_dedup_expand(dedup_args(b), S)) != hipSuccess) return e;
            if (!cap && (e = hipEventRecord(b->evx1, S)) != hipSuccess) return e;
        }
        if (cap && csr_too)   // (ev2 is recorded after the graph's launch)
            return hipMemcpyAsync(b->h_hdr, b->d_hdr, tm_batch::HDR_FIXED, hipMemcpyDeviceToHost, S);
        return csr_too ? enqueue_csr(b, s, S) : hipSuccess;
    };
    int grc = 1;
    if (graph) {   // a repeated tokenised batch: memset + walk + read-back replayed
        grc = launch_graph(b, a, s, S);
        if (grc != 1 && grc) return grc;
    }
    bool csr_done = false;
    if (dedup_now && (rc = clear_dedup_table(b, S))) return rc;   // (outside the capture below)
    if (dgraph) {
        const DedupArgs d = dedup_args(b);
        std::vector<uint8_t> key(sizeof t + sizeof ts + sizeof a + sizeof s + sizeof d);
        uint8_t* k = key.data();
        memcpy(k, &t, sizeof t); k += sizeof t;
        memcpy(k, &ts, sizeof ts); k += sizeof ts;
        memcpy(k, &a, sizeof a); k += sizeof a;
        memcpy(k, &s, sizeof s); k += sizeof s;
        memcpy(k, &d, sizeof d);
        if (b->gexec && b->gkey == key) {
            HIP_OK(graph_replay(b, S));
            grc = 0;
        } else {
            if (kn.par_trace && b->gkey.size() == key.size()) {   // which arguments changed (offsets per struct)
                const size_t ends[5] = {sizeof t, sizeof t + sizeof ts, sizeof t + sizeof ts + sizeof a,
                                        sizeof t + sizeof ts + sizeof a + sizeof s, key.size()};
                const char* names[5] = {"tok", "tscan", "match", "scan", "dedup"};
                fprintf(stderr, "[graph key miss]");
                size_t st = 0;
                for (int q = 0; q < 5; ++q) {
                    for (size_t i = st; i < ends[q]; i += 4)
                        if (memcmp(&key[i], &b->gkey[i], std::min<size_t>(4, ends[q] - i)))
                            fprintf(stderr, " %s+%zu", names[q], i - st);
                    st = ends[q];
                }
                fprintf(stderr, "\n");
            }
            if (b->gexec) (void)hipGraphExecDestroy(b->gexec);
            b->gexec = nullptr;
            if (b->gkey == key) {   // the second launch with these arguments: capture them
                hipGraph_t g = nullptr;
                if (hipStreamBeginCapture(S, hipStreamCaptureModeRelaxed) == hipSuccess) {
                    const hipError_t e = enqueue(true, true);
                    const hipError_t e2 = hipStreamEndCapture(S, &g);
                    if (e == hipSuccess && e2 == hipSuccess && g &&
                        hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0) == hipSuccess) {
                        (void)hipGraphDestroy(g);
                        HIP_OK(graph_replay(b, S));
                        grc = 0;
                    } else {
                        if (g) (void)hipGraphDestroy(g);
                        (void)hipGetLastError();
                        b->gexec = nullptr;
                        b->gbad = true;   // the direct way from now on
                    }
                } else {
                    (void)hipGetLastError();
                    b->gbad = true;
                }
            }
            b->gkey.swap(key);
        }
        csr_done = grc == 0;
        if (csr_done) { b->tok_timed = false; b->graphed = true; }   // (replayed: see the enqueue above)
    }
    // A bounded batch (an async slot's): the same arguments every launch, so
    // from its second launch on the tokeniser, the walk, the generic path and
    // the slot's tail (export + flag) replay as one captured graph: ~10
    // enqueues of ~3 us host time each become one
    b->tail_done = false;
    if (!csr && b->bounded && b->tail && tokenize_now && use_graphs && !checked && !b->gbad && grc == 1) {
        std::vector<uint8_t> key(sizeof t + sizeof ts + sizeof a + sizeof s + b->tail_key.size());
        uint8_t* k = key.data();
        memcpy(k, &t, sizeof t); k += sizeof t;
        memcpy(k, &ts, sizeof ts); k += sizeof ts;
        memcpy(k, &a, sizeof a); k += sizeof a;
        memcpy(k, &s, sizeof s); k += sizeof s;
        if (!b->tail_key.empty()) memcpy(k, b->tail_key.data(), b->tail_key.size());
        if (b->gexec && b->gkey == key) {
            HIP_OK(hipGraphLaunch(b->gexec, S));
            ++graph_launches;
            grc = 0;
        } else {
            if (b->gexec) (void)hipGraphExecDestroy(b->gexec);
            b->gexec = nullptr;
            if (b->gkey == key) {   // the second launch with these arguments: capture them
                hipGraph_t g = nullptr;
                if (hipStreamBeginCapture(S, hipStreamCaptureModeRelaxed) == hipSuccess) {
                    hipError_t e = enqueue(true, false);
                    if (e == hipSuccess) e = b->tail(S);
                    const hipError_t e2 = hipStreamEndCapture(S, &g);
                    if (e == hipSuccess && e2 == hipSuccess && g &&
                        hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0) == hipSuccess) {
                        (void)hipGraphDestroy(g);
                        HIP_OK(hipGraphLaunch(b->gexec, S));
                        ++graph_launches;
                        grc = 0;
                    } else {
                        if (g) (void)hipGraphDestroy(g);
                        (void)hipGetLastError();
                        b->gexec = nullptr;
                        b->gbad = true;   // the direct way from now on
                    }
                } else {
                    (void)hipGetLastError();
                    b->gbad = true;
                }
            }
            b->gkey.swap(key);
        }
        b->tail_done = grc == 0;
    }
    if (grc == 1) {
        const hipError_t e = enqueue(false, false);
        if (e != hipSuccess) {
            snprintf(last_error(), 512, "%s at launch (%s)", hipGetErrorString(e), __FILE_NAME__);
            return TM_EIO;
        }
    }
    if (dedup_now) {   // (enqueued: a failed launch dedups again next time)
        b->dedup_stale = false;
        b->rowof_host = false;
    }
    note_launch(b);
    b->launched = true;
    b->done = false;
    b->dense = false;
    b->csr = csr;
    if (!csr) return TM_OK;   // the async slot enqueues its read-back and event
    if (grc == 1 && !csr_done) HIP_OK(enqueue_csr(b, s, S));   // (a graph holds it)
    b->scan_args = s;
    if (b->check_tokens) HIP_OK(hipMemcpyAsync(b->h_bad, b->d_nslow, 2 * 4, hipMemcpyDeviceToHost, S));
    if (checked) HIP_OK(hipMemcpyAsync(R.h_dbg, R.d_dbg, 8 * 4, hipMemcpyDeviceToHost, S));
    if (b->oneshot || b->eager_dense) {
        if ((rc = enqueue_dense_tail(b, S))) return rc;
        b->dense_enq = true;
    }
    HIP_OK(hipEventRecord(b->ev_end, S));
    b->end_recorded = true;
    return TM_OK;
}

hipError_t tm_engine::enqueue_csr(tm_batch* b, const ScanArgs& s, hipStream_t S, unsigned ev_flags) {
    (void)s;
    hipError_t e;
    if ((e = hipEventRecordWithFlags(b->ev2, S, ev_flags)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(b->h_hdr, b->d_hdr, tm_batch::HDR_FIXED, hipMemcpyDeviceToHost, S)) != hipSuccess)
        return e;   // ctrl + stats
    return hipSuccess;
}

int tm_engine::enqueue_dense_tail(tm_batch* b, hipStream_t S) {
    int rc;
    ScanArgs s = b->scan_args;
    s.ids = b->d_ids;
    s.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull);
    b->dense_cap = s.ids_cap;
    if (!b->oneshot) {   // the dense CSR only (the pipelined tm_match_batch copies it by DMA)
        HIP_OK(hipEventRecord(b->evc0, S));
        HIP_OK(launch_scan(s, S, b->d_total));
        HIP_OK(launch_finalize(s, S, false));
        HIP_OK(hipEventRecord(b->evc1, S));
        return TM_OK;
    }
    if ((rc = host_reserve_coherent(b->h_xrow, b->c_xrow, ((size_t)b->n + 1) * 4))) return rc;
    if ((rc = host_reserve_coherent(b->h_xids, b->c_xids, std::max<size_t>(b->c_ids, 1) * 4))) return rc;
    void *d_row = nullptr, *d_ids = nullptr;
    HIP_OK(hipHostGetDevicePointer(&d_row, b->h_xrow, 0));
    HIP_OK(hipHostGetDevicePointer(&d_ids, b->h_xids, 0));
    b->x_cap = std::min<uint64_t>(s.ids_cap, b->c_xids / 4);
    HIP_OK(hipEventRecord(b->evc0, S));
    HIP_OK(launch_scan(s, S, b->d_total));
    HIP_OK(launch_finalize(s, S, false));
    HIP_OK(hipEventRecord(b->evc1, S));
    HIP_OK(launch_csr_to_host(b->d_rowoff, b->d_ids, b->n, b->d_total, b->x_cap, static_cast<uint32_t*>(d_row),
                              static_cast<uint32_t*>(d_ids), S));
    return TM_OK;
}

int tm_engine::oneshot_result(tm_batch* b, tm_result* out) {
    const uint32_t* row = reinterpret_cast<const uint32_t*>(b->h_xrow);
    if (!b->oneshot || !b->done || b->total > b->x_cap || row[b->n] != b->total || row[0] != 0) return 1;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, b->evc0, b->evc1);
    b->st.ms_csr = ms;
    b->dense = true;
    out->n_topics = b->n;
    out->n_matches = b->total;
    out->row_offsets = row;
    out->filter_ids = reinterpret_cast<const uint32_t*>(b->h_xids);
    return TM_OK;
}

int tm_engine::ensure_dense(tm_batch* b) {
    if (!b->done) return TM_EINVAL;
    if (b->dense) return TM_OK;
    const hipStream_t S = st(b);
    int rc;
    if (b->total > b->c_ids) {
        if ((rc = dev_reserve(b->d_ids, b->c_ids, (size_t)b->total + b->total / 4))) return rc;
    }
    b->scan_args.ids = b->d_ids;
    b->scan_args.ids_cap = (uint32_t)std::min<size_t>(b->c_ids, 0xFFFFFFF0ull);
    HIP_OK(hipEventRecord(b->evc0, S));
    HIP_OK(launch_scan(b->scan_args, S, b->d_total));
    HIP_OK(launch_finalize(b->scan_args, S, checked));
    HIP_OK(hipEventRecord(b->evc1, S));
    HIP_OK(hipMemcpyAsync(b->h_total, b->d_total, 4, hipMemcpyDeviceToHost, S));
    HIP_OK(hipStreamSynchronize(S));
    if (b->h_total[0] != b->total) {
        snprintf(last_error(), 512, "inconsistent CSR: scanned %u entries, kernel count %llu", b->h_total[0],
                 (unsigned long long)b->total);
        return TM_EIO;
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, b->evc0, b->evc1);
    b->st.ms_csr = ms;
    b->dense = true;
    return TM_OK;
}

int tm_engine::launch_graph(tm_batch* b, const MatchArgs& a, const ScanArgs& s, hipStream_t S) {
    std::vector<uint8_t> key(sizeof(MatchArgs) + sizeof(ScanArgs));
    memcpy(key.data(), &a, sizeof a);
    memcpy(key.data() + sizeof a, &s, sizeof s);
    if (!b->gexec || b->gkey != key) {
        if (b->gexec) (void)hipGraphExecDestroy(b->gexec);
        b->gexec = nullptr;
        if (b->gkey != key) {   // captured only when a launch repeats the last one's arguments
            b->gkey.swap(key);
            return 1;
        }
        hipGraph_t g = nullptr;
        if (hipStreamBeginCapture(S, hipStreamCaptureModeRelaxed) != hipSuccess) {
            (void)hipGetLastError();
            b->gbad = true;
            return 1;
        }
        hipError_t e = hipMemsetAsync(b->d_hdr, 0, tm_batch::HDR_FIXED, S);
        // timing events as external nodes: every replay re-records them
        if (e == hipSuccess) e = launch_match(a, S, b->ev0, b->ev1, false, hipEventRecordExternal);
        if (e == hipSuccess) e = enqueue_csr(b, s, S, hipEventRecordExternal);
        const hipError_t e2 = hipStreamEndCapture(S, &g);
        if (e != hipSuccess || e2 != hipSuccess || !g ||
            hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0) != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            b->gexec = nullptr;
            b->gbad = true;
            return 1;
        }
        (void)hipGraphDestroy(g);
        b->gkey.swap(key);
    }
    HIP_OK(hipGraphLaunch(b->gexec, S));
    ++graph_launches;
    return TM_OK;
}

int tm_engine::check_ctrl(const uint32_t* ctrl, const unsigned long long* stats, uint32_t* err, uint64_t* need,
               uint64_t* staged_out) {
    *err = ctrl[CTRL_ERR];
    uint64_t staged = 0, top = 0;
    for (uint32_t g = 0; g < TICKET_GROUPS; ++g) {
        const uint64_t t = xg_top_read(ctrl, g);
        staged += t;
        top = std::max(top, t);
    }
    *need = top * TICKET_GROUPS;   // staging capacity that holds every region's reservation
    if (staged_out) *staged_out = staged;
    const uint64_t nmatch = stats[ST_MATCHES];
    // a CSR with u32 offsets cannot hold more (tm_result): refuse, never wrap
    if ((*err & ERR_CSR_RANGE) || staged > result_limit || nmatch > result_limit) {
        snprintf(last_error(), 512, "batch result too large: %llu staged / %llu matched > limit %llu",
                 (unsigned long long)staged, (unsigned long long)nmatch, (unsigned long long)result_limit);
        return TM_EOVERFLOW;
    }
    return TM_OK;
}

int tm_engine::grow_for(tm_batch* b, uint32_t err, uint64_t need, uint64_t staged) {
    if (err & ERR_STAGING) {
        // per-group regions of the largest group's size: unless that exceeds
        // the limit while the batch as a whole fits (skew concentrated in one
        // walk group) -- then one region for all groups, sized by the total
        const uint64_t limit = std::min<uint64_t>(MAX_RESULT, result_limit + 1024);
        if (!b->one_region && need + need / 4 + 1024 > limit && staged <= result_limit) b->one_region = true;
        if (b->one_region) need = staged;
        int rc = dev_reserve(b->d_sfids, b->c_sfids, std::min<uint64_t>(need + need / 4 + 1024, limit));
        if (rc) return rc;
    }
    if (err & ERR_SLOW_SCRATCH) {
        b->s_qcap *= 4;
        b->s_ocap *= 4;
    }
    return TM_OK;
}

void tm_engine::fill_stats(tm_batch* b) {
    float ms_match = 0, ms_total = 0, ms_tok = 0, ms_dd = 0, ms_x = 0;
    (void)hipEventElapsedTime(&ms_match, b->ev0, b->ev1);
    (void)hipEventElapsedTime(&ms_total, b->ev0, b->ev2);
    if (b->tok_timed) (void)hipEventElapsedTime(&ms_tok, b->evt, b->ev0);
    if (b->dedup_timed) (void)hipEventElapsedTime(&ms_dd, b->evd, b->tok_timed ? b->evt : b->ev0);
    if (b->dedup_dev && !b->graphed) (void)hipEventElapsedTime(&ms_x, b->evx0, b->evx1);
    b->st.ms_tokenize = ms_tok;
    b->st.ms_dedup = ms_dd;
    b->st.ms_expand = ms_x;
    b->st.publishes = b->dedup ? b->n_pub : b->n;
    float ms_q = 0;
    (void)hipEventElapsedTime(&ms_q, b->evq, b->dedup_timed ? b->evd : b->tok_timed ? b->evt : b->ev0);
    b->st.ms_queue = ms_q;
    b->st.ms_csr = 0;   // set by ensure_dense
    b->st.topics = b->n;
    b->st.visits = b->h_stats[ST_VISITS];
    b->st.hash_hits = b->h_stats[ST_HASH];
    b->st.words = b->h_stats[ST_WORDS];
    b->st.matches = b->h_stats[ST_MATCHES];
    b->st.slow_topics = b->h_stats[ST_SLOW];
    b->st.probes = b->h_stats[ST_PROBES];
    b->st.iterations = b->h_stats[ST_ITERS];
    b->st.overflow_tiles = b->h_ctrl[CTRL_NOVF];
    b->st.ms_match = ms_match;
    b->st.ms_total = ms_total;
    b->total = b->st.matches;
    b->st.delivered = b->dedup_dev ? b->h_stats[ST_DELIVERED] : b->st.matches;
}

int tm_engine::wait(tm_batch* b, bool drained, uint32_t* relaunched) {
    if (!b->launched) return TM_EINVAL;
    const hipStream_t S = st(b);
    if (!b->csr) {   // an async launch stopped after the walk: redo it the CSR way
        int rc = launch(b, true);
        if (rc) return rc;
        drained = false;
    }
    for (int attempt = 0;; ++attempt) {
        if (!drained || attempt) {
            if (b->end_recorded) HIP_OK(hipEventSynchronize(b->ev_end));
            else HIP_OK(hipStreamSynchronize(S));
        }
        if (attempt && relaunched) ++*relaunched;
        if (b->dedup_dev) {   // the walk's rows: the distinct publishes counted by the dedup pass
            b->n = b->h_ctrl[CTRL_NROWS];
            b->scan_args.n = b->n;
        }
        if (b->check_tokens && b->n && b->h_bad[1]) {
            snprintf(last_error(), 512, "token batch failed the device check (word offsets or flags)");
            return TM_EINVAL;
        }
        const uint32_t* h_dbg = b->rep->h_dbg;
        if (checked && h_dbg[0]) {
            snprintf(last_error(), 512, "bounds check %u failed: index %u bound %u (count %u, extra %u)",
                     h_dbg[0], h_dbg[1], h_dbg[2], h_dbg[3], h_dbg[4]);
            return TM_EIO;
        }
        uint32_t err;
        uint64_t need, staged;
        int rc = check_ctrl(b->h_ctrl, b->h_stats, &err, &need, &staged);
        if (rc) return rc;
        if (!err) break;
        if (attempt >= 6) {
            snprintf(last_error(), 512, "capacity misses did not settle after %d relaunches (err %#x, %llu staged)",
                     attempt, err, (unsigned long long)staged);
            return TM_EOVERFLOW;
        }
        if ((rc = grow_for(b, err, need, staged))) return rc;
        if ((rc = launch(b))) return rc;
    }
    fill_stats(b);
    b->done = true;
    if (b->dedup_dev) b->dtab_dirty = false;   // (its expansion cleared the claimed slots)
    // (dense_enq, not eager_dense: the pipelined caller clears eager_dense
    // right after launch, while the tail it asked for is already queued)
    b->dense = b->dense_enq && !b->oneshot && b->total <= b->dense_cap;
    if (b->dense) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, b->evc0, b->evc1);
        b->st.ms_csr = ms;
    }
    return TM_OK;
}

int tm_engine::result(tm_batch* b, tm_result* out) {
    if (!b->done) return TM_EINVAL;
    int rc;
    if ((rc = ensure_dense(b))) return rc;
    const hipStream_t S = st(b);
    // the match count is known since wait(): both copies go out behind one sync
    const uint64_t total = b->total;
    if (total > b->c_ids) {
        snprintf(last_error(), 512, "inconsistent CSR: kernel count %llu, capacity %zu",
                 (unsigned long long)total, b->c_ids);
        return TM_EIO;
    }
    if ((rc = host_reserve(b->h_rowoff, b->ch_rowoff, (size_t)b->n + 1))) return rc;
    if ((rc = host_reserve(b->h_ids, b->ch_ids, std::max<uint64_t>(total, 1)))) return rc;
    HIP_OK(hipMemcpyAsync(b->h_rowoff, b->d_rowoff, ((size_t)b->n + 1) * 4, hipMemcpyDeviceToHost, S));
    if (total) HIP_OK(hipMemcpyAsync(b->h_ids, b->d_ids, total * 4, hipMemcpyDeviceToHost, S));
    HIP_OK(hipStreamSynchronize(S));
    if (b->h_rowoff[b->n] != total) {
        snprintf(last_error(), 512, "inconsistent CSR: row offsets end at %u, kernel count %llu",
                 b->h_rowoff[b->n], (unsigned long long)total);
        return TM_EIO;
    }
    out->n_topics = b->n;
    out->n_matches = total;
    out->row_offsets = b->h_rowoff;
    out->filter_ids = b->h_ids;
    return TM_OK;
}

// tm_result with the ids packed to 3 bytes on the device (while the trie's
// node ids fit 24 bits), copied into the batch's own pinned buffer: a quarter
// less D2H and nothing to unpack on the host (tm_filters_copy_packed reads them)
int tm_engine::result_packed(tm_batch* b, tm_result_packed* out) {
    if (nd.size() > (1u << 24)) {   // 4-byte ids: the plain result
        tm_result r{};
        int rc = result(b, &r);
        if (rc) return rc;
        out->n_topics = r.n_topics;
        out->id_bytes = 4;
        out->n_matches = r.n_matches;
        out->row_offsets = r.row_offsets;
        out->ids = reinterpret_cast<const uint8_t*>(r.filter_ids);
        return TM_OK;
    }
    if (!b->done) return TM_EINVAL;
    int rc;
    if ((rc = ensure_dense(b))) return rc;
    const hipStream_t S = st(b);
    const uint64_t total = b->total;
    if (total > b->c_ids) {
        snprintf(last_error(), 512, "inconsistent CSR: kernel count %llu, capacity %zu",
                 (unsigned long long)total, b->c_ids);
        return TM_EIO;
    }
    if ((rc = host_reserve(b->h_rowoff, b->ch_rowoff, (size_t)b->n + 1))) return rc;
    if ((rc = host_reserve(b->h_ids8, b->ch_ids8, (size_t)total * 3 + 16))) return rc;
    HIP_OK(hipMemcpyAsync(b->h_rowoff, b->d_rowoff, ((size_t)b->n + 1) * 4, hipMemcpyDeviceToHost, S));
    if (total) {
        if ((rc = dev_reserve(b->d_pack, b->c_pack, total * 3 + 16))) return rc;
        HIP_OK(launch_pack_ids(b->d_ids, total, b->d_pack, S));
        HIP_OK(hipMemcpyAsync(b->h_ids8, b->d_pack, total * 3, hipMemcpyDeviceToHost, S));
    }
    HIP_OK(hipStreamSynchronize(S));
    if (b->h_rowoff[b->n] != total) {
        snprintf(last_error(), 512, "inconsistent CSR: row offsets end at %u, kernel count %llu",
                 b->h_rowoff[b->n], (unsigned long long)total);
        return TM_EIO;
    }
    out->n_topics = b->n;
    out->id_bytes = 3;
    out->n_matches = total;
    out->row_offsets = b->h_rowoff;
    out->ids = b->h_ids8;
    return TM_OK;
}

int tm_engine::sample(tm_batch* b, const uint32_t* rows, uint32_t k, tm_result* out) {
    if (!b->done || !b->csr) return TM_EINVAL;
    for (uint32_t i = 0; i < k; ++i)
        if (rows[i] >= b->n) return TM_EINVAL;
    const hipStream_t S = st(b);
    b->h_smp_off.assign((size_t)k + 1, 0);
    b->h_smp_ids.clear();
    if (k) {
        int rc;
        // [rows u32 k | cnt u32 k | pad | src u64 k | off u64 k + 1], batch-owned
        const size_t o_src = (((size_t)k * 8) + 15) & ~(size_t)15, o_off = o_src + (size_t)k * 8;
        if ((rc = dev_reserve(b->d_smp_meta, b->c_smp_meta, o_off + ((size_t)k + 1) * 8))) return rc;
        uint8_t* m = b->d_smp_meta;
        uint32_t* d_rows = reinterpret_cast<uint32_t*>(m);
        uint32_t* d_cnt = d_rows + k;
        unsigned long long* d_src = reinterpret_cast<unsigned long long*>(m + o_src);
        uint64_t* d_off = reinterpret_cast<uint64_t*>(m + o_off);
        std::vector<uint32_t> cnt(k);
        HIP_OK(hipMemcpyAsync(d_rows, rows, (size_t)k * 4, hipMemcpyHostToDevice, S));
        HIP_OK(launch_sample_meta(b->d_count, b->d_src, d_rows, k, d_cnt, d_src, S));
        HIP_OK(hipMemcpyAsync(cnt.data(), d_cnt, (size_t)k * 4, hipMemcpyDeviceToHost, S));
        HIP_OK(hipStreamSynchronize(S));
        std::vector<uint64_t> off((size_t)k + 1, 0);
        for (uint32_t i = 0; i < k; ++i) off[i + 1] = off[i] + cnt[i];
        if (off[k] > MAX_RESULT) return TM_EOVERFLOW;   // u32 CSR offsets
        for (uint32_t i = 0; i <= k; ++i) b->h_smp_off[i] = (uint32_t)off[i];
        b->h_smp_ids.resize(off[k]);
        if (off[k]) {
            if ((rc = dev_reserve(b->d_smp_ids, b->c_smp_ids, off[k]))) return rc;
            HIP_OK(hipMemcpyAsync(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, S));
            HIP_OK(launch_sample_ids(b->d_sfids, d_cnt, d_src, d_off, k, b->d_smp_ids, S));
            HIP_OK(hipMemcpyAsync(b->h_smp_ids.data(), b->d_smp_ids, off[k] * 4, hipMemcpyDeviceToHost, S));
            HIP_OK(hipStreamSynchronize(S));
        }
    }
    if (b->h_smp_ids.empty()) b->h_smp_ids.push_back(0);   // (a valid pointer for an empty result)
    out->n_topics = k;
    out->n_matches = b->h_smp_off[k];
    out->row_offsets = b->h_smp_off.data();
    out->filter_ids = b->h_smp_ids.data();
    return TM_OK;
}
