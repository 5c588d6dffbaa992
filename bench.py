"""bench.py -- publishes matched/sec at 1M wildcard subscriptions (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload: 1,000,000 distinct wildcard filters
(depth <= 7, V = 1024, Zipf 1.1, p+ = 0.15, p# = 0.25, seed 2) compiled into
the HBM trie replica; a batch of 10,000,000 synthetic publishes per GPU
(seed 1000 + rank) whose bytes are resident in HBM before timing and are
tokenised + interned there by the device tokeniser on the first launch; the
timed steps reuse those tokens (the dictionary does not change), and a fresh
batch (tokeniser + walk every launch) is timed beside them
("fresh_publishes_per_s").  One step = the frontier-walk kernel and the
generic slow path over the batch -- every topic's complete, byte-sorted,
deduplicated match set lands in HBM as the walk's rows (tm_batch_rows: per
topic a count and a start in the staging array; the per-publish path and the
fan-out consume them there).  The dense CSR (row offsets + ids in topic
order: scan + one copy, built on request by tm_batch_result / routes /
export) is timed beside it as "dense_csr".

Multi-GPU: one process per GPU (torchrun), the trie replicated on every GPU,
each rank matching its own 10M batch (replicated mode, no data-path
collective) -> "scaling": "weak"; value = all ranks' publishes / max rank time.

Extra fields: roofline (HBM, algorithmic bytes per launch counted by the kernel,
over the match kernel's HIP-event time), cpu_baseline (the CPU restatement of
emqx_router:match_routes/1 on this host, rank 0 / N = 1 only), p99 batch latency
at B = 65,536 as §8d defines it (submit -> results ready: new publishes from
host memory to sorted ids in host memory; the device-resident replay beside it
as p99_resident_ms), the per-publish drop-in path (coalesce: async and
blocking calls, the CPU port beside them), the host-inclusive end-to-end rate,
C1 on the CPU port and the device, and C5 (K = 100, 10 and 1000: skew + 10k
subscribe/unsubscribe deltas per step).

Self-checks, after the timed regions (the oracle only as the checker): at
N = 1 3,000 evenly spaced rows of the timed C2 launch against the CPU
restatement, and 3,000 distinct rows of every C5 leg's last (graph-replayed)
batch against the oracle on that step's snapshot; at N > 1 every rank's
sampled rows against rank 0's replica on device 0 (emqx_amd/selfcheck.py).
All of them -> parity_sample_ok.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
ALG_BYTES_PER_VISIT = 64       # one 64-B DRAM request per visited trie node


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def host_cpu_share() -> dict:
    """CPUs this process may really use: the affinity mask capped by the cgroup
    CPU quota (cpu.max).  On the GPU box os.cpu_count() / nproc report the whole
    machine (256 threads of two EPYC 9575F) while the lease's cgroup grants 16
    CPUs of bandwidth, so more threads than the quota only time-slice."""
    info = {"nproc": os.cpu_count() or 1, "affinity": len(os.sched_getaffinity(0)), "cgroup_quota": None}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            info["cgroup_quota"] = float(q) / float(per)
    except (OSError, ValueError):
        pass
    share = info["affinity"]
    if info["cgroup_quota"]:
        share = min(share, max(1, int(info["cgroup_quota"] + 0.5)))
    info["threads"] = share
    info["model"] = cpu_info()
    mhz = None
    for p in ("/sys/devices/system/cpu/cpu0/cpufreq/cpuinfo_max_freq",):
        try:
            with open(p) as f:
                mhz = int(f.read().strip()) / 1000.0
        except (OSError, ValueError):
            pass
    info["max_mhz"] = mhz
    return info


def cpu_baseline(filters, topics, sample_1t, sample_mt, host, label="C2 trie (1M filters"):
    """emqx_router:match_routes/1 restated in C (oracle/, prefix-string ETS layout),
    timed on this host's cores over a bounded sample of the same workload:
    1 thread, and host['threads'] threads (the lease's CPU share) each taking a
    contiguous slice."""
    from oracle import pyoracle
    threads = host["threads"]
    orc = pyoracle.Oracle()
    t0 = time.time()
    for f in filters.tolist():
        orc.add_route(f)
    build_s = time.time() - t0
    s1 = topics.slice(0, sample_1t)
    t0 = time.time()
    orc.match_routes_batch(s1.buf, s1.offs, nthreads=1)
    dt1 = time.time() - t0
    sm = topics.slice(0, sample_mt)
    # repeat short samples until the timed region is >= 2 s (a C1 pass is ~20 ms)
    reps, dtm = 0, 0.0
    while dtm < 2.0:
        t0 = time.time()
        st = orc.match_routes_batch(sm.buf, sm.offs, nthreads=threads)
        dtm += time.time() - t0
        reps += 1
    orc.close()
    return {
        "value": reps * sample_mt / dtm,
        "unit": "publishes/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{label}, ETS-layout C restatement, build {build_s:.1f}s); "
                   f"{reps} x {sample_mt} publishes on {threads} threads in {dtm:.2f}s; "
                   f"{sample_1t} publishes on 1 thread in {dt1:.2f}s = {sample_1t / dt1:.0f}/s; "
                   f"routes returned {st['routes']}; cpu {host['model']} (max {host['max_mhz']} MHz), "
                   f"nproc {host['nproc']}, affinity {host['affinity']}, cgroup quota {host['cgroup_quota']} CPUs"),
        "value_1thread": sample_1t / dt1,
        "host": host,
    }


def c1_leg(host, device=0):
    """BASELINE config 1: 10k mixed '+'/'#' filters (10 %
    exact), 100k publishes.  The CPU restatement of match_routes/1 on the
    lease's cores and the device pipeline on the same workload."""
    from emqx_amd import gen
    from emqx_amd.engine import Engine
    p = gen.C1
    filters = gen.gen_filters(p)
    topics = gen.gen_topics(p, filters, 1001, 100_000)
    out = {"workload": "C1: 10k filters (10% exact), 100k publishes",
           "cpu_baseline": cpu_baseline(filters, topics, len(topics), len(topics), host,
                                        label="C1 trie (10k filters")}
    eng = Engine(device=device)
    for f in filters.tolist():
        eng.route_add(f, 0)
    eng.sync()
    b = eng.prepare(topics)
    for _ in range(3):
        b.launch().wait()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        b.launch().wait()
    dt = (time.perf_counter() - t0) / reps
    out["gpu_publishes_per_s"] = len(topics) / dt
    out["gpu_ms_per_batch"] = 1e3 * dt
    out["speedup_vs_cpu_allcore"] = out["gpu_publishes_per_s"] / out["cpu_baseline"]["value"]
    b.free()
    eng.close()
    return out


def pmc_traffic(workload, topics, filters=None):
    """HBM bytes per walk launch from the committed PMC pass of this workload
    (`tools/gpu.sh TAG 'traffic c2'` -> profiles/pmc_latest.json for C2,
    `'traffic c4'` -> profiles/pmc_c4.json for C4), or None.  The counters are
    NOT collected in this run (a --pmc pass is a rocprofv3 run of its own):
    roofline.traffic_source names the file they come from."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json" if workload == "C2" else "pmc_c4.json")
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    if pmc.get("workload") != workload or pmc.get("topics") != topics:
        return None
    if filters is not None and pmc.get("filters") not in (None, filters):
        return None
    return pmc.get("hbm_bytes_per_launch")


def traffic_source(workload):
    return ("profiles/" + ("pmc_latest.json" if workload == "C2" else "pmc_c4.json")
            + " (rocprofv3 FETCH_SIZE and WRITE_SIZE passes of this workload, committed; not counted in this run)")


def c2_selfcheck(eng, b, filters, topics) -> dict:
    """THE CHECKER, after the timed region (oracle/ is used here only as the
    checker, like cpu_baseline): >= 3,000 evenly spaced rows of the timed
    launch, gathered on the device (tm_batch_sample), as filter bytes against
    the CPU restatement of emqx_trie:match/1 (oracle/tm_oracle.c, ETS layout,
    src/emqx_trie.erl:96-99,162-186) over the same 1M filters."""
    from emqx_amd import selfcheck as SC
    from oracle import pyoracle
    t0 = time.time()
    idx = SC.sample_index(len(topics))
    so, si = b.sample(idx)
    got = SC.rows_from_csr(so, si, np.arange(len(idx)), SC.engine_names(eng))
    orc = pyoracle.Oracle()
    for f in filters.tolist():
        orc.register(f)
        orc.insert(f)
    ts = [topics[int(i)] for i in idx]
    buf, offs = pyoracle.pack(ts)
    counts, oidx, _ = orc.match_batch(buf, offs, nthreads=8)
    cut = np.concatenate([[0], np.cumsum(counts.astype(np.int64))])
    names = {}

    def name(j):
        if j not in names:
            names[j] = orc.filter_bytes(j)
        return names[j]
    exp = [[name(int(j)) for j in oidx[cut[i]:cut[i + 1]]] for i in range(len(ts))]
    orc.close()
    bad = [i for i in range(len(ts)) if got[i] != exp[i]]
    return {"parity_sample_ok": not bad and len(ts) > 0, "sampled_rows": len(ts),
            "matches_checked": int(cut[-1]), "mismatches": [ts[i].decode("latin-1") for i in bad[:3]],
            "checker": "oracle/tm_oracle.c trie restatement over the same filters (rows as filter bytes)",
            "seconds": round(time.time() - t0, 2)}


def c5_selfcheck(eng, b, pubs, derived, allf, live, added) -> dict:
    """THE CHECKER, after the timed region (oracle/ only as the checker): the
    last step's batch -- a fresh deduplicated launch replayed from its captured
    graph and matched after every delta of the run -- against the CPU
    restatement on that snapshot (the trie's state now; oracle/c5_checker.py
    FinalSnapshot: inverted index + live set for the derived filters, trie
    oracle for the background ones, brute-force emqx_topic:match/2 for the
    churned-in ones).  3,000 evenly spaced distinct rows (by their first
    publish's bytes, gathered on the device) and the publish -> row map at
    3,000 evenly spaced publishes (equal bytes <=> equal row)."""
    from emqx_amd import selfcheck as SC
    from oracle.c5_checker import FinalSnapshot, _word_id
    t0 = time.time()
    row_of, n_rows = b.row_map()
    u, first = np.unique(row_of, return_index=True)
    rows_ok = len(u) == n_rows and (u == np.arange(n_rows)).all() and (np.diff(first) > 0).all()
    ridx = SC.sample_index(n_rows)
    ts = [pubs[int(first[r])] for r in ridx]
    distinct_ok = len(set(ts)) == len(ts)
    pidx = SC.sample_index(len(row_of))
    map_ok = all(pubs[int(i)] == pubs[int(first[row_of[i]])] for i in pidx)
    so, si = b.sample(ridx)
    got = SC.rows_from_csr(so, si, np.arange(len(ridx)), SC.engine_names(eng))
    chk = FinalSnapshot(derived, allf.slice(len(derived), len(allf)).tolist(), live, added)
    exp = chk.rows(ts)
    chk.close()
    bad = [i for i in range(len(ts)) if got[i] != exp[i]]
    hot = sum(1 for t in ts if all(_word_id(w) >= 0 for w in t.split(b"/")))
    return {"parity_sample_ok": bool(not bad and rows_ok and distinct_ok and map_ok and ts),
            "sampled_rows": len(ts), "sampled_hot_rows": hot, "sampled_publishes": len(pidx),
            "matches_checked": int(sum(len(e) for e in exp)), "row_map_ok": bool(rows_ok and map_ok and distinct_ok),
            "mismatches": [ts[i].decode("latin-1")[:80] for i in bad[:3]],
            "checker": "oracle/c5_checker.py FinalSnapshot on the last step's snapshot",
            "seconds": round(time.time() - t0, 2)}


def timed_steps(bs, steps, ms_match=None, ms_total=None):
    """steps launches cycling over the batches in bs: batch i + len(bs) - 1 is
    launched before batch i is waited for (each on its own stream when
    len(bs) > 1); ends on a wait, so the device is idle at both ends."""
    nb = len(bs)
    for i in range(min(nb - 1, steps)):
        bs[i].launch()
    for i in range(steps):
        if i + nb - 1 < steps:
            bs[(i + nb - 1) % nb].launch()
        cur = bs[i % nb]
        cur.wait()
        if ms_match is not None:
            s = cur.stats()
            ms_match.append(s["ms_match"])
            ms_total.append(s["ms_total"])


def run_c4(args, ws, rank, local, pg):
    """Config C4: IoT filters partitioned over the WORLD_SIZE GPUs by their literal
    (w0, w1) prefix (root-wildcard filters replicated), each rank publishing its
    own batch; one step = owner kernel + all_to_all of the tokenised topics (RCCL)
    + the owner's device walk + all_to_all of the counts and global filter ids +
    reassembly in publish order (emqx_amd/sharded.py)."""
    import torch

    from emqx_amd import gen
    from emqx_amd.engine import Engine
    from emqx_amd.sharded import ShardedMatcher

    p = gen.IotParams(n_filters=args.c4_filters) if args.c4_filters else gen.C4
    t0 = time.time()
    vocab = gen.gen_iot_vocab(p)
    eng = Engine(device=local, frozen_dict=True)
    eng.dict_load(vocab)
    del vocab
    inserted = 0
    chunk = 5_000_000
    for lo in range(0, p.n_filters, chunk):
        fl = gen.gen_iot_filters(p, lo, min(p.n_filters, lo + chunk))
        inserted += eng.insert_many(fl, rank, ws)
        log(f"[rank {rank}] C4 filters {min(p.n_filters, lo + chunk)}/{p.n_filters}: {inserted} on this shard, "
            f"{time.time() - t0:.0f}s")
    eng.sync()
    est = eng.stats()
    log(f"[rank {rank}] shard trie built+uploaded in {time.time() - t0:.1f}s: {est}")
    topics = gen.gen_iot_topics(p, 4000 + rank, args.topics)
    tok = eng.tokenize(topics)
    del topics
    dev = torch.device("cuda", local)
    words = torch.from_numpy(tok.words.view(np.int32)).to(dev)
    toff = torch.from_numpy(tok.toff.view(np.int32)).to(dev)
    tflags = torch.from_numpy(tok.tflags).to(dev)
    n = len(tok)
    sm = ShardedMatcher(eng, rank, ws, device=dev)
    for _ in range(args.warmup):
        sm.step(words, toff, tflags)
    torch.cuda.synchronize()
    if pg is not None:
        pg.barrier()
    t0 = time.perf_counter()
    ms_match = []
    for _ in range(args.steps):
        row_off, gids = sm.step(words, toff, tflags)
        ms_match.append(sm.last["ms_match"])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pg is not None:
        pg.barrier()
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        pg.all_reduce(tt, op=pg.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = sm._batch.stats()
    alg_bytes = (ALG_BYTES_PER_VISIT * (st["visits"] + st["hash_hits"]) + 4 * st["words"]
                 + 4 * st["matches"] + 4 * st["topics"])
    k_ms = float(np.mean(ms_match))
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    out = {
        "metric": "publishes matched/sec (node) at 100M IoT filters, filter-sharded",
        "value": ws * n * args.steps / elapsed,
        "unit": "publishes/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded IoT generator, SURVEY.md §8d C4)",
        "config": {"workload": f"C4: {p.n_filters} IoT filters sharded over {ws} GPU(s), "
                               f"{n} publishes per GPU", "filters": p.n_filters,
                   "filters_on_rank0_shard": inserted, "mode": "filter-sharded",
                   "parallelism": f"filters sharded x{ws}, all_to_all exchange"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic("C4", n, p.n_filters),
                     "kernel": "tm_match_tiles", "kernel_ms": k_ms, "alg_bytes_per_launch": alg_bytes,
                     "per_publish": {k: st[v] / max(st["topics"], 1) for k, v in
                                     (("V", "visits"), ("H", "hash_hits"), ("d", "words"), ("M", "matches"))}},
        "matches_per_step": int(gids.numel()),
        "device_match_ms": k_ms,
        "exchange": {"sent_topics": sm.last["sent_topics"], "recv_topics": sm.last["recv_topics"]},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.destroy_process_group()


def run_c4_group(args):
    """Config C4 in ONE process (tm_sharded_*, no torch, no collective): the IoT
    filters partitioned over shard engines on the listed devices (default
    0..N-1; 0,0 rehearses two shards on one GPU), one slice of --topics
    publishes per shard, tokenised on its shard's device at prepare.  One step
    = every slice partitioned by owner on its own device + every shard
    receiving its parts and walking them, one host wait (tm_sharded_run); the
    rows stay in each shard's HBM.  The publish-order CSR (global ids) is built
    on request and timed beside it; a fresh batch (tokenise + plan + step) too.
    Self-check: >= 3,000 sampled rows of every slice against one engine on
    device 0 over the filters that can match them (a topic
    device/d<X>/sensor/... can only match filters whose second level is d<X>)."""
    from emqx_amd import gen
    from emqx_amd import selfcheck as SC
    from emqx_amd.engine import Engine, ShardedGroup

    devs = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    G = len(devs)
    p = gen.IotParams(n_filters=args.c4_filters) if args.c4_filters else gen.C4
    t0 = time.time()
    n = args.topics * G
    parts = [gen.gen_iot_topics(p, 4000 + k, args.topics) for k in range(G)]
    topics = gen.Strings.concat(parts) if G > 1 else parts[0]
    del parts
    lo = [n * k // G for k in range(G + 1)]                         # the group's slices
    sample = np.concatenate([lo[k] + SC.sample_index(lo[k + 1] - lo[k]) for k in range(G)])
    want = np.unique(gen.iot_device_ids(gen.Strings.from_list([topics[int(i)] for i in sample])))
    grp = ShardedGroup(devs)
    vocab = gen.gen_iot_vocab(p)
    grp.dict_load(vocab)
    inserted, cand = 0, []
    chunk = 5_000_000
    for c0 in range(0, p.n_filters, chunk):
        fl = gen.gen_iot_filters(p, c0, min(p.n_filters, c0 + chunk))
        inserted += grp.insert_many(fl)
        keep = np.flatnonzero(np.isin(gen.iot_device_ids(fl), want))
        cand.extend(fl[int(i)] for i in keep)
        log(f"[c4 group] filters {min(p.n_filters, c0 + chunk)}/{p.n_filters} over {G} shard(s), "
            f"{time.time() - t0:.0f}s")
    b = grp.prepare(topics)
    for _ in range(max(args.warmup, 1)):
        b.run()
    ms_match, phases, waits = [], [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.run()
        st = b.stats()
        ms_match.append(st["ms_match"])
        phases.append((st["ms_partition"], st["ms_exchange"], st["ms_step"]))
        waits.append(st["host_waits"])
    elapsed = time.perf_counter() - t0
    st = b.stats()
    alg_bytes = (ALG_BYTES_PER_VISIT * (st["visits"] + st["hash_hits"]) + 4 * st["words"]
                 + 4 * st["matches"] + 4 * st["topics"]) / G      # per shard (device)
    k_ms = float(np.mean(ms_match))                                 # slowest part per step
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    ph = np.mean(np.array(phases), 0).tolist()
    if args.profile:   # rocprofv3 runs: only the timed steps' launches
        print(json.dumps({"workload": "c4", "value": n * args.steps / elapsed, "kernel_ms": k_ms,
                          "frac": achieved / HBM_PEAK_GBS}), flush=True)
        b.free()
        grp.close()
        return
    # the publish-order CSR with global ids, built on request from the step's rows
    tr = time.perf_counter()
    offs, ids = b.result()
    csr_ms = b.stats()["ms_unpartition"]
    result_ms = 1e3 * (time.perf_counter() - tr)
    # a fresh batch: slices tokenised on their devices + the plan + one step
    fresh, fresh_phases = [], []
    for _ in range(3):
        tf = time.perf_counter()
        b.reprepare(topics)
        tp = time.perf_counter()
        b.run()
        te = time.perf_counter()
        fresh.append(1e3 * (te - tf))
        s_ = b.stats()
        fresh_phases.append((s_["ms_stage"], s_["ms_plan"], 1e3 * (tp - tf), 1e3 * (te - tp)))
    # self-check against one engine on device 0 (fresh batch's rows = the timed batch's: same publishes)
    ref = Engine(device=0, frozen_dict=True)
    ref.dict_load(vocab)
    ref.insert_many(cand)
    cache = {}

    def gname(g):
        g = int(g)
        if g not in cache:
            cache[g] = grp.filter_bytes(g)
        return cache[g]

    def grp_rows(idx):
        return [[gname(x) for x in ids[int(offs[i]):int(offs[i + 1])]] for i in idx]
    sc = group_selfcheck(grp_rows, topics, lo, [f"slice {k} (device {d})" for k, d in enumerate(devs)], ref)
    ref.close()
    out = {
        "metric": "publishes matched/sec (node) at 100M IoT filters, filter-sharded",
        "value": n * args.steps / elapsed,
        "unit": "publishes/s",
        "n_gpus": len(set(devs)),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded IoT generator, SURVEY.md §8d C4)",
        "config": {"workload": f"C4: {p.n_filters} IoT filters sharded over {G} shard(s) on devices {devs}, "
                               f"{args.topics} publishes per shard, one process (tm_sharded)", "filters": p.n_filters,
                   "filters_inserted_over_shards": inserted, "mode": "filter-sharded, in-process",
                   "parallelism": f"filters sharded x{G}, per-device partition + part exchange (no collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic("C4", args.topics, p.n_filters) if G == 1
                     else None, "kernel": "tm_match_tiles", "kernel_ms": k_ms, "alg_bytes_per_launch": alg_bytes,
                     "per_publish": {k: st[v] / max(st["topics"], 1) for k, v in
                                     (("V", "visits"), ("H", "hash_hits"), ("d", "words"), ("M", "matches"))}},
        "matches_per_step": st["matches"],
        "device_match_ms": k_ms,
        "phase_ms": {"partition_device": ph[0], "exchange_device": ph[1], "step_host": ph[2]},
        "host_waits_per_step": float(np.mean(waits)),
        "publish_order_csr": {"ms": csr_ms, "with_d2h_ms": result_ms,
                              "publishes_per_s_with_csr": n / (1e-3 * (1e3 * elapsed / args.steps + csr_ms))},
        "fresh_publishes_per_s": n / (1e-3 * float(np.median(fresh))),
        "fresh_ms": float(np.median(fresh)),
        # a fresh batch's phases: bytes into pinned memory, the plan (uploads,
        # device tokenisers, part counts), the whole prepare call, the step
        "fresh_phase_ms": dict(zip(("stage", "plan", "prepare", "step"),
                                   np.median(np.array(fresh_phases), 0).tolist())),
        "part_topics": st["part_topics"],
        "links": [[grp.link(i, j) for j in range(G)] for i in range(G)],
        "devices": devs,
        "selfcheck": sc,
        "parity_sample_ok": sc["parity_sample_ok"],
    }
    b.free()
    grp.close()
    print(json.dumps(out), flush=True)


def c5_leg(k, steps, n_deltas, n_topics, device=0, seed=5, sync=None, warmup=2, n_batches=3, selfcheck=True):
    """Config C5: 10k hot topics take 90% of the publishes, each matched by ~k
    filters derived from it (+ 100k background C2-style filters).  Every step
    is a NEW batch of n_topics publishes (n_batches pre-generated batches,
    their bytes resident in HBM, taken in turn) and n_deltas subscribe /
    unsubscribe deltas:
      host    the deltas applied to the trie (emqx_trie:delete/1, insert/1)
              and their upload enqueued;
      device  the batch deduplicated (equal bytes walk once, TM_BATCH_DEDUP
              on the device), its distinct topics tokenised
              (emqx_topic:words/1) and walked (rows longer than K by the
              generic kernel), and every publish's row expanded in HBM
              (tm_batch_publish_rows: the per-publish result; its total is
              "delivered").
    Pipelined: the host applies deltas i + 1 while the device runs step i;
    their upload is queued behind walk i and batch i + 1 behind the upload
    (read-your-writes) before batch i is waited for, so a step costs about
    max(host, device).  From a batch's second launch on, the launch replays a
    captured HIP graph; the device phase split comes from the direct launches
    (each batch's first, in the warm-up).  After the timed region the last
    step's batch is checked against the oracle on its snapshot (c5_selfcheck)."""
    from emqx_amd import gen
    from emqx_amd.engine import Engine
    from emqx_amd.skew import Churn, workload

    p = gen.SkewParams(k_per_hot=k)
    t0 = time.time()
    allf, derived, hot, batches = workload(p, 100_000, n_topics, seed=seed, batches=n_batches)
    log(f"[c5 k={k}] workload: {len(allf)} filters, {n_batches} x {len(batches[0])} publishes in "
        f"{time.time() - t0:.1f}s")
    eng = Engine(device=device)
    eng.insert_many(allf)
    eng.sync()
    churn = Churn(hot, derived.tolist(), seed=seed + 6)
    tp = time.perf_counter()
    bs = [eng.prepare(pubs, dedup=True) for pubs in batches]    # bytes to HBM (inputs resident)
    prepare_ms = 1e3 * (time.perf_counter() - tp) / n_batches
    split = []
    for w in range(warmup):
        for b in bs:
            b.retokenize().launch().wait()
            if w == 0:       # each batch's first launch is direct: its events time every phase
                st = b.stats()
                split.append((st["ms_dedup"], st["ms_tokenize"], st["ms_match"], st["ms_expand"],
                              st["ms_dedup"] + st["ms_tokenize"] + st["ms_total"]))
    if sync is not None:
        sync.barrier()
    # The deltas are drawn before timing, as packed binaries (what the NIF's
    # route_apply hands over).  Step i applies deltas i and matches batch
    # i mod n_batches against the result.
    deltas, added = [], []
    for _ in range(steps):
        dels, adds = churn.step(n_deltas)
        added += adds
        deltas.append((gen.Strings.from_list(dels), gen.Strings.from_list(adds)))
    ms_dev, ms_queue, ms_churn = [], [], []
    rows, delivered = [], []

    def collect(bb):
        st = bb.stats()
        # a graph replay times its whole span (reported as its walk), a direct
        # launch each phase: their sum is the launch's device time either way
        ms_dev.append(st["ms_tokenize"] + st["ms_dedup"] + st["ms_total"])
        ms_queue.append(st["ms_queue"])
        rows.append(st["topics"])
        delivered.append(st["delivered"])

    ms_host = {"sync_async": [], "wait": [], "launch": []}   # the step's host time beside the churn
    g0 = eng.stats()["graph_launches"]
    cg0 = cgroup_cpu_stat()
    t0 = time.perf_counter()
    tc = time.perf_counter()
    Churn.apply(eng, *deltas[0])
    ms_churn.append(1e3 * (time.perf_counter() - tc))
    bs[0].retokenize().launch()
    for i in range(steps):
        b = bs[i % n_batches]
        if i + 1 < steps:
            tc = time.perf_counter()
            Churn.apply(eng, *deltas[i + 1])
            ms_churn.append(1e3 * (time.perf_counter() - tc))
            tc = time.perf_counter()
            eng.sync_async()     # the upload, queued behind step i on the engine stream
            ms_host["sync_async"].append(1e3 * (time.perf_counter() - tc))
            # batch i + 1 is queued behind the upload before batch i is waited
            # for: the device goes from walk i to upload i + 1 to batch i + 1
            # without waiting for the host (the batches rotate, so i's rows
            # stay intact until it is read below)
            tc = time.perf_counter()
            bs[(i + 1) % n_batches].retokenize().launch()
            ms_host["launch"].append(1e3 * (time.perf_counter() - tc))
        tc = time.perf_counter()
        b.wait()
        if i + 1 < steps:   # (the last step's wait is the device's tail, no churn beside it)
            ms_host["wait"].append(1e3 * (time.perf_counter() - tc))
    elapsed = time.perf_counter() - t0
    # the device times, rows and deliveries of the rotated batches' last
    # launches, read after the timed region: a batch's stats (event times)
    # read after every wait sat on the churn's critical path (~0.1 ms of host
    # time per step), and a relaunch overwrites them
    for j in range(max(0, steps - n_batches), steps):
        collect(bs[j % n_batches])
    cg1 = cgroup_cpu_stat()
    if sync is not None:
        sync.barrier()
        elapsed = sync.allmax(elapsed)
    graph_launches = eng.stats()["graph_launches"] - g0
    last = (steps - 1) % n_batches
    st = bs[last].stats()
    n = len(batches[0])
    sp = np.median(np.array(split), 0).tolist() if split else [0.0] * 5
    out = {
        "k": k, "publishes_per_s": n * steps / elapsed, "ms_per_step": 1e3 * elapsed / steps, "steps": steps,
        "distinct_topics_per_s": float(np.mean(rows)) * steps / elapsed,
        "batches": n_batches, "dedup_tokenise_walk_expand_every_step": True,
        # the rotated batches' bytes were uploaded before timing (prepare_ms
        # per batch, host copy + H2D): the timed rate is HBM-resident input
        "inputs_resident_in_hbm": True,
        "publishes_per_s_with_prepare": n / (1e-3 * (1e3 * elapsed / steps + prepare_ms)),
        "deltas_per_step": n_deltas, "filters": len(allf), "publishes": n, "distinct_topics": int(np.mean(rows)),
        "prepare_ms": prepare_ms,
        "device_ms": float(np.mean(ms_dev)),
        # per-phase device times of a direct (non-graph) launch of each batch
        "device_split_direct_ms": dict(zip(("dedup", "tokenize", "walk", "expand", "total"), sp)),
        "device_queue_ms": float(np.mean(ms_queue)),
        "churn_ms": float(np.mean(ms_churn)), "churn_ms_max": float(np.max(ms_churn)),
        "churn_ms_steps": [round(x, 3) for x in ms_churn],   # [0]: before the first launch (no walk beside it)
        "host_ms": {k: float(np.mean(v)) if v else 0.0 for k, v in ms_host.items()},
        "churn_overlapped_with_device": True,
        # (publish, filter) matches per step, every publish's row materialised
        # in HBM (tm_batch_publish_rows), summed on the device
        "delivered_matches_per_step": int(np.mean(delivered)),
        "generic_path_topics": int(st["slow_topics"]),
        "uploads_delta": eng.stats()["uploads_delta"],
        # timed launches replayed as a captured HIP graph
        "graph_launches": graph_launches,
        # CFS quota throttling of the process over the timed steps, and the
        # CPU time it used (cgroup cpu.stat): the churn runs on the box's
        # 16-CPU share
        "cgroup": {k: cg1[k] - cg0.get(k, 0) for k in ("nr_throttled", "throttled_usec", "usage_usec") if k in cg1},
    }
    if selfcheck:
        out["selfcheck"] = c5_selfcheck(eng, bs[last], batches[last], derived, allf, churn.live_set, added)
        out["parity_sample_ok"] = out["selfcheck"]["parity_sample_ok"]
        if not out["parity_sample_ok"]:
            log(f"[c5 k={k}] PARITY SAMPLE FAILED: {out['selfcheck']}")
    for b in bs:
        b.free()
    eng.close()
    return out


def run_c5(args, ws, rank, local, sync):
    """--workload c5: the C5 leg alone as the bench line (K = --c5-k)."""
    leg = c5_leg(args.c5_k, args.steps, args.c5_deltas, args.topics, device=local, seed=5 + rank, sync=sync,
                 warmup=args.warmup, selfcheck=not args.profile)
    out = {
        "metric": "publishes matched/sec (node), hot-topic skew + churn (C5)",
        "value": ws * leg["publishes_per_s"],
        "unit": "publishes/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": leg["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded skew generator, SURVEY.md §8d C5)",
        "config": {"workload": f"C5: 10k hot topics x ~{args.c5_k} filters + 100k background, "
                               f"{leg['publishes']} publishes per GPU (90% hot, Zipf 1.0), {args.c5_deltas} deltas per step",
                   "filters": leg["filters"], "distinct_topics": leg["distinct_topics"],
                   "mode": "replicated, a new batch every step, deduplicated on the device"},
        "device_pipeline_ms": leg["device_ms"],
        "churn_apply_ms": leg["churn_ms"],
        "distinct_topics_per_s": ws * leg["distinct_topics_per_s"],
        "leg": leg,
    }
    if not args.profile:
        out["parity_sample_ok"] = leg.get("parity_sample_ok")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if sync is not None:
        sync.close()


COALESCE_LEGS = (("async", 1, 8, 256), ("async_4096", 1, 16, 256), ("sync", 0, 64, 1))


def cgroup_cpu_stat() -> dict:
    """The process's cgroup CPU accounting (cgroup v2 cpu.stat; {} if absent):
    nr_throttled / throttled_usec tell whether the box's CFS quota paused the
    whole process during a leg (a multi-ms stall every thread sees)."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if len(ln.split()) == 2)}
    except (OSError, ValueError):
        return {}


def coalesce_legs(eng, topics, legs, exp_c=None, exp_h=None) -> dict:
    """Per-publish emqx_trie:match/1 calls through the drop-in boundary, driven
    by the native load generator (emqx_amd/csrc/tm_load.cpp): legs = (name,
    mode, threads, calls in flight per thread, calls).  Every call's row is
    checked against the batch path (length + hash)."""
    from emqx_amd import load as LD
    if exp_c is None:
        offs, ids = eng.match_batch(topics)
        exp_c = np.diff(offs.astype(np.int64))
        exp_h = LD.row_hashes(offs, ids)
    out = {}
    for name, mode, th, win, cnt in legs:
        sub = topics if cnt == len(topics) else topics.slice(0, cnt)
        # untimed warm-up at the leg's own concurrency: the batch sizes it
        # forms get their slot graphs captured here (a one-time setup cost
        # per size class and slot, milliseconds each), not inside the timed
        # calls.  (20k calls left some slot / size-class pairs to the timed
        # run: 9-29 ms max latencies with no CPU throttling, round 6)
        if mode == 1:   # (and a burst of large batches first: every slot's largest size class)
            LD.run(eng, topics.slice(0, min(200_000, len(topics))), mode, 8, 2048, hashes=False)
        LD.run(eng, topics.slice(0, min(max(200_000, 8 * th * win), len(topics))), mode, th, win, hashes=False)
        b0 = eng.async_stats()
        c0 = cgroup_cpu_stat()
        st, counts, hashes = LD.run(eng, sub, mode, th, win)
        c1 = cgroup_cpu_stat()
        b1 = eng.async_stats()
        ok = (st["errors"] == 0 and np.array_equal(counts.astype(np.int64), exp_c[:cnt])
              and np.array_equal(hashes, exp_h[:cnt]))
        nb = max(b1["batches"] - b0["batches"], 1)
        out[name] = {"calls_per_s": cnt / st["seconds"], "calls": cnt, "threads": th, "outstanding_per_thread": win,
                     "in_flight": th * win, "p50_us": st["p50_us"], "p99_us": st["p99_us"], "mean_us": st["mean_us"],
                     "max_us": st["max_us"], "max_at_s": st["max_at_s"], "seconds": st["seconds"],
                     "rows_equal_batch_path": bool(ok),
                     "batches": b1["batches"] - b0["batches"],
                     "mean_batch": (b1["requests"] - b0["requests"]) / nb,
                     "recoveries": b1["recoveries"] - b0["recoveries"],
                     "host_us_per_batch": {k: (b1[k] - b0[k]) / nb for k in ("us_launch", "us_wait", "us_deliver")},
                     "inline_launches": b1["inline_launches"] - b0["inline_launches"],
                     # CFS quota throttling of the process during the leg (cgroup cpu.stat)
                     "cgroup_throttled": {k: c1[k] - c0.get(k, 0) for k in ("nr_throttled", "throttled_usec")
                                          if k in c1}}
        log(f"[coalesce] {name}: {out[name]}")
    return out


def coalesce_brief(eng, topics) -> dict:
    """The default line's per-publish sub-object (~2 s): async with 2,048
    calls in flight (8 threads x 256) and 64 blocking threads, on the C2 trie
    of the headline; the CPU port's rate is added beside it by the caller."""
    n = min(len(topics), 1_000_000)
    sub = topics.slice(0, n)
    legs = coalesce_legs(eng, sub, (("async", 1, 8, 256, n), ("sync", 0, 64, 1, min(n, 300_000))))
    return {"workload": f"C2 1M filters, {n} single-topic tm_match_async / tm_match_coalesced calls",
            "async_calls_per_s": legs["async"]["calls_per_s"], "async_p50_us": legs["async"]["p50_us"],
            "async_p99_us": legs["async"]["p99_us"], "async_max_us": legs["async"]["max_us"],
            "async_in_flight": legs["async"]["in_flight"],
            "sync_calls_per_s": legs["sync"]["calls_per_s"], "sync_threads": 64,
            "sync_p99_us": legs["sync"]["p99_us"],
            "rows_equal_batch_path": legs["async"]["rows_equal_batch_path"] and legs["sync"]["rows_equal_batch_path"],
            "legs": legs}


def run_coalesce(args, ws, rank, local, sync):
    """Per-publish emqx_trie:match/1 calls (what the NIF's match/2 does) on the
    C2 trie, driven by the native load generator (emqx_amd/csrc/tm_load.cpp):
      async  8 submitter threads x 256 outstanding tm_match_async calls --
             2048 publishing processes each awaiting its reply (enif_send);
      async_4096  16 x 256: with the engine's launcher and completers, more
             threads than the box's 16-CPU quota (CFS throttling shows as
             multi-ms outliers there);
      sync   64 threads blocking in tm_match_coalesced (a NIF on dirty
             schedulers).
    value = async calls/s; every call's row is checked against the batch path
    (length + hash).  The CPU baseline is the oracle restatement of
    match_routes/1 on the lease's cores over the same topics."""
    from emqx_amd import gen
    from emqx_amd.engine import Engine

    p = gen.C2
    filters = gen.gen_filters(p)
    n = min(args.topics, 2_000_000)
    topics = gen.gen_topics(p, filters, 1000 + rank, n)
    eng = Engine(device=local)
    eng.insert_many(filters)
    eng.sync()
    eng.coalesce_config(max_batch=args.coalesce_max_batch, linger_us=args.coalesce_linger_us)
    legs = coalesce_legs(eng, topics, [(name, mode, th, win, n if mode else min(n, 400_000))
                                       for name, mode, th, win in COALESCE_LEGS])
    out = {"metric": "emqx_trie:match/1 calls/sec, one call per publish (tm_match_async, 2048 in flight)",
           "value": legs["async"]["calls_per_s"], "unit": "calls/s", "n_gpus": 1, "steps": 1, "warmup": 1,
           "ms_per_step": 1e3 * n / legs["async"]["calls_per_s"], "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32", "data": "synthetic (seeded C2 generator)",
           "config": {"workload": f"coalesce: C2 1M filters, {n} single-topic calls",
                      "max_batch": args.coalesce_max_batch, "linger_us": args.coalesce_linger_us,
                      "depth": eng.async_stats()["depth"]},
           "legs": legs}
    if not args.no_cpu:
        host = host_cpu_share()
        out["cpu_baseline"] = cpu_baseline(filters, topics, min(200_000, n), min(args.cpu_sample, n), host)
        out["speedup_async_vs_cpu_allcore"] = out["value"] / out["cpu_baseline"]["value"]
        out["speedup_sync_vs_cpu_allcore"] = legs["sync"]["calls_per_s"] / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)


def run_dispatch(args, ws, rank, local, sync):
    """Publish -> match -> fan-out on the device: the C2
    trie and publishes, every filter with local subscribers (75% one, 24% 2-8,
    64 hot filters with 4096 each; ids from a pool of 1M subscribers).  One step
    = the match pipeline (tm_batch_launch/wait) + tm_batch_dispatch kept in HBM
    (per-match delivery scan + the load-balanced subscriber copy)."""
    from emqx_amd import gen
    from emqx_amd.engine import Engine

    p = gen.C2
    filters = gen.gen_filters(p)
    topics = gen.gen_topics(p, filters, 1000 + rank, args.topics)
    eng = Engine(device=local)
    fl = filters.tolist()
    eng.insert_many(fl)
    rng = np.random.default_rng(77)
    u = rng.random(len(fl))
    nsub = np.where(u < 0.75, 1, rng.integers(2, 9, len(fl)))
    nsub[rng.choice(len(fl), 64, replace=False)] = 4096
    t0 = time.time()
    pool = rng.integers(0, 1_000_000, int(nsub.sum()), dtype=np.uint32)
    k = 0
    for f, c in zip(fl, nsub.tolist()):
        for s in pool[k:k + c].tolist():
            eng.subscribe(f, s)
        k += c
    log(f"[rank {rank}] {k} subscriptions in {time.time() - t0:.1f}s")
    eng.sync()
    b = eng.prepare(topics)
    for _ in range(max(args.warmup, 1)):
        b.launch().wait()
        b.dispatch_rows_device()
        b.dispatch_device()
    if sync is not None:
        sync.barrier()
    # one step = the match pipeline + the fan-out over the walk's rows as they
    # lie in staging (TM_DISPATCH_ROWS: no dense CSR first), kept in HBM
    ms_match, ms_fill, ms_disp = [], [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.launch().wait()
        td = time.perf_counter()
        total, fill_ms = b.dispatch_rows_device()
        ms_disp.append(1e3 * (time.perf_counter() - td))
        ms_fill.append(fill_ms)
        ms_match.append(b.stats()["ms_total"])
    elapsed = time.perf_counter() - t0
    if sync is not None:
        sync.barrier()
        elapsed = sync.allmax(elapsed)
    # the same with the publish-order CSR form (dense CSR built first)
    csr_disp, csr_fill = [], []
    for _ in range(args.steps):
        b.launch().wait()
        td = time.perf_counter()
        tot2, f2, *_ = b.dispatch_device()
        csr_disp.append(1e3 * (time.perf_counter() - td))
        csr_fill.append(f2)
    assert tot2 == total
    st = b.stats()
    n, m = len(topics), int(st["matches"])
    f_ms = float(np.mean(ms_fill))
    alg = 8 * total + 20 * m          # read + write a subscriber id; ids[j], moff[j], soff[f] per entry
    achieved = alg / (f_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_dispatch.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("workload") == "dispatch" and pmc.get("topics") == n:
                traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    out = {
        "metric": "publishes matched + fanned out/sec (node), C2 trie with local subscribers",
        "value": ws * n * args.steps / elapsed,
        "unit": "publishes/s",
        "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (seeded C2 generator + seeded subscriber counts)",
        "config": {"workload": f"dispatch: C2 1M filters, {k} subscriptions, {n} publishes per GPU",
                   "filters": len(fl), "subscriptions": k, "mode": "replicated"},
        "deliveries_per_step": int(total),
        "deliveries_per_s": ws * total * args.steps / elapsed,
        "match_pipeline_ms": float(np.mean(ms_match)),
        "dispatch_ms": float(np.mean(ms_disp)),
        "dispatch_form": "rows (TM_DISPATCH_ROWS: the walk's rows where they lie)",
        "dispatch_csr": {"dispatch_ms": float(np.mean(csr_disp)), "fill_ms": float(np.mean(csr_fill))},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "tm_fan_fill",
                     "kernel_ms": f_ms, "alg_bytes_per_launch": alg},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if sync is not None:
        sync.close()


def run_group(args):
    """Config C3 in ONE process (tm_group_*): the C2 trie replicated on devices
    0..N-1, one batch of N x the per-GPU publishes split into N contiguous
    slices matched concurrently (no collective).  Weak scaling like the
    torchrun form: every device gets --topics publishes."""
    from emqx_amd import gen
    from emqx_amd.engine import Group

    devs = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    ng = len(devs)
    p = gen.C2
    t0 = time.time()
    filters = gen.gen_filters(p)
    one = gen.gen_topics(p, filters, 1000, args.topics)
    # device k's slice is the publishes rank k would generate (seed 1000 + k)
    parts = [one] + [gen.gen_topics(p, filters, 1000 + k, args.topics) for k in range(1, ng)]
    topics = gen.Strings.concat(parts)
    del parts, one
    log(f"[group] {len(filters)} filters, {len(topics)} topics in {time.time() - t0:.1f}s")
    grp = Group(devs)
    t0 = time.time()
    grp.insert_many(filters)
    grp.sync()
    log(f"[group] {ng} replicas built+uploaded in {time.time() - t0:.1f}s")
    b = grp.prepare(topics)
    for _ in range(max(args.warmup, 1)):
        b.launch().wait()
    ms_match = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.launch().wait()
        ms_match.append(b.stats()["ms_match"])
    elapsed = time.perf_counter() - t0
    st = b.stats()
    n = len(topics)
    alg_bytes = (ALG_BYTES_PER_VISIT * (st["visits"] + st["hash_hits"]) + 4 * st["words"]
                 + 4 * st["matches"] + 4 * n) / ng      # per device
    k_ms = float(np.mean(ms_match))                      # slowest slice per step
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    out = {
        "metric": "publishes matched/sec (node) at 1M wildcard subs; p99 batch match latency",
        "value": n * args.steps / elapsed,
        "unit": "publishes/s",
        "n_gpus": ng,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded generator, SURVEY.md §8d C2/C3)",
        "config": {"workload": f"C3: 1M wildcard filters replicated on {ng} devices, {args.topics} publishes per "
                               f"device, one process (tm_group)", "devices": devs,
                   "filters": len(filters), "publishes_per_gpu": args.topics, "mode": "replicated, in-process",
                   "parallelism": f"replicated trie x{ng}, batch split in {ng} slices"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "tm_match_tiles",
                     "kernel_ms": k_ms, "alg_bytes_per_launch": alg_bytes},
        "matches_per_step": st["matches"],
    }
    # self-check: >= 3,000 sampled rows of every device's slice against one
    # replica on device 0 (a separate engine over the same filters).  The
    # sampled rows are gathered on each slice's device (tm_group_sample):
    # nothing else of the N x 10M-row result crosses to the host
    from emqx_amd import selfcheck as SC
    from emqx_amd.engine import Engine
    rep = grp.engine()
    lo = [n * k // ng for k in range(ng + 1)]
    host_bytes = [0]

    def grp_rows(idx):
        so, si = b.sample(idx)
        host_bytes[0] += so.nbytes + si.nbytes
        return SC.rows_from_csr(so, si, np.arange(len(idx)), SC.engine_names(rep))
    ref = Engine(device=0)
    ref.insert_many(filters)
    sc = group_selfcheck(grp_rows, topics, lo, [f"slice {k} (device {d})" for k, d in enumerate(devs)], ref)
    ref.close()
    sc["host_result_bytes"] = host_bytes[0]
    out["selfcheck"] = sc
    out["parity_sample_ok"] = sc["parity_sample_ok"]
    out["devices"] = devs
    b.free()
    grp.close()
    # per device the workload is the N = 1 line's (C2 trie, --topics publishes):
    # the committed PMC pass of that launch gives its HBM traffic
    out["roofline"]["traffic"] = pmc_traffic("C2", args.topics)
    if not args.no_cpu:
        # north_star: the CPU reference on this host's cores in the same run, at every N
        host = host_cpu_share()
        out["cpu_baseline"] = cpu_baseline(filters, topics, min(200_000, n), min(args.cpu_sample, n), host)
        out["speedup_vs_cpu_allcore"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out), flush=True)


def replica_selfcheck(eng, b, topics, sync, rank, label) -> dict:
    """After the timed region: this rank's waited batch b gives an evenly
    spaced sample of >= 3,000 rows (as filter bytes, digested); rank 0's engine
    -- one replica on device 0 -- matches every rank's sampled publishes and
    compares bit-exactly.  Rank 0 returns the verdict, every rank the same."""
    from emqx_amd import selfcheck as SC
    idx = SC.sample_index(len(topics))
    sample = [topics[int(i)] for i in idx]
    so, si = b.sample(idx)               # gathered on the device: ~3,000 rows, not the 10M-row CSR
    rows = SC.rows_from_csr(so, si, np.arange(len(idx)), SC.engine_names(eng))
    payloads = sync.allgather(SC.payload(sample, rows, label))
    verdict = "{}"
    if rank == 0:
        names = SC.engine_names(eng)

        def match_rows(ts):
            o, i = eng.match_batch(ts)
            return SC.rows_from_csr(o, i, np.arange(len(ts)), names)
        verdict = json.dumps(SC.check(payloads, match_rows))
    return json.loads(sync.allgather(verdict)[0])


def group_selfcheck(grp_rows, topics, lo, labels, ref_engine) -> dict:
    """In-process groups: slice k = publishes [lo[k], lo[k+1]) of the batch;
    grp_rows(idx) -> rows (filter bytes) of those publishes from the group's
    result; ref_engine = one replica on device 0 over the same filters."""
    from emqx_amd import selfcheck as SC
    payloads = []
    for k in range(len(lo) - 1):
        idx = lo[k] + SC.sample_index(lo[k + 1] - lo[k])
        payloads.append(SC.payload([topics[int(i)] for i in idx], grp_rows(idx), labels[k]))
    names = SC.engine_names(ref_engine)

    def match_rows(ts):
        o, i = ref_engine.match_batch(ts)
        return SC.rows_from_csr(o, i, np.arange(len(ts)), names)
    return SC.check(payloads, match_rows)


def fresh_latency(eng, filters, topics, batches: int) -> dict:
    """p50/p99 of tm_match_batch over `batches` never-repeated batches of B
    publishes (B = 4,096 and 65,536): host bytes -> host CSR of sorted ids.
    The batches are disjoint slices of the C2 publishes (more are generated
    when the resident ones run out); slicing happens before timing."""
    import ctypes as C

    from emqx_amd import _native as N
    from emqx_amd import gen
    out = {}
    pool = topics
    for bsz in (4096, 65536):
        need = bsz * (batches + 5)
        if len(pool) < need:
            extra = gen.gen_topics(gen.C2, filters, 7000 + len(pool), need - len(pool))
            pool = gen.Strings.concat([pool, extra])
        subs = []
        for i in range(batches + 5):
            sl = pool.slice(i * bsz, (i + 1) * bsz)
            subs.append((np.ascontiguousarray(sl.buf), np.ascontiguousarray(sl.offs.astype(np.uint64))))
        r = N.Result()
        lat = []
        for i, (buf, offs) in enumerate(subs):
            t = time.perf_counter()
            N.check(eng.L.tm_match_batch(eng.h, buf.ctypes.data, offs.ctypes.data, bsz, C.byref(r)), "tm_match_batch")
            dt = 1e3 * (time.perf_counter() - t)
            if i >= 5:                   # the first five size the pinned buffers
                lat.append(dt)
        out[str(bsz)] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                         "batches": len(lat), "distinct_batches": True,
                         "path": "host bytes -> tm_match_batch -> host CSR"}
    return out


def e2e_rate(eng, sub, reps: int = 3) -> dict:
    """tm_match_batch over `sub` from host bytes to the host CSR, best of `reps`
    after one warm-up call (pinned result buffers sized)."""
    import ctypes as C

    from emqx_amd import _native as N
    buf = np.ascontiguousarray(sub.buf)
    offs = np.ascontiguousarray(sub.offs.astype(np.uint64))
    r = N.Result()

    def call():
        N.check(eng.L.tm_match_batch(eng.h, buf.ctypes.data, offs.ctypes.data, len(sub), C.byref(r)), "tm_match_batch")

    call()
    best = float("inf")
    for _ in range(reps):
        t = time.perf_counter()
        call()
        best = min(best, time.perf_counter() - t)
    # stage breakdown through the split API (same work, separate calls)
    h = C.c_void_p()
    stages = {"prepare_h2d": [], "launch_wait": [], "result_d2h": []}
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        N.check(eng.L.tm_batch_prepare(eng.h, buf.ctypes.data, offs.ctypes.data, len(sub), C.byref(h)), "prepare")
        t1 = time.perf_counter()
        N.check(eng.L.tm_batch_launch(eng.h, h), "launch")
        N.check(eng.L.tm_batch_wait(eng.h, h), "wait")
        t2 = time.perf_counter()
        N.check(eng.L.tm_batch_result(eng.h, h, C.byref(r)), "result")
        t3 = time.perf_counter()
        for k, v in zip(stages, (t1 - t0, t2 - t1, t3 - t2)):
            stages[k].append(1e3 * v)
    eng.L.tm_batch_free(eng.h, h)
    return {"publishes_per_s": len(sub) / best, "topics": len(sub), "ms": 1e3 * best,
            "stages_ms": {k: min(v[1:]) for k, v in stages.items()},
            "bytes_in": int(offs[-1] - offs[0]), "matches_out": int(r.n_matches),
            "path": ("tm_match_batch: H2D bytes, device tokeniser, match, D2H CSR, chunks of 2^20 publishes "
                     "pipelined over two streams (best of %d; stages_ms: the same steps unpipelined)" % reps)}


def e2e_packed_rate(eng, sub, ref: dict, reps: int = 3) -> dict:
    """tm_match_batch_packed over `sub`: the same walk as e2e_rate, but the
    host receives 3-byte filter ids (n_filters <= 2^24) instead of uint32, a
    quarter less D2H. Checked against the uint32 call: same match count and
    row offsets, and the first 2^20 packed ids widen to the uint32 ids."""
    import ctypes as C

    from emqx_amd import _native as N
    buf = np.ascontiguousarray(sub.buf)
    offs = np.ascontiguousarray(sub.offs.astype(np.uint64))
    r = N.ResultPacked()

    def call():
        N.check(eng.L.tm_match_batch_packed(eng.h, buf.ctypes.data, offs.ctypes.data, len(sub), C.byref(r)),
                "tm_match_batch_packed")

    call()
    best = float("inf")
    for _ in range(reps):
        t = time.perf_counter()
        call()
        best = min(best, time.perf_counter() - t)
    n, m, ib = int(r.n_topics), int(r.n_matches), int(r.id_bytes)
    ok = m == ref["matches_out"]
    ro_p = np.ctypeslib.as_array(r.row_offsets, shape=(n + 1,)).copy()  # the u32 call reuses this buffer
    k = min(m, 1 << 20)
    head = np.ctypeslib.as_array(r.ids, shape=(k * ib,)).copy() if k else None
    u = N.Result()
    N.check(eng.L.tm_match_batch(eng.h, buf.ctypes.data, offs.ctypes.data, len(sub), C.byref(u)), "tm_match_batch")
    ro_u = np.ctypeslib.as_array(u.row_offsets, shape=(n + 1,))
    ok = ok and bool(np.array_equal(ro_p, ro_u))
    if k:
        raw = head.reshape(k, ib).astype(np.uint32)
        wide = np.zeros(k, np.uint32)
        for b in range(ib):
            wide |= raw[:, b] << np.uint32(8 * b)
        ok = ok and bool(np.array_equal(wide, np.ctypeslib.as_array(u.filter_ids, shape=(k,))))
    return {"publishes_per_s": len(sub) / best, "topics": len(sub), "ms": 1e3 * best, "id_bytes": ib,
            "matches_out": m, "bytes_out": m * ib + 4 * (n + 1), "parity_vs_u32_ok": ok,
            "path": ("tm_match_batch_packed: as e2e (uint32 ids) but ids packed to %d bytes on the device "
                     "before D2H (best of %d)" % (ib, reps))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 C2 steps = ~1 s timed: long enough for an outside utilisation sampler to see the GPU busy
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--topics", type=int, default=10_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="N = 1: skip the C5 legs of the default line")
    ap.add_argument("--inflight", type=int, default=1,
                    help="C2: batches in flight in the headline steps, each on its own stream (1 = one "
                         "batch on the engine stream: walk events and rocprof durations stay un-overlapped)")
    ap.add_argument("--cpu-sample", type=int, default=2_000_000)
    ap.add_argument("--latency-batches", type=int, default=200)
    ap.add_argument("--e2e-topics", type=int, default=10_000_000,
                    help="publishes of the host-inclusive end-to-end measurement")
    ap.add_argument("--profile", action="store_true",
                    help="only the timed steps (no latency / e2e / cpu legs): for rocprofv3 runs")
    ap.add_argument("--workload", choices=["c2", "c4", "c5", "dispatch", "coalesce"], default="c2",
                    help="c2: 1M wildcard filters, replicated (the BASELINE metric); c4: IoT filters, sharded; "
                         "c5: hot-topic skew + churn")
    ap.add_argument("--coalesce-linger-us", type=int, default=0, help="coalesce leg: batch linger")
    ap.add_argument("--coalesce-max-batch", type=int, default=16384, help="coalesce leg: largest device batch")
    ap.add_argument("--c5-k", type=int, default=100, help="C5 filters per hot topic (10 / 100 / 1000)")
    ap.add_argument("--c5-deltas", type=int, default=10_000, help="C5 subscribe/unsubscribe deltas per step")
    ap.add_argument("--c4-filters", type=int, default=0, help="C4 filter count (default 100M)")
    ap.add_argument("--devices", type=str, default="",
                    help="comma list of HIP devices: replicas of the in-process group (--gpus N without torchrun), "
                         "or the device of each local rank; default 0..N-1 (e.g. 0,0 rehearses 2 on one GPU)")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    devs = [int(x) for x in args.devices.split(",")] if args.devices else None
    if devs and ws > 1:
        local = devs[local]
    if ws > 1 and ws != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {ws}; using WORLD_SIZE")
    pg = None
    if ws == 1 and args.workload == "c4":
        return run_c4_group(args)   # one process, torch-free (tm_sharded)
    if ws > 1 and args.workload == "c4":
        # the filter-sharded exchange is RCCL: torch (and its HIP runtime) is
        # initialised before the engine library loads, so both share one runtime
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        pg = dist
    if args.workload == "c4":
        return run_c4(args, ws, rank, local, pg)
    sync = None
    if ws > 1:
        # replicated mode has no data-path collective: a host file barrier and
        # max-reduce line the ranks up (emqx_amd/hostsync.py), no torch
        from emqx_amd.hostsync import FileGroup
        sync = FileGroup(rank, ws)
    if args.workload == "c5":
        return run_c5(args, ws, rank, local, sync)
    if args.workload == "dispatch":
        return run_dispatch(args, ws, rank, local, sync)
    if args.workload == "coalesce":
        return run_coalesce(args, ws, rank, local, sync)
    if ws == 1 and args.gpus > 1:
        return run_group(args)

    from emqx_amd import gen
    from emqx_amd.engine import Engine

    p = gen.C2
    t0 = time.time()
    filters = gen.gen_filters(p)
    topics = gen.gen_topics(p, filters, 1000 + rank, args.topics)
    log(f"[rank {rank}] generated {len(filters)} filters, {len(topics)} topics in {time.time() - t0:.1f}s")

    eng = Engine(device=local)
    t0 = time.time()
    eng.insert_many(filters)
    eng.sync()
    est = eng.stats()
    log(f"[rank {rank}] trie built+uploaded in {time.time() - t0:.1f}s: {est}")

    t0 = time.time()
    # args.inflight batches of the same publishes, each on a stream of its own
    # (TM_BATCH_STREAM): batch i + 1 is launched before batch i is waited for,
    # so one batch's CSR pass overlaps the next one's walk
    nb = max(1, args.inflight)
    bs = [eng.prepare(topics, stream=nb > 1) for _ in range(nb)]
    b = bs[0]
    log(f"[rank {rank}] {nb} batch(es) resident in HBM in {time.time() - t0:.1f}s")

    # the first launch tokenises the resident bytes on the device (tm_tok_*);
    # the timed steps reuse the tokens (the dictionary does not change), so a
    # step is the trie walk (+ generic path) over a tokenised batch in HBM,
    # leaving the rows where the walk wrote them
    for _ in range(max(args.warmup, 1)):
        for x in bs:
            x.launch().wait()
    st = b.stats()
    if st["topics"] != len(topics):
        raise RuntimeError(f"batch stats inconsistent: {st}")

    # every step's wait() drains that batch's stream; the loop ends on a wait,
    # so the device is idle at both ends of the timed region
    if sync is not None:
        sync.barrier()
    ms_match, ms_total = [], []
    t0 = time.perf_counter()
    timed_steps(bs, args.steps, ms_match, ms_total)
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if sync is not None:
        sync.barrier()
        elapsed = sync.allmax(elapsed)

    n = len(topics)
    value = ws * n * args.steps / elapsed
    ms_step = 1e3 * elapsed / args.steps
    # the timed launch checks itself (oracle as the checker, outside the timed
    # region): N = 1 against the CPU restatement; N > 1 below against rank 0's
    # replica on device 0
    c2_check = None
    if ws == 1 and not args.profile:
        c2_check = c2_selfcheck(eng, b, filters, topics)
        if not c2_check["parity_sample_ok"]:
            log(f"[rank 0] C2 PARITY SAMPLE FAILED: {c2_check}")

    # fresh batches: the same resident bytes tokenised again every launch, so a
    # step is the whole device pipeline of a never-seen batch (tokenise + walk
    # + CSR); reported beside the headline, which reuses the tokens
    fresh_ms, fresh_tok = [], []
    for _ in range(max(3, min(args.steps, 10))):
        b.retokenize().launch().wait()
        s = b.stats()
        fresh_ms.append(s["ms_tokenize"] + s["ms_total"])
        fresh_tok.append(s["ms_tokenize"])

    # roofline of the dominant kernel (tm_match_tiles): algorithmic bytes per launch
    alg_bytes = (ALG_BYTES_PER_VISIT * (st["visits"] + st["hash_hits"]) + 4 * st["words"]
                 + 4 * st["matches"] + 4 * n)
    k_ms = float(np.mean(ms_match))
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    traffic = pmc_traffic("C2", n)

    out = {
        "metric": "publishes matched/sec (node) at 1M wildcard subs; p99 batch match latency",
        "value": value,
        "unit": "publishes/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded generator, SURVEY.md §8d C2)",
        "config": {"workload": "C2: 1M wildcard filters depth<=7, 10M-publish batch per GPU",
                   "filters": len(filters), "publishes_per_gpu": n, "mode": "replicated",
                   "parallelism": f"replicated trie x{ws}, batches split per GPU",
                   "batches_in_flight": nb},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_source("C2") if traffic else None,
                     "kernel": "tm_match_tiles", "kernel_ms": k_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "per_publish": {"V": st["visits"] / n, "H": st["hash_hits"] / n,
                                     "d": st["words"] / n, "M": st["matches"] / n,
                                     "bucket_reads": st["probes"] / n},
                     # frontier iterations: each pops <= 64 probes and waits for their reads
                     "iterations_per_tile": st["iterations"] / max(1, -(-n // 64)),
                     "probes_per_iteration": st["probes"] / max(1, st["iterations"])},
        "pipeline_ms": float(np.mean(ms_total)),
        "pipeline_fresh_ms": float(np.median(fresh_ms)),
        "tokenize_ms": float(np.median(fresh_tok)),
        "fresh_publishes_per_s": ws * n / (1e-3 * float(np.median(fresh_ms))),
        "matches_per_step": st["matches"],
        "slow_path_topics": st["slow_topics"],
    }
    if c2_check is not None:
        out["selfcheck"] = c2_check
        out["parity_sample_ok"] = c2_check["parity_sample_ok"]

    # the same steps with the dense CSR built after every wait (scan + copy
    # of every row into topic order, tm_batch_device_csr): what a consumer
    # that indexes the result by offsets pays per batch
    if nb == 1:
        csr_ms = []
        t2 = time.perf_counter()
        for _ in range(args.steps):
            b.launch().wait()
            b.device_csr()
            csr_ms.append(b.stats()["ms_csr"])
        e2 = time.perf_counter() - t2
        if sync is not None:
            e2 = sync.allmax(e2)
        out["dense_csr"] = {"publishes_per_s": ws * n * args.steps / e2, "ms_per_step": 1e3 * e2 / args.steps,
                            "csr_ms": float(np.mean(csr_ms))}

    if nb == 1 and not args.profile:
        # two batches in flight on streams of their own (TM_BATCH_STREAM): one
        # batch's CSR pass and walk tail overlap the next one's walk.  Beside
        # the headline, which keeps one batch so its walk events and rocprof
        # durations are un-overlapped
        b2 = [eng.prepare(topics, stream=True) for _ in range(2)]
        for x in b2:
            x.launch().wait()
        if sync is not None:
            sync.barrier()
        t2 = time.perf_counter()
        timed_steps(b2, args.steps)
        e2 = time.perf_counter() - t2
        if sync is not None:
            sync.barrier()
            e2 = sync.allmax(e2)
        out["two_in_flight"] = {"publishes_per_s": ws * n * args.steps / e2, "ms_per_step": 1e3 * e2 / args.steps}
        for x in b2:
            x.free()

    if ws > 1:
        # self-check of the multi-GPU run: every rank's sampled rows (as filter
        # bytes) must equal what rank 0's replica on device 0 returns for the
        # same publishes (emqx_amd/selfcheck.py)
        out["devices"] = [int(x) for x in sync.allgather(str(local))]
        out["selfcheck"] = replica_selfcheck(eng, b, topics, sync, rank, f"rank {rank} (device {local})")
        out["parity_sample_ok"] = out["selfcheck"]["parity_sample_ok"]
        if rank == 0 and not out["parity_sample_ok"]:
            log(f"[rank 0] PARITY SAMPLE FAILED: {out['selfcheck']}")

    if args.profile:
        args.no_cpu = True
    if rank == 0 and not args.profile:
        # p99 batch latency (device-resident batches, launch -> results in HBM)
        # at B = 4,096 / 65,536 / 1,048,576; the headline
        # p99_batch_ms is B = 65,536
        sweep = {}
        for bsz in (4096, 65536, 1 << 20):
            try:
                lb = eng.prepare(topics.slice(0, min(bsz, n)))
                for _ in range(5):
                    lb.launch().wait()
                lat = []
                for _ in range(args.latency_batches):
                    t = time.perf_counter()
                    lb.launch().wait()
                    lat.append(1e3 * (time.perf_counter() - t))
                lb.free()
                sweep[str(bsz)] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                                   "batches": len(lat)}
            except Exception as e:  # report, don't hide
                sweep[str(bsz)] = {"error": str(e)}
        main_lat = sweep.get("65536", {})
        out["p99_resident_ms"] = main_lat.get("p99_ms")
        out["p50_resident_ms"] = main_lat.get("p50_ms")
        out["latency_sweep"] = sweep
        if "error" in main_lat:
            out["latency_error"] = main_lat["error"]
        # the headline latency, SURVEY.md §8d's "batch submit -> results
        # ready": new topic bytes in host memory -> tm_match_batch (H2D,
        # device tokeniser, walk, CSR, D2H) -> sorted ids in host memory, a
        # different slice of publishes every batch, B = 65,536
        out["fresh_latency_sweep"] = fresh_latency(eng, filters, topics, args.latency_batches)
        fl = out["fresh_latency_sweep"]["65536"]
        out["p99_batch_ms"] = fl["p99_ms"]
        out["p50_batch_ms"] = fl["p50_ms"]
        out["latency_batch"] = 65536
        out["latency_path"] = "submit -> results ready: " + fl["path"] + " (fresh publishes every batch)"
        # the drop-in per-publish path: emqx_trie:match/1 once per publish
        # (the NIF's match/2), async and blocking, on this C2 trie
        out["coalesce"] = coalesce_brief(eng, topics)
        # host-inclusive end to end, timed at the C ABI (tm_match_batch): topic
        # bytes in host RAM -> H2D -> device tokenise -> match -> sorted CSR in
        # the engine's pinned host buffers (what a NIF hands to the broker)
        e2e_sub = topics.slice(0, min(n, args.e2e_topics))
        out["e2e"] = e2e_rate(eng, e2e_sub)
        # the same with 3-byte ids on the wire: the host-delivered headline
        out["e2e_packed"] = e2e_packed_rate(eng, e2e_sub, out["e2e"])
        out["e2e_u32_publishes_per_s"] = out["e2e"]["publishes_per_s"]
        out["e2e_host_publishes_per_s"] = max(out["e2e"]["publishes_per_s"],
                                              out["e2e_packed"]["publishes_per_s"])

    for x in bs:
        x.free()

    if rank == 0 and not args.no_cpu:
        # north_star: the CPU reference timed on this host's cores in the same
        # run at every N (rank 0, after the timed region; the other ranks are done)
        host = host_cpu_share()
        out["cpu_baseline"] = cpu_baseline(filters, topics, min(200_000, n), min(args.cpu_sample, n), host)
        out["speedup_vs_cpu_allcore"] = value / out["cpu_baseline"]["value"]
        if "coalesce" in out:
            cv = out["cpu_baseline"]["value"]
            out["coalesce"]["cpu_port_publishes_per_s"] = cv
            out["coalesce"]["async_vs_cpu_port"] = out["coalesce"]["async_calls_per_s"] / cv
            out["coalesce"]["sync_vs_cpu_port"] = out["coalesce"]["sync_calls_per_s"] / cv
        if ws == 1:
            out["c1"] = c1_leg(host, device=local)
    if rank == 0 and ws == 1 and not args.profile and not args.no_c5:
        # config C5 in the driver's line: K = 100, 10 and 1000 filters per hot
        # topic, 10k subscribe/unsubscribe deltas per step; each leg checks
        # its last step's batch against the oracle on that step's snapshot
        # 30 steps: the timed region holds the first delta's churn (nothing
        # on the device beside it) and the last batch's walk (no churn beside
        # it) -- ~2-4 ms of fill and drain, 0.2-0.4 ms per step over 10
        # steps, ~0.1 over 30 (the device runs back to back in between:
        # profiles/r06/s3/c5_k1000_timeline.txt)
        out["c5"] = {f"k{k}": c5_leg(k, 30, 10_000, args.topics, device=local) for k in (100, 10, 1000)}
        out["parity_sample_ok"] = bool(out.get("parity_sample_ok", True)
                                       and all(v.get("parity_sample_ok") for v in out["c5"].values()))

    if rank == 0:
        print(json.dumps(out), flush=True)
    if sync is not None:
        sync.close()


if __name__ == "__main__":
    main()
