"""One-screen summary of a bench.py JSON line (tools/gpu.sh): the headline,
roofline, and whichever legs the line carries.

    python tools/summarize.py FILE.json
"""
import json
import sys


def g(v, d=3):
    return round(v / 1e9, d) if isinstance(v, (int, float)) else v


def main(path):
    lines = [x for x in open(path).read().strip().splitlines() if x.startswith("{")]
    if not lines:
        print("no JSON line in", path)
        return
    d = json.loads(lines[-1])
    out = [f"{d.get('metric', '?')[:48]}: {g(d.get('value'))} G {d.get('unit', '')}, n_gpus {d.get('n_gpus')}, "
           f"ms/step {round(d.get('ms_per_step', 0), 3)}"]
    r = d.get("roofline")
    if r:
        out.append(f"  roofline {r.get('kernel')}: {round(r['kernel_ms'], 3)} ms, frac {round(r['frac'], 3)}, "
                   f"traffic {r.get('traffic')}")
    for k in ("fresh_publishes_per_s", "e2e_host_publishes_per_s", "two_in_flight", "dense_csr", "tokenize_ms",
              "p99_batch_ms", "parity_sample_ok", "speedup_vs_cpu_allcore", "distinct_topics_per_s",
              "device_pipeline_ms", "churn_apply_ms", "prepare_ms", "dispatch_ms", "deliveries_per_s", "fresh_ms"):
        if k in d:
            v = d[k]
            if isinstance(v, dict) and "publishes_per_s" in v:
                v = g(v["publishes_per_s"])
            elif isinstance(v, float) and v > 1e6:
                v = g(v)
            elif isinstance(v, float):
                v = round(v, 3)
            out.append(f"  {k}: {v}")
    if "fresh_latency_sweep" in d:
        out.append("  fresh lat " + str({k: (round(v['p50_ms'], 3), round(v['p99_ms'], 3))
                                         for k, v in d["fresh_latency_sweep"].items()}))
    if "selfcheck" in d:
        sc = d["selfcheck"]
        out.append(f"  selfcheck ok {sc.get('parity_sample_ok')} rows {sc.get('sampled_rows')} "
                   f"host bytes {sc.get('host_result_bytes')}")
    if "cpu_baseline" in d:
        out.append(f"  cpu {round(d['cpu_baseline']['value'])} /s on {d['cpu_baseline']['cores']}")
    for k, v in (d.get("c5") or {}).items():
        out.append(f"  c5 {k}: {g(v['publishes_per_s'])} G, ms {round(v['ms_per_step'], 3)}, dev "
                   f"{round(v['device_ms'], 3)}, churn {round(v['churn_ms'], 3)}")
    if "legs" in d:
        for k, v in d["legs"].items():
            out.append(f"  {k}: {round(v['calls_per_s'] / 1e6, 3)} M/s p50 {round(v['p50_us'])} p99 "
                       f"{round(v['p99_us'])} us")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1])
