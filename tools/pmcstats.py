"""Per-kernel PMC counter sums from rocprofv3 SQLite databases (dev tool).

    python tools/pmcstats.py KERNEL_SUBSTRING db [db ...]
Prints, per counter, the value summed over the kernel's dispatches divided by
the number of dispatches (per-launch average)."""
import collections
import sqlite3
import sys

pat = sys.argv[1]
for db in sys.argv[2:]:
    c = sqlite3.connect(db)
    vals = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    dur = {}
    for name, cn, v, d, s, e in c.execute(
            "select kernel_name, counter_name, value, dispatch_id, start, end from counters_collection"):
        if pat in name:
            vals[cn] += v
            disp[cn].add(d)
            dur[d] = e - s
    for k in sorted(vals):
        print(f"{k:28s} {vals[k] / max(len(disp[k]), 1):16.0f}")
    if dur:
        print(f"{'duration_us':28s} {sum(dur.values()) / len(dur) / 1e3:16.1f}")
