"""Per-kernel durations from a rocprofv3 SQLite database (dev tool).

    python tools/kstats.py path/to/results.db [top]
"""
import collections
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = sqlite3.connect(db)
syms = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
d = collections.defaultdict(list)
for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
    d[syms.get(kid, kid)].append((e - s) / 1e3)
print(f"{'kernel':64s} {'calls':>6s} {'mean_us':>10s} {'min_us':>10s} {'max_us':>10s} {'total_ms':>10s}")
for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:top]:
    print(f"{k[:64]:64s} {len(v):6d} {sum(v)/len(v):10.1f} {min(v):10.1f} {max(v):10.1f} {sum(v)/1e3:10.3f}")
