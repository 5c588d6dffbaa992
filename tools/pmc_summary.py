"""Fold rocprofv3 --pmc CSVs (tools/pmc_round.sh) into per-kernel averages.

    python tools/pmc_summary.py gpurun_out/TAG [--topics N] [--write profiles/pmc_latest.json]

Prints, per kernel and counter, the mean over dispatches.  With --write, stores
the HBM traffic of one tm_match_tiles launch as the guide prescribes
(MI355X_MICROARCH.md "HBM"): FETCH_SIZE doubled (gfx950 tallies wide reads at
half their bytes) plus WRITE_SIZE, both reported by rocprofv3 in KiB.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values per dispatch]
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?")
                c = row.get("Counter_Name", "?")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                acc[k][(c, row.get("Dispatch_Id"))].append(v)
    out = defaultdict(dict)
    for k, d in acc.items():
        per = defaultdict(list)
        for (c, _disp), vals in d.items():
            per[c].append(sum(vals))        # sum over dimensions/instances of one dispatch
        for c, vals in per.items():
            out[k][c] = sum(vals) / len(vals)
    return out


def short(k):
    return k.split("(")[0].replace("void ", "").replace("etm::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--topics", type=int, default=10_000_000)
    ap.add_argument("--write", default=None)
    ap.add_argument("--workload", default="C2")
    ap.add_argument("--filters", type=int, default=0)
    ap.add_argument("--kernel", default="tm_match_tiles")
    args = ap.parse_args()
    res = load(args.root)
    if not res:
        print("no counter_collection.csv under", args.root)
        return 1
    for k in sorted(res):
        print(short(k))
        for c in sorted(res[k]):
            print(f"    {c:32s} {res[k][c]:.6g}")
    if args.write:
        mt = [k for k in res if args.kernel in k]
        if not mt:
            print(args.kernel, "not found")
            return 1
        r = res[mt[0]]
        fetch_kib = r.get("FETCH_SIZE")
        write_kib = r.get("WRITE_SIZE")
        info = {"workload": args.workload, "topics": args.topics, "kernel": short(mt[0]),
                "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
                "hbm_bytes_per_launch": None, "filters": args.filters or None,
                "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB -> bytes; "
                        "the 16-B bucket loads are the calibrated width, the 4/8-B stores are not"}
        if fetch_kib is not None and write_kib is not None:
            info["hbm_bytes_per_launch"] = (2 * fetch_kib + write_kib) * 1024
        for key in ("TCC_HIT_sum", "TCC_MISS_sum"):
            if key in r:
                info[key] = r[key]
        if "TCC_HIT_sum" in r and "TCC_MISS_sum" in r and r["TCC_HIT_sum"] + r["TCC_MISS_sum"] > 0:
            info["l2_hit_rate"] = r["TCC_HIT_sum"] / (r["TCC_HIT_sum"] + r["TCC_MISS_sum"])
        with open(args.write, "w") as f:
            json.dump(info, f, indent=1)
        print(json.dumps(info, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
