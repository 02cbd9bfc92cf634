#!/usr/bin/env python3
"""Summarise rocprofv3 CSVs (tools/profile.sh) per kernel: mean duration and mean PMC counters per
dispatch. gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of wide
streaming reads, so hbm_read_bytes = 2 * FETCH_SIZE * 1024 (an upper bound for narrower reads);
WRITE_SIZE is taken at face value (exact for 16-B/lane stores; ours are 4-B/lane dword stores)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    """Kernel name without namespace / parameter list: k_raster<false, 5, *> and k_raster_plain<false, ..>
    -> k_raster (the fast build, the one the bench runs), k_raster<true, 5, *> -> k_raster_exact; k_setup<true, *> (the
    shadow pre-pass set-up) -> k_setup_shadow, k_setup<false, *> -> k_setup."""
    m = re.search(r"(k_[a-z_]+)(<([a-z]+)[^>]*>)?\(", name)
    if m:
        first = m.group(3) == "true"
        if m.group(1) == "k_setup":
            return "k_setup_shadow" if first else "k_setup"
        # k_raster_plain (frames without the shadow pre-pass) and k_raster<.., true> (with it) are the
        # frame's raster kernel either way
        base = "k_raster" if m.group(1) == "k_raster_plain" else m.group(1)
        return base + ("_exact" if first else "")
    for k in ("copyBuffer", "fillBuffer"):
        if k in name:
            return k
    return name[:40]


def main(root, workload, out_json):
    res = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            res[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    stats = {}
    for f in glob.glob(os.path.join(root, "*", "*_kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            stats[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                         "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}
    summary = {}
    for k in sorted(set(res) | set(stats)):
        e = {"trace": stats.get(k)}
        for c, v in res[k].items():
            e[c] = sum(v) / len(v)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_read_bytes_corrected"] = 2 * e["FETCH_SIZE"] * 1024
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]
        summary[k] = e
    doc = {}
    if os.path.exists(out_json):
        doc = json.load(open(out_json))
    doc[workload] = summary
    json.dump(doc, open(out_json, "w"), indent=1, sort_keys=True)
    for k, e in summary.items():
        t = e.get("trace") or {}
        print(f"{k:16s} avg {t.get('avg_ns', 0)/1e3:8.1f} us  " +
              "  ".join(f"{c}={v:.4g}" for c, v in sorted(e.items()) if c != "trace"))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
