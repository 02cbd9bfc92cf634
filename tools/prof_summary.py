#!/usr/bin/env python3
"""Summarise rocprofv3 CSVs (tools/profile.sh) per kernel: mean duration and mean PMC counters per
dispatch.

Read bytes: FETCH_SIZE on gfx950 counts every 128-B L2->fabric read request as 64 B (MI355X_MICROARCH.md
§HBM). The calibration probe (tools/fetch_calib.sh, profiles/round3/fetch_calib.json) measured the sized
request counters against known bytes for every access shape k_raster uses -- coalesced 16-B and 12-B
streams, whole-line chunks in scrambled order, one 12-B / 16-B gather per distinct line, packed 12-B / 16-B
records gathered in random order, all over 1 GiB (4x the Infinity Cache):
32 * TCC_EA0_RDREQ_32B + 64 * TCC_EA0_RDREQ_64B + 128 * TCC_EA0_RDREQ_128B equals the known bytes exactly
on every shape with a known answer, and FETCH_SIZE is exactly half of it on all eight. So hbm_read_bytes is
that sized sum when the pass was collected (tools/profile.sh pmc_sized), else 2 * FETCH_SIZE * 1024: the
factor 2 is measured for 12-B and 16-B gathers as well, not only for streaming reads. These count requests
that leave L2, Infinity-Cache hits included. WRITE_SIZE is taken at face value (k_raster's colour + depth
stores: 66.4 MB per C3 launch, the algorithmic 8 B per pixel exactly)."""
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
        sized = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
        if all(c in e for c in sized):
            e["hbm_read_bytes_sized"] = 32 * e[sized[0]] + 64 * e[sized[1]] + 128 * e[sized[2]]
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes_corrected"] = 2 * e["FETCH_SIZE"] * 1024
        read = e.get("hbm_read_bytes_sized", e.get("hbm_read_bytes_corrected"))
        if read is not None and "WRITE_SIZE" in e:
            e["hbm_read_bytes"] = read
            e["hbm_read_method"] = ("sized TCC_EA0_RDREQ_{32B,64B,128B}" if "hbm_read_bytes_sized" in e
                                    else "2 x FETCH_SIZE")
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = read + e["hbm_write_bytes"]
        summary[k] = e
    doc = {}
    if os.path.exists(out_json):
        doc = json.load(open(out_json))
    doc[workload] = summary
    json.dump(doc, open(out_json, "w"), indent=1, sort_keys=True)
    for k, e in summary.items():
        t = e.get("trace") or {}
        print(f"{k:16s} avg {t.get('avg_ns', 0)/1e3:8.1f} us  " +
              "  ".join(f"{c}={v:.4g}" for c, v in sorted(e.items()) if isinstance(v, float)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
