#!/usr/bin/env python3
"""Summarise the FETCH_SIZE calibration (tools/fetch_calib.sh) into one JSON document.

Per probe kernel: the known bytes of its access shape, FETCH_SIZE in bytes, the sized-request byte count
32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B, and the ratios. The ratio truth / FETCH_SIZE on the shapes
with known truth is the calibration tools/prof_summary.py applies (see its docstring)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def kname(name):
    m = re.match(r"\s*(?:void\s+)?(k_cal_[a-z0-9]+)", name)
    return m.group(1) if m else None


def load(root):
    res = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = kname(row["Kernel_Name"])
            if k:
                res[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    trace = {}
    for f in glob.glob(os.path.join(root, "*", "*_kernel_stats.csv")):
        for row in csv.DictReader(open(f)):
            k = kname(row["Name"])
            if k:
                trace[k] = float(row["AverageNs"])
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in res.items()}, trace


def main(root, out_json=None):
    plain = json.load(open(os.path.join(root, "plain.json")))["cases"]
    pmc, trace = load(root)
    rows = []
    for case in plain:
        k = case["kernel"]
        e = pmc.get(k, {})
        fetch = e.get("FETCH_SIZE", 0.0) * 1024
        sized = (32 * e.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64 * e.get("TCC_EA0_RDREQ_64B_sum", 0.0)
                 + 128 * e.get("TCC_EA0_RDREQ_128B_sum", 0.0))
        truth = case["truth_bytes"] or None
        row = {"kernel": k, "truth_bytes": truth, "footprint": case["footprint"], "fetch_size_bytes": fetch,
               "sized_bytes": sized, "trace_avg_ns": trace.get(k), "event_ms_min": case["ms_min"],
               "counters": e}
        if fetch:
            row["sized_over_fetch"] = sized / fetch
        if truth and fetch:
            row["truth_over_fetch"] = truth / fetch
        if truth and sized:
            row["sized_over_truth"] = sized / truth
        row["sized_over_footprint"] = sized / case["footprint"] if sized else None
        if trace.get(k):
            row["sized_gbs"] = sized / trace[k]
        rows.append(row)
    doc = {"probe": "tools/fetch_calib/fetch_calib.hip", "runner": "tools/fetch_calib.sh", "cases": rows}
    for r in rows:
        print(f"{r['kernel']:16s} truth {r['truth_bytes'] or 0:12.4g} fetch {r['fetch_size_bytes']:12.4g} "
              f"sized {r['sized_bytes']:12.4g} sized/fetch {r.get('sized_over_fetch', 0):.3f} "
              f"truth/fetch {r.get('truth_over_fetch', 0):.3f} sized/foot {r['sized_over_footprint'] or 0:.3f} "
              f"{(r['trace_avg_ns'] or 0) / 1e3:8.1f} us")
    out_json = out_json or os.path.join(root, "fetch_calib.json")
    json.dump(doc, open(out_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
