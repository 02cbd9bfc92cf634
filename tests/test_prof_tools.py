"""The HBM traffic accounting behind bench.py's roofline.traffic (tools/prof_summary.py) and the committed
FETCH_SIZE calibration it rests on (profiles/round3/fetch_calib.json, tools/fetch_calib.sh)."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import prof_summary  # noqa: E402


def write_csv(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_sized_read_requests_preferred_over_fetch_size(tmp_path):
    name = "void (anonymous namespace)::k_raster_plain<false, 5, true>(TriFrameParams, TriDeviceBuffers)"
    counters = [("FETCH_SIZE", 1000.0), ("WRITE_SIZE", 500.0), ("TCC_EA0_RDREQ_32B_sum", 2.0),
                ("TCC_EA0_RDREQ_64B_sum", 3.0), ("TCC_EA0_RDREQ_128B_sum", 10.0)]
    write_csv(str(tmp_path / "p" / "p_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
              [(name, c, v) for c, v in counters])
    write_csv(str(tmp_path / "t" / "t_kernel_stats.csv"), ["Name", "Calls", "AverageNs", "MinNs", "MaxNs"],
              [(name, 4, 96000.0, 95000.0, 97000.0)])
    out = str(tmp_path / "s.json")
    prof_summary.main(str(tmp_path), "w", out)
    e = json.load(open(out))["w"]["k_raster"]
    assert e["hbm_read_bytes"] == 32 * 2 + 64 * 3 + 128 * 10
    assert e["hbm_read_bytes_corrected"] == 2 * 1000 * 1024
    assert e["hbm_bytes_per_launch"] == e["hbm_read_bytes"] + 500 * 1024
    assert e["hbm_read_method"].startswith("sized")
    assert e["trace"]["avg_ns"] == 96000.0


def test_fetch_size_fallback_without_sized_pass(tmp_path):
    name = "(anonymous namespace)::k_vertex(TriFrameParams, TriDeviceBuffers)"
    write_csv(str(tmp_path / "p" / "p_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
              [(name, "FETCH_SIZE", 10.0), (name, "WRITE_SIZE", 4.0)])
    out = str(tmp_path / "s.json")
    prof_summary.main(str(tmp_path), "w", out)
    e = json.load(open(out))["w"]["k_vertex"]
    assert e["hbm_read_bytes"] == 2 * 10 * 1024 and e["hbm_read_method"] == "2 x FETCH_SIZE"


def test_committed_calibration_pins_the_factor():
    """On every probe shape with a known byte count the sized requests equal it, and FETCH_SIZE is half of
    the sized count on all of them (12-B and 16-B gathers included)."""
    doc = json.load(open(os.path.join(ROOT, "profiles", "round3", "fetch_calib.json")))
    cases = {c["kernel"]: c for c in doc["cases"]}
    for k in ("k_cal_stream16", "k_cal_stream12", "k_cal_chunk16", "k_cal_chunk12", "k_cal_line16", "k_cal_line12",
              "k_cal_dense16", "k_cal_dense12"):
        c = cases[k]
        assert abs(c["sized_over_fetch"] - 2.0) < 0.01, k
        if c["truth_bytes"]:
            assert abs(c["sized_over_truth"] - 1.0) < 0.01, k
    # one 12-B or 16-B read per distinct line moves the whole 128-B line
    assert abs(cases["k_cal_line12"]["sized_over_footprint"] - 1.0) < 0.01
