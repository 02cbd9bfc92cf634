"""Host-side bench logic (no GPU): the CPU baseline's core count."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _cg(tmp_path, text):
    (tmp_path / "cpu.max").write_text(text)
    return str(tmp_path)


def test_effective_cpus_cgroup_quota(tmp_path):
    aff = len(os.sched_getaffinity(0))
    r = bench.effective_cpus(_cg(tmp_path, "150000 100000\n"))  # 1.5 CPUs -> 2 threads
    assert r["quota"] == 2 and r["affinity"] == aff and r["effective"] == min(aff, 2)


def test_effective_cpus_unlimited(tmp_path):
    r = bench.effective_cpus(_cg(tmp_path, "max 100000\n"))
    assert r["quota"] is None and r["effective"] == r["affinity"] == len(os.sched_getaffinity(0))


def test_effective_cpus_cgroup_v1(tmp_path):
    d = tmp_path / "cpu"
    d.mkdir()
    (d / "cpu.cfs_quota_us").write_text("100000\n")
    (d / "cpu.cfs_period_us").write_text("100000\n")
    r = bench.effective_cpus(str(tmp_path))
    assert r["quota"] == 1 and r["effective"] == 1


def test_effective_cpus_missing(tmp_path):
    r = bench.effective_cpus(str(tmp_path / "absent"))
    assert r["quota"] is None and r["effective"] >= 1


def _gpurun_excluded(rel, patterns):
    """tar-style exclusion as gpurun applies .gpurunignore: a pattern with a leading './' is anchored at the
    tree's top, others match any path component suffix; a match on a directory excludes what is under it."""
    import fnmatch

    rel = rel.lstrip("./")
    parts = rel.split("/")
    for p in patterns:
        if p.startswith("./"):
            pat = p[2:]
            for i in range(1, len(parts) + 1):
                if fnmatch.fnmatch("/".join(parts[:i]), pat):
                    return True
        else:
            for i in range(len(parts)):
                for j in range(i + 1, len(parts) + 1):
                    if fnmatch.fnmatch("/".join(parts[i:j]), p):
                        return True
    return False


def test_pmc_summary_travels_and_names_k_raster():
    """bench.py fills roofline.traffic and roofline_valu from profiles/pmc_summary.json on the GPU box (VERDICT r4
    'What's weak' #2: .gpurunignore once dropped it, and both fields went null on the driver's line)."""
    pats = [l.strip() for l in open(os.path.join(ROOT, ".gpurunignore")) if l.strip() and not l.startswith("#")]
    assert not _gpurun_excluded("./profiles/pmc_summary.json", pats)
    assert _gpurun_excluded("./profiles/round4/c3_kernel_stats.csv", pats)  # the self-test of the matcher
    e = bench.pmc_kernel("c3_grid1m_3840x2160", "k_raster")
    assert e is not None
    assert e["hbm_bytes_per_launch"] > 66e6 and e["SQ_INSTS_VALU"] > 1e7
    assert bench.valu_floor_frac(e, 8.0 * 3840 * 2160) > 0.05


def test_pmc_summary_missing_is_loud(tmp_path, capsys):
    assert bench.pmc_kernel("c3_grid1m_3840x2160", "k_raster", path=str(tmp_path / "absent.json")) is None
    assert "WARNING" in capsys.readouterr().err
    (tmp_path / "s.json").write_text('{"c3_grid1m_3840x2160": {}}')
    assert bench.pmc_kernel("c3_grid1m_3840x2160", "k_raster", path=str(tmp_path / "s.json")) is None
    assert "no k_raster entry" in capsys.readouterr().err
