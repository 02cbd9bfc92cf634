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
