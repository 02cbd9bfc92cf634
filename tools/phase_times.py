#!/usr/bin/env python3
"""k_raster phase durations per workgroup (diagnostics build):
    bash tools/build_variant.sh phase -DTRI_PHASE_TIMING
    TRI_RASTER_LIB=3d-renderer_amd/lib/variants/phase.so python tools/phase_times.py [c3|c2|c5] [world/rank]
Phases (wave 0's s_memtime after each workgroup barrier): init (LDS clear + queue count), coverage,
large triangles, shading + stores, skybox. Prints the mean / median / p90 cycles per phase and the
workgroup duration distribution."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-renderer_amd", "python"))
from trident_raster import raster, scenes  # noqa: E402


def setup_phases(lib, n):
    """k_setup per workgroup: first round's fetch + set-up, its binning, the rest to the end."""
    buf = (C.c_ulonglong * (n * 4))()
    assert lib.tri_debug_setup_times(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)
    a = a[a[:, 0] != 0]
    d = np.diff(a, axis=1)
    tot = a[:, 3] - a[:, 0]
    span = a[:, 3].max() - a[:, 0].min()
    print(f"k_setup: {len(a)} workgroups; span of the launch {span} ticks")
    for k, nm in enumerate(["fetch+setup", "binning", "rest"]):
        x = d[:, k]
        print(f"  {nm:12s} mean {x.mean():9.0f}  median {np.median(x):9.0f}  p90 {np.percentile(x, 90):9.0f}")
    print(f"  {'total':12s} mean {tot.mean():9.0f}  median {np.median(tot):9.0f}  p90 {np.percentile(tot, 90):9.0f}")
    st = a[:, 0] - a[:, 0].min()
    print(f"  start offsets: median {np.median(st):.0f}  p90 {np.percentile(st, 90):.0f}  max {st.max()}")


def main(which="c3", band=None):
    lib = raster.load_library()
    s = {"c3": scenes.scene_c3_grid, "c2": scenes.scene_c2_sphere, "c5": scenes.scene_c5_textured}[which]()
    n = 65536
    buf = (C.c_ulonglong * (n * 6))()
    if band:  # "world/rank": the rows of that band (cluster culling on)
        world, rank = (int(x) for x in band.split("/"))
        band = (s.height * rank // world, s.height * (rank + 1) // world)
    with raster.TriRaster(s.width, s.height, band=band) as r:
        scenes.load_scene(r, s)
        for _ in range(8):
            r.render_frame()
        r.synchronize()
        assert lib.tri_debug_phase_times(buf, n) == 0
        setup_phases(lib, n)
        st = {}
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 6).astype(np.int64)
    nb = int((a[:, 0] != 0).sum())
    a = a[:nb]
    names = ["init", "coverage", "big", "shade", "sky"]
    d = np.diff(a, axis=1)
    tot = a[:, 5] - a[:, 0]
    print(f"{which}: {nb} workgroups; cycles per workgroup (s_memtime ticks)")
    for k, nm in enumerate(names):
        x = d[:, k]
        print(f"  {nm:9s} mean {x.mean():9.0f}  median {np.median(x):9.0f}  p90 {np.percentile(x, 90):9.0f}  "
              f"share {x.sum() / tot.sum():6.1%}")
    print(f"  {'total':9s} mean {tot.mean():9.0f}  median {np.median(tot):9.0f}  p90 {np.percentile(tot, 90):9.0f}  "
          f"max {tot.max():9.0f}")
    print("  stats:", st)


if __name__ == "__main__":
    main(*(sys.argv[1:] or ["c3"]))
