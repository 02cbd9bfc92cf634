#!/usr/bin/env python3
"""tri_render's host time by phase, from a diagnostics build (tools/build_variant.sh hostt -DTRI_HOST_TIMING,
selected with TRI_RASTER_LIB): bursts of 16 calls after a drain, so the queue never fills.
    python tools/host_breakdown.py [c2|c3] [bursts]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-renderer_amd", "python"))
from trident_raster import raster, scenes  # noqa: E402

PHASES = ("make_current", "state checks + buffers", "frame arguments + plan", "launches", "total")


def main(which="c2", bursts=50):
    s = {"c2": scenes.scene_c2_sphere, "c3": scenes.scene_c3_grid}[which]()
    lib = raster.load_library()
    if not hasattr(lib, "tri_debug_host_times"):
        sys.exit("the loaded library is not a TRI_HOST_TIMING build")
    out = (C.c_double * 5)()
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        for _ in range(50):
            lib.tri_render(r._ctx)
        r.synchronize()
        lib.tri_debug_host_times(out, 1)
        for _ in range(int(bursts)):
            r.synchronize()
            for _ in range(16):
                lib.tri_render(r._ctx)
        r.synchronize()
        lib.tri_debug_host_times(out, 1)
    print(f"{which}: tri_render host ns per call: " + ", ".join(f"{p} {v:.0f}" for p, v in zip(PHASES, out)))


if __name__ == "__main__":
    main(*sys.argv[1:])
