#!/usr/bin/env python3
"""Distinct primitives per wave in k_raster_plain's shading loop (diagnostics build), the number a triangle-grouped
fragment set-up would loop over:
    bash tools/build_variant.sh groups -DTRI_PRIM_GROUPS
    TRI_RASTER_LIB=3d-renderer_amd/lib/variants/groups.so python tools/prim_groups.py [c3|c2|c3trs]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-renderer_amd", "python"))
from trident_raster import raster, scenes  # noqa: E402


def main(which="c3"):
    lib = raster.load_library()
    s = {"c3": scenes.scene_c3_grid, "c2": scenes.scene_c2_sphere, "c3trs": scenes.scene_c3_trs}[which]()
    buf = (C.c_ulonglong * 3)()
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        r.synchronize()
        assert lib.tri_debug_prim_groups(buf, 1) == 0
        r.render_frame()
        r.synchronize()
        assert lib.tri_debug_prim_groups(buf, 0) == 0
    it, groups, lanes = buf[0], buf[1], buf[2]
    print(f"{which}: {it} wave-iterations with shaded lanes, {lanes} shaded lanes "
          f"({lanes / it:.1f} per iteration), {groups / it:.2f} distinct primitives per iteration "
          f"({lanes / groups:.2f} lanes per primitive)")


if __name__ == "__main__":
    main(*(sys.argv[1:] or ["c3"]))
