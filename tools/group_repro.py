#!/usr/bin/env python3
"""Diagnostics: render the full C3 frame as a tri_group of 8 bands on device 0 a few times and compare
each frame (colour + depth) with the single-context frame; prints the mismatching rows per band."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-renderer_amd", "python"))
from trident_raster import abi, raster, scenes  # noqa: E402


def main(mode="exact", reps=4):
    flags = abi.TRI_FLAG_EXACT_SHADING if mode == "exact" else 0
    s = scenes.scene_c3_grid()
    with raster.TriRaster(s.width, s.height, flags=flags) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        fc, fd = r.readback()
    rows = s.height // 8
    with raster.TriGroup(s.width, s.height, [0] * 8, display=0, flags=flags) as grp:
        scenes.load_scene(grp, s)
        for k in range(int(reps)):
            grp.render_frame()
            gc, gd = grp.readback()
            bad_d = np.argwhere(gd != fd)
            bad_c = np.argwhere((gc != fc).any(-1))
            per_band = [int(((bad_d[:, 0] >= b * rows) & (bad_d[:, 0] < (b + 1) * rows)).sum()) for b in range(8)]
            print(f"{mode} frame {k}: depth mismatches {len(bad_d)} per band {per_band}, colour mismatches {len(bad_c)}")
            if len(bad_d):
                y, x = bad_d[0]
                print("   first", y, x, hex(gd[y, x]), hex(fd[y, x]), "rows", np.unique(bad_d[:, 0])[:20])


if __name__ == "__main__":
    main(*sys.argv[1:])
