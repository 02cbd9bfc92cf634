#!/usr/bin/env python3
"""Diagnostics: render the full C3 frame as a tri_group of 8 bands on device 0 and compare each frame (colour +
depth) with the single-context frame; prints the mismatching rows per band.
    python tools/group_repro.py [exact|fast] [frames] [poison byte, e.g. 0x5a]
With a poison byte, device memory is filled with it and released before the group is created, so buffers the
group's contexts read before writing hold that garbage instead of fresh zeros."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-renderer_amd", "python"))
from trident_raster import abi, raster, scenes  # noqa: E402


def poison(byte, chunks=48, size=64 << 20):
    hip = C.CDLL("libamdhip64.so")
    ptrs = []
    for _ in range(chunks):
        p = C.c_void_p()
        if hip.hipMalloc(C.byref(p), C.c_size_t(size)) != 0:
            break
        hip.hipMemset(p, C.c_int(byte), C.c_size_t(size))
        ptrs.append(p)
    hip.hipDeviceSynchronize()
    for p in ptrs:
        hip.hipFree(p)
    return len(ptrs)


def main(mode="exact", reps=2, poison_byte=None):
    flags = abi.TRI_FLAG_EXACT_SHADING if mode == "exact" else 0
    s = scenes.scene_c3_grid()
    with raster.TriRaster(s.width, s.height, flags=flags) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        fc, fd = r.readback()
    if poison_byte is not None:
        print("poisoned", poison(int(poison_byte, 0)), "chunks with", poison_byte)
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
