#!/usr/bin/env python3
"""Host cost of enqueueing frames: time N back-to-back tri_render calls (no synchronisation inside) on one
context, then the drain; if the enqueue rate is the frame rate, the bench is host-bound at that size.
    python tools/host_overhead.py [c2|c3] [frames]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "3d-renderer_amd", "python"))
from trident_raster import abi, raster, scenes  # noqa: E402


def main(which="c2", n=2000):
    n = int(n)
    s = {"c2": scenes.scene_c2_sphere, "c3": scenes.scene_c3_grid}[which]()
    lib = raster.load_library()
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        ctx = r._ctx
        ubo, clear = C.byref(s.ubo), C.byref((C.c_float * 4)(*s.clear))
        draws, nd = abi.draws_array(s.draws)
        for _ in range(50):
            lib.tri_render(ctx)
        r.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            lib.tri_render(ctx)
        t1 = time.perf_counter()
        r.synchronize()
        t2 = time.perf_counter()
        burst = []  # short bursts after a drain: the queue never fills, so this is the host cost alone
        for _ in range(20):
            r.synchronize()
            b0 = time.perf_counter()
            for _ in range(16):
                lib.tri_render(ctx)
            burst.append((time.perf_counter() - b0) / 16)
        r.synchronize()
        burst.sort()
        print(f"{which}: host cost of tri_render in bursts of 16 (queue not full): median {1e6 * burst[len(burst) // 2]:.1f} us")
        t2 = time.perf_counter()
        for _ in range(n):
            lib.tri_set_frame(ctx, ubo, clear)
            lib.tri_set_draws(ctx, draws, nd)
            lib.tri_render(ctx)
        t3 = time.perf_counter()
        r.synchronize()
        t4 = time.perf_counter()
    print(f"{which}: tri_render enqueue {1e6 * (t1 - t0) / n:.1f} us/frame, drained at {1e6 * (t2 - t0) / n:.1f} us/frame; "
          f"with set_frame + set_draws: enqueue {1e6 * (t3 - t2) / n:.1f}, drained {1e6 * (t4 - t2) / n:.1f} us/frame")


if __name__ == "__main__":
    main(*sys.argv[1:])
