#!/usr/bin/env python3
"""Host cost per frame of tri_xfer_frame (render + the exchange stream's fences; one rank, so no transfer) against
the torch-side path bench.py takes at N = 1 (four ctypes calls under a torch stream context), for one C4 band
(3840 x 270 of C3) with 3 contexts in flight. Prints host us per call and frames/s."""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-renderer_amd", "python"))
from trident_raster import abi, raster, scenes  # noqa: E402


def main(frames=3000):
    lib = raster.load_library()
    s = scenes.scene_c3_grid()
    W, H = s.width, s.height
    band = (4 * H // 8, 5 * H // 8)
    geo = raster.TriGeometry(0)
    geo.upload(s.vertices, s.indices, s.meshes)
    rs = []
    for _ in range(3):
        r = raster.TriRaster(W, H, band=band)
        scenes.load_scene(r, s, geometry=geo)
        r.render_frame()
        rs.append(r)
    uid = (C.c_uint8 * 128)()
    raster._check(lib.tri_xfer_unique_id(uid))
    comm = C.c_void_p()
    raster._check(lib.tri_xfer_comm_create(uid, 1, 0, 0, C.byref(comm)))
    rows = band[1] - band[0]
    band_y = (C.c_uint32 * 2)(0, rows)
    cfg = abi.TriXferConfig(W, band_y, 0, abi.TRI_GROUP_FMT_DBP, 6400, 255, 3)
    x = C.c_void_p()
    raster._check(lib.tri_xfer_create((C.c_void_p * 1)(comm.value), 1, C.byref(cfg), C.byref(x)))
    bufs = [torch.empty(rows * W, dtype=torch.int32, device="cuda:0") for _ in range(3)]
    for k, b in enumerate(bufs):
        raster._check(lib.tri_xfer_bind_slot(x, k, C.c_void_p(b.data_ptr())))
    draws, nd = abi.draws_array(s.draws)
    ubo, clear = C.byref(s.ubo), (C.c_float * 4)(*s.clear)
    ctxs = [r._ctx for r in rs]
    for rep in range(2):
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for k in range(frames):
            h = time.perf_counter()
            rc = lib.tri_xfer_frame(x, k % 3, ctxs[k % 3], None, ubo, clear, draws, nd, 1)
            host += time.perf_counter() - h
            if rc:
                raster._check(rc)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"tri_xfer_frame: host {host / frames * 1e6:.1f} us per call, {frames / dt:.0f} frames/s", flush=True)
    streams = [torch.cuda.Stream() for _ in range(3)]
    for r, st in zip(rs, streams):
        r.set_stream(st.cuda_stream)
    dptrs = [C.c_void_p(b.data_ptr()) for b in bufs]
    for rep in range(2):
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for k in range(frames):
            h = time.perf_counter()
            ctx = ctxs[k % 3]
            with torch.cuda.stream(streams[k % 3]):
                rc = (lib.tri_bind_output(ctx, dptrs[k % 3], None) or lib.tri_set_frame(ctx, ubo, clear) or
                      lib.tri_set_draws(ctx, draws, nd) or lib.tri_render(ctx))
            host += time.perf_counter() - h
            if rc:
                raster._check(rc)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"ctypes path (bench N = 1): host {host / frames * 1e6:.1f} us per frame, {frames / dt:.0f} frames/s",
              flush=True)
    lib.tri_xfer_destroy(x)
    lib.tri_xfer_comm_destroy(comm)


if __name__ == "__main__":
    main()
