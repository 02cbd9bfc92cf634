"""tri_xfer, the native band exchange bench.py uses at N > 1 (include/tri_raster.h): on one GPU, a one-rank RCCL
communicator created from the library's own unique id inside a torch process, frames rendered through
tri_xfer_frame into caller-owned slots bit-exact with the plain render (slot reuse behind the device-side fence),
the transfer sizes, and the argument checks. The multi-rank send / receive / decode path needs N GPUs (one process
per GPU: RCCL refuses two ranks on one device, tools/rccl_dup_probe.py); bench.py checks the assembled frame against
the one-GPU frame on every N > 1 run (verify_assembly) and falls back to torch.distributed if it differs."""
import ctypes as C

import numpy as np
import pytest

import scene_cases as sc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from trident_raster import raster

    lib = raster.load_library()
    uid = (C.c_uint8 * 128)()
    raster._check(lib.tri_xfer_unique_id(uid))
    c = C.c_void_p()
    raster._check(lib.tri_xfer_comm_create(uid, 1, 0, 0, C.byref(c)))
    yield lib, c
    lib.tri_xfer_comm_destroy(c)


def _xfer(lib, comm, W, H, fmt, nbuf=2, slot=8192):
    from trident_raster import abi, raster

    band_y = (C.c_uint32 * 2)(0, H)
    cfg = abi.TriXferConfig(W, band_y, 0, fmt, slot if fmt == abi.TRI_GROUP_FMT_DBP else 0, 255, nbuf)
    x = C.c_void_p()
    raster._check(lib.tri_xfer_create((C.c_void_p * 1)(comm.value), 1, C.byref(cfg), C.byref(x)))
    return x


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_xfer_frames_match_the_plain_render(comm, fmt):
    import torch
    from trident_raster import abi, raster, scenes

    lib, c = comm
    s = sc.grid_c3(320, 180, 30)
    W, H = s.width, s.height
    with raster.TriRaster(W, H) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        want, _ = r.readback(depth=False)
        x = _xfer(lib, c, W, H, fmt)
        try:
            bufs = [torch.zeros(W * H, dtype=torch.int32, device="cuda:0") for _ in range(2)]
            for k, b in enumerate(bufs):
                raster._check(lib.tri_xfer_bind_slot(x, k, C.c_void_p(b.data_ptr())))
            draws, nd = abi.draws_array(s.draws)
            clear = (C.c_float * 4)(*s.clear)
            for k in range(5):  # slots 0, 1, 0, 1, 0: each reuse waits for the slot's previous frame on the device
                raster._check(lib.tri_xfer_frame(x, k % 2, r._ctx, None, C.byref(s.ubo), clear, draws, nd, 1))
            raster._check(lib.tri_xfer_synchronize(x))
            torch.cuda.synchronize()
            for b in bufs:
                got = b.cpu().numpy().view(np.uint8).reshape(H, W, 4)
                assert np.array_equal(got, want)
            sent, recv, mx = C.c_uint64(), C.c_uint64(), C.c_uint32()
            raster._check(lib.tri_xfer_info(x, C.byref(sent), C.byref(recv), C.byref(mx)))
            assert (sent.value, recv.value) == (0, 0)  # one rank: nothing crosses a link
            # an exchange-only frame (no context) and a render-only frame are accepted too
            raster._check(lib.tri_xfer_frame(x, 0, None, None, None, None, None, 0, 1))
            raster._check(lib.tri_xfer_frame(x, 1, r._ctx, None, None, None, None, 0, 0))
            # slot 0 moves to another context's stream (fenced behind its last frame) and renders the same pixels
            with raster.TriRaster(W, H) as r2:
                scenes.load_scene(r2, s)
                bufs[0].zero_()
                torch.cuda.synchronize()
                raster._check(lib.tri_xfer_frame(x, 0, r2._ctx, None, None, None, None, 0, 1))
                raster._check(lib.tri_xfer_synchronize(x))
                torch.cuda.synchronize()
                assert np.array_equal(bufs[0].cpu().numpy().view(np.uint8).reshape(H, W, 4), want)
        finally:
            lib.tri_xfer_destroy(x)


def test_xfer_rejects_bad_arguments(comm):
    from trident_raster import abi, raster

    lib, c = comm
    band_y = (C.c_uint32 * 2)(0, 16)
    x = C.c_void_p()
    bad = abi.TriXferConfig(64, band_y, 1, 0, 0, 255, 2)  # display rank outside the world
    assert lib.tri_xfer_create((C.c_void_p * 1)(c.value), 1, C.byref(bad), C.byref(x)) == abi.TRI_E_INVALID
    bad = abi.TriXferConfig(64, band_y, 0, abi.TRI_GROUP_FMT_DBP, 100, 255, 2)  # slot below the minimum
    assert lib.tri_xfer_create((C.c_void_p * 1)(c.value), 1, C.byref(bad), C.byref(x)) == abi.TRI_E_INVALID
    empty = (C.c_uint32 * 2)(5, 5)  # a band without rows
    bad = abi.TriXferConfig(64, empty, 0, 0, 0, 255, 2)
    assert lib.tri_xfer_create((C.c_void_p * 1)(c.value), 1, C.byref(bad), C.byref(x)) == abi.TRI_E_INVALID
    x = _xfer(lib, c, 64, 16, 0)
    try:
        assert lib.tri_xfer_frame(x, 0, None, None, None, None, None, 0, 1) == abi.TRI_E_INVALID  # slot not bound
        assert lib.tri_xfer_bind_slot(x, 2, C.c_void_p(256)) == abi.TRI_E_INVALID  # slot out of range
        assert lib.tri_xfer_bind_slot(x, 0, C.c_void_p(258)) == abi.TRI_E_INVALID  # misaligned
    finally:
        raster._check(lib.tri_xfer_destroy(x))


def test_xfer_exchange_only_slots_run_on_their_own_streams(comm):
    """Slots that never rendered (an assemble-only display rank's, which passes no context) take streams of their
    own, one per slot; the frames are accepted and synchronise."""
    import torch
    from trident_raster import raster

    lib, c = comm
    x = _xfer(lib, c, 64, 16, 0, nbuf=3)
    try:
        bufs = [torch.zeros(64 * 16, dtype=torch.int32, device="cuda:0") for _ in range(3)]
        for k, b in enumerate(bufs):
            raster._check(lib.tri_xfer_bind_slot(x, k, C.c_void_p(b.data_ptr())))
        for k in range(7):
            raster._check(lib.tri_xfer_frame(x, k % 3, None, None, None, None, None, 0, 1))
        raster._check(lib.tri_xfer_synchronize(x))
    finally:
        raster._check(lib.tri_xfer_destroy(x))
