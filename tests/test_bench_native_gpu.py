"""bench.py's native exchange plumbing on one GPU (the part of the N > 1 path a one-GPU box can run): a BandRenderer
given a tri_xfer over a one-rank RCCL communicator renders every frame through tri_xfer_frame into its context's
slot, the assembled frame the bench reads is the latest slot's, and verify_assembly (the in-bench parity check every
N > 1 run makes) finds it bit-exact against the frame rendered whole by one context. The transfers themselves need
N GPUs (tests/test_xfer_gpu.py covers the library side)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def test_band_renderer_native_exchange_plumbing():
    import ctypes as C

    import torch
    from trident_raster import abi, raster

    import bench
    import scene_cases as sc

    scene = sc.grid_c3(640, 360, 60)
    br = bench.BandRenderer(scene, 0, 1, 0, inflight=3)
    try:
        assert br.xfer is None  # one rank: the plain path, unless attached as below
        lib = raster.load_library()
        uid = (C.c_uint8 * 128)()
        raster._check(lib.tri_xfer_unique_id(uid))
        comm = C.c_void_p()
        raster._check(lib.tri_xfer_comm_create(uid, 1, 0, 0, C.byref(comm)))
        bench._XFER_COMMS[:] = [comm]  # what xfer_comms() would have built over torch.distributed
        try:
            br._attach_xfer(0)
            assert br.xfer is not None and br.nbuf == 3 and len(br.xbufs) == 3
            for _ in range(7):  # slots 0, 1, 2, 0, ... each on its own context's stream
                br.step()
            torch.cuda.synchronize()
            br.check()
            assert br._kx == (7 - 1) % 3
            assert br.inbound_bytes() == 0
            parity = bench.verify_assembly(br, scene, False)
            assert parity["bit_exact"], parity
            assert br.render_only_ms(frames=6) > 0 and br.assembly_only_ms(frames=6) >= 0
        finally:
            br.close()
            lib.tri_xfer_comm_destroy(comm)
            bench._XFER_COMMS[:] = []
    finally:
        if br.xfer is not None:
            br.close()
    assert abi.TRI_XFER_ID_BYTES == 128


def test_forge_editor_frame_secondary():
    """bench.forge_frame (the frame Forge runs, through RenderCommand::DrawFrame with its deferred fence): two small
    panels and the present blit complete and report a rate and a host cost (the shim's pixel parity after the deferred
    fence is covered by test_host_shim.py / test_present.py, which read through FinishFrame)."""
    import bench

    layout = {"viewports": ((2, 212, 160), (1, 200, 150)), "present": (320, 240)}
    r = bench.forge_frame(layout, frames=12, warm_seconds=0.02)
    assert r["frames_per_s"] > 0 and r["host_ms_per_drawframe_idle_gpu"] > 0
    assert r["viewports"] == [[212, 160], [200, 150]] and r["triangles"] == 999698
