"""tri_xfer's multi-rank exchange executed on one GPU (VERDICT r5 #1a): N exchanges in one process over the loopback
transport (tri_xfer_comm_create_loopback) stand in for N ranks, each with its own band contexts and streams, driven
frame by frame with every sender before the display. Only ncclSend / ncclRecv are replaced (by an event-ordered
device copy into the same receive buffers); the pack, the receive buffers, the batched dbp decode, the senders'
status carried to the display and an assemble-only display's own streams are the N-GPU code. The assembled C4 frame
(3840 x 2160, 999,698 triangles) must equal the one-context frame bit for bit, at N = 2, 4 and 8, over equal,
rebalanced and 0-row display splits, in the dbp, 3-byte and 4-byte formats, with 3 frames in flight."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NBUF = 3  # frames in flight (slots), as the bench's C3 default
FRAMES = 7  # every slot used at least twice: the reuse waits for the slot's previous transfer


@pytest.fixture(scope="module")
def c4():
    """The C4 scene, one shared geometry on device 0, and the one-context reference frame."""
    from trident_raster import raster, scenes

    import bench

    s = bench.build_scene("c3")
    geo = raster.TriGeometry(0)
    geo.upload(s.vertices, s.indices, s.meshes)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s, geometry=geo)
        r.render_frame()
        want, _ = r.readback(depth=False)
        alpha = r.frame_alpha()
    yield s, geo, want, alpha
    geo.close()


class Ranks:
    """N loopback ranks on device 0: rank r's band contexts (one per slot), its slot buffers and its tri_xfer."""

    def __init__(self, scene, geo, bands, fmt, alpha, slot_bytes=0, ncomm=NBUF):
        import torch
        from trident_raster import abi, raster, scenes

        self.lib = raster.load_library()
        self.scene, self.bands, self.N = scene, bands, len(bands)
        W, H = scene.width, scene.height
        self.hub = C.c_void_p()
        raster._check(self.lib.tri_xfer_loopback_create(self.N, C.byref(self.hub)))
        self.comms = [[C.c_void_p() for _ in range(ncomm)] for _ in range(self.N)]
        for r in range(self.N):
            for c in self.comms[r]:
                raster._check(self.lib.tri_xfer_comm_create_loopback(self.hub, r, 0, C.byref(c)))
        self.ctx = [[None] * NBUF for _ in range(self.N)]
        self.rs = []
        for r, (y0, y1) in enumerate(bands):
            if y1 == y0:
                continue  # an assemble-only display renders nothing (ctx NULL every frame)
            for k in range(NBUF):
                t = raster.TriRaster(W, H, band=(y0, y1))
                scenes.load_scene(t, scene, geometry=geo)
                self.rs.append(t)
                self.ctx[r][k] = t._ctx
        band_y = (C.c_uint32 * (self.N + 1))(*([y0 for y0, _ in bands] + [H]))
        self.bufs, self.x = [], []
        for r in range(self.N):
            cfg = abi.TriXferConfig(W, band_y, 0, fmt, slot_bytes, alpha, NBUF)
            x = C.c_void_p()
            arr = (C.c_void_p * ncomm)(*[c.value for c in self.comms[r]])
            raster._check(self.lib.tri_xfer_create(arr, ncomm, C.byref(cfg), C.byref(x)))
            n = H * W if r == 0 else (bands[r][1] - bands[r][0]) * W
            bs = [torch.full((n,), -1, dtype=torch.int32, device="cuda:0") for _ in range(NBUF)]
            for k, b in enumerate(bs):
                raster._check(self.lib.tri_xfer_bind_slot(x, k, C.c_void_p(b.data_ptr())))
            self.x.append(x)
            self.bufs.append(bs)
        self.ubo = C.byref(scene.ubo)
        self.clear = (C.c_float * 4)(*scene.clear)
        self.draws, self.nd = abi.draws_array(scene.draws)

    def frame(self, k):
        """Frame k on slot k % NBUF: every sender renders and sends, then the display renders (if it has rows),
        receives and decodes."""
        from trident_raster import raster

        slot = k % NBUF
        for r in list(range(1, self.N)) + [0]:
            c = self.ctx[r][slot]
            raster._check(self.lib.tri_xfer_frame(self.x[r], slot, c, None, self.ubo if c else None,
                                                  self.clear if c else None, self.draws if c else None, self.nd, 1))

    def sync(self):
        return [self.lib.tri_xfer_synchronize(x) for x in self.x]

    def close(self):
        import torch

        torch.cuda.synchronize()
        for x in self.x:
            self.lib.tri_xfer_destroy(x)
        for t in self.rs:
            t.close()
        for cs in self.comms:
            for c in cs:
                self.lib.tri_xfer_comm_destroy(c)
        self.lib.tri_xfer_loopback_destroy(self.hub)


def _splits(N, H):
    import bench

    out = {"equal": bench.band_split(H, N)}
    # a rebalanced split: the display band kept, sender bands re-cut from uneven (synthetic) render times
    eq = out["equal"]
    ms = [1.0] + [1.0 + 0.15 * r for r in range(1, N)]
    # (at N = 2 there is one sender band: an uneven display band instead, as the split autotune picks)
    out["rebalanced"] = (bench.band_split(H, N, tuple(bench.rebalance_sizes(eq, ms))) if N > 2
                         else bench.band_split(H, N, int(0.6 * H)))
    if N > 2:
        out["display0"] = bench.band_split(H, N, 0)
    return out


CASES = [(N, sp) for N in (2, 4, 8) for sp in ("equal", "rebalanced", "display0") if not (N == 2 and sp == "display0")]


@pytest.mark.parametrize("N,split", CASES, ids=[f"N{n}-{s}" for n, s in CASES])
def test_loopback_assembles_c4_bit_exact(c4, N, split):
    import torch
    from trident_raster import abi, raster

    s, geo, want, alpha = c4
    assert alpha == 255
    bands = _splits(N, s.height)[split]
    if split == "rebalanced":
        assert len({b - a for a, b in bands}) > 1, bands  # really uneven
    for fmt in (abi.TRI_GROUP_FMT_DBP, abi.TRI_GROUP_FMT_BGR24, abi.TRI_GROUP_FMT_BGRA32):
        slot = 6656 if fmt == abi.TRI_GROUP_FMT_DBP else 0  # C3 bands need 5920-6528 B
        ranks = Ranks(s, geo, bands, fmt, alpha, slot)
        try:
            for k in range(FRAMES):
                ranks.frame(k)
            assert ranks.sync() == [0] * N, (fmt, ranks.lib.tri_last_error())
            torch.cuda.synchronize()
            for k in range(NBUF):
                got = ranks.bufs[0][k].cpu().numpy().view(np.uint8).reshape(s.height, s.width, 4)
                bad = int((got != want).any(-1).sum())
                assert bad == 0, f"fmt {fmt} slot {k}: {bad} pixels differ"
            sent, recv = C.c_uint64(), C.c_uint64()
            raster._check(ranks.lib.tri_xfer_info(ranks.x[0], C.byref(sent), C.byref(recv), None))
            remote_px = sum((b - a) * s.width for a, b in bands[1:])
            if fmt == abi.TRI_GROUP_FMT_BGRA32:
                assert recv.value == 4 * remote_px
            elif fmt == abi.TRI_GROUP_FMT_DBP:
                assert recv.value < 1.7 * remote_px  # ≈ 1.5-1.6 B per pixel
        finally:
            ranks.close()


def test_loopback_display_sees_the_senders_lossy_bands(c4):
    """The senders' status travels with their bands: a dbp slot too small for the band (every slot overflows) and a
    promised alpha the pixels do not have are reported by tri_xfer_synchronize on the display rank too."""
    from trident_raster import abi

    s, geo, want, alpha = c4
    bands = _splits(4, s.height)["display0"]
    ranks = Ranks(s, geo, bands, abi.TRI_GROUP_FMT_DBP, alpha, 176)  # TRI_DBP_MIN_SLOT: every slot overflows
    try:
        ranks.frame(0)
        assert ranks.sync() == [abi.TRI_E_OVERFLOW] * 4
    finally:
        ranks.close()
    for fmt in (abi.TRI_GROUP_FMT_DBP, abi.TRI_GROUP_FMT_BGR24):
        ranks = Ranks(s, geo, bands, fmt, 7, 12448 if fmt == abi.TRI_GROUP_FMT_DBP else 0)  # the pixels' alpha is 255
        try:
            ranks.frame(0)
            assert ranks.sync() == [abi.TRI_E_STATE] * 4, fmt
        finally:
            ranks.close()


def test_loopback_one_communicator_shared_by_three_slots(c4):
    """Fewer communicators than frames in flight (the fallback when a second ncclCommInitRank fails): the shared
    communicator's operations are fenced across the slots' streams, and the frame is still bit-exact."""
    import torch
    from trident_raster import abi, raster

    s, geo, want, alpha = c4
    bands = _splits(4, s.height)["equal"]
    ranks = Ranks(s, geo, bands, abi.TRI_GROUP_FMT_DBP, alpha, 6656, ncomm=1)
    try:
        n = C.c_uint32()
        raster._check(ranks.lib.tri_xfer_comm_count(ranks.x[0], C.byref(n)))
        assert n.value == 1
        for k in range(FRAMES):
            ranks.frame(k)
        assert ranks.sync() == [0] * 4
        torch.cuda.synchronize()
        for k in range(NBUF):
            got = ranks.bufs[0][k].cpu().numpy().view(np.uint8).reshape(s.height, s.width, 4)
            assert np.array_equal(got, want), k
    finally:
        ranks.close()


def test_loopback_order_and_deadline(c4):
    """A display that receives before its senders posted is refused (TRI_E_STATE), a sender that reuses a slot its
    display never received is refused, and the synchronise deadline expires on work that outlasts it
    (TRI_E_TIMEOUT; the work itself completes)."""
    import torch
    from trident_raster import abi, raster

    s, geo, want, alpha = c4
    bands = _splits(2, s.height)["equal"]
    ranks = Ranks(s, geo, bands, abi.TRI_GROUP_FMT_BGRA32, alpha)
    L = ranks.lib
    try:
        c0 = ranks.ctx[0][0]
        assert L.tri_xfer_frame(ranks.x[0], 0, c0, None, None, None, None, 0, 1) == abi.TRI_E_STATE
        c1 = ranks.ctx[1][0]
        raster._check(L.tri_xfer_frame(ranks.x[1], 0, c1, None, None, None, None, 0, 1))
        assert L.tri_xfer_frame(ranks.x[1], 0, c1, None, None, None, None, 0, 1) == abi.TRI_E_STATE
        raster._check(L.tri_xfer_frame(ranks.x[0], 0, c0, None, None, None, None, 0, 1))  # receives the posted band
        raster._check(L.tri_xfer_set_timeout(ranks.x[1], 1))
        for _ in range(200):  # ≈ 10 ms of band frames behind a 1-ms deadline
            raster._check(L.tri_xfer_frame(ranks.x[1], 1, ranks.ctx[1][1], None, None, None, None, 0, 0))
        assert L.tri_xfer_synchronize(ranks.x[1]) == abi.TRI_E_TIMEOUT
        torch.cuda.synchronize()
        raster._check(L.tri_xfer_set_timeout(ranks.x[1], 60000))
        assert L.tri_xfer_synchronize(ranks.x[1]) == 0
    finally:
        ranks.close()
