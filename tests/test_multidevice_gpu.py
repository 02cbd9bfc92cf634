"""C4 readiness on one GPU: the full C3 frame (3840x2160, 999,698 triangles, the reference cubemap) split
into 8 row bands, as 8 band contexts and as a tri_group of 8 bands, bit-exact against the single-context
frame and depth bit-exact against the oracle's full frame (BASELINE configs[3]); the group's
double-buffered frame with its consumer fence; and the Trident::Renderer shim driving a group
(Renderer::SetDeviceCount, the tri_config.device_count of SURVEY 8(b)).

On a one-GPU box every band sits on device 0 (the stand-in for N devices): the RCCL send/recv branch of
tri_group runs only on the driver's 8-GPU node. The band split, cluster culling, in-place assembly, the
per-device geometry, the buffer rotation and the fences are the same code either way.
"""
import ctypes as C

import numpy as np
import pytest

import scene_cases as sc

pytestmark = pytest.mark.gpu

COLOR_TOL = 1


@pytest.fixture(scope="module")
def c3_full():
    from trident_raster import scenes

    return scenes.scene_c3_grid()


def _render_single(scene, flags):
    from trident_raster import raster, scenes

    with raster.TriRaster(scene.width, scene.height, flags=flags) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        return r.readback()


@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_c4_full_frame_eight_bands(oracle, c3_full, mode):
    """C4 = C3 on 8 GPUs: eight 270-row bands of the full 4K / 1M-triangle frame, rendered (a) as eight
    band contexts sharing one tri_geometry and (b) as a tri_group over devices [0]*8, assemble to the
    single-context frame bit for bit; depth is bit-exact against the oracle's full frame."""
    from trident_raster import abi, raster, scenes

    flags = abi.TRI_FLAG_EXACT_SHADING if mode == "exact" else 0
    s = c3_full
    full_c, full_d = _render_single(s, flags)
    rows = s.height // 8
    g = raster.TriGeometry(0)
    g.upload(s.vertices, s.indices, s.meshes)
    parts = []
    for r in range(8):
        with raster.TriRaster(s.width, s.height, band=(r * rows, (r + 1) * rows), device=0, flags=flags) as ctx:
            scenes.load_scene(ctx, s, geometry=g)
            ctx.render_frame()
            parts.append(ctx.readback())
    g.close()
    band_c = np.concatenate([p[0] for p in parts])
    band_d = np.concatenate([p[1] for p in parts])
    assert np.array_equal(band_d, full_d), int((band_d != full_d).sum())
    assert np.array_equal(band_c, full_c), int((band_c != full_c).any(-1).sum())
    with raster.TriGroup(s.width, s.height, [0] * 8, display=0, flags=flags) as grp:
        scenes.load_scene(grp, s)
        grp.render_frame()
        grp_c, grp_d = grp.readback()
    bad = np.argwhere((grp_d != full_d) | (grp_c != full_c).any(-1))
    assert len(bad) == 0, f"group frame: {len(bad)} pixels differ, rows {np.unique(bad[:, 0] // rows)} (bands), " \
                          f"first {bad[:3].tolist()} depth {grp_d[tuple(bad[0])]:#x} vs {full_d[tuple(bad[0])]:#x}"
    oc, od, _ = oracle.render(s)
    assert np.array_equal(full_d, od), int((full_d != od).sum())
    assert int(np.abs(full_c.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL


def _poison_device_memory(byte=0xFF, chunks=48, size=64 << 20):
    """Fill device memory with `byte` and release it: buffers allocated next hold that garbage, not fresh zeros."""
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


def test_first_frame_over_reused_device_memory(c3_full):
    """Regression (round 3): a context's bin counters were zeroed by a null-stream hipMemset that the context's
    non-blocking stream did not wait for; over recycled device memory the first frame of an 8-band group lost a
    whole bin (1024 pixels left at the clear depth). Now every reset is stream-ordered. Device memory is
    poisoned with 0xFF before each fresh context / group renders its first frame. A race, so a guard rather than
    a proof: tools/group_repro.py caught the pre-fix build in one run of four."""
    from trident_raster import raster, scenes

    s = c3_full
    ref_c, ref_d = _render_single(s, 0)
    for attempt in range(2):
        assert _poison_device_memory() > 0
        with raster.TriGroup(s.width, s.height, [0] * 8, display=0) as grp:
            scenes.load_scene(grp, s)
            grp.render_frame()
            gc, gd = grp.readback()
        bad = np.argwhere((gd != ref_d) | (gc != ref_c).any(-1))
        assert len(bad) == 0, f"group, attempt {attempt}: {len(bad)} pixels differ, bands {np.unique(bad[:, 0] // 270)}"
        assert _poison_device_memory() > 0
        c, d = _render_single(s, 0)
        assert np.array_equal(d, ref_d) and np.array_equal(c, ref_c), f"single context, attempt {attempt}"


def _copy_frame(ptr, dev, w, h):
    from trident_raster import raster

    return raster.copy_device_to_host(ptr, w * h * 4, dev).reshape(h, w, 4)


def test_group_double_buffer_and_present_fence(oracle):
    """Frame k lands in buffer k % 2: while frame k + 1 renders into the other buffer, frame k's image
    stays intact for its presenter; frame k + 2 reuses frame k's buffer after the consumer fence
    (tri_group_present). Three different camera positions, so every frame differs."""
    from trident_raster import raster, scenes

    base = sc.primitives_row(oracle, 320, 240)
    cams = [(0.0, 1.0, 6.0), (0.6, 1.3, 6.5), (-0.7, 0.8, 5.5)]
    frames = []
    for cam in cams:
        s = sc.primitives_row(oracle, 320, 240)
        view, proj = scenes.editor_camera(cam, (0, 0, 0), 60.0, (320, 240))
        s.ubo = scenes.pack_ubo(view, proj, cam, [{"type": "directional"}])
        frames.append(s)
    with raster.TriGroup(base.width, base.height, [0] * 3, display=1) as g:
        scenes.load_scene(g, frames[0])
        g.render_frame()
        p0, dev = g.frame_pointer()
        img0 = _copy_frame(p0, dev, 320, 240)
        g.present()  # the presenter of frame 0 is done with it
        g.set_frame(frames[1].ubo, frames[1].clear)
        g.render_frame()
        p1, _ = g.frame_pointer()
        assert p1 != p0
        # frame 0's buffer was not touched by frame 1
        assert np.array_equal(_copy_frame(p0, dev, 320, 240), img0)
        img1 = _copy_frame(p1, dev, 320, 240)
        g.set_frame(frames[2].ubo, frames[2].clear)
        g.render_frame()  # frame 2 reuses buffer 0 (after the fence)
        p2, _ = g.frame_pointer()
        assert p2 == p0
        assert np.array_equal(_copy_frame(p1, dev, 320, 240), img1)  # frame 1 intact
        col2, dep2 = g.readback()
        img = g.output_image()
        assert img.device_ptr == p2 and (img.width, img.height) == (320, 240)
    for (col, want) in ((img0, frames[0]), (img1, frames[1]), (col2, frames[2])):
        oc, od, _ = oracle.render(want)
        assert int(np.abs(col.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL
    assert not np.array_equal(img0, img1)
    _, od2, _ = oracle.render(frames[2])
    assert np.array_equal(dep2, od2)


def test_group_shares_one_geometry_per_device(oracle):
    """Caller-owned geometry (tri_group_bind_geometry): every band on device 0 binds the one object;
    the frame equals the oracle's, and binding back to the group's own copy (after its upload) too."""
    from trident_raster import raster, scenes

    s = sc.primitives_row(oracle, 320, 240)
    geo = raster.TriGeometry(0)
    geo.upload(s.vertices, s.indices, s.meshes)
    oc, od, _ = oracle.render(s)
    with raster.TriGroup(s.width, s.height, [0] * 4) as g:
        g.bind_geometry([geo])
        g.upload_materials(s.materials)
        g.upload_skybox(s.skybox)
        g.set_frame(s.ubo, s.clear)
        g.set_draws(s.draws)
        g.render_frame()
        col, dep = g.readback()
        assert np.array_equal(dep, od)
        assert int(np.abs(col.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL
        g.upload_geometry(s.vertices, s.indices, s.meshes)  # back to the group's own per-device copy
        g.render_frame()
        col2, dep2 = g.readback()
    geo.close()
    assert np.array_equal(dep2, od) and np.array_equal(col2, col)


def test_group_blit_matches_single_context():
    """tri_group_blit_linear over the assembled frame == tri_blit_linear of the single-context frame."""
    from trident_raster import raster, scenes

    s = sc.grid_c3(640, 360, 80)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        r.blit(500, 281)
        want = r.read_present()
    with raster.TriGroup(s.width, s.height, [0] * 3) as g:
        scenes.load_scene(g, s)
        g.render_frame()
        g.blit(500, 281)
        got = g.read_present()
    assert np.array_equal(got, want)


def _hip_device_count():
    n = C.c_int(0)
    return n.value if C.CDLL("libamdhip64.so").hipGetDeviceCount(C.byref(n)) == 0 else 0


def _camera_frames(oracle, cams, w=320, h=240):
    from trident_raster import scenes

    frames = []
    for cam in cams:
        s = sc.primitives_row(oracle, w, h)
        view, proj = scenes.editor_camera(cam, (0, 0, 0), 60.0, (w, h))
        s.ubo = scenes.pack_ubo(view, proj, cam, [{"type": "directional"}])
        frames.append(s)
    return frames


def test_group_blit_is_fenced_against_the_next_but_one_frame(oracle):
    """render k, blit k into a caller buffer, render k + 1 and k + 2 without a present fence or a
    sync: frame k + 2 reuses frame k's buffer, and its in-place bands (context streams) must wait for the
    blit (assembly stream). The blitted image equals the single-context blit of frame k; read_present
    refuses after a blit into a caller buffer (the owned target is stale)."""
    from trident_raster import abi, raster, scenes

    frames = _camera_frames(oracle, [(0.0, 1.0, 6.0), (0.6, 1.3, 6.5), (-0.7, 0.8, 5.5)], 640, 480)
    with raster.TriRaster(640, 480) as r:
        scenes.load_scene(r, frames[0])
        r.render_frame()
        r.blit(800, 600)
        want = r.read_present()
    import torch

    dst = torch.empty((600, 800, 4), dtype=torch.uint8, device="cuda:0")
    with raster.TriGroup(640, 480, [0] * 4, display=2) as g:
        scenes.load_scene(g, frames[0])
        g.render_frame()
        g.blit(800, 600, dst_ptr=dst.data_ptr())
        for s in frames[1:]:
            g.set_frame(s.ubo, s.clear)
            g.render_frame()
        g.synchronize()
        with pytest.raises(RuntimeError):
            g.read_present()
        got = dst.cpu().numpy()
    assert np.array_equal(got, want), int((got != want).any(-1).sum())


def test_hip_band_codec_round_trip():
    """tri_pack_bgr24 / tri_unpack_bgr24 (band_codec.hip) against numpy: aligned bands (4 pixels per lane) and
    unaligned ones (a band of an odd-width frame), the odd tail, and the alpha check."""
    import torch

    from trident_raster import raster

    rng = np.random.default_rng(5)
    for n, off in ((3840 * 270, 0), (333 * 17 + 3, 1), (5, 0), (1, 3)):
        px = rng.integers(0, 2 ** 24, n, dtype=np.int64)
        host = (px | (255 << 24)).astype(np.uint32)
        src = torch.from_numpy(np.concatenate([np.zeros(off, np.uint32), host]).view(np.int32)).cuda()
        band = src[off:]
        packed = torch.zeros(3 * n + 1, dtype=torch.uint8, device="cuda")[1:] if off else \
            torch.zeros(3 * n, dtype=torch.uint8, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        raster.pack_bgr24(band.data_ptr(), packed.data_ptr(), n, 255, flag.data_ptr())
        want = host.view(np.uint8).reshape(n, 4)[:, :3].reshape(-1)
        assert np.array_equal(packed.cpu().numpy(), want)
        out = torch.zeros(n + off, dtype=torch.int32, device="cuda")[off:]
        raster.unpack_bgr24(packed.data_ptr(), out.data_ptr(), n, 255)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), host)
        assert int(flag.item()) == 0
        raster.pack_bgr24(band.data_ptr(), packed.data_ptr(), n, 254, flag.data_ptr())  # wrong promise
        assert int(flag.item()) != 0


def test_frame_alpha_proof(oracle):
    """tri_frame_alpha: 255 for the opaque C3-style grid and the sprites' tint-alpha-1 frames; -1 for the
    textured grid (its texture carries alpha), a tint alpha below 1 or a translucent clear colour."""
    from trident_raster import raster, scenes

    for scene, want in ((sc.grid_c3(320, 180, 30), 255), (sc.textured_grid(), -1), (sc.c1_cube_skybox(1), 255)):
        with raster.TriRaster(scene.width, scene.height) as r:
            scenes.load_scene(r, scene)
            assert r.frame_alpha() == want, scene.name
    s = sc.grid_c3(320, 180, 30)
    s.draws[0].pc.tint[3] = 0.5
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        assert r.frame_alpha() == -1
        s.draws[0].pc.tint[3] = 1.0
        r.set_draws(s.draws)
        assert r.frame_alpha() == 255
        r.set_frame(s.ubo, (0.1, 0.1, 0.1, 0.5))
        assert r.frame_alpha() == -1


@pytest.mark.parametrize("scene_name,group_flags,fmt", [("grid", 0, 2), ("grid", 4, 1), ("grid", 1, 0), ("textured", 0, 0)])
def test_group_staged_bands_packed_transfer(oracle, scene_name, group_flags, fmt):
    """VERDICT r3 #3 / r4 #5 on one GPU: TRI_GROUP_STAGE_BANDS sends every non-display band through the remote path
    (band buffer, packed when the alpha is proven uniform — the delta bit-plane format by default, 3-byte pixels
    with TRI_GROUP_PACK_BGR24 (4) — transfer, unpack into the frame). Four frames with different cameras; each
    assembled frame equals the single-context frame bit for bit, with every format and with packing off
    (TRI_GROUP_NO_PACK = 1), and a frame with non-uniform alpha travels as 4 bytes. dbp: the first frame uses the
    largest slot, later ones the slot refitted at each synchronize (render_frame re-renders after an overflow)."""
    from trident_raster import abi, raster, scenes

    cams = [(0.0, 0.0, 3.0), (0.3, 0.2, 3.2), (-0.4, -0.1, 2.8), (0.1, 0.3, 3.5)]
    frames = []
    for cam in cams:
        s = sc.grid_c3(480, 270, 40) if scene_name == "grid" else sc.textured_grid(480, 270, 30)
        view, proj = scenes.editor_camera(cam, (0, 0, 0), 60.0, (480, 270))
        s.ubo = scenes.pack_ubo(view, proj, cam, [{"type": "directional"}])
        frames.append(s)
    want = [_render_single(s, 0) for s in frames]
    gf = abi.TRI_GROUP_STAGE_BANDS | group_flags
    slots = []
    with raster.TriGroup(480, 270, [0] * 4, display=1, group_flags=gf) as g:
        scenes.load_scene(g, frames[0])
        for k, s in enumerate(frames):
            g.set_frame(s.ubo, s.clear)
            g.render_frame()
            col, dep = g.readback()
            f, slot = g.transfer_format()
            bpp, inbound = g.transfer_info()
            assert f == fmt and inbound == 0
            assert bpp == {0: 4, 1: 3}.get(fmt, bpp)
            if fmt == 2:
                slots.append(slot)
                assert 1 <= bpp <= (4 if k == 0 else 3) and abi.TRI_DBP_MIN_SLOT <= slot <= abi.TRI_DBP_MAX_SLOT
            assert np.array_equal(dep, want[k][1]), f"frame {k} depth"
            assert np.array_equal(col, want[k][0]), f"frame {k}: {int((col != want[k][0]).any(-1).sum())} pixels differ"
            g.present()
    if fmt == 2:
        assert slots[0] == abi.TRI_DBP_MAX_SLOT and max(slots[1:]) < abi.TRI_DBP_MAX_SLOT  # refitted after frame 0


def test_group_dbp_slot_overflow_rerenders(oracle):
    """A dbp slot fitted to a clear-only frame (header-only slots) is outgrown by the next frame's geometry:
    tri_group_synchronize reports TRI_E_OVERFLOW once and refits the slot, and the frame rendered again equals the
    single-context frame bit for bit."""
    from trident_raster import abi, raster, scenes

    s = scenes.scene_c3_grid(480, 270, 40, skybox="solid")  # a solid sky: the geometry-free frame is uniform
    want = _render_single(s, 0)
    with raster.TriGroup(480, 270, [0] * 3, display=0, group_flags=abi.TRI_GROUP_STAGE_BANDS) as g:
        scenes.load_scene(g, s)
        g.set_draws([])
        g.render_frame()  # largest slot; synchronize fits the slot to the clear colour's header-only slots
        assert g.transfer_format() == (abi.TRI_GROUP_FMT_DBP, abi.TRI_DBP_MAX_SLOT)
        g.set_draws(s.draws)
        g.render()
        with pytest.raises(raster.TriError) as e:
            g.synchronize()
        assert e.value.code == abi.TRI_E_OVERFLOW
        assert g.transfer_format() == (abi.TRI_GROUP_FMT_DBP, abi.TRI_DBP_MIN_SLOT)  # the overflowed frame's slot
        g.render_frame()
        f, slot = g.transfer_format()
        assert f == abi.TRI_GROUP_FMT_DBP and abi.TRI_DBP_MIN_SLOT < slot < abi.TRI_DBP_MAX_SLOT
        col, dep = g.readback()
        assert np.array_equal(col, want[0]) and np.array_equal(dep, want[1])


@pytest.mark.skipif(_hip_device_count() < 2, reason="the RCCL branch of tri_group needs two HIP devices")
@pytest.mark.parametrize("devices,display", [([0, 1, 0, 1], 0), ([1, 0, 1, 0, 1], 3)])
@pytest.mark.parametrize("gflags", [0, 4, 1])
def test_group_distinct_devices_rccl_assembly(oracle, devices, display, gflags):
    """the cross-device branch of tri_group (ncclCommInitAll, grouped ncclSend/ncclRecv into the
    rotating frame buffer, band buffers reused after asm_done), with the band packing in the delta bit-plane format
    (the default when the frame's alpha is proven), as 3-byte pixels (TRI_GROUP_PACK_BGR24 = 4) and off
    (TRI_GROUP_NO_PACK = 1). Four frames with different cameras; each assembled frame equals the single-context
    render, the k - 1 buffer stays untouched while frame k renders, and transfer_info / transfer_format report the
    format, the bytes per pixel and the display device's inbound bytes of the remote bands. Skipped on a one-GPU box
    (runs on the driver's multi-GPU node)."""
    from trident_raster import abi, raster, scenes

    frames = _camera_frames(oracle, [(0.0, 1.0, 6.0), (0.6, 1.3, 6.5), (-0.7, 0.8, 5.5), (0.2, 1.6, 7.0)])
    want = [_render_single(s, 0)[0] for s in frames]
    with raster.TriRaster(320, 240, device=0) as r:
        scenes.load_scene(r, frames[0])
        alpha = r.frame_alpha()
    fmt = 0 if (gflags == 1 or alpha < 0) else (1 if gflags == 4 else 2)
    n, H, W = len(devices), 240, 320
    remote = [((k + 1) * H // n - k * H // n) * W for k in range(n) if devices[k] != devices[display]]
    with raster.TriGroup(320, 240, devices, display=display, group_flags=gflags) as g:
        scenes.load_scene(g, frames[0])
        prev = None
        for k, s in enumerate(frames):
            g.set_frame(s.ubo, s.clear)
            g.render_frame()
            g.synchronize()
            f, slot = g.transfer_format()
            assert f == fmt
            if fmt == 2:
                inbound = sum(raster.dbp_bytes(px, slot) for px in remote)
                assert g.transfer_info()[1] == inbound
            else:
                bpp = 4 if fmt == 0 else 3
                assert g.transfer_info() == (bpp, sum(px * bpp for px in remote))
            p, dev = g.frame_pointer()
            img = _copy_frame(p, dev, 320, 240)
            assert np.array_equal(img, want[k]), f"frame {k}: {int((img != want[k]).any(-1).sum())} pixels differ"
            if prev is not None:
                assert np.array_equal(_copy_frame(prev[0], dev, 320, 240), want[k - 1]), f"frame {k - 1} overwritten"
            prev = (p, k)
            g.present()


@pytest.fixture(scope="module")
def app_mod():
    from trident_raster import app

    app.load_library()
    return app


def _shim_scene(app_mod, devices):
    from trident_raster import scenes

    a = app_mod.TridentApp()
    if devices:
        a.set_device_count(len(devices), devices)
    a.set_camera("editor", (0, 1, 6))
    a.set_camera("runtime", (2, 2, 5), (-10, 20, 0), fov=50.0, ready=True)
    a.set_viewport(2, 200, 150)
    a.set_viewport(1, 320, 240)
    v, i = scenes.uv_sphere_mesh(20, 28, 1.0)
    m = a.append_mesh(v, i, base_color=(0.7, 0.8, 0.9, 1), metallic=0.3, roughness=0.5)
    a.add_mesh_entity("none", m, position=(0, 0.5, 0))
    a.add_mesh_entity("cube", position=(-1.5, 0, 0), rotation=(10, 20, 30))
    a.add_light("point", position=(0, 2, 2), color=(1, 0.9, 0.8), intensity=8.0, range=6.0)
    a.set_present_extent(400, 300)
    a.draw_frame()
    a.draw_frame()
    return a


def test_gpu_shim_device_group_equals_single_viewport(app_mod):
    """Renderer::SetDeviceCount(4, [0, 0, 0, 0]): both viewports render as 4-band groups; every frame,
    the viewport textures and the presented image equal the one-context shim's, and the geometry went
    to the (single distinct) device once for both viewports."""
    from trident_raster import abi, raster

    single = _shim_scene(app_mod, None)
    multi = _shim_scene(app_mod, [0, 0, 0, 0])
    for vp, (w, h) in ((1, (320, 240)), (2, (200, 150))):
        sc_, sd = single.read_pixels(vp, w, h)
        mc, md = multi.read_pixels(vp, w, h)
        assert np.array_equal(md, sd) and np.array_equal(mc, sc_)
        img = multi.viewport_texture(vp)
        assert (img.width, img.height, img.format, img.device) == (w, h, abi.TRI_FORMAT_B8G8R8A8_UNORM, 0)
        bgra = raster.copy_device_to_host(img.device_ptr, h * img.pitch_bytes, img.device).reshape(h, w, 4)
        assert np.array_equal(bgra[..., [2, 1, 0, 3]], mc)
    assert np.array_equal(multi.read_present(400, 300), single.read_present(400, 300))
    assert multi.geometry_uploads() == 1
    multi.set_device_count(1)  # back to one context per viewport: the same frame again
    multi.draw_frame()
    mc, md = multi.read_pixels(1, 320, 240)
    sc_, sd = single.read_pixels(1, 320, 240)
    assert np.array_equal(md, sd) and np.array_equal(mc, sc_)
    single.close()
    multi.close()
    assert C.sizeof(abi.TriImage) == 32
