"""Second viewport + presentation blit. The editor renders every viewport, then
blits the primary one onto the swapchain image with vkCmdBlitImage(..., VK_FILTER_LINEAR)
(Renderer.cpp:5208-5221, :5346-5361); the primary viewport is the one SetViewport was called for
last (:2751-2754).

CPU: known answers of the oracle's blit restatement (Vulkan "Image Blits": destination texel centres
scaled into the source, bilinear over clamp-to-edge taps of UNORM values, UNORM8 rounding). GPU: the
HIP blit (tri_blit_linear) and the shim's present image against that restatement, bit-exact.
Parity against a Vulkan driver's blit is unpinned (no Vulkan here; its filter precision is
implementation-defined).
"""
import numpy as np
import pytest

import scene_cases as sc


def blit_ref(src, dw, dh):
    """numpy float32 restatement with the oracle's operation order (checks the C restatement)."""
    h, w = src.shape[:2]
    f32 = np.float32
    sx, sy = f32(w) / f32(dw), f32(h) / f32(dh)
    x = np.arange(dw, dtype=f32)
    y = np.arange(dh, dtype=f32)
    u = (x + f32(0.5)) * sx - f32(0.5)
    v = (y + f32(0.5)) * sy - f32(0.5)
    fu, fv = np.floor(u), np.floor(v)
    a, b = (u - fu).astype(f32), (v - fv).astype(f32)
    i0, j0 = fu.astype(np.int64), fv.astype(np.int64)
    xa, xb = np.clip(i0, 0, w - 1), np.clip(i0 + 1, 0, w - 1)
    ya, yb = np.clip(j0, 0, h - 1), np.clip(j0 + 1, 0, h - 1)
    t = src.astype(f32) / f32(255.0)
    t00, t10 = t[ya][:, xa], t[ya][:, xb]
    t01, t11 = t[yb][:, xa], t[yb][:, xb]
    A, B = a[None, :, None], b[:, None, None]
    l0 = t00 + A * (t10 - t00)
    l1 = t01 + A * (t11 - t01)
    c = np.clip(l0 + B * (l1 - l0), 0, 1)
    return np.floor(c * f32(255.0) + f32(0.5)).astype(np.uint8)


def test_blit_identity_and_known_answers(oracle):
    rng = np.random.default_rng(7)
    src = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    assert np.array_equal(oracle.blit_linear(src, 53, 37), src)  # same extent: a copy
    # 2x downscale: every destination centre falls between 4 source texels at weights 1/2, 1/2
    sq = rng.integers(0, 256, (8, 8, 4), dtype=np.uint8)
    half = oracle.blit_linear(sq, 4, 4)
    avg = sq.reshape(4, 2, 4, 2, 4).astype(np.float64).mean(axis=(1, 3))
    assert np.abs(half.astype(np.float64) - avg).max() <= 0.5 + 1e-6
    # upscale: clamp-to-edge keeps the corner texels
    up = oracle.blit_linear(sq, 32, 32)
    assert np.array_equal(up[0, 0], sq[0, 0]) and np.array_equal(up[-1, -1], sq[-1, -1])


@pytest.mark.parametrize("shape", [(480, 640, 720, 1280), (480, 640, 240, 320), (37, 53, 177, 333), (64, 64, 1, 1)])
def test_blit_restatements_agree(oracle, shape):
    h, w, dh, dw = shape
    src = np.random.default_rng(h * w + dw).integers(0, 256, (h, w, 4), dtype=np.uint8)
    assert np.array_equal(oracle.blit_linear(src, dw, dh), blit_ref(src, dw, dh))


# ---- GPU ----------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("dw,dh", [(1280, 720), (320, 240), (333, 177), (640, 480), (640, 301), (1001, 480)])
def test_gpu_blit_matches_oracle(oracle, dw, dh):
    from trident_raster import raster, scenes

    s = sc.c1_cube_skybox(1)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        col, _ = r.readback(depth=False)
        r.blit(dw, dh)
        got = r.read_present()
    assert np.array_equal(got, oracle.blit_linear(col, dw, dh))


@pytest.mark.gpu
def test_gpu_blit_rejects_bands():
    from trident_raster import raster, scenes

    s = sc.c1_cube_skybox(1)
    with raster.TriRaster(s.width, s.height, band=(0, 240)) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        with pytest.raises(raster.TriError):
            r.blit(320, 240)


@pytest.mark.gpu
def test_gpu_shim_presents_the_active_viewport(oracle):
    """Scene (id 1) and Game (id 2) viewports render every frame; the one SetViewport touched last is
    blitted to the swapchain-sized present image."""
    from trident_raster import app

    a = app.TridentApp()
    a.set_camera("editor", (0.0, 3.0, 8.0))
    a.set_camera("runtime", (2.0, 2.0, 6.0), (-10.0, 20.0, 0.0), fov=70.0, ready=True)
    a.set_viewport(2, 320, 200)
    a.set_viewport(1, 480, 270)  # active
    a.add_mesh_entity("cube", position=(0.0, 3.0, -2.0), rotation=(0.0, 30.0, 0.0))
    a.add_mesh_entity("sphere", position=(1.5, 3.0, -1.0))
    a.set_present_extent(960, 540)
    a.draw_frame()
    a.draw_frame()
    vp1, _ = a.read_pixels(1, 480, 270, depth=False)
    present = a.read_present(960, 540)
    want = oracle.blit_linear(vp1[..., [2, 1, 0, 3]], 960, 540)[..., [2, 1, 0, 3]]  # RGBA <-> BGRA
    assert np.array_equal(present, want)
    a.set_viewport(2, 320, 200)  # the Game view becomes primary
    a.draw_frame()
    vp2, _ = a.read_pixels(2, 320, 200, depth=False)
    present = a.read_present(960, 540)
    assert np.array_equal(present, oracle.blit_linear(vp2[..., [2, 1, 0, 3]], 960, 540)[..., [2, 1, 0, 3]])


# ---- legacy direct-to-swapchain path (Renderer.cpp:5233, :5498-5590) --------------------------------
def _legacy_app(with_viewport=False, flags=0):
    from trident_raster import app, scenes

    a = app.TridentApp(raster_flags=flags)
    a.set_assets_dir(scenes.ASSETS_DIR)
    a.set_camera("editor", (0.0, 3.0, 8.0), (-8.0, 15.0, 0.0))
    a.add_mesh_entity("cube", position=(0.0, 3.0, -2.0), rotation=(0.0, 30.0, 0.0))
    a.add_mesh_entity("sphere", position=(1.5, 3.0, -1.0))
    a.add_sprite_entity(position=(-1.5, 2.5, 0.0), tint=(1.0, 0.5, 0.25, 1.0))
    if with_viewport:
        a.set_viewport(1, 320, 200)
    a.set_present_extent(400, 300)
    return a


def test_legacy_pass_inputs_without_viewports():
    """With no viewport registered, the present pass's uniform block comes from GetActiveCamera() (the
    reference's null-camera UpdateUniformBuffer, Renderer.cpp:5223-5226): frame_inputs(0) exposes it; once
    a viewport exists, id 0 names no pass."""
    a = _legacy_app()
    ubo, draws = a.frame_inputs(0)
    assert len(draws) == 3  # cube, sphere, then the sprite (GatherSpriteDraws after the meshes)
    assert abs(ubo.camera_position[1] - 3.0) < 1e-6
    a.close()
    b = _legacy_app(with_viewport=True)
    with pytest.raises(Exception):
        b.frame_inputs(0)
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [False, True])
def test_gpu_shim_legacy_present_without_viewport(oracle, exact):
    """No SetViewport call: DrawFrame renders the skybox, the meshes and the sprite straight into the present
    image at the present (swapchain) extent; the image matches the oracle's frame of the same inputs (depth
    is not stored by that pass, Pipeline.cpp:395)."""
    from trident_raster import abi, scenes

    a = _legacy_app(flags=abi.TRI_FLAG_EXACT_SHADING if exact else 0)
    a.draw_frame()
    a.draw_frame()
    present = a.read_present(400, 300)
    ubo, draws = a.frame_inputs(0)
    vb, ib, ranges = a.geometry()
    s = scenes.Scene("legacy", 400, 300, vb, ib, ranges, draws, ubo,
                     materials=[(m[0], m[1]) for m in a.materials()], skybox=scenes.reference_skybox())
    oc, od, _ = oracle.render(s)
    assert (od != 0x3F800000).sum() > 1000  # the meshes and the sprite are on screen
    diff = np.abs(present.astype(np.int16) - oc[..., [2, 1, 0, 3]].astype(np.int16))
    assert int(diff.max()) <= 1, int(diff.max())
    # registering a viewport switches the present back to the blit of the primary viewport
    a.set_viewport(1, 320, 200)
    a.draw_frame()
    vp1, _ = a.read_pixels(1, 320, 200, depth=False)
    assert np.array_equal(a.read_present(400, 300),
                          oracle.blit_linear(vp1[..., [2, 1, 0, 3]], 400, 300)[..., [2, 1, 0, 3]])
    a.close()


@pytest.mark.gpu
@pytest.mark.parametrize("with_viewport", [False, True])
def test_gpu_present_read_after_extent_change(with_viewport):
    """a SetPresentExtent between DrawFrame and ReadPresentPixels (a window resize) must not change
    the size of the image the read returns — it is the one the last present produced, legacy or blit."""
    a = _legacy_app(with_viewport=with_viewport)
    a.draw_frame()
    before = a.read_present(400, 300)
    a.set_present_extent(200, 150)  # smaller: the old code sized the host buffer from this
    assert np.array_equal(a.read_present(400, 300), before)
    with pytest.raises(Exception):
        a.read_present(200, 150)
    a.draw_frame()  # the next present is produced at the new extent
    assert a.read_present(200, 150).shape == (150, 200, 4)
    a.close()
