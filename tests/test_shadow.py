"""Shadow-map pre-pass (BASELINE.json config 5; tri_set_shadow).

The reference only reserves the switch (LightComponent::m_ShadowCaster, LightComponent.h:33), so the
pass is defined by this build and restated by the oracle (oracle/tri_oracle.cpp shadow_raster_triangle,
shadow_visibility, oracle_shadow_fit_ortho): parity is against that restatement, pinned here by
known-answer tests. GPU bar as everywhere: depth and the shadow map bit-exact, colour within 1 LSB.
"""
import ctypes as C

import numpy as np
import pytest

import scene_cases as sc

COLOR_TOL = 1


def corners(lo, hi):
    return np.array([[(hi if k & 1 else lo)[0], (hi if k & 2 else lo)[1], (hi if k & 4 else lo)[2], 1.0]
                     for k in range(8)], np.float32)


@pytest.mark.parametrize("case", [((-0.5, -1.0, -0.3), (-5, -3, -6), (5, 3, -4)),
                                  ((0.0, -1.0, 0.0), (-1, 0, -1), (1, 2, 1)),
                                  ((1.0, 0.2, 0.0), (0, 0, 0), (10, 1, 3)),
                                  ((0.0, 0.0, 0.0), (-2, -2, -2), (2, 2, 2))])
def test_fit_ortho_matches_oracle_and_contains_box(oracle, case):
    from trident_raster import raster

    d, lo, hi = case
    got = raster.shadow_fit_ortho(d, lo, hi)
    want = oracle.shadow_fit_ortho(d, lo, hi)
    assert got.tobytes() == want.tobytes()  # the product's host helper == the oracle's restatement
    m = got.reshape(4, 4)  # [col][row]
    assert np.array_equal(m[:, 3], np.array([0, 0, 0, 1], np.float32))  # affine
    ndc = corners(np.array(lo, np.float32), np.array(hi, np.float32)) @ m
    assert np.all(np.abs(ndc[:, :2]) < 1.0) and np.all(ndc[:, 2] > 0.0) and np.all(ndc[:, 2] < 1.0)
    assert np.all(np.abs(ndc[:, :2]).max(0) > 0.95)  # fitted: the box spans the map (1 % margin)


def test_fit_ortho_rejects_bad_box():
    from trident_raster import raster

    with pytest.raises(raster.TriError):
        raster.shadow_fit_ortho((0, -1, 0), (1, 0, 0), (0, 1, 1))


def quad_scene(depth_ndc, size, lvp=None):
    """One light-facing quad covering light NDC [-0.5, 0.5]^2 at light depth depth_ndc (camera
    anywhere: only the shadow map is inspected)."""
    from trident_raster import abi, scenes

    v = np.zeros(4, abi.VERTEX_DTYPE)
    v["position"] = [(-0.5, -0.5, depth_ndc), (0.5, -0.5, depth_ndc), (0.5, 0.5, depth_ndc), (-0.5, 0.5, depth_ndc)]
    v["normal"] = (0, 0, 1)
    v["color"] = 1.0
    idx = np.array([0, 1, 2, 0, 2, 3], np.uint32)
    view, proj = scenes.editor_camera((0, 0, 3), (0, 0, 0), 60.0, (64, 64))
    s = scenes.Scene("quad", 64, 64, v, idx, np.array([(0, 6, 0, 0)], abi.MESH_RANGE_DTYPE),
                     [abi.make_draw(0, np.eye(4, dtype=np.float32))], scenes.pack_ubo(view, proj, (0, 0, 3)))
    s.shadow = abi.make_shadow(np.eye(4, dtype=np.float32) if lvp is None else lvp, size, 0.0, 0.0)
    return s


def test_oracle_shadow_map_quad_kat(oracle):
    """Identity light transform: the quad covers exactly the 32 x 32 texel centres inside
    [-0.5, 0.5]^2 of a 64^2 map (no centre lies on an edge), at its depth; the rest stays at the clear 1.0."""
    s = quad_scene(0.25, 64)
    smap = np.zeros((64, 64), np.uint32)
    oracle.render(s, shadow_map_out=smap)
    d = smap.view(np.float32)
    assert np.all(d[16:48, 16:48] == np.float32(0.25))
    outside = np.ones((64, 64), bool)
    outside[16:48, 16:48] = False
    assert np.all(d[outside] == 1.0)


def test_oracle_shadow_map_depth_clamp_and_no_cull(oracle):
    """Depth clamp instead of near/far clipping: a caster in front of the light's near plane lands at
    0 and one beyond the far plane at 1. A clockwise copy (no culling) covers the same texels."""
    from trident_raster import abi

    for z, want in ((-0.5, 0.0), (1.5, 1.0)):
        s = quad_scene(z, 64)
        smap = np.zeros((64, 64), np.uint32)
        oracle.render(s, shadow_map_out=smap)
        assert np.all(smap.view(np.float32)[16:48, 16:48] == np.float32(want))
    s = quad_scene(0.25, 64)
    s.indices = np.array([0, 2, 1, 0, 3, 2], np.uint32)  # clockwise in light space
    smap = np.zeros((64, 64), np.uint32)
    oracle.render(s, shadow_map_out=smap)
    assert np.all(smap.view(np.float32)[16:48, 16:48] == np.float32(0.25))
    assert abi.TRI_OK == 0


def test_oracle_shadow_lookup_kat(oracle):
    """Visibility only scales the sun: with the pre-pass on, every pixel equals either the unshadowed
    render (lit), the render with a zero-intensity sun (fully shadowed) or lies between them (2x2
    compare edges); the unoccluded ground is lit (the bias prevents self-shadowing) and the casters
    leave a shadow of plausible size."""
    s = sc.shadow_scene(oracle, 320, 240, 256)
    lit, lit_d, _ = oracle.render(s)
    shadow = s.shadow
    s.shadow = None
    plain, plain_d, _ = oracle.render(s)
    sun = s.ubo.directional_light_color[3]
    s.ubo.directional_light_color[3] = 0.0
    dark, _, _ = oracle.render(s)
    s.ubo.directional_light_color[3] = sun
    s.shadow = shadow
    assert np.array_equal(lit_d, plain_d)
    a, p, k = (x.astype(np.int16) for x in (lit, plain, dark))
    lo, hi = np.minimum(p, k), np.maximum(p, k)
    assert np.all((a >= lo) & (a <= hi))
    covered = plain_d != 0x3F800000
    full_shadow = np.all(a == k, -1) & np.any(p != k, -1) & covered
    lit_px = np.all(a == p, -1) & covered
    assert full_shadow.sum() > 500, full_shadow.sum()
    assert lit_px.sum() > 10 * full_shadow.sum() // 4


def test_oracle_shadow_rejects_projective_light(oracle):
    s = quad_scene(0.25, 64)
    m = np.eye(4, dtype=np.float32)
    m[2, 3] = -1.0  # perspective w row
    s.shadow.light_view_proj = (C.c_float * 16)(*m.reshape(16).tolist())
    with pytest.raises(RuntimeError):
        oracle.render(s)


# ---------------------------------------------------------------------------------------------------
# GPU parity
# ---------------------------------------------------------------------------------------------------
@pytest.fixture(params=["fast", "exact"])
def flags(request):
    from trident_raster import abi

    return abi.TRI_FLAG_EXACT_SHADING if request.param == "exact" else 0


def render_gpu(scene, band=None, flags=0):
    from trident_raster import raster, scenes

    with raster.TriRaster(scene.width, scene.height, band=band, flags=flags) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        col, dep = r.readback()
        smap = r.read_shadow_map() if scene.shadow is not None else None
        stats = r.frame_stats()
    return col, dep, smap, stats


def assert_shadow_parity(scene, oracle, flags=0, band=None, min_covered=1):
    gc, gd, gm, gs = render_gpu(scene, band, flags)
    om = np.zeros((scene.shadow.size, scene.shadow.size), np.uint32)
    oc, od, os_ = oracle.render(scene, band=band, shadow_map_out=om)
    assert int((gm != om).sum()) == 0, "shadow map mismatch"
    assert int((gd != od).sum()) == 0, "depth mismatch"
    diff = np.abs(gc.astype(np.int16) - oc.astype(np.int16))
    assert int(diff.max(initial=0)) <= COLOR_TOL, f"colour diff {diff.max()}"
    assert int((od != 0x3F800000).sum()) >= min_covered
    assert gs["triangles_setup"] == os_["triangles_setup"]
    return om


@pytest.mark.gpu
def test_gpu_shadow_scene(oracle, flags):
    om = assert_shadow_parity(sc.shadow_scene(oracle, 480, 320, 512), oracle, flags, min_covered=50000)
    assert (om != 0x3F800000).sum() > 10000  # casters landed in the map


@pytest.mark.gpu
def test_gpu_shadow_map_kats():
    """The GPU map reproduces the oracle KATs: the 32 x 32 quad footprint, clamped depths, no culling."""
    for z, want in ((0.25, 0.25), (-0.5, 0.0), (1.5, 1.0)):
        _, _, gm, _ = render_gpu(quad_scene(z, 64))
        d = gm.view(np.float32)
        assert np.all(d[16:48, 16:48] == np.float32(want))
        d = d.copy()
        d[16:48, 16:48] = 1.0
        assert np.all(d == 1.0)


@pytest.mark.gpu
def test_gpu_shadow_clipped_casters_and_receivers(oracle, flags):
    """Near-plane clipped receivers (their polygon vertices carry light-space positions) under a
    shadow-casting sun."""
    from trident_raster import scenes

    s = scenes.with_shadow(sc.near_clip_grid(320, 240, 40), 256)
    assert_shadow_parity(s, oracle, flags, min_covered=10000)


@pytest.mark.gpu
def test_gpu_shadow_row_bands(oracle):
    """Each band renders the whole map (replicated pre-pass) and shades its rows: bands == full frame."""
    s = sc.shadow_scene(oracle, 320, 240, 256)
    full_c, full_d, full_m, _ = render_gpu(s)
    parts = [render_gpu(s, band=(a, b)) for a, b in ((0, 80), (80, 160), (160, 240))]
    assert np.array_equal(np.concatenate([p[0] for p in parts]), full_c)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), full_d)
    for p in parts:
        assert np.array_equal(p[2], full_m)


@pytest.mark.gpu
def test_gpu_shadow_off_again_matches_plain(oracle):
    """tri_set_shadow(NULL) returns the context to the reference's frame exactly."""
    from trident_raster import raster, scenes

    s = sc.shadow_scene(oracle, 256, 192, 256)
    shadow = s.shadow
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        r.set_shadow(None)
        r.render_frame()
        col, dep = r.readback()
    s.shadow = None
    oc, od, _ = oracle.render(s)
    assert np.array_equal(dep, od)
    assert int(np.abs(col.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL
    assert shadow.size == 256


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_gpu_c5_full_4k_textures_and_shadow(oracle, mode):
    """BASELINE C5 at full size: 3840x2160, 1M triangles in 4 draws with four 2048^2 sRGB textures and
    the 2048^2 shadow pre-pass, in both shading builds. Map and depth bit-exact, colour within 1 LSB."""
    from trident_raster import abi, scenes

    s = scenes.scene_c5_textured()
    assert s.shadow is not None and s.shadow.size == 2048
    flags = abi.TRI_FLAG_EXACT_SHADING if mode == "exact" else 0
    om = assert_shadow_parity(s, oracle, flags, min_covered=3840 * 2160 // 2)
    assert (om != 0x3F800000).sum() > 100000


@pytest.mark.gpu
def test_gpu_shadow_map_refreshed_every_frame(oracle):
    """The map is rebuilt from scratch each frame: after a frame without any draw it is all 1.0 (no caster, no
    set-up pass), and the next frame with casters matches the oracle again (the bins' counts were reset)."""
    from trident_raster import raster, scenes

    s = sc.shadow_scene(oracle, 256, 192, 256)
    om = np.zeros((s.shadow.size, s.shadow.size), np.uint32)
    oracle.render(s, shadow_map_out=om)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        first = r.read_shadow_map()
        r.set_draws([])
        r.render_frame()
        empty = r.read_shadow_map()
        r.set_draws(s.draws)
        r.render_frame()
        again = r.read_shadow_map()
    assert np.array_equal(first, om) and (om != 0x3F800000).sum() > 1000
    assert (empty == 0x3F800000).all()
    assert np.array_equal(again, om)
