"""Default.frag's AI frame-generation blend (Default.frag:182-191): with AiBlendConfig.w > 0 every mesh fragment's
output becomes mix(colour, texture(AiBlendTexture, gl_FragCoord.xy * AiBlendConfig.yz), clamp(AiBlendConfig.x, 0, 1)),
the texture being the R8G8B8A8_UNORM frame UploadAiInterpolationToGpu fills (Renderer.cpp:1560-1700; LINEAR,
CLAMP_TO_EDGE). CPU: known answers of the oracle's restatement. GPU: the HIP path (k_raster_ai) against it."""
import numpy as np
import pytest

import scene_cases as sc


def _cube(frame=2, w=320, h=240):
    """The C3 grid at 320x240 (it covers most of the frame) over the solid sky."""
    s = sc.grid_c3(w, h, 60)
    from trident_raster import scenes

    s.skybox = scenes.DEFAULT_SKYBOX
    return s


def _bgra_to_rgba(c):
    return c[..., [2, 1, 0, 3]]


def test_oracle_full_weight_returns_the_ai_frame(oracle):
    """Weight 1: mix(c, ai, 1) = ai exactly, so every mesh pixel holds its AI texel (sampled at its own centre on a
    frame of the same extent) and every background pixel keeps the sky."""
    from trident_raster import scenes

    base = _cube()
    c0, d0, _ = oracle.render(base)
    s = scenes.with_ai_blend(_cube(), strength=1.0)
    c1, d1, _ = oracle.render(s)
    assert np.array_equal(d0, d1)
    mesh = d0 != 0x3F800000
    assert mesh.sum() > 5000
    assert np.array_equal(_bgra_to_rgba(c1)[mesh], s.ai_frame[mesh])
    assert np.array_equal(c1[~mesh], c0[~mesh])


def test_oracle_weights_and_switch(oracle):
    """AiBlendConfig.w = 0 or a weight clamped to 0 leaves the frame as it was; weight 0.35 is the GLSL mix of the two
    (within the 1-LSB rounding of the unblended frame's stored bytes); strengths above 1 clamp to 1."""
    from trident_raster import scenes

    c0, _, _ = oracle.render(_cube())
    off = scenes.with_ai_blend(_cube(), strength=0.35)
    off.ubo.ai_blend_config[3] = 0.0
    assert np.array_equal(oracle.render(off)[0], c0)
    assert np.array_equal(oracle.render(scenes.with_ai_blend(_cube(), strength=-2.0))[0], c0)
    s = scenes.with_ai_blend(_cube(), strength=0.35)
    c, d, _ = oracle.render(s)
    mesh = d != 0x3F800000
    want = _bgra_to_rgba(c0).astype(np.float64) * 0.65 + s.ai_frame.astype(np.float64) * 0.35
    diff = np.abs(_bgra_to_rgba(c).astype(np.float64) - want)[mesh]
    assert diff.max() <= 1.0, diff.max()
    full = oracle.render(scenes.with_ai_blend(_cube(), strength=7.0))[0]
    assert np.array_equal(full, oracle.render(scenes.with_ai_blend(_cube(), strength=1.0))[0])


def test_oracle_ai_frame_of_another_extent_is_filtered(oracle):
    """uv = gl_FragCoord.xy * AiBlendConfig.yz: a constant frame of another extent stays constant (the coordinates
    leave it and clamp); a 2x2 ramp addressed with the frame's own 1 / extent is filtered LINEAR between its texel
    centres and clamped at the edges."""
    from trident_raster import scenes

    flat = np.full((120, 160, 4), (10, 200, 90, 255), np.uint8)
    s = scenes.with_ai_blend(_cube(), strength=1.0, ai_frame=flat)
    c, d, _ = oracle.render(s)
    mesh = d != 0x3F800000
    assert (_bgra_to_rgba(c)[mesh] == (10, 200, 90, 255)).all()
    ramp = np.zeros((2, 2, 4), np.uint8)
    ramp[:, 1] = 255  # left column 0, right column 255: the frame's x ramp after bilinear filtering
    s = scenes.with_ai_blend(_cube(), strength=1.0, ai_frame=ramp)
    s.ubo.ai_blend_config[1] = np.float32(1.0) / np.float32(320)  # uv = gl_FragCoord / the frame's extent
    s.ubo.ai_blend_config[2] = np.float32(1.0) / np.float32(240)
    c, d, _ = oracle.render(s)
    rgba = _bgra_to_rgba(c).astype(np.int32)
    ys, xs = np.nonzero(d != 0x3F800000)
    u = (xs + 0.5) / 320 * 2 - 0.5
    want = np.clip(u, 0.0, 1.0) * 255
    assert np.abs(rgba[ys, xs, 0] - want).max() <= 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("case", ["cube", "grid_one", "textured", "multi"])
def test_gpu_ai_blend_matches_oracle(oracle, exact, case):
    """k_raster_ai against the oracle, depth bit-exact and colour within 1 LSB, on the single-draw solid frame (which
    otherwise takes the ONE instantiation), a textured draw and several draws; the frame alpha is not claimed
    uniform."""
    from test_parity_gpu import assert_parity
    from trident_raster import abi, raster, scenes

    s = {"cube": _cube, "grid_one": lambda: sc.grid_c3(640, 360, 120), "textured": sc.textured_grid,
         "multi": lambda: sc.primitives_row(oracle)}[case]()
    scenes.with_ai_blend(s, strength=0.35)
    flags = abi.TRI_FLAG_EXACT_SHADING if exact else 0
    assert_parity(s, oracle, min_covered=2000, flags=flags)
    with raster.TriRaster(s.width, s.height, flags=flags) as r:
        scenes.load_scene(r, s)
        assert r.frame_alpha() == -1


@pytest.mark.gpu
def test_gpu_ai_blend_errors(oracle):
    """A blending UBO without an AI frame is TRI_E_STATE at tri_render; with the shadow pre-pass TRI_E_UNSUPPORTED;
    removing the frame and the blend brings back the plain frame."""
    from trident_raster import abi, raster, scenes

    s = scenes.with_ai_blend(_cube(), strength=0.35)
    frame = s.ai_frame
    with raster.TriRaster(s.width, s.height) as r:
        s.ai_frame = None
        scenes.load_scene(r, s)
        with pytest.raises(raster.TriError) as e:
            r.render_frame()
        assert e.value.code == abi.TRI_E_STATE
        r.upload_ai_frame(frame)
        r.set_shadow(abi.make_shadow(np.eye(4, dtype=np.float32), 256, 0.001, 2.0))
        with pytest.raises(raster.TriError) as e:
            r.render_frame()
        assert e.value.code == abi.TRI_E_UNSUPPORTED
        r.set_shadow(None)
        r.upload_ai_frame(None)
        plain = _cube()
        r.set_frame(plain.ubo, plain.clear)
        r.render_frame()
        col, dep = r.readback()
    oc, od, _ = oracle.render(plain)
    assert np.array_equal(dep, od) and int(np.abs(col.astype(np.int16) - oc.astype(np.int16)).max()) <= 1


def _shim_app():
    from trident_raster import app, scenes

    a = app.TridentApp()
    a.set_assets_dir(scenes.ASSETS_DIR)
    a.set_camera("editor", (0.0, 3.0, 8.0), (-8.0, 15.0, 0.0))
    a.add_mesh_entity("cube", position=(0.0, 3.0, -2.0), rotation=(0.0, 30.0, 0.0))
    a.add_mesh_entity("sphere", position=(1.2, 3.0, -1.0), scale=(2.0, 2.0, 2.0))
    a.set_viewport(1, 320, 240)
    return a


def test_shim_packs_ai_blend_config():
    """UpdateUniformBuffer's AiBlendConfig (Renderer.cpp:5916-5925): zero without a frame; (strength, 1 / w, 1 / h, 1)
    with one; SetAiBlendStrength clamps to [0, 1]; dropping the frame zeroes it again."""
    a = _shim_app()
    ubo, _ = a.frame_inputs(1)
    assert list(ubo.ai_blend_config) == [0.0, 0.0, 0.0, 0.0]
    a.submit_ai_frame(np.zeros((240, 320, 3), np.float32))
    ubo, _ = a.frame_inputs(1)
    assert list(ubo.ai_blend_config) == [np.float32(0.35), np.float32(1 / 320), np.float32(1 / 240), 1.0]
    a.set_ai_blend_strength(3.0)
    assert a.frame_inputs(1)[0].ai_blend_config[0] == 1.0
    a.submit_ai_frame(None)
    assert list(a.frame_inputs(1)[0].ai_blend_config) == [0.0, 0.0, 0.0, 0.0]
    a.close()


@pytest.mark.gpu
def test_gpu_shim_ai_blend_viewport(oracle):
    """SubmitAiInterpolation's packing (clamp, round(v * 255), alpha 1 for a 3-channel frame) and the blend through
    the shim: the viewport equals the oracle's frame of the same inputs with the same AI texture."""
    from trident_raster import scenes

    a = _shim_app()
    rng = np.random.default_rng(5)
    gen = rng.uniform(-0.2, 1.2, size=(240, 320, 3)).astype(np.float32)  # out-of-range values clamp
    a.submit_ai_frame(gen)
    a.draw_frame()
    rgba, _ = a.read_pixels(1, 320, 240, depth=False)
    ubo, draws = a.frame_inputs(1)
    vb, ib, ranges = a.geometry()
    packed = np.empty((240, 320, 4), np.uint8)
    packed[..., :3] = np.round(np.clip(gen, 0.0, 1.0) * np.float32(255.0)).astype(np.uint8)
    packed[..., 3] = 255
    s = scenes.Scene("shim_ai", 320, 240, vb, ib, ranges, draws, ubo, materials=[(m[0], m[1]) for m in a.materials()],
                     skybox=scenes.reference_skybox(), ai_frame=packed)
    oc, od, _ = oracle.render(s)
    assert (od != 0x3F800000).sum() > 2000
    diff = np.abs(rgba.astype(np.int16) - oc[..., [2, 1, 0, 3]].astype(np.int16))
    assert int(diff.max()) <= 1, int(diff.max())
    a.close()
