"""Known-answer tests that pin the CPU oracle to the reference's definitions (SURVEY.md §8(c) KATs).

The reference has no tests or golden images of its own, so these restate expected
values from the reference's sources: glm's documented matrix conventions (EditorCamera.cpp:126-160,
Renderer.cpp:417-427), Default.frag's BRDF evaluated independently in float64 numpy, the sampler
state (Renderer.cpp:3592-3607), the fill/cull/depth state (Pipeline.cpp:611-666) and
UpdateUniformBuffer's light packing (Renderer.cpp:5822-5925).
"""
import numpy as np
import pytest

from trident_raster import abi, scenes


# ---------------------------------------------------------------------------------------------
# matrices
# ---------------------------------------------------------------------------------------------
def test_perspective_rh_zo_with_vulkan_flip(oracle):
    view, proj, fwd = oracle.editor_camera((0, 3, 8), (0, 0, 0), 60.0, (640, 480), 0.1, 1000.0)
    P = proj  # [col][row]
    assert P[0, 0] == pytest.approx(1.299038, abs=1e-6)
    assert P[1, 1] == pytest.approx(-1.732051, abs=1e-6)
    assert P[2, 2] == pytest.approx(-1.0001, abs=1e-6)
    assert P[3, 2] == pytest.approx(-0.10001, abs=1e-7)
    assert P[2, 3] == -1.0 and P[3, 3] == 0.0
    # view = mat4_cast(conj(q)) * translate(-p): identity rotation -> translation column (0,-3,-8)
    assert np.array_equal(view[3], np.array([0, -3, -8, 1], np.float32))
    assert np.allclose(fwd, [0, 0, -1])


def test_editor_camera_rotation_and_spawn_point(oracle):
    view, proj, fwd = oracle.editor_camera((0, 3, 8), (0, 90.0, 0), 60.0, (640, 480))
    assert np.allclose(fwd, [-1, 0, 0], atol=1e-6)  # yaw 90 deg looks down -x
    # Forge spawns primitives at camera + 10 * forward (ApplicationLayer.cpp:688)
    _, _, f0 = oracle.editor_camera((0, 3, 8), (0, 0, 0))
    assert np.allclose(np.array([0, 3, 8]) + 10 * f0, [0, 3, -2])


def test_runtime_camera_is_gl_depth_range(oracle):
    view, proj = oracle.runtime_camera((0, 1.8, 6), (0, 0, 0), 60.0, (1280, 720), 0.1, 1000.0)
    assert proj[2, 2] == pytest.approx(-(1000.1) / 999.9, rel=1e-6)  # perspectiveRH_NO
    assert proj[3, 2] == pytest.approx(-(2 * 1000 * 0.1) / 999.9, rel=1e-6)
    assert proj[1, 1] < 0  # Y flip
    assert np.allclose(view[3, :3], [0, -1.8, -6], atol=1e-6)


def test_compose_transform_trs_order(oracle):
    m = oracle.compose_transform((1, 2, 3), (0, 90, 0), (2, 1, 1))
    v = m.T @ np.array([1, 0, 0, 1], np.float32)  # column-major: M * v = m.T @ v
    assert np.allclose(v, [1, 2, 1, 1], atol=1e-6)  # x scaled by 2, rotated +90 about y -> -z
    # the numpy restatement used by bench scenes agrees bit-for-bit
    assert np.array_equal(m, scenes.compose_transform((1, 2, 3), (0, 90, 0), (2, 1, 1)))


# ---------------------------------------------------------------------------------------------
# helpers: direct clip-space scenes (view = projection = identity -> clip = world, w = 1)
# ---------------------------------------------------------------------------------------------
def ndc_quad(x0, x1, y0, y1, z=0.5, uv=None):
    v = np.zeros(4, abi.VERTEX_DTYPE)
    v["position"] = [(x0, y0, z), (x1, y0, z), (x1, y1, z), (x0, y1, z)]
    v["normal"] = (0, 0, 1)
    v["color"] = 1.0
    v["texcoord"] = uv if uv is not None else [(0, 0), (1, 0), (1, 1), (0, 1)]
    # identity projection has no Y flip: framebuffer y grows with NDC y, so CCW-on-screen (front)
    # is the cube-style winding (0,2,1),(0,3,2)
    return v, np.array([0, 2, 1, 0, 3, 2], np.uint32)


def identity_scene(v, idx, w, h, lights=(), materials=(), textures=(), draws=None, cam=(0, 0, 3),
                   ambient=(0.03, 0.03, 0.03), counts=None):
    I = np.eye(4, dtype=np.float32)
    ubo = scenes.pack_ubo(I, I, cam, list(lights), ambient=ambient)
    if counts is not None:
        ubo.light_counts = (abi.C.c_uint32 * 4)(*counts, 0, 0)
    meshes = np.array([(0, idx.size, 0, 0)], abi.MESH_RANGE_DTYPE)
    return scenes.Scene("kat", w, h, v, idx, meshes, draws or [abi.make_draw(0, I)], ubo,
                        materials=list(materials), textures=list(textures))


# ---------------------------------------------------------------------------------------------
# rasterization rules
# ---------------------------------------------------------------------------------------------
def test_top_left_fill_rule_and_shared_edge_once(oracle):
    W = H = 32
    nx = lambda x: 2 * x / W - 1  # noqa: E731  framebuffer x -> NDC
    v, idx = ndc_quad(nx(10.5), nx(20.5), nx(5.5), nx(15.5))  # every edge passes through centres
    col, dep, st = oracle.render(identity_scene(v, idx, W, H))
    covered = dep != 0x3F800000
    ys, xs = np.nonzero(covered)
    assert (xs.min(), xs.max(), ys.min(), ys.max()) == (10, 19, 5, 14)  # left/top in, right/bottom out
    assert covered.sum() == 100
    assert st["fragments_tested"] == 100  # the shared diagonal's centre pixels are owned exactly once


def test_backface_cull_and_cube_quirk(oracle):
    """Pipeline.cpp:637-638 cull BACK / front CCW; the cube's (0,2,1),(0,3,2) faces are CW from outside
    (Renderer.cpp:163-168): from Forge's camera the +Z face is culled and the interior renders."""
    base = scenes.scene_c1_cube(0)
    plus_z = scenes.Scene("pz", base.width, base.height, base.vertices, base.indices[:6], base.meshes.copy(),
                          base.draws, base.ubo, base.materials)
    plus_z.meshes["index_count"] = 6
    _, dep, st = oracle.render(plus_z)
    assert st["triangles_setup"] == 0 and (dep == 0x3F800000).all()
    minus_z = scenes.Scene("mz", base.width, base.height, base.vertices, base.indices[6:12], base.meshes.copy(),
                           base.draws, base.ubo, base.materials)
    minus_z.meshes["index_count"] = 6
    _, dep, st = oracle.render(minus_z)
    assert st["triangles_setup"] == 2 and (dep != 0x3F800000).sum() > 500


def test_depth_is_screen_linear_and_less_or_equal(oracle):
    W = H = 16
    v, idx = ndc_quad(-0.9, 0.9, -0.9, 0.9, z=0.25)
    I = np.eye(4, dtype=np.float32)
    draws = [abi.make_draw(0, I, tint=(1, 0, 0, 1)), abi.make_draw(0, I, tint=(0, 0, 1, 1))]
    col, dep, _ = oracle.render(identity_scene(v, idx, W, H, draws=draws, counts=(0, 0), ambient=(1, 1, 1)))
    inside = dep != 0x3F800000
    assert (dep[inside].view(np.float32) == np.float32(0.25)).all()
    # equal depth: the later draw (blue) passes LESS_OR_EQUAL and overwrites
    assert (col[inside][:, 0] > 0).all() and (col[inside][:, 2] == 0).all()


def test_near_plane_clip_depth_range(oracle):
    from scene_cases import near_clip_grid

    _, dep, st = oracle.render(near_clip_grid())
    assert st["triangles_clipped"] > 0
    d = dep.view(np.float32)
    assert (d >= 0).all() and (d <= 1).all()


# ---------------------------------------------------------------------------------------------
# sampler: sRGB decode before bilinear, REPEAT, level 0
# ---------------------------------------------------------------------------------------------
def srgb_to_linear(c):
    c = c / 255.0
    return np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)


def expected_ambient_only(albedo):
    c = albedo / (albedo + 1.0)
    return np.floor(np.clip(c ** (1 / 2.2), 0, 1) * 255 + 0.5).astype(int)


@pytest.mark.parametrize("u,expect_linear", [(0.5, 0.5), (1.25, 0.0), (-0.25, 1.0), (0.375, 0.25)])
def test_srgb_decode_then_bilinear_repeat(oracle, u, expect_linear):
    tex = np.array([[[0, 0, 0, 255], [255, 255, 255, 255]]], np.uint8)  # 2x1: black, white
    v, idx = ndc_quad(-1, 1, -1, 1, uv=[(u, 0.5)] * 4)
    s = identity_scene(v, idx, 8, 8, textures=[(0, tex)], counts=(0, 0), ambient=(1, 1, 1),
                       materials=[((1, 1, 1, 1), (0, 1, 1, 0))])
    col, dep, _ = oracle.render(s)
    got = col[4, 4, :3].astype(int)
    exp = expected_ambient_only(np.float64(expect_linear))
    assert (np.abs(got - exp) <= 1).all(), (got, exp)
    if u == 0.5:  # filtering the encoded bytes instead would give ~116
        assert abs(int(got[0]) - 116) > 20


# ---------------------------------------------------------------------------------------------
# Default.frag in float64 (independent restatement of Default.frag:67-192)
# ---------------------------------------------------------------------------------------------
def frag_f64(P, N, cam, albedo, metallic, roughness, amb, sun, points):
    N = N / np.linalg.norm(N)
    V = (cam - P) / np.linalg.norm(cam - P)
    F0 = 0.04 * (1 - metallic) + albedo * metallic

    def pbr(L, rad):
        H = (V + L) / np.linalg.norm(V + L)
        a2 = (roughness * roughness) ** 2
        ndh = max(N @ H, 0)
        D = a2 / (np.pi * (ndh * ndh * (a2 - 1) + 1) ** 2)
        k = (roughness + 1) ** 2 / 8
        g = lambda x: x / max(x * (1 - k) + k, 1e-4)  # noqa: E731
        ndv, ndl = max(N @ V, 0), max(N @ L, 0)
        F = F0 + (1 - F0) * np.clip(1 - max(H @ V, 0), 0, 1) ** 5
        spec = D * g(ndv) * g(ndl) * F / max(4 * ndv * ndl, 1e-4)
        kd = (1 - F) * (1 - metallic)
        return (kd * albedo / np.pi + spec) * rad * ndl

    c = amb * albedo
    if sun is not None:
        c = c + pbr(-sun[0] / np.linalg.norm(sun[0]), sun[1])
    for pos, rng, rad in points:
        d = np.linalg.norm(pos - P)
        att = (1 - np.clip(d / max(rng, 1e-4), 0, 1)) ** 2
        c = c + pbr((pos - P) / d, rad * att)
    c = c / (c + 1)
    return np.floor(np.clip(c ** (1 / 2.2), 0, 1) * 255 + 0.5).astype(int)


def test_pbr_brdf_against_float64(oracle):
    W, H = 48, 32
    v, idx = ndc_quad(-1, 1, -1, 1, z=0.5, uv=[(0.5, 0.5)] * 4)
    v["color"] = (0.9, 0.7, 0.5)
    lights = [{"type": "directional", "direction": (-0.3, -0.6, -1.0), "color": (1.0, 0.95, 0.9), "intensity": 3.0},
              {"type": "point", "position": (0.4, 0.3, 0.8), "range": 3.0, "intensity": 5.0, "color": (1, 0.8, 0.6)},
              {"type": "point", "position": (-0.6, -0.2, 1.2), "range": 4.0, "intensity": 2.0, "color": (0.5, 0.7, 1)}]
    mat = ((1.0, 0.9, 0.8, 1.0), (0.3, 0.5, 1.0, 0.0))
    s = identity_scene(v, idx, W, H, lights=lights, materials=[mat], cam=(0.1, 0.2, 2.5))
    col, dep, _ = oracle.render(s)
    base = np.array(mat[0][:3])
    albedo = base * np.array([0.9, 0.7, 0.5])
    sun = (np.array([-0.3, -0.6, -1.0]), np.array([1.0, 0.95, 0.9]) * 3.0)
    pts = [(np.array(L["position"]), L["range"], np.array(L["color"]) * L["intensity"]) for L in lights[1:]]
    worst = 0
    for py in range(0, H, 3):
        for px in range(0, W, 3):
            P = np.array([(px + 0.5) * 2 / W - 1, (py + 0.5) * 2 / H - 1, 0.5])
            exp = frag_f64(P, np.array([0, 0, 1.0]), np.array([0.1, 0.2, 2.5]), albedo, 0.3, 0.5,
                           np.full(3, 0.03), sun, pts)
            got = col[py, px, [2, 1, 0]].astype(int)  # BGRA -> RGB
            worst = max(worst, int(np.abs(got - exp).max()))
    assert worst <= 1, worst


def test_unorm_output_is_bgra_and_clear_colour(oracle):
    v, idx = ndc_quad(2, 3, 2, 3)  # off-screen: nothing drawn
    s = identity_scene(v, idx, 4, 4)
    s.clear = (0.005, 0.5, 1.0, 1.0)
    col, dep, _ = oracle.render(s)
    assert (col.reshape(-1, 4) == [255, 128, 1, 255]).all()  # B, G, R, A; round-to-nearest
    assert (dep == 0x3F800000).all()


# ---------------------------------------------------------------------------------------------
# UpdateUniformBuffer packing (Renderer.cpp:5822-5925)
# ---------------------------------------------------------------------------------------------
def ubo_of(oracle, lights):
    I = np.eye(4, dtype=np.float32)
    return oracle.pack_ubo(I, I, (0, 0, 0), lights)


def test_ubo_fallback_sun_when_no_lights(oracle):
    u = ubo_of(oracle, [])
    assert list(u.light_counts) == [1, 0, 0, 0]
    d = np.array(u.directional_light_direction[:3])
    assert np.allclose(d, np.array([-0.5, -1, -0.3]) / np.linalg.norm([-0.5, -1, -0.3]), atol=1e-6)
    assert list(u.directional_light_color) == pytest.approx([1.0, 0.98, 0.92, 5.0])
    assert list(u.ambient_color_intensity) == pytest.approx([0.03, 0.03, 0.03, 1.0])
    assert list(u.ai_blend_config) == [0, 0, 0, 0]


def test_ubo_point_lights_only_disable_the_sun(oracle):
    u = ubo_of(oracle, [{"type": "point", "position": (1, 2, 3), "range": -5.0, "intensity": -1.0}])
    assert list(u.light_counts) == [0, 1, 0, 0]
    assert list(u.point_lights[0].position_range) == [1, 2, 3, 0.0]  # range clamped to >= 0
    assert u.point_lights[0].color_intensity[3] == 0.0  # intensity clamped to >= 0


def test_ubo_first_directional_wins_and_eight_point_cap(oracle):
    lights = [{"type": "directional", "direction": (0, -1, 0), "intensity": 2.0},
              {"type": "directional", "direction": (1, 0, 0), "intensity": 7.0},
              {"type": "directional", "enabled": False}]
    lights += [{"type": "point", "position": (k, 0, 0)} for k in range(11)]
    u = ubo_of(oracle, lights)
    assert list(u.light_counts) == [1, 8, 0, 0]
    assert list(u.directional_light_direction[:3]) == [0, -1, 0] and u.directional_light_color[3] == 2.0
    assert [u.point_lights[k].position_range[0] for k in range(8)] == list(range(8))


def test_numpy_scene_packer_matches_oracle(oracle):
    lights = [{"type": "directional", "direction": (0.2, -1, 0.1), "intensity": 4.0},
              {"type": "point", "position": (1, 2, 3), "range": 7.0}]
    I = np.eye(4, dtype=np.float32)
    a = bytes(oracle.pack_ubo(I, I, (1, 2, 3), lights))
    b = bytes(scenes.pack_ubo(I, I, (1, 2, 3), lights))
    assert a == b
