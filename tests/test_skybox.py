"""Skybox pass: Skybox.cpp:13-79, Skybox.vert:30-41, Skybox.frag:28-35, pipeline
Pipeline.cpp:727-880 (cull FRONT, depth LEQUAL, no depth write), recorded before the meshes
(Renderer.cpp:5076-5082); cubemap from CreateSkyboxCubemap (Renderer.cpp:3818-4110).

CPU: known answers for the oracle's restatement. GPU: the HIP pass against the oracle (depth bit-exact,
colour within 1 LSB). Parity against the reference renderer itself is unpinned (no Vulkan here).
"""
import numpy as np
import pytest

import scene_cases as sc

FACE_COLOURS = np.array([[200, 30, 30], [30, 200, 30], [30, 30, 200], [200, 200, 30], [30, 200, 200],
                         [200, 30, 200]], np.uint8)


def uniform_faces(n=8):
    f = np.zeros((6, n, n, 4), np.uint8)
    f[..., :3] = FACE_COLOURS[:, None, None, :]
    f[..., 3] = 255
    return f


def srgb_to_unorm(c):
    v = c / 255.0
    lin = np.where(v <= 0.04045, v / 12.92, ((v + 0.055) / 1.055) ** 2.4)
    return np.floor(np.float32(lin) * np.float32(255.0) + np.float32(0.5)).astype(np.int64)


def bgra(col, y, x):
    b, g, r, a = (int(v) for v in col[y, x])
    return r, g, b, a


def test_solid_fallback_skybox_is_linear_grey(oracle):
    """CreateSolidColor(0x808080) (Renderer.cpp:3925-3926): sRGB 128 decoded to 0.2159 and written
    to the UNORM target without gamma -> 55 per channel; alpha 1 (Skybox.frag: vec4(sky, 1.0))."""
    s = sc.skybox_only(64, 48, fov=60.0, faces=sc.SOLID_0x808080)
    col, dep, _ = oracle.render(s)
    assert np.all(col[..., 0] == 55) and np.all(col[..., 1] == 55) and np.all(col[..., 2] == 55)
    assert np.all(col[..., 3] == 255)
    assert np.all(dep == 0x3F800000)  # no depth writes


def test_face_selection_and_orientation(oracle):
    """Vulkan major-axis face selection on the view-space direction: the view looks down -Z, so the
    centre is face -Z; with a 120-degree field of view the left/right edges reach -X/+X and the top
    row (+Y after the projection's Y flip) reaches +Y."""
    w, h = 200, 150
    s = sc.skybox_only(w, h, fov=120.0, faces=uniform_faces())
    col, _, _ = oracle.render(s)
    expect = srgb_to_unorm(FACE_COLOURS.astype(np.float64))
    assert bgra(col, h // 2, w // 2)[:3] == tuple(expect[5])  # -Z
    assert bgra(col, h // 2, 0)[:3] == tuple(expect[1])       # -X
    assert bgra(col, h // 2, w - 1)[:3] == tuple(expect[0])   # +X
    assert bgra(col, 0, w // 2)[:3] == tuple(expect[2])       # +Y
    assert bgra(col, h - 1, w // 2)[:3] == tuple(expect[3])   # -Y


def test_sky_is_locked_to_the_view(oracle):
    """Skybox.vert samples mat3(View) * world — a view-space direction — so camera rotation does not
    move the sky (reference behaviour, kept)."""
    a, _, _ = oracle.render(sc.skybox_only(96, 64, fov=90.0))
    b, _, _ = oracle.render(sc.skybox_only(96, 64, fov=90.0, rot=(15.0, 40.0, 0.0)))
    assert np.array_equal(a, b)


def test_meshes_cover_the_sky(oracle):
    s = sc.c1_cube_skybox(1, 160, 120)
    col, dep, _ = oracle.render(s)
    covered = dep != 0x3F800000
    assert covered.sum() > 100 and (~covered).sum() > 100
    s2 = sc.c1_cube_skybox(1, 160, 120)
    s2.skybox = None
    col2, dep2, _ = oracle.render(s2)
    assert np.array_equal(dep, dep2)  # the sky never writes depth
    assert np.array_equal(col[covered], col2[covered])
    assert not np.array_equal(col[~covered], col2[~covered])


# ---- GPU ----------------------------------------------------------------------------------------
def render_gpu(scene, band=None, flags=0):
    from trident_raster import raster, scenes

    with raster.TriRaster(scene.width, scene.height, band=band, flags=flags) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        return r.readback()


def assert_sky_parity(scene, oracle, band=None, flags=0):
    gc, gd = render_gpu(scene, band, flags)
    oc, od, _ = oracle.render(scene, band=band)
    assert np.array_equal(gd, od)
    diff = np.abs(gc.astype(np.int16) - oc.astype(np.int16))
    assert int(diff.max(initial=0)) <= 1, int(diff.max())
    return int((diff > 0).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("fov", [60.0, 100.0, 150.0])
def test_gpu_skybox_only(oracle, fov):
    assert_sky_parity(sc.skybox_only(320, 240, fov=fov), oracle)


@pytest.mark.gpu
def test_gpu_skybox_solid_and_uniform(oracle):
    assert_sky_parity(sc.skybox_only(128, 96, fov=60.0, faces=sc.SOLID_0x808080), oracle)
    assert_sky_parity(sc.skybox_only(200, 150, fov=120.0, faces=uniform_faces()), oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [False, True])
def test_gpu_cube_over_skybox(oracle, exact):
    from trident_raster import abi

    flags = abi.TRI_FLAG_EXACT_SHADING if exact else 0
    assert_sky_parity(sc.c1_cube_skybox(1), oracle, flags=flags)


@pytest.mark.gpu
def test_gpu_skybox_bands(oracle):
    s = sc.skybox_only(256, 192, fov=110.0)
    for band in [(0, 64), (64, 128), (128, 192)]:
        assert_sky_parity(s, oracle, band=band)


def skybox_runtime_camera(ptype, w=240, h=160, ortho=12.0):
    """RuntimeCamera projections (RuntimeCamera.cpp:177-195): GL-style perspective (ptype 0) or
    glm::ortho (ptype 1). Orthographic rays do not start at the cube's centre, so the kernel takes
    the general ray/cube path there; some rays miss the 20-unit cube and keep the clear colour."""
    import oracle_py

    s = sc.skybox_only(w, h, fov=70.0)
    view, proj = oracle_py.runtime_camera((0.0, 3.0, 8.0), (10.0, 25.0, 0.0), 70.0, (w, h), 0.1, 1000.0,
                                          ortho=ortho, ptype=ptype)
    s.ubo = oracle_py.pack_ubo(view, proj, (0.0, 3.0, 8.0))
    s.name = f"skybox_runtime_p{ptype}"
    return s


def test_orthographic_sky_has_uncovered_pixels(oracle):
    s = skybox_runtime_camera(1, ortho=30.0)
    col, _, _ = oracle.render(s)
    clear = np.array([1, 1, 1, 255], np.uint8)  # unorm8(0.005) = 1
    missed = np.all(col == clear, axis=-1)
    assert missed.any() and (~missed).any()


@pytest.mark.gpu
@pytest.mark.parametrize("ptype,ortho", [(0, 12.0), (1, 12.0), (1, 30.0)])
def test_gpu_skybox_runtime_camera(oracle, ptype, ortho):
    assert_sky_parity(skybox_runtime_camera(ptype, ortho=ortho), oracle)


# ---- the reference's own cubemap (Trident-Forge/Assets/Skyboxes, "PNG fallback") ---------------------
@pytest.mark.gpu
@pytest.mark.parametrize("exact", [False, True])
def test_gpu_reference_skybox_c1(oracle, exact):
    """C1 at full size over the cubemap a default Forge frame shows (512^2 PNG faces found by the
    discovery of Renderer.cpp:3840-3915 and decoded without flip, TextureLoader.cpp:773)."""
    from trident_raster import abi, scenes

    s = scenes.scene_c1_cube(1, 640, 480)
    assert s.skybox.shape == (6, 512, 512, 4)
    assert_sky_parity(s, oracle, flags=abi.TRI_FLAG_EXACT_SHADING if exact else 0)


@pytest.mark.gpu
def test_gpu_reference_skybox_c2(oracle):
    """C2 at full size (1920x1080, 50k triangles, ~60 % of the pixels are sky)."""
    s = sc.sphere_c2(oracle=oracle)
    assert s.skybox.shape == (6, 512, 512, 4)
    assert_sky_parity(s, oracle)


@pytest.mark.gpu
def test_gpu_shim_renders_reference_skybox(oracle):
    """The shim's Init-time discovery under assets/ (Renderer::SetAssetsDirectory) feeds the same cubemap."""
    import os

    from trident_raster import app, scenes

    a = app.TridentApp()
    assert a.set_assets_dir(scenes.ASSETS_DIR) == "PNG fallback"
    a.set_camera("editor", (0.0, 3.0, 8.0), (-10.0, 25.0, 0.0))
    a.set_viewport(1, 320, 240)
    a.add_mesh_entity("sphere", position=(0.0, 3.0, 4.0))
    a.draw_frame()
    a.draw_frame()
    rgba, depth = a.read_pixels(1, 320, 240)
    ubo, draws = a.frame_inputs(1)
    vb, ib, ranges = a.geometry()
    s = scenes.Scene("shim_sky", 320, 240, vb, ib, ranges, draws, ubo,
                     materials=[(m[0], m[1]) for m in a.materials()], skybox=scenes.reference_skybox())
    oc, od, _ = oracle.render(s)
    assert np.array_equal(depth.view(np.uint32), od)
    assert int(np.abs(rgba.astype(np.int16) - oc[..., [2, 1, 0, 3]].astype(np.int16)).max()) <= 1
    assert os.path.isdir(scenes.ASSETS_DIR)
    a.close()
