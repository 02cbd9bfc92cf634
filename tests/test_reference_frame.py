"""Parity against the reference's OWN rendered pixels: the sky pass of a real Trident-Forge frame.

`Screenshots/Screenshot1.png` in the reference checkout is a Forge window over a skybox-only scene, rendered by
the reference's Vulkan path. Its two viewport images are cropped losslessly into `tests/golden/
reference_sky_{scene,game}.png` by `tests/golden/make_reference_sky.py` (crop rectangles and the Game panel's
FPS-label mask documented there).

Why the crop is reproducible without the camera pose: Skybox.vert:30-41 samples `mat3(View) * world`, a
view-space direction, so the sky image depends only on the projection (fov 60 degrees: EditorCamera.h:64,
RuntimeCamera.h:72; aspect = the panel size) and on the cubemap (Forge's Assets/Skyboxes PNG faces, found by
Renderer.cpp:3830-3927, committed under assets/Skyboxes). Skybox.frag:28-35 writes the LINEAR-filtered,
sRGB-decoded texel into the B8G8R8A8_UNORM target (Swapchain.cpp:161-172); ImGui displays it 1:1.

What this pins: perspectiveRH_ZO / the GL-style runtime perspective with the Y flip, the
cube-face selection, seamless LINEAR filtering, sRGB decode before filtering and the UNORM store — against real
Vulkan output. A one-pixel shift of the crop moves the comparison to >=26 LSB (scene) / 188 (game), so the bar
below is sharp. The mesh path is not pinned by this (the screenshots with meshes use FBX assets the snapshot
lacks).

Bar: max 2 LSB per channel, >= 99.99 % of the pixels within 1 LSB.
"""
import os

import numpy as np
import pytest

import scene_cases as sc

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
MAX_LSB = 2
WITHIN1 = 0.9999
GAME_LABEL_MASK = (slice(8, 36), slice(8, 161))  # the Game panel's "FPS: ..." text (make_reference_sky.py)


def reference_crop(name):
    from PIL import Image

    a = np.asarray(Image.open(os.path.join(GOLDEN, f"reference_sky_{name}.png")).convert("RGB"))
    mask = np.ones(a.shape[:2], bool)
    if name == "game":
        mask[GAME_LABEL_MASK] = False
    return a.astype(np.int16), mask


def editor_sky(w, h):
    from trident_raster import scenes

    return sc.skybox_only(w, h, 60.0, (0.0, 0.0, 0.0), scenes.reference_skybox())


def runtime_sky(w, h, rot=(0.0, 0.0, 0.0)):
    """The Game viewport with a ready runtime camera: RuntimeCamera's GL-style perspective (fov 60)."""
    import oracle_py
    from trident_raster import scenes

    s = sc.skybox_only(w, h, 60.0, (0.0, 0.0, 0.0), scenes.reference_skybox())
    view, proj = oracle_py.runtime_camera((0.0, 3.0, 8.0), rot, 60.0, (w, h), 0.1, 1000.0, ptype=0)
    s.ubo = oracle_py.pack_ubo(view, proj, (0.0, 3.0, 8.0))
    s.name = f"reference_sky_runtime_{w}x{h}"
    return s


def compare(bgra, name):
    ref, mask = reference_crop(name)
    assert bgra.shape[:2] == ref.shape[:2], (bgra.shape, ref.shape)
    rgb = bgra[..., [2, 1, 0]].astype(np.int16)
    d = np.abs(rgb - ref).max(-1)[mask]
    stats = {"max": int(d.max()), "within1": float((d <= 1).mean()), "exact": float((d == 0).mean()),
             "mean": float(d.mean())}
    assert stats["max"] <= MAX_LSB, stats
    assert stats["within1"] >= WITHIN1, stats
    return stats


def test_fixture_is_the_viewport_image():
    """The crops are exactly the viewport images (no panel border inside) and the bar is sharp: shifting the
    expected image by one pixel breaks it."""
    for name in ("scene", "game"):
        ref, mask = reference_crop(name)
        assert ref.shape == ((1078, 992, 3) if name == "scene" else (1078, 1064, 3))
        assert not np.all(ref[0] == 15) and not np.all(ref[:, 0] == 15)
        shifted = np.abs(ref[:, 1:] - ref[:, :-1]).max(-1)[mask[:, 1:]]
        assert shifted.max() > 2 * MAX_LSB


@pytest.mark.parametrize("name,w", [("scene", 992), ("game", 1064)])
def test_oracle_matches_reference_sky(oracle, name, w):
    col, dep, _ = oracle.render(editor_sky(w, 1078))
    assert np.all(dep == 0x3F800000)  # the sky writes no depth (Pipeline.cpp:727-880)
    compare(col, name)


def test_oracle_runtime_camera_matches_reference_game_sky(oracle):
    """The Game viewport through RuntimeCamera's projection (RuntimeCamera.cpp:177-195), with a rotated pose:
    the sky is view-locked, so the pose does not matter."""
    col, _, _ = oracle.render(runtime_sky(1064, 1078, rot=(-12.0, 33.0, 0.0)))
    compare(col, "game")


# ---- GPU: the HIP sky pass against the reference's pixels directly (no oracle in between) -------------
def render_gpu(scene, flags=0):
    from trident_raster import raster, scenes

    with raster.TriRaster(scene.width, scene.height, flags=flags) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        return r.readback()


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("name,w", [("scene", 992), ("game", 1064)])
def test_gpu_matches_reference_sky(name, w, exact):
    from trident_raster import abi

    col, dep = render_gpu(editor_sky(w, 1078), abi.TRI_FLAG_EXACT_SHADING if exact else 0)
    assert np.all(dep == 0x3F800000)
    compare(col, name)


@pytest.mark.gpu
def test_gpu_runtime_camera_matches_reference_game_sky():
    col, _ = render_gpu(runtime_sky(1064, 1078, rot=(-12.0, 33.0, 0.0)))
    compare(col, "game")


@pytest.mark.gpu
def test_gpu_shim_two_viewports_match_reference_frame():
    """The whole editor frame through the Trident::Renderer shim, as Forge drives it: Scene viewport (id 1,
    editor camera) and Game viewport (id 2, the ready runtime camera) at the screenshot's panel sizes, the
    cubemap discovered under Assets/Skyboxes by Init, no meshes."""
    from trident_raster import app, scenes

    a = app.TridentApp()
    try:
        assert a.set_assets_dir(scenes.ASSETS_DIR) == "PNG fallback"
        a.set_camera("editor", (0.0, 3.0, 8.0), (-8.0, 20.0, 0.0))
        a.set_camera("runtime", (4.0, 1.0, -3.0), (5.0, -70.0, 0.0))
        a.set_viewport(1, 992, 1078)
        a.set_viewport(2, 1064, 1078)
        a.draw_frame()
        a.draw_frame()
        for vid, name, w in ((1, "scene", 992), (2, "game", 1064)):
            rgba, _ = a.read_pixels(vid, w, 1078, depth=False)
            compare(rgba[..., [2, 1, 0, 3]], name)  # read_pixels returns RGBA; compare() takes BGRA
    finally:
        a.close()
