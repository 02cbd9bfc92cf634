"""JPEG textures (host/src/JpegDecoder.cpp): the reference loads every 2D texture through stb_image
(stbi_load(..., STBI_rgb_alpha) after stbi_set_flip_vertically_on_load(true), TextureLoader.cpp:290-304),
which decodes JPEG as well as PNG; stb is an un-vendored submodule, so its JPEG algorithm is restated.

Pinned against Pillow (libjpeg-turbo, an independent decoder) on seeded synthetic files: baseline and
progressive, 4:4:4 / 4:2:2 / 4:2:0 / greyscale, restart intervals, odd sizes. The two decoders implement
the same standard with different integer IDCT / colour-conversion rounding, so samples agree within 3
levels and on average within a fraction of one. stb's one deliberate deviation from libjpeg's upsampling
-- its 2x1 filter weights the second-to-last chroma sample 3:1 for the second-to-last output pair
(stbi__resample_row_h_2) -- is kept and excluded from the Pillow comparison at that column; bit-exact parity
with stb itself is unpinned (stb is absent here).
"""
import io

import numpy as np
import pytest

from test_png import app  # noqa: F401  (fixture)

TOL = 3


def synthetic(w, h, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    a = np.stack([128 + 100 * np.sin(xx / 7.0 + yy / 11.0), 128 + 90 * np.cos(xx / 5.0 - yy / 9.0),
                  (xx * 3 + yy * 5) % 256], -1)
    return np.clip(a + rng.normal(0, 12, a.shape), 0, 255).astype(np.uint8)


def encode(tmp_path, name, arr, **kw):
    from PIL import Image

    im = Image.fromarray(arr)
    p = str(tmp_path / name)
    im.save(p, "JPEG", **kw)
    return p


def pillow_rgba(path):
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGBA")).astype(np.int16)


def compare(app, path, skip_cols=()):  # noqa: F811
    want = pillow_rgba(path)
    got = app.load_image(path, flip=False).astype(np.int16)
    assert got.shape == want.shape
    d = np.abs(got - want)
    if skip_cols:
        d[:, list(skip_cols)] = 0
    assert int(d.max()) <= TOL, int(d.max())
    assert float(d[..., :3].mean()) < 0.6
    assert (got[..., 3] == 255).all()
    return got


@pytest.mark.parametrize("size", [(64, 48), (37, 29), (1, 1), (17, 3), (256, 130)])
@pytest.mark.parametrize("subsampling", [0, 2])  # 4:4:4, 4:2:0 (h2v2)
@pytest.mark.parametrize("progressive", [False, True])
@pytest.mark.parametrize("quality", [50, 95])
def test_colour_matches_pillow(app, tmp_path, size, subsampling, progressive, quality):  # noqa: F811
    w, h = size
    p = encode(tmp_path, "c.jpg", synthetic(w, h, w * h + quality), quality=quality, subsampling=subsampling,
               progressive=progressive)
    compare(app, p)


@pytest.mark.parametrize("size", [(64, 48), (37, 29), (17, 3), (2, 5)])
@pytest.mark.parametrize("progressive", [False, True])
def test_h2v1_matches_pillow_except_stbs_edge_pair(app, tmp_path, size, progressive):  # noqa: F811
    w, h = size
    p = encode(tmp_path, "c.jpg", synthetic(w, h, 7), quality=90, subsampling=1, progressive=progressive)
    cw = (w + 1) // 2
    compare(app, p, skip_cols=[2 * (cw - 1)] if cw > 1 and 2 * (cw - 1) < w else [])


@pytest.mark.parametrize("progressive", [False, True])
def test_greyscale(app, tmp_path, progressive):  # noqa: F811
    a = synthetic(45, 33, 3)[..., 0]
    p = encode(tmp_path, "g.jpg", a, quality=85, progressive=progressive)
    got = compare(app, p)
    assert (got[..., 0] == got[..., 1]).all() and (got[..., 1] == got[..., 2]).all()


@pytest.mark.parametrize("blocks", [1, 3, 7])
def test_restart_intervals(app, tmp_path, blocks):  # noqa: F811
    p = encode(tmp_path, "r.jpg", synthetic(90, 50, blocks), quality=80, restart_marker_blocks=blocks)
    assert b"\xff\xdd" in open(p, "rb").read()
    compare(app, p)


def test_texture_loader_flips_jpeg_rows(app, tmp_path):  # noqa: F811
    p = encode(tmp_path, "t.jpg", synthetic(40, 24, 9), quality=92)
    a = app.load_image(p, flip=False)
    assert np.array_equal(app.load_image(p, flip=True), a[::-1])  # stbi_set_flip_vertically_on_load(true)


def test_unsupported_and_malformed_fail_cleanly(app, tmp_path):  # noqa: F811
    from PIL import Image

    good = encode(tmp_path, "ok.jpg", synthetic(32, 32, 1), quality=80)
    data = open(good, "rb").read()
    cases = {
        "truncated.jpg": data[: len(data) // 3],
        "header_only.jpg": data[:20],
        "soi_only.jpg": b"\xff\xd8\xff\xd9",
        # an arithmetic-coded frame (SOF9) is rejected as stb rejects it
        "arith.jpg": data.replace(b"\xff\xc0", b"\xff\xc9", 1),
    }
    b = io.BytesIO()
    Image.fromarray(synthetic(16, 16, 2)).convert("CMYK").save(b, "JPEG")
    cases["cmyk.jpg"] = b.getvalue()
    for name, blob in cases.items():
        p = tmp_path / name
        p.write_bytes(blob)
        with pytest.raises(RuntimeError):
            app.load_image(str(p), flip=False)


def test_shim_resolves_a_jpeg_texture_slot(tmp_path):
    """ResolveTextureSlot on a .jpg path loads it (Renderer.cpp:3700-3745) instead of falling back to slot 0."""
    from trident_raster import app as appmod

    appmod.load_library()
    p = encode(tmp_path, "tex.jpg", synthetic(16, 16, 4), quality=90)
    a = appmod.TridentApp()
    a.set_camera("editor", (0, 0, 3))
    a.set_viewport(1, 64, 64)
    e = a.add_mesh_entity("quad")
    a.set_entity_texture(e, p)
    _, draws = a.frame_inputs(1)
    assert draws[0].pc.texture_slot == 1
    a.close()
