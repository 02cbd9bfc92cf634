"""PNG decoding (host/src/ImageDecoder.cpp) and the skybox discovery of Renderer::CreateSkyboxCubemap.

The reference decodes images with stb_image (an un-vendored submodule): stbi_load(..., STBI_rgb_alpha)
with flip-on-load for 2D textures (TextureLoader.cpp:290-304) and without it for cube faces (:773). The
decoder is pinned here against Pillow (an independent decoder) on the reference's own skybox faces and
on synthetic files covering every colour type, bit depth, tRNS form and Adam7 interlacing; where stb's
conversion differs from Pillow's (16-bit samples keep their high byte) the expectation is written out.
"""
import os
import struct
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKY = os.path.join(ROOT, "assets", "Skyboxes")
FACES = ["px", "nx", "py", "ny", "pz", "nz"]


@pytest.fixture(scope="module")
def app():
    from trident_raster import app as a

    a.load_library()
    return a


def pil_rgba(path):
    from PIL import Image

    return np.asarray(Image.open(path).convert("RGBA"))


@pytest.mark.parametrize("face", FACES)
def test_reference_faces_match_pillow(app, face):
    path = os.path.join(SKY, face + ".png")
    want = pil_rgba(path)
    assert want.shape == (512, 512, 4)
    assert np.array_equal(app.load_image(path, flip=False), want)  # cube faces: no flip (:773)
    assert np.array_equal(app.load_image(path, flip=True), want[::-1])  # 2D textures: flipped (:290)


def save(tmp_path, name, im, **kw):
    p = str(tmp_path / name)
    im.save(p, **kw)
    return p


def test_colour_types_and_depths(app, tmp_path):
    from PIL import Image

    rng = np.random.default_rng(1)
    rgba = rng.integers(0, 256, (13, 17, 4), dtype=np.uint8)
    cases = {
        "rgba": Image.fromarray(rgba, "RGBA"),
        "rgb": Image.fromarray(rgba[..., :3].copy(), "RGB"),
        "l": Image.fromarray(rgba[..., 0].copy(), "L"),
        "la": Image.fromarray(rgba[..., :2].copy(), "LA"),
        "bit1": Image.fromarray(rgba[..., 0] > 127).convert("1"),
        "pal": Image.fromarray(rgba[..., :3].copy(), "RGB").convert("P", palette=Image.ADAPTIVE, colors=200),
    }
    for name, im in cases.items():
        p = save(tmp_path, name + ".png", im)
        assert np.array_equal(app.load_image(p, flip=False), pil_rgba(p)), name
    p = save(tmp_path, "pal4.png", cases["pal"].quantize(12), bits=4)
    assert np.array_equal(app.load_image(p, flip=False), pil_rgba(p))


def test_transparency_keys(app, tmp_path):
    """tRNS: palette alpha table, grey and RGB colour keys (alpha 0 where equal, 255 elsewhere)."""
    from PIL import Image

    rng = np.random.default_rng(2)
    g = rng.integers(0, 4, (9, 11), dtype=np.uint8) * 60
    p = save(tmp_path, "lkey.png", Image.fromarray(g, "L"), transparency=120)
    got = app.load_image(p, flip=False)
    assert np.array_equal(got[..., 3], np.where(g == 120, 0, 255))
    assert np.array_equal(got, pil_rgba(p))
    rgb = rng.integers(0, 2, (9, 11, 3), dtype=np.uint8) * 200
    p = save(tmp_path, "rgbkey.png", Image.fromarray(rgb, "RGB"), transparency=(200, 0, 200))
    got = app.load_image(p, flip=False)
    assert np.array_equal(got[..., 3], np.where((rgb == (200, 0, 200)).all(-1), 0, 255))
    assert np.array_equal(got, pil_rgba(p))
    pal = Image.fromarray(rgb, "RGB").convert("P", palette=Image.ADAPTIVE, colors=8)
    p = save(tmp_path, "palkey.png", pal, transparency=bytes([0, 128, 255, 7]))
    assert np.array_equal(app.load_image(p, flip=False), pil_rgba(p))


def chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def encode_png(pixels, ctype, depth, interlace=False, filt=lambda y: y % 5):
    """A minimal PNG writer (any filter per row, optional Adam7) for cases Pillow cannot write.
    pixels: [h, w, channels] of integers at `depth` bits."""
    h, w, ch = pixels.shape

    def pack_rows(img):
        rows = []
        for r in img:
            if depth == 16:
                raw = b"".join(struct.pack(">H", int(v)) for v in r.reshape(-1))
            elif depth == 8:
                raw = bytes(int(v) for v in r.reshape(-1))
            else:
                bits = "".join(format(int(v), f"0{depth}b") for v in r.reshape(-1))
                bits += "0" * (-len(bits) % 8)
                raw = bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))
            rows.append(raw)
        return rows

    def filtered(rows):
        out = b""
        bpp = max(1, ch * depth // 8)
        prev = bytes(len(rows[0])) if rows else b""
        for y, raw in enumerate(rows):
            f = filt(y)
            line = bytearray()
            for i, x in enumerate(raw):
                a = raw[i - bpp] if i >= bpp else 0
                b = prev[i]
                c = prev[i - bpp] if i >= bpp else 0
                pred = [0, a, b, (a + b) >> 1, None][f]
                if f == 4:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                line.append((x - pred) & 255)
            out += bytes([f]) + bytes(line)
            prev = raw
        return out

    if interlace:
        data = b""
        for x0, y0, dx, dy in [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]:
            sub = pixels[y0::dy, x0::dx]
            if sub.size:
                data += filtered(pack_rows(sub))
    else:
        data = filtered(pack_rows(pixels))
    hdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0)
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", hdr) + chunk(b"IDAT", zlib.compress(data)) + chunk(b"IEND", b"")


@pytest.mark.parametrize("interlace", [False, True])
def test_adam7_filters_and_16_bit(app, tmp_path, interlace):
    rng = np.random.default_rng(3)
    px = rng.integers(0, 256, (19, 23, 4))
    p = tmp_path / "a.png"
    p.write_bytes(encode_png(px, 6, 8, interlace))
    assert np.array_equal(app.load_image(str(p), flip=False), px.astype(np.uint8))
    # 16-bit RGB: stb keeps the high byte of each sample (stbi__convert_16_to_8); alpha 255
    px16 = rng.integers(0, 65536, (7, 9, 3))
    p.write_bytes(encode_png(px16, 2, 16, interlace))
    want = np.concatenate([(px16 >> 8), np.full((7, 9, 1), 255)], -1).astype(np.uint8)
    assert np.array_equal(app.load_image(str(p), flip=False), want)
    # 2-bit grey: scaled by 0x55 (stbi__depth_scale_table)
    g2 = rng.integers(0, 4, (6, 13, 1))
    p.write_bytes(encode_png(g2, 0, 2, interlace))
    v = (g2[..., 0] * 0x55).astype(np.uint8)
    assert np.array_equal(app.load_image(str(p), flip=False), np.stack([v, v, v, np.full_like(v, 255)], -1))


def test_malformed_inputs_fail_cleanly(app, tmp_path):
    from trident_raster.raster import TriError

    good = (tmp_path / "g.png")
    good.write_bytes(encode_png(np.zeros((4, 4, 4), int), 6, 8))
    data = good.read_bytes()
    for name, blob in (("trunc", data[:40]), ("sig", b"\x88" + data[1:]), ("empty", b"")):
        p = tmp_path / f"{name}.png"
        p.write_bytes(blob)
        with pytest.raises((TriError, RuntimeError, OSError)):
            app.load_image(str(p))


def test_reference_discovery(app):
    """Renderer.cpp:3840-3915: no KTX, no Default/ directory -> the loose px/nx/... PNG faces."""
    faces, src = app.load_default_skybox(os.path.join(ROOT, "assets"))
    assert src == "PNG fallback"
    for k, f in enumerate(FACES):
        assert np.array_equal(faces[k], pil_rgba(os.path.join(SKY, f + ".png")))


def test_discovery_order_and_fallbacks(app, tmp_path):
    import shutil

    faces = {f: np.full((4, 4, 4), 10 * k + 5, np.uint8) for k, f in enumerate(FACES)}
    from PIL import Image

    root = tmp_path / "Assets" / "Skyboxes"
    root.mkdir(parents=True)
    long_names = {"px": "sky_posx", "nx": "sky_negx", "py": "sky_posy", "ny": "sky_negy", "pz": "sky_posz", "nz": "sky_negz"}
    for f, img in faces.items():
        Image.fromarray(img, "RGBA").save(str(root / (long_names[f] + ".png")))
    got, src = app.load_default_skybox(str(tmp_path / "Assets"))
    assert src == "PNG fallback" and np.array_equal(got, np.stack([faces[f] for f in FACES]))
    os.remove(str(root / "sky_negz.png"))  # incomplete -> nothing (the renderer then uses the solid colour)
    got, src = app.load_default_skybox(str(tmp_path / "Assets"))
    assert got is None and src == ""
    d = root / "Default"  # a Default/ directory takes precedence (LoadFromDirectory)
    d.mkdir()
    for f, img in faces.items():
        Image.fromarray(255 - img, "RGBA").save(str(d / (f + ".png")))
    got, src = app.load_default_skybox(str(tmp_path / "Assets"))
    assert src == "Default directory" and np.array_equal(got, 255 - np.stack([faces[f] for f in FACES]))
    shutil.rmtree(str(d))
    (root / "DefaultSkybox.ktx").write_bytes(b"\xabKTX 11\xbb")  # KTX first; not restated -> invalid
    got, src = app.load_default_skybox(str(tmp_path / "Assets"))
    assert got is None and src == "DefaultSkybox.ktx"


def test_shim_init_discovers_reference_skybox(app):
    a = app.TridentApp()
    assert a.set_assets_dir(os.path.join(ROOT, "assets")) == "PNG fallback"
    assert a.set_assets_dir(os.path.join(ROOT, "no-such-dir")) == "solid 0x808080"
    a.close()
