"""Committed fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py): full scene inputs +
expected B8G8R8A8 / D32 outputs. CPU: the oracle reproduces them bit-for-bit. GPU: the HIP path
matches them (depth bit-exact, colour within 1 LSB), independently of a live oracle."""
import glob
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(glob.glob(os.path.join(HERE, "*.npz")))


def load(path):
    import sys

    sys.path.insert(0, HERE)
    from make_golden import unpack

    z = np.load(path, allow_pickle=False)
    return unpack(z), z["out_bgra"], z["out_depth"], z["stats"]


def test_fixtures_exist():
    assert len(FIXTURES) >= 8


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_oracle_reproduces_golden(oracle, path):
    scene, bgra, depth, stats = load(path)
    col, dep, st = oracle.render(scene)
    assert np.array_equal(dep, depth)
    assert np.array_equal(col, bgra)
    assert [st["triangles_in"], st["triangles_setup"], st["triangles_clipped"]] == list(stats)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_hip_matches_golden(path):
    from trident_raster import raster, scenes

    scene, bgra, depth, _ = load(path)
    with raster.TriRaster(scene.width, scene.height) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        col, dep = r.readback()
    assert np.array_equal(dep, depth)
    assert int(np.abs(col.astype(np.int16) - bgra.astype(np.int16)).max()) <= 1
