"""Object-space varyings outside the single-draw solid instantiation (TriFrameParams::obj48): frames with
several draws, textures or the shadow pre-pass whose draws are affine, unskinned, conformal and keep the identity
texture transform. k_vertex then writes no varyings; the fragment stage gathers the geometry's own 48-B input records
at slot + vdelta[draw] and carries them through its draw's model and normal matrices. Parity bar as everywhere: depth
bit-exact, colour within 1 LSB of the oracle (which interpolates world-space varyings), in both shading builds.
tri_frame_stats.path says which path a frame took."""
import numpy as np
import pytest

import scene_cases as sc
from test_parity_gpu import assert_parity, flags  # noqa: F401 (the fixture)

pytestmark = pytest.mark.gpu


def frame_path(scene, flags=0):
    from trident_raster import raster, scenes

    with raster.TriRaster(scene.width, scene.height, flags=flags) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        st = r.frame_stats()
    return st["path"], st["triangles_clipped"]


def test_obj48_transformed_draws_clipped(oracle, flags):
    """Two textured draws with different models, near-plane clipped: per-draw matrices per pixel, and the
    clipper's polygon vertices interpolated from the object records."""
    from trident_raster import abi

    s = sc.near_clip_multi()
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    path, clipped = frame_path(s, flags)
    assert path & abi.TRI_PATH_OBJ48 and clipped > 0, (hex(path), clipped)


def test_obj48_identity_draws_with_shadow_clipped(oracle, flags):
    """C5's shape at test size: identity draws, textures, the shadow pre-pass (k_vertex's light-space positions from
    the position stream), clipping."""
    from trident_raster import abi

    s = sc.near_clip_multi(identity=True, shadow=True)
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    path, clipped = frame_path(s, flags)
    assert path & abi.TRI_PATH_OBJ48 and path & abi.TRI_PATH_SHADOW and clipped > 0, (hex(path), clipped)


def test_obj48_off_for_transformed_draws_with_shadow(oracle, flags):
    """The shadow instantiation carries no per-draw transform: such frames keep world-space varyings."""
    from trident_raster import abi

    s = sc.near_clip_multi(shadow=True)
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    path, _ = frame_path(s, flags)
    assert path & abi.TRI_PATH_SHADOW and not path & abi.TRI_PATH_OBJ48, hex(path)


def test_obj48_single_textured_draw_clipped(oracle, flags):
    """ONE textured draw, near-plane clipped: k_setup's single-draw instantiation on an obj48 frame (its clipper reads
    the input records, not the varyings k_vertex did not write)."""
    from trident_raster import abi

    s = sc.near_clip_single()
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    path, clipped = frame_path(s, flags)
    assert path & abi.TRI_PATH_OBJ48 and clipped > 0, (hex(path), clipped)


def test_obj48_single_draw_ai_blend_clipped(oracle, flags):
    """The same single clipped draw on a solid slot with the AI-frame blend (k_raster_ai, obj48)."""
    from trident_raster import abi, scenes

    s = sc.near_clip_grid()
    scenes.with_ai_blend(s, strength=0.35)
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    path, clipped = frame_path(s, flags)
    assert path & abi.TRI_PATH_OBJ48 and clipped > 0, (hex(path), clipped)


def test_obj48_c5_and_fallbacks(oracle):
    """C5 (4 textured identity draws + the pre-pass) takes obj48; a texture transform, skinning or a non-conformal
    model does not."""
    from trident_raster import abi, scenes

    s = scenes.scene_c5_textured(640, 360, 80, 64, shadow_size=256)
    s.skybox = None
    assert_parity(s, oracle, min_covered=100000)
    assert frame_path(s)[0] & abi.TRI_PATH_OBJ48
    t = sc.textured_grid()  # uv scale / offset / tiling: world-space varyings
    assert not frame_path(t)[0] & abi.TRI_PATH_OBJ48
    p = sc.shadow_scene(oracle)  # the ground quad's non-uniform scale
    assert not frame_path(p)[0] & abi.TRI_PATH_OBJ48


def test_idx_route_on_and_off(oracle, flags):
    """Several draws over concatenated meshes in draw order reach their vertex slots through the index buffer
    (TRI_PATH_IDX_ROUTE: no per-primitive prim_vs record); the same meshes drawn in the other order (index rows no
    longer follow the primitive numbers) keep the records. Both frames match the oracle, clipped primitives
    included."""
    from trident_raster import abi

    s = sc.near_clip_multi()
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    path, clipped = frame_path(s, flags)
    assert path & abi.TRI_PATH_IDX_ROUTE and clipped > 0, hex(path)
    s.draws = [s.draws[1], s.draws[0]]  # mesh 1 first: the route's one offset no longer fits
    s.name += "_swapped"
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    assert not frame_path(s, flags)[0] & abi.TRI_PATH_IDX_ROUTE
