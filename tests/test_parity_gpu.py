"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Bar: depth is bit-exact (D32 bits compared as uint32); colour (B8G8R8A8_UNORM) is
within 1 LSB per channel. Shading uses the same IEEE float operation order on both sides except the
transcendental library calls (powf), hence the 1-LSB colour tolerance.
"""
import numpy as np
import pytest

import scene_cases as sc

pytestmark = pytest.mark.gpu

COLOR_TOL = 1  # LSB per channel


@pytest.fixture(params=["fast", "exact"])
def flags(request):
    """fast: hardware rcp/rsq/exp/log shading (default); exact: IEEE div/sqrt/powf (TRI_FLAG_EXACT_SHADING)."""
    from trident_raster import abi

    return abi.TRI_FLAG_EXACT_SHADING if request.param == "exact" else 0


def render_gpu(scene, band=None, flags=0):
    from trident_raster import raster, scenes

    with raster.TriRaster(scene.width, scene.height, band=band, flags=flags) as r:
        scenes.load_scene(r, scene)
        r.render_frame()
        col, dep = r.readback()
        stats = r.frame_stats()
    return col, dep, stats


def assert_parity(scene, oracle, band=None, min_covered=1, flags=0):
    gc, gd, gs = render_gpu(scene, band, flags)
    oc, od, os_ = oracle.render(scene, band=band)
    assert gd.shape == od.shape and gc.shape == oc.shape
    depth_mismatch = int((gd != od).sum())
    assert depth_mismatch == 0, f"{scene.name}: {depth_mismatch} depth mismatches"
    diff = np.abs(gc.astype(np.int16) - oc.astype(np.int16))
    assert int(diff.max(initial=0)) <= COLOR_TOL, f"{scene.name}: colour diff {diff.max()} (> {COLOR_TOL})"
    covered = int((od != 0x3F800000).sum())
    assert covered >= min_covered, f"{scene.name}: only {covered} covered pixels"
    assert gs["triangles_setup"] == os_["triangles_setup"], (gs, os_)
    return covered, int((diff > 0).sum())


def test_c1_spinning_cube(oracle, flags):
    for frame in range(6):
        assert_parity(sc.c1_cube(frame), oracle, min_covered=1000, flags=flags)


def test_primitives(oracle, flags):
    assert_parity(sc.primitives_row(oracle), oracle, min_covered=2000, flags=flags)


def test_c5_four_textured_draws(oracle, flags):
    """BASELINE C5's sampler stress within the reference's model: 4 draws, 4 sRGB texture slots
    (bilinear, REPEAT), reduced size so the oracle finishes in seconds."""
    from trident_raster import scenes

    s = scenes.scene_c5_textured(640, 360, 80, 64)
    s.skybox = None
    assert_parity(s, oracle, min_covered=100000, flags=flags)


@pytest.mark.parametrize("one_draw", [True, False])
def test_large_triangles_per_wave_binning(oracle, one_draw):
    """Triangles spanning more bins than k_setup's workgroup grid: the per-wave reservation fallback."""
    assert_parity(sc.large_quads(one_draw=one_draw), oracle, min_covered=1920 * 1080 // 2)


def test_c2_sphere_1080p(oracle, flags):
    assert_parity(sc.sphere_c2(oracle=oracle), oracle, min_covered=300000, flags=flags)


def test_c3_grid_720p(oracle, flags):
    assert_parity(sc.grid_c3(1280, 720, 200), oracle, min_covered=1280 * 720 // 2, flags=flags)


def test_c3_trs_draw_720p(oracle, flags):
    """The C3 grid (all 999,698 triangles) under bench.py's c3trs draw: translate + 20 deg yaw + uniform 0.95 scale
    (ComposeTransform, Renderer.cpp:417-427). The fragment stage takes the general object-space path: the
    interpolated position and normal carried through the model and normal matrices per pixel."""
    from trident_raster import abi, raster, scenes

    s = scenes.scene_c3_trs(1280, 720, 708)
    assert_parity(s, oracle, min_covered=1280 * 720 // 2, flags=flags)
    with raster.TriRaster(s.width, s.height, flags=flags) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        path = r.frame_stats()["path"]
    want = abi.TRI_PATH_ONE_DRAW | abi.TRI_PATH_VARY_OBJ | abi.TRI_PATH_OBJ_XFORM
    assert path & want == want, hex(path)


def test_c3_full_4k_1m_triangles(oracle, flags):
    from trident_raster import scenes

    assert_parity(scenes.scene_c3_grid(), oracle, min_covered=3840 * 2160 // 2, flags=flags)


@pytest.mark.parametrize("seed", [11, 12])
def test_pixel_aligned_span_walk(oracle, flags, seed):
    """Edges through pixel centres (exact-integer row crossings), horizontal/vertical edges, slivers and
    triangles either side of the 64-px 32-bit set-up limit: the span walk's boundary cases, depth bit-exact
    against the oracle's per-pixel LEQUAL raster."""
    assert_parity(sc.pixel_aligned_triangles(seed=seed), oracle, min_covered=100000, flags=flags)


def test_textured_srgb_bilinear_repeat(oracle, flags):
    assert_parity(sc.textured_grid(), oracle, min_covered=10000, flags=flags)


def test_near_plane_clipping(oracle, flags):
    from trident_raster import raster, scenes

    s = sc.near_clip_grid()
    assert_parity(s, oracle, min_covered=10000, flags=flags)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        assert r.frame_stats()["triangles_clipped"] > 0


@pytest.mark.parametrize("case", ["scaled", "offset", "nonuniform", "unnormalised"])
def test_object_space_varyings(oracle, flags, case):
    """Single-draw solid frames keep their varyings in object space (TriFrameParams::vary_obj) when the draw
    is affine with a conformal normal matrix over unit normals: the near-clip ground plane (clipped polygons)
    under a uniformly scaled, turned model, and with its vertex records offset in the buffer (base vertex and
    minimum index). A non-uniform scale and non-unit normals take the world-space varyings instead. Every
    case stays within the 1-LSB bar with depth bit-exact."""
    from trident_raster import abi, scenes

    s = sc.near_clip_grid()
    if case == "scaled":
        s.draws = [abi.make_draw(0, scenes.compose_transform((0.3, 0.0, -5.0), (-90.0, 20.0, 0.0), (1.7, 1.7, 1.7)),
                                 material_index=0)]
    elif case == "nonuniform":
        s.draws = [abi.make_draw(0, scenes.compose_transform((0.0, 0.0, -5.0), (-90.0, 0.0, 0.0), (1.0, 2.0, 0.5)),
                                 material_index=0)]
    elif case == "unnormalised":
        v = s.vertices.copy()
        v["normal"] *= np.random.default_rng(5).uniform(0.5, 1.5, size=(v.shape[0], 1)).astype(np.float32)
        s.vertices = v
    else:  # 1000 records ahead of the mesh, 7 of them below its smallest index
        pad = np.zeros(1000 + 7, s.vertices.dtype)
        pad["position"] = 1e30  # never referenced (finite, with unit normals: the records stay eligible)
        pad["normal"] = (0.0, 0.0, 1.0)
        s.vertices = np.concatenate([pad[:1000], pad[1000:], s.vertices])
        s.indices = s.indices + np.uint32(7)
        s.meshes = np.array([(0, s.indices.size, 1000, 0)], abi.MESH_RANGE_DTYPE)
    assert_parity(s, oracle, min_covered=10000, flags=flags)


def test_depth_ties_and_far_clip(oracle, flags):
    assert_parity(sc.depth_ties(), oracle, min_covered=1000, flags=flags)


def test_skinning(oracle, flags):
    assert_parity(sc.skinned_quad(oracle), oracle, min_covered=1000, flags=flags)


def test_invalid_inputs_skipped(oracle, flags):
    assert_parity(sc.invalid_inputs(oracle), oracle, min_covered=100, flags=flags)


def test_empty_scene_clear_colour(oracle):
    col, dep, _ = render_gpu(sc.empty_scene())
    assert (dep == 0x3F800000).all()
    expect = np.array([int(0.3 * 255 + 0.5), int(0.2 * 255 + 0.5), int(0.1 * 255 + 0.5), 255], np.uint8)
    assert (col == expect).all()


@pytest.mark.parametrize("nbands", [2, 3, 8])
def test_row_bands_assemble_to_full_frame(nbands):
    """Multi-GPU screen partition: bands rendered independently == the full frame, bit for bit."""
    s = sc.grid_c3(640, 360, 80)
    full_c, full_d, _ = render_gpu(s)
    cuts = np.linspace(0, s.height, nbands + 1).astype(int)
    parts = [render_gpu(s, band=(int(a), int(b))) for a, b in zip(cuts[:-1], cuts[1:])]
    assert np.array_equal(np.concatenate([p[0] for p in parts]), full_c)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), full_d)


@pytest.mark.parametrize("case", ["near_clip", "primitives", "textured"])
def test_row_bands_clip_draws_textures(oracle, case):
    """Row bands with clipped primitives, several draws and textured draws assemble to the full
    frame bit for bit, and each band matches the oracle's band (set-up counts included)."""
    s = {"near_clip": lambda: sc.near_clip_grid(), "primitives": lambda: sc.primitives_row(oracle),
         "textured": lambda: sc.textured_grid()}[case]()
    full_c, full_d, _ = render_gpu(s)
    cuts = np.linspace(0, s.height, 5).astype(int)
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        parts.append(render_gpu(s, band=(int(a), int(b))))
        assert_parity(s, oracle, band=(int(a), int(b)), min_covered=0)
    assert np.array_equal(np.concatenate([p[0] for p in parts]), full_c)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), full_d)


def test_repeat_render_is_deterministic():
    from trident_raster import raster, scenes

    s = sc.grid_c3(960, 540, 150)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        outs = []
        for _ in range(3):
            r.render_frame()
            outs.append(r.readback())
    for c, d in outs[1:]:
        assert np.array_equal(c, outs[0][0]) and np.array_equal(d, outs[0][1])


def test_texture_upload_switches_specialised_raster(oracle, flags):
    """One context, one draw: while its texture slot is empty (it aliases the 1x1 white default) the frame
    takes the single-draw solid instantiation (texel and tint as kernel arguments); uploading the texture
    must switch it to the sampling path on the next frame, and clearing the tint back to the default
    slot must switch it back (the shade record a frame uses is refreshed with the slot)."""
    import copy

    from trident_raster import raster, scenes

    textured = sc.textured_grid()
    solid = copy.copy(textured)
    solid.textures = []  # slot 3 empty: the draw samples the default white 1x1 slot
    with raster.TriRaster(textured.width, textured.height, flags=flags) as r:
        scenes.load_scene(r, solid)
        frames = []
        for scene, upload in ((solid, None), (textured, textured.textures[0]), (solid, None)):
            if upload is not None:
                r.upload_texture(*upload)
            elif scene is solid and frames:  # back to the 1x1 default: a 1x1 white texel in slot 3
                r.upload_texture(3, np.full((1, 1, 4), 255, np.uint8))
            r.render_frame()
            frames.append((scene, *r.readback()))
    for scene, col, dep in frames:
        oc, od, _ = oracle.render(scene)
        assert np.array_equal(dep, od), scene.name
        assert int(np.abs(col.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL, scene.name


def test_bin_overflow_grows_and_recovers():
    """A frame that overflows the bin list reports TRI_E_OVERFLOW, grows, and re-renders correctly."""
    from trident_raster import abi, raster, scenes

    s = sc.grid_c3(1280, 720, 300)
    with raster.TriRaster(s.width, s.height) as r:
        scenes.load_scene(r, s)
        r.render_frame()
        ref = r.readback()
    # many overlapping large triangles: far more bin entries than the initial capacity heuristic
    v, idx = scenes.cube_mesh()
    draws = [abi.make_draw(0, scenes.compose_transform((0, 0, -3.0 - 0.01 * k), (10.0 * k, 7.0 * k, 0), (4, 4, 4)))
             for k in range(400)]
    s2 = scenes.Scene("overflow", 1280, 720, v, idx, np.array([(0, idx.size, 0, 0)], abi.MESH_RANGE_DTYPE), draws,
                      s.ubo)
    with raster.TriRaster(s2.width, s2.height) as r:
        scenes.load_scene(r, s2)
        r.render()
        with pytest.raises(raster.TriError) as ei:
            r.synchronize()
        assert ei.value.code == abi.TRI_E_OVERFLOW
        r.render_frame()  # grown buffers: succeeds
    assert ref[0].shape == (720, 1280, 4)


@pytest.mark.parametrize("case", ["grid_turned", "primitives", "invalid", "skinned", "near_clip", "dense",
                                  "near_far_planes"])
def test_cluster_cull_is_exact(oracle, case):
    """TRI_FLAG_CLUSTER_CULL on a whole frame (row bands always cull): frames bit-identical to the
    unculled path and to the oracle, with geometry partly off screen, several draws, invalid vertices,
    skinned draws (never culled), clipped primitives, and clusters cut by both the near and the far plane
    (the cull's depth margin, raster_kernels.hip cluster_visible)."""
    from trident_raster import abi, scenes

    if case == "near_far_planes":  # the displaced grid spans z in [-5.9, -4.1]: both planes cut its clusters
        s = sc.grid_c3(640, 360, 120)
        view, proj = scenes.editor_camera((0.0, 0.0, 0.0), (0, 0, 0), 60.0, (640, 360), 4.6, 5.3)
        s.ubo = scenes.pack_ubo(view, proj, (0.0, 0.0, 0.0), [{"type": "directional"}])
    elif case == "grid_turned":
        s = sc.grid_c3(640, 360, 120)
        view, proj = scenes.editor_camera((1.5, 0.5, 0.0), (8.0, 35.0, 0.0), 60.0, (640, 360))
        s.ubo = scenes.pack_ubo(view, proj, (1.5, 0.5, 0.0), [{"type": "directional"}])
    elif case == "dense":  # 47 clusters over 24 vertex slots: every cluster flag still gets a k_vertex lane
        s = scenes.scene_c1_cube(1, 320, 240)
        s.indices = np.tile(s.indices, 2000)
        s.meshes = s.meshes.copy()
        s.meshes[0]["index_count"] = s.indices.size
    else:
        s = {"primitives": lambda: sc.primitives_row(oracle), "invalid": lambda: sc.invalid_inputs(oracle),
             "skinned": lambda: sc.skinned_quad(oracle), "near_clip": lambda: sc.near_clip_grid()}[case]()
    plain_c, plain_d, plain_s = render_gpu(s)
    cull_c, cull_d, cull_s = render_gpu(s, flags=abi.TRI_FLAG_CLUSTER_CULL)
    assert np.array_equal(cull_c, plain_c) and np.array_equal(cull_d, plain_d)
    assert cull_s["triangles_setup"] == plain_s["triangles_setup"]
    assert_parity(s, oracle, flags=abi.TRI_FLAG_CLUSTER_CULL)
    if case in ("dense", "near_far_planes"):  # and in row bands (which always cull), assembled
        cuts = np.linspace(0, s.height, 5).astype(int)
        parts = [render_gpu(s, band=(int(a), int(b))) for a, b in zip(cuts[:-1], cuts[1:])]
        assert np.array_equal(np.concatenate([q[0] for q in parts]), plain_c)
        assert np.array_equal(np.concatenate([q[1] for q in parts]), plain_d)


@pytest.mark.parametrize("nbands,display", [(1, 0), (3, 1), (8, 5)])
def test_group_bands_on_one_device_assemble_in_place(oracle, nbands, display):
    """tri_group with every band on device 0 (the 1-GPU stand-in for N devices): bands render in place
    into the display frame; the assembled frame and the per-band depth equal the oracle's full frame."""
    from trident_raster import raster, scenes

    s = sc.primitives_row(oracle, 320, 240)
    with raster.TriGroup(s.width, s.height, [0] * nbands, display=display) as g:
        scenes.load_scene(g, s)
        g.render_frame()
        col, dep = g.readback()
        g.render_frame()  # steady state: a second frame over the same buffers
        col2, dep2 = g.readback()
        ptr, dev = g.frame_pointer()
    oc, od, _ = oracle.render(s)
    assert np.array_equal(dep, od) and np.array_equal(dep2, od)
    assert int(np.abs(col.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL
    assert np.array_equal(col, col2)
    assert ptr and dev == 0


def test_external_stream_orders_output():
    """tri_set_stream with a torch stream: the frame is enqueued on THAT stream, so a reader on another
    stream ordered behind it (wait_stream, no device-wide sync) sees the finished band — what the bench's
    collectives rely on (a default-stream handle of 0 used to mean the context's own
    unordered stream)."""
    import torch
    from trident_raster import scenes

    s = sc.grid_c3(1920, 1080, 300)
    W, H = s.width, s.height
    color = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    depth = torch.zeros(W * H, dtype=torch.float32, device="cuda")
    st, reader = torch.cuda.Stream(), torch.cuda.Stream()
    with raster_ctx(W, H) as r:
        scenes.load_scene(r, s)
        r.render_frame()  # sizes the queues
        ref_c, _ = r.readback()
        r.set_stream(st.cuda_stream)
        r.bind_output(color.data_ptr(), depth.data_ptr())
        for _ in range(3):
            torch.cuda.synchronize()
            color.zero_()
            torch.cuda.synchronize()
            with torch.cuda.stream(st):
                r.render()
            reader.wait_stream(st)
            with torch.cuda.stream(reader):
                snap = color.clone()
            reader.synchronize()
            got = snap.cpu().numpy().view(np.uint8).reshape(H, W, 4)
            assert np.array_equal(got, ref_c.reshape(H, W, 4))
        r.synchronize()


def raster_ctx(W, H):
    from trident_raster import raster

    return raster.TriRaster(W, H)


def test_own_geometry_after_a_shared_one(oracle):
    """A context that rendered a shared tri_geometry, then uploads geometry of its own with an unchanged
    draw list, resolves its draws against the new buffers (per-object geometry versions could
    collide): both frames match the oracle."""
    from trident_raster import raster, scenes

    s1, s2 = sc.grid_c3(320, 240, 24), sc.grid_c3(320, 240, 37)
    g = raster.TriGeometry(0)
    g.upload(s1.vertices, s1.indices, s1.meshes)
    with raster.TriRaster(320, 240, device=0) as r:
        scenes.load_scene(r, s1, geometry=g)
        r.render_frame()
        got1 = r.readback()
        r.upload_geometry(s2.vertices, s2.indices, s2.meshes)  # own geometry; same draws
        r.set_draws(s2.draws)
        r.render_frame()
        got2 = r.readback()
    g.close()
    for (gc, gd), s in ((got1, s1), (got2, s2)):
        oc, od, _ = oracle.render(s)
        assert np.array_equal(gd, od)
        assert int(np.abs(gc.astype(np.int16) - oc.astype(np.int16)).max()) <= COLOR_TOL
    assert not np.array_equal(got1[1], got2[1])


def test_gpu_against_float64_pipeline(flags):
    """The HIP frame against the float64 restatement of the Vulkan rules and the reference shaders
    (tests/test_oracle_clip_f64.py), without the oracle in between: interior pixels of the textured grid, the
    near-clip grid and a sphere out to grazing angles, and the skybox pass. Both builds are within 1 LSB of the
    oracle (the exact build's powf / IEEE divides may round a channel differently from glibc's) and the oracle
    within 1 LSB of float64, so the bar is 2 LSB."""
    import test_oracle_clip_f64 as f64

    tol = 2
    for s in (sc.textured_grid(320, 180, 30), sc.near_clip_grid(320, 240, 24), sc.sphere_c2(320, 240, 40, 60)):
        s.skybox = None
        gc, gd, _ = render_gpu(s, flags=flags)
        fd, margin, _, _ = f64.f64_depth(s)
        ref, mask = f64.f64_colour(s, fd, margin)
        assert mask.sum() > 6000
        want = np.rint(np.clip(ref, 0, 1) * 255.0)
        diff = np.abs(gc[..., [2, 1, 0, 3]].astype(np.float64) - want)[mask]
        assert diff.max() <= tol, (s.name, diff.max())
    s = sc.skybox_only(160, 120, 90.0, (-80.0, 30.0, 0.0), sc.cubemap_faces(32, seed=5))
    gc, _, _ = render_gpu(s, flags=flags)
    ref = f64.f64_sky(s)
    mask = ~np.isnan(ref[..., 0])
    diff = np.abs(gc[..., [2, 1, 0]].astype(np.float64) - np.rint(np.clip(ref, 0, 1) * 255.0))[mask]
    assert mask.mean() > 0.6 and diff.max() <= tol, diff.max()
