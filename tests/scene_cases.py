"""Parity scenes shared by the CPU golden tests and the GPU parity tests.

Each builder returns a trident_raster.scenes.Scene whose inputs are fully determined (Forge-style
camera/entities, reference primitive meshes restated by the oracle, procedural meshes)."""
import numpy as np

from trident_raster import abi, scenes

F = np.float32


def c1_cube(frame=0, w=640, h=480):
    return scenes.scene_c1_cube(frame, w, h)


def primitives_row(oracle, w=320, h=240):
    """Cube, sphere and quad primitives side by side (CreatePrimitiveEntity), editor camera (0,3,8)."""
    cam = (0.0, 3.0, 8.0)
    view, proj, fwd = oracle.editor_camera(cam, (0, 0, 0), 60.0, (w, h))
    verts, idxs, meshes = [], [], []
    vbase = ibase = 0
    for kind in (1, 2, 3):
        v, i = oracle.build_primitive(kind)
        meshes.append((ibase, i.size, vbase, len(meshes)))
        verts.append(v)
        idxs.append(i)
        vbase += v.size
        ibase += i.size
    m = np.array(meshes, dtype=abi.MESH_RANGE_DTYPE)
    draws = []
    for k, x in enumerate((-1.6, 0.0, 1.6)):
        model = oracle.compose_transform((x, 3.0, 3.0), (20.0 * k, 35.0 + 10 * k, 5.0 * k), (1.0, 1.0, 1.0))
        draws.append(abi.make_draw(k, model, texture_slot=0, material_index=k))
    ubo = oracle.pack_ubo(view, proj, cam, [])
    return scenes.Scene("primitives", w, h, np.concatenate(verts), np.concatenate(idxs), m, draws, ubo,
                        materials=[((1, 1, 1, 1), (0.0, 1.0, 1.0, 0.0))] * 3)


def sphere_c2(w=1920, h=1080, rings=125, segments=200, oracle=None):
    s = scenes.scene_c2_sphere(w, h, rings, segments)
    if oracle is not None:  # reference sphere builder restated by the oracle (glibc sin/cos)
        v, i = oracle.build_uv_sphere(rings, segments, 3.0)
        s.vertices, s.indices = v, i
        s.meshes = np.array([(0, i.size, 0, 0)], dtype=abi.MESH_RANGE_DTYPE)
    return s


def grid_c3(w=1280, h=720, n=200):
    return scenes.scene_c3_grid(w, h, n)


def checker_texture(wt=16, ht=8, seed=7):
    rng = np.random.default_rng(seed)
    t = rng.integers(0, 256, size=(ht, wt, 4), dtype=np.uint8)
    t[..., 3] = rng.integers(128, 256, size=(ht, wt), dtype=np.uint8)
    return t


def textured_grid(w=640, h=360, n=40):
    s = scenes.scene_c3_grid(w, h, n)
    s.textures = [(3, checker_texture())]
    s.draws = [abi.make_draw(0, np.eye(4, dtype=F), texture_slot=3, material_index=0, tint=(1.0, 0.9, 0.8, 0.75),
                             texture_scale=(1.5, 0.75), texture_offset=(0.1, -0.2), tiling=1.25)]
    return s


def near_clip_grid(w=640, h=480, n=60):
    """Camera pitched down over a ground plane that passes through the near plane and behind the
    eye: exercises homogeneous clipping (w <= 0, z < 0) and the guard band."""
    cam = (0.0, 0.35, 0.0)
    view, proj = scenes.editor_camera(cam, (-28.0, 12.0, 0.0), 70.0, (w, h), 0.1, 40.0)
    v, idx = scenes.displaced_grid_mesh(n, extent=(30.0, 30.0), depth=0.0, amplitude=0.15)
    # grid lies in x-y; rotate it to the x-z ground plane facing +y
    model = scenes.compose_transform((0.0, 0.0, -5.0), (-90.0, 0.0, 0.0), (1.0, 1.0, 1.0))
    lights = [{"type": "point", "position": (0.5, 1.0, -2.0), "range": 6.0, "intensity": 8.0}]
    return scenes.Scene("near_clip", w, h, v, idx, np.array([(0, idx.size, 0, 0)], abi.MESH_RANGE_DTYPE),
                        [abi.make_draw(0, model, material_index=0)], scenes.pack_ubo(view, proj, cam, lights),
                        materials=[((0.8, 0.8, 0.8, 1.0), (0.5, 0.3, 1.0, 0.0))])


def depth_ties(w=256, h=256):
    """Two coplanar quads: the later draw must win every tie (LESS_OR_EQUAL), plus a far-plane
    straddling quad (per-pixel far clip)."""
    quad_v, quad_i = scenes.cube_mesh()  # reuse vertex layout; build a quad by hand below
    v = np.zeros(4, abi.VERTEX_DTYPE)
    v["position"] = [(-1, -1, 0), (1, -1, 0), (1, 1, 0), (-1, 1, 0)]
    v["normal"] = (0, 0, 1)
    v["color"] = 1.0
    v["texcoord"] = [(0, 0), (1, 0), (1, 1), (0, 1)]
    idx = np.array([0, 1, 2, 0, 2, 3], np.uint32)
    meshes = np.array([(0, 6, 0, 0)], abi.MESH_RANGE_DTYPE)
    cam = (0.0, 0.0, 4.0)
    view, proj = scenes.editor_camera(cam, (0, 0, 0), 60.0, (w, h), 0.1, 6.0)
    m1 = scenes.compose_transform((0, 0, 0), (0, 0, 0), (1, 1, 1))
    m2 = scenes.compose_transform((0.3, 0.2, 0), (0, 0, 0), (1, 1, 1))
    m3 = scenes.compose_transform((0.0, -0.5, -1.0), (70.0, 0, 0), (3, 3, 3))  # pokes past far = 6
    draws = [abi.make_draw(0, m1, tint=(1, 0.2, 0.2, 1)), abi.make_draw(0, m2, tint=(0.2, 1, 0.2, 1)),
             abi.make_draw(0, m1, tint=(0.2, 0.2, 1, 1)), abi.make_draw(0, m3, tint=(1, 1, 0.3, 1))]
    return scenes.Scene("depth_ties", w, h, v, idx, meshes, draws, scenes.pack_ubo(view, proj, cam, []),
                        materials=[((1, 1, 1, 1), (0.2, 0.5, 1.0, 0.0))])


def pixel_aligned_triangles(w=512, h=256, n=8000, seed=11):
    """Triangles whose vertices sit on quarter-pixel positions under an exact orthographic mapping (world
    x, y in pixels: the snap lands on them exactly), so edges run through pixel centres and their row
    crossings are exact integers — the boundary cases of k_raster's span walk (ceil/floor of -F/A, the
    top-left bias) — plus horizontal and vertical edges, slivers, and triangles on both sides of the
    64-px limit of the 32-bit edge set-up. Random depths overlap them (key resolve); both windings are
    emitted at random, so about half are culled. 8000 triangles over 512x256 keep the frame on 32x32 bins
    (choose_bin_grid: density >= 0.05), the bin size whose per-lane walk is the span walk."""
    rng = np.random.default_rng(seed)
    tris = []
    for k in range(n):
        kind = k % 6
        size = [3, 10, 40, 62, 70, 24][kind] * (0.5 + rng.random())
        cx, cy = rng.uniform(-20, w + 20), rng.uniform(-20, h + 20)
        if kind == 5:  # axis-aligned right triangle (one horizontal, one vertical edge)
            a, b = size * rng.choice([-1, 1]), size * rng.choice([-1, 1])
            p = [(cx, cy), (cx + a, cy), (cx, cy + b)]
        elif kind == 3 and k % 12 == 3:  # sliver
            p = [(cx, cy), (cx + size, cy + 0.25 * rng.integers(1, 4)), (cx + size * 0.5, cy + 0.25)]
        else:
            p = [(cx + size * rng.uniform(-1, 1), cy + size * rng.uniform(-1, 1)) for _ in range(3)]
        q = np.round(np.asarray(p, np.float64) * 4.0) / 4.0  # quarter pixels: exact in float and on the snap
        z = rng.uniform(0.05, 0.95, size=3)
        if rng.random() < 0.3:
            z[:] = z[0]  # flat: depth ties between overlapping flat triangles at equal depth are rarer but exact
        tris.append([(q[i, 0], q[i, 1], z[i]) for i in range(3)])
    v = np.zeros(3 * n, abi.VERTEX_DTYPE)
    v["position"] = np.asarray(tris, F).reshape(-1, 3)
    v["normal"] = (0, 0, 1)
    v["color"] = rng.uniform(0.2, 1.0, size=(3 * n, 3)).astype(F)
    v["texcoord"] = rng.uniform(0, 1, size=(3 * n, 2)).astype(F)
    idx = np.arange(3 * n, dtype=np.uint32)
    meshes = np.array([(0, idx.size, 0, 0)], abi.MESH_RANGE_DTYPE)
    view = np.eye(4, dtype=F)
    proj = np.eye(4, dtype=F)  # [col][row]: clip = (2x/W - 1, 2y/H - 1, z, 1), powers of two, products exact
    proj[0, 0], proj[3, 0] = F(2.0 / w), F(-1.0)
    proj[1, 1], proj[3, 1] = F(2.0 / h), F(-1.0)
    cam = (w / 2.0, h / 2.0, 50.0)
    draws = [abi.make_draw(0, np.eye(4, dtype=F), material_index=0)]
    return scenes.Scene("pixel_aligned", w, h, v, idx, meshes, draws, scenes.pack_ubo(view, proj, cam, []),
                        materials=[((1, 1, 1, 1), (0.1, 0.5, 1.0, 0.0))])


def large_quads(w=1920, h=1080, one_draw=False):
    """Screen-filling quads over 1920x1080 (2040 bins of 32x32): a set-up round whose bins span more than
    k_setup's 1024-cell LDS grid, so binning takes the per-wave reservation path."""
    s = depth_ties(w, h)
    big = scenes.compose_transform((0.0, 0.0, 0.0), (0, 0, 0), (3.5, 3.5, 1.0))
    tilted = scenes.compose_transform((0.4, -0.3, 0.5), (25.0, 35.0, 0), (2.5, 2.5, 1.0))
    s.draws = [abi.make_draw(0, big, tint=(1, 0.3, 0.2, 1))] if one_draw else \
        [abi.make_draw(0, big, tint=(1, 0.3, 0.2, 1)), abi.make_draw(0, tilted, tint=(0.2, 0.9, 0.4, 1))]
    s.name = "large_quads_1" if one_draw else "large_quads_2"
    return s


def skinned_quad(oracle, w=256, h=256):
    """GPU skinning branch (Default.vert:64-85): 2-bone palette at an offset, weights per vertex,
    one out-of-range bone index (skipped)."""
    v, i = oracle.build_primitive(3)
    v["bone_indices"] = [(0, 1, 0, 0), (1, 0, 0, 0), (0, 5, 0, 0), (1, 1, 0, 0)]
    v["bone_weights"] = [(0.75, 0.25, 0, 0), (1.0, 0, 0, 0), (0.6, 0.4, 0, 0), (0.5, 0.5, 0, 0)]
    bones = np.stack([np.eye(4, dtype=F).reshape(16),
                      np.eye(4, dtype=F).reshape(16),
                      oracle.compose_transform((0.2, 0.1, 0.0), (0, 0, 25.0), (1.2, 0.9, 1.0)).reshape(16)])
    cam = (0.0, 0.0, 2.0)
    view, proj, _ = oracle.editor_camera(cam, (0, 0, 0), 60.0, (w, h))
    model = oracle.compose_transform((0.0, 0.0, 0.0), (0.0, 0.0, 0.0), (1, 1, 1))
    d = abi.make_draw(0, model, bone_offset=1, bone_count=2)
    return scenes.Scene("skinned", w, h, v, i, np.array([(0, i.size, 0, 0)], abi.MESH_RANGE_DTYPE), [d],
                        oracle.pack_ubo(view, proj, cam, []), materials=[], bones=bones)


def invalid_inputs(oracle, w=200, h=150):
    """Bad mesh index, out-of-range vertex index, empty mesh: silently skipped (Renderer.cpp:2946-2956,
    :5118-5127); the valid cube still renders."""
    v, i = oracle.build_primitive(1)
    bad = np.concatenate([i, np.array([0, 1, 999], np.uint32)])
    meshes = np.array([(0, i.size, 0, 0), (i.size, 3, 0, 0), (0, 0, 0, 0)], abi.MESH_RANGE_DTYPE)
    cam = (0.0, 0.0, 3.0)
    view, proj, _ = oracle.editor_camera(cam, (0, 0, 0), 60.0, (w, h))
    model = oracle.compose_transform((0.0, 0.0, 0.0), (30.0, 40.0, 0.0), (1, 1, 1))
    draws = [abi.make_draw(7, model), abi.make_draw(1, model), abi.make_draw(2, model), abi.make_draw(0, model)]
    return scenes.Scene("invalid", w, h, v, bad, meshes, draws, oracle.pack_ubo(view, proj, cam, []))


def empty_scene(w=128, h=96):
    view, proj = scenes.editor_camera((0, 0, 5), (0, 0, 0), 60.0, (w, h))
    return scenes.Scene("empty", w, h, np.zeros(0, abi.VERTEX_DTYPE), np.zeros(0, np.uint32),
                        np.zeros(0, abi.MESH_RANGE_DTYPE), [], scenes.pack_ubo(view, proj, (0, 0, 5)),
                        clear=(0.1, 0.2, 0.3, 1.0))


# ---- skybox ----------------------------------------------------------------
SOLID_0x808080 = scenes.DEFAULT_SKYBOX  # CreateSolidColor(0x808080)


def cubemap_faces(n=16, seed=11):
    """A cubemap whose faces are distinct seeded gradients with noise (exercises filtering and the
    seamless edges), uint8 [6, n, n, 4] sRGB, faces +X,-X,+Y,-Y,+Z,-Z."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:n, 0:n].astype(np.float32) / max(n - 1, 1)
    faces = np.empty((6, n, n, 4), np.uint8)
    for f in range(6):
        base = rng.integers(30, 200, size=3)
        g = np.stack([base[0] + 50 * xx, base[1] + 50 * yy, base[2] + 25 * (xx + yy)], -1)
        g += rng.integers(-8, 9, size=g.shape)
        faces[f, ..., :3] = np.clip(g, 0, 255).astype(np.uint8)
        faces[f, ..., 3] = 255
    return faces


def skybox_only(w=320, h=240, fov=100.0, rot=(0.0, 0.0, 0.0), faces=None):
    """No meshes: every pixel is the skybox pass (Renderer.cpp:5076-5082 before any mesh draw)."""
    s = scenes.scene_c1_cube(0, w, h)
    view, proj = scenes.editor_camera((0.0, 3.0, 8.0), rot, fov, (w, h), 0.1, 1000.0)
    s.ubo = scenes.pack_ubo(view, proj, (0.0, 3.0, 8.0))
    s.draws = []
    s.name = f"skybox_only_{w}x{h}_fov{fov:g}"
    s.skybox = cubemap_faces() if faces is None else faces
    return s


def c1_cube_skybox(frame=1, w=640, h=480):
    s = scenes.scene_c1_cube(frame, w, h)
    s.skybox = cubemap_faces(32, seed=5)
    s.name = "c1_cube_skybox"
    return s


# ---- shadow-map pre-pass (BASELINE C5; tri_set_shadow) ------------------------------
def shadow_scene(oracle, w=480, h=320, size=256, sun=(-0.45, -1.0, -0.35), bias=0.001, slope=2.0):
    """A ground quad under a floating cube and sphere, lit by a shadow-casting sun (plus one point
    light): the primitives (Renderer.cpp:72-246) as Forge spawns them, light frustum fitted by
    tri_shadow_fit_ortho over the draws' world box."""
    cam = (0.0, 4.0, 8.0)
    view, proj, _ = oracle.editor_camera(cam, (-25.0, 0.0, 0.0), 60.0, (w, h))
    verts, idxs, meshes = [], [], []
    vbase = ibase = 0
    for kind in (1, 2, 3):
        v, i = oracle.build_primitive(kind)
        meshes.append((ibase, i.size, vbase, len(meshes)))
        verts.append(v)
        idxs.append(i)
        vbase += v.size
        ibase += i.size
    m = np.array(meshes, dtype=abi.MESH_RANGE_DTYPE)
    draws = [
        abi.make_draw(2, oracle.compose_transform((0.0, 0.0, 0.0), (-90.0, 0.0, 0.0), (12.0, 12.0, 1.0)), material_index=0),
        abi.make_draw(0, oracle.compose_transform((-1.2, 1.4, 0.5), (15.0, 30.0, 0.0), (1.2, 1.2, 1.2)), material_index=0),
        abi.make_draw(1, oracle.compose_transform((1.3, 1.0, -0.4), (0.0, 0.0, 0.0), (1.6, 1.6, 1.6)), material_index=0),
    ]
    lights = [{"type": "directional", "direction": sun, "intensity": 4.0},
              {"type": "point", "position": (2.0, 2.5, 2.0), "range": 7.0, "intensity": 3.0}]
    s = scenes.Scene("shadow", w, h, np.concatenate(verts), np.concatenate(idxs), m, draws,
                     oracle.pack_ubo(view, proj, cam, lights), materials=[((0.9, 0.85, 0.8, 1.0), (0.1, 0.6, 1.0, 0.0))],
                     skybox=SOLID_0x808080)
    return scenes.with_shadow(s, size, bias, slope)


def near_clip_multi(w=640, h=480, n=60, identity=False, shadow=False):
    """near_clip_grid as two textured draws (the grid's index halves, each with its own sRGB slot): clipped primitives
    on a frame outside the single-draw solid instantiation (obj48's object records through the clipper). identity:
    the ground-plane rotation baked into the vertices, so both draws have identity models (the C5 case); otherwise
    the second draw carries its own translation on top of the rotation (a per-draw transform per pixel)."""
    s = near_clip_grid(w, h, n)
    model = np.array(s.draws[0].pc.model, F).reshape(4, 4)  # [col][row]
    if identity:
        v = s.vertices.copy()
        p = v["position"].astype(F)
        nn = v["normal"].astype(F)
        v["position"] = (p @ model[:3, :3] + model[3, :3]).astype(F)
        v["normal"] = (nn @ model[:3, :3]).astype(F)
        s.vertices = v
        m0 = m1 = np.eye(4, dtype=F)
    else:
        m0 = model
        m1 = scenes.compose_transform((0.4, 0.05, -5.3), (-90.0, 0.0, 0.0), (1.0, 1.0, 1.0))
    half = (s.indices.size // 6) * 3
    s.meshes = np.array([(0, half, 0, 0), (half, s.indices.size - half, 0, 0)], abi.MESH_RANGE_DTYPE)
    s.textures = [(1, checker_texture(16, 8, 3)), (2, checker_texture(8, 16, 4))]
    s.draws = [abi.make_draw(0, m0, texture_slot=1, material_index=0),
               abi.make_draw(1, m1, texture_slot=2, material_index=0)]
    s.ubo = scenes.pack_ubo(*scenes.editor_camera((0.0, 0.35, 0.0), (-28.0, 12.0, 0.0), 70.0, (w, h), 0.1, 40.0),
                            (0.0, 0.35, 0.0), [{"type": "directional", "direction": (-0.3, -1.0, -0.2), "intensity": 3.0},
                                               {"type": "point", "position": (0.5, 1.0, -2.0), "range": 6.0,
                                                "intensity": 8.0}])
    s.name = f"near_clip_multi{'_id' if identity else ''}{'_shadow' if shadow else ''}"
    if shadow:
        scenes.with_shadow(s, 512)
    return s


def near_clip_single(w=640, h=480, n=60, shadow=False):
    """near_clip_grid as ONE textured draw (a non-1x1 sRGB slot, the identity uv transform, the ground-plane rotation
    as its model): a single-draw frame outside the solid instantiation, so k_setup runs its single-draw form while
    k_vertex writes no varyings (obj48). The clipper must read the geometry's input records."""
    s = near_clip_grid(w, h, n)
    model = np.array(s.draws[0].pc.model, F).reshape(4, 4)
    s.textures = [(1, checker_texture(16, 8, 3))]
    s.draws = [abi.make_draw(0, model, texture_slot=1, material_index=0)]
    s.name = f"near_clip_single{'_shadow' if shadow else ''}"
    if shadow:
        scenes.with_shadow(s, 512)
    return s
