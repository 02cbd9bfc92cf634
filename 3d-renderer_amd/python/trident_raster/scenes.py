"""Synthetic scenes for BASELINE.json's configs, built the way Trident-Forge builds
them: an editor camera (EditorCamera.cpp:126-160), entities with Transform (ComposeTransform,
Renderer.cpp:417-427), mesh draws and lights packed by UpdateUniformBuffer (Renderer.cpp:5822-5925).

The reference's sample assets (Assimp FBX) are not in the snapshot, so C2/C3 use procedural meshes:
C2 = the reference UV-sphere builder at rings 125 x segments 200 (50,000 tris), C3 = a PCG32-seeded
displaced 708 x 708 grid (999,698 tris). Everything is float32 numpy; glm operation order is kept for
the matrices.
"""
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi

F = np.float32


# ---------------------------------------------------------------------------------------------
# PCG32 (O'Neill, pcg32_random_r), seed 0x5EED
# ---------------------------------------------------------------------------------------------
class PCG32:
    MULT = 6364136223846793005
    MASK = (1 << 64) - 1

    def __init__(self, seed=0x5EED, seq=54):
        self.state = 0
        self.inc = ((seq << 1) | 1) & self.MASK
        self.next_u32()
        self.state = (self.state + seed) & self.MASK
        self.next_u32()

    def next_u32(self):
        old = self.state
        self.state = (old * self.MULT + self.inc) & self.MASK
        xorshifted = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xorshifted >> rot) | (xorshifted << ((-rot) & 31))) & 0xFFFFFFFF

    def uniform(self, n=None):
        if n is None:
            return self.next_u32() / 4294967296.0
        return np.array([self.next_u32() / 4294967296.0 for _ in range(n)], dtype=np.float64)


# ---------------------------------------------------------------------------------------------
# glm restatements (float32, column-major m[col][row])
# ---------------------------------------------------------------------------------------------
def radians(d):
    return F(d) * F(0.01745329251994329576923690768489)


def mat_mul(a, b):
    r = np.zeros((4, 4), F)
    for j in range(4):
        for i in range(4):
            s = F(a[0, i] * b[j, 0])
            s = F(s + F(a[1, i] * b[j, 1]))
            s = F(s + F(a[2, i] * b[j, 2]))
            s = F(s + F(a[3, i] * b[j, 3]))
            r[j, i] = s
    return r


def translate(m, v):
    r = m.copy()
    for i in range(4):
        r[3, i] = F(F(F(F(m[0, i] * F(v[0])) + F(m[1, i] * F(v[1]))) + F(m[2, i] * F(v[2]))) + m[3, i])
    return r


def rotate(m, angle, axis):
    c, s = F(np.cos(F(angle))), F(np.sin(F(angle)))
    a = np.asarray(axis, F)
    a = a * F(F(1.0) / F(np.sqrt(F(F(a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]))))
    t = a * F(F(1.0) - c)
    R = np.zeros((3, 3), F)
    R[0, 0] = c + t[0] * a[0]; R[0, 1] = t[0] * a[1] + s * a[2]; R[0, 2] = t[0] * a[2] - s * a[1]
    R[1, 0] = t[1] * a[0] - s * a[2]; R[1, 1] = c + t[1] * a[1]; R[1, 2] = t[1] * a[2] + s * a[0]
    R[2, 0] = t[2] * a[0] + s * a[1]; R[2, 1] = t[2] * a[1] - s * a[0]; R[2, 2] = c + t[2] * a[2]
    r = np.zeros((4, 4), F)
    for j in range(3):
        for i in range(4):
            r[j, i] = F(F(m[0, i] * R[j, 0] + m[1, i] * R[j, 1]) + m[2, i] * R[j, 2])
    r[3] = m[3]
    return r


def scale(m, v):
    r = m.copy()
    for k in range(3):
        r[k] = m[k] * F(v[k])
    return r


def compose_transform(position, rotation_deg, scl=(1, 1, 1)):
    """ComposeTransform (Renderer.cpp:417-427): T * Rx * Ry * Rz * S."""
    m = np.eye(4, dtype=F)
    m = translate(m, position)
    m = rotate(m, radians(rotation_deg[0]), (1, 0, 0))
    m = rotate(m, radians(rotation_deg[1]), (0, 1, 0))
    m = rotate(m, radians(rotation_deg[2]), (0, 0, 1))
    return scale(m, scl)


def quat_from_euler(e):
    c = np.cos(np.asarray(e, F) * F(0.5)).astype(F)
    s = np.sin(np.asarray(e, F) * F(0.5)).astype(F)
    w = c[0] * c[1] * c[2] + s[0] * s[1] * s[2]
    x = s[0] * c[1] * c[2] - c[0] * s[1] * s[2]
    y = c[0] * s[1] * c[2] + s[0] * c[1] * s[2]
    z = c[0] * c[1] * s[2] - s[0] * s[1] * c[2]
    return np.array([w, x, y, z], F)


def mat4_cast(q):
    w, x, y, z = q
    r = np.eye(4, dtype=F)
    r[0, 0] = F(1) - F(2) * (y * y + z * z); r[0, 1] = F(2) * (x * y + w * z); r[0, 2] = F(2) * (x * z - w * y)
    r[1, 0] = F(2) * (x * y - w * z); r[1, 1] = F(1) - F(2) * (x * x + z * z); r[1, 2] = F(2) * (y * z + w * x)
    r[2, 0] = F(2) * (x * z + w * y); r[2, 1] = F(2) * (y * z - w * x); r[2, 2] = F(1) - F(2) * (x * x + y * y)
    return r


def perspective_rh_zo(fovy, aspect, n, f):
    t = F(np.tan(F(fovy) / F(2)))
    r = np.zeros((4, 4), F)
    r[0, 0] = F(1) / (F(aspect) * t)
    r[1, 1] = F(1) / t
    r[2, 2] = F(f) / (F(n) - F(f))
    r[2, 3] = F(-1)
    r[3, 2] = -(F(f) * F(n)) / (F(f) - F(n))
    return r


def editor_camera(position, rotation_deg=(0, 0, 0), fov=60.0, viewport=(1280, 720), near=0.1, far=1000.0):
    """EditorCamera view/projection (EditorCamera.cpp:131-160), perspectiveRH_ZO + Vulkan Y flip."""
    q = quat_from_euler(np.array([radians(a) for a in rotation_deg], F))
    qc = np.array([q[0], -q[1], -q[2], -q[3]], F)
    view = mat_mul(mat4_cast(qc), translate(np.eye(4, dtype=F), -np.asarray(position, F)))
    aspect = max(F(viewport[0]) / max(F(viewport[1]), F(0.0001)), F(0.0001))
    proj = perspective_rh_zo(radians(fov), aspect, near, far)
    proj[1, 1] *= F(-1)
    return view, proj


def pack_ubo(view, proj, cam_pos, lights=(), ambient=(0.03, 0.03, 0.03), ambient_intensity=1.0):
    """UpdateUniformBuffer (Renderer.cpp:5822-5925). lights: dicts with type 'directional'|'point'."""
    u = abi.TriGlobalUbo()
    u.view = abi.mat_to_c(view)
    u.projection = abi.mat_to_c(proj)
    u.camera_position = (abi.C.c_float * 4)(cam_pos[0], cam_pos[1], cam_pos[2], 1.0)
    u.ambient_color_intensity = (abi.C.c_float * 4)(*ambient, ambient_intensity)
    d = np.array([-0.5, -1.0, -0.3], F)
    direction = d * F(F(1) / F(np.sqrt(F(F(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))))
    color, intensity = (1.0, 0.98, 0.92), 5.0
    ndir = npt = 0
    for L in lights:
        if not L.get("enabled", True):
            continue
        if L["type"] == "directional":
            if ndir == 0:
                dd = np.asarray(L.get("direction", (-0.5, -1.0, -0.3)), F)
                l2 = F(F(dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2])
                if l2 > F(0.0001):
                    direction = dd * F(F(1) / F(np.sqrt(l2)))
                color = L.get("color", (1.0, 0.98, 0.92))
                intensity = max(L.get("intensity", 5.0), 0.0)
            ndir += 1
        elif L["type"] == "point" and npt < abi.TRI_MAX_POINT_LIGHTS:
            p = L.get("position", (0, 0, 0))
            u.point_lights[npt].position_range = (abi.C.c_float * 4)(*p, max(L.get("range", 10.0), 0.0))
            u.point_lights[npt].color_intensity = (abi.C.c_float * 4)(*L.get("color", (1.0, 0.98, 0.92)),
                                                                       max(L.get("intensity", 5.0), 0.0))
            npt += 1
    fallback = ndir == 0 and npt == 0
    u.directional_light_direction = (abi.C.c_float * 4)(*direction.tolist(), 0.0)
    u.directional_light_color = (abi.C.c_float * 4)(*color, intensity)
    u.light_counts = (abi.C.c_uint32 * 4)(1 if (ndir > 0 or fallback) else 0, npt, 0, 0)
    return u


# ---------------------------------------------------------------------------------------------
# geometry
# ---------------------------------------------------------------------------------------------
def _vertices(n):
    v = np.zeros(n, dtype=abi.VERTEX_DTYPE)
    v["color"] = 1.0
    return v


def cube_mesh():
    """BuildPrimitiveCubeMesh (Renderer.cpp:106-173), indices (0,2,1),(0,3,2) per face."""
    faces = [
        ((0, 0, 1), (1, 0, 0), (0, 1, 0), [(-.5, -.5, .5), (.5, -.5, .5), (.5, .5, .5), (-.5, .5, .5)]),
        ((0, 0, -1), (-1, 0, 0), (0, 1, 0), [(.5, -.5, -.5), (-.5, -.5, -.5), (-.5, .5, -.5), (.5, .5, -.5)]),
        ((1, 0, 0), (0, 0, -1), (0, 1, 0), [(.5, -.5, .5), (.5, -.5, -.5), (.5, .5, -.5), (.5, .5, .5)]),
        ((-1, 0, 0), (0, 0, 1), (0, 1, 0), [(-.5, -.5, -.5), (-.5, -.5, .5), (-.5, .5, .5), (-.5, .5, -.5)]),
        ((0, 1, 0), (1, 0, 0), (0, 0, -1), [(-.5, .5, .5), (.5, .5, .5), (.5, .5, -.5), (-.5, .5, -.5)]),
        ((0, -1, 0), (1, 0, 0), (0, 0, 1), [(-.5, -.5, -.5), (.5, -.5, -.5), (.5, -.5, .5), (-.5, -.5, .5)]),
    ]
    v = _vertices(24)
    idx = []
    uvs = [(0, 0), (1, 0), (1, 1), (0, 1)]
    for f, (n, t, b, ps) in enumerate(faces):
        for k in range(4):
            o = 4 * f + k
            v[o]["position"] = ps[k]
            v[o]["normal"] = n
            v[o]["tangent"] = t
            v[o]["bitangent"] = b
            v[o]["texcoord"] = uvs[k]
        o = 4 * f
        idx += [o, o + 2, o + 1, o, o + 3, o + 2]
    return v, np.array(idx, np.uint32)


def uv_sphere_mesh(rings=16, segments=24, radius=0.5):
    """BuildPrimitiveSphereMesh (Renderer.cpp:175-246) with parameterised rings/segments/radius."""
    r = np.arange(rings + 1, dtype=F)[:, None]
    s = np.arange(segments + 1, dtype=F)[None, :]
    V = r / F(rings)
    U = s / F(segments)
    phi = V * F(np.pi)
    theta = U * F(2 * np.pi)
    sp, cp, st, ct = np.sin(phi), np.cos(phi), np.sin(theta), np.cos(theta)
    px = F(radius) * sp * ct
    py = np.broadcast_to(F(radius) * cp, px.shape)
    pz = F(radius) * sp * st
    pos = np.stack([px, py, pz], -1).reshape(-1, 3).astype(F)
    ln = np.sqrt((pos * pos).sum(-1, keepdims=True))
    nrm = np.where(ln > 0, pos / np.maximum(ln, F(1e-30)), 0).astype(F)
    tan = np.stack([-np.broadcast_to(st, px.shape), np.zeros_like(px), np.broadcast_to(ct, px.shape)], -1).reshape(-1, 3)
    v = _vertices(pos.shape[0])
    v["position"] = pos
    v["normal"] = nrm
    v["tangent"] = tan
    v["bitangent"] = np.cross(nrm, tan)
    v["texcoord"] = np.stack([np.broadcast_to(U, px.shape), np.broadcast_to(F(1) - V, px.shape)], -1).reshape(-1, 2)
    row = segments + 1
    rr, ss = np.meshgrid(np.arange(rings), np.arange(segments), indexing="ij")
    i0 = rr * row + ss
    i1 = (rr + 1) * row + ss
    i2 = (rr + 1) * row + ss + 1
    i3 = rr * row + ss + 1
    idx = np.stack([i0, i2, i1, i0, i3, i2], -1).reshape(-1).astype(np.uint32)
    return v, idx


def displaced_grid_mesh(n=708, extent=(5.4, 3.1), depth=-5.0, amplitude=0.9, seed=0x5EED, uv_repeat=4.0):
    """n x n vertices spanning the frustum at z in [depth-1, depth+1], analytic
    normals, per-vertex colour in [0.5, 1]^3 and uv = uv_repeat * grid (exercises REPEAT)."""
    rng = PCG32(seed)
    f1, f2 = 1.0 + 2.0 * rng.uniform(), 1.0 + 2.0 * rng.uniform()
    p1, p2 = 6.283185307179586 * rng.uniform(), 6.283185307179586 * rng.uniform()
    g = np.linspace(0.0, 1.0, n)
    gx, gy = np.meshgrid(g, g, indexing="xy")  # row j (y), column i (x)
    x = (gx * 2 - 1) * extent[0]
    y = (gy * 2 - 1) * extent[1]
    kx, ky = 2 * np.pi * f1 / (2 * extent[0]), 2 * np.pi * f2 / (2 * extent[1])
    sx, cx = np.sin(kx * x + p1), np.cos(kx * x + p1)
    sy, cy = np.sin(ky * y + p2), np.cos(ky * y + p2)
    z = depth + amplitude * sx * cy
    dzdx = amplitude * kx * cx * cy
    dzdy = -amplitude * ky * sx * sy
    nrm = np.stack([-dzdx, -dzdy, np.ones_like(z)], -1)
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    tan = np.stack([np.ones_like(z), np.zeros_like(z), dzdx], -1)
    tan /= np.linalg.norm(tan, axis=-1, keepdims=True)
    v = _vertices(n * n)
    v["position"] = np.stack([x, y, z], -1).reshape(-1, 3)
    v["normal"] = nrm.reshape(-1, 3)
    v["tangent"] = tan.reshape(-1, 3)
    v["bitangent"] = np.cross(nrm, tan).reshape(-1, 3)
    col = np.random.default_rng(seed).random((n * n, 3))  # seeded colour field in [0.5, 1]
    v["color"] = 0.5 + 0.5 * col
    v["texcoord"] = np.stack([gx * uv_repeat, gy * uv_repeat], -1).reshape(-1, 2)
    jj, ii = np.meshgrid(np.arange(n - 1), np.arange(n - 1), indexing="ij")
    v00 = jj * n + ii
    v10 = v00 + 1
    v11 = v00 + n + 1
    v01 = v00 + n
    idx = np.stack([v00, v10, v11, v00, v11, v01], -1).reshape(-1).astype(np.uint32)  # front-facing (quad winding)
    return v, idx


# ---------------------------------------------------------------------------------------------
# scenes
# ---------------------------------------------------------------------------------------------
@dataclass
class Scene:
    name: str
    width: int
    height: int
    vertices: np.ndarray
    indices: np.ndarray
    meshes: np.ndarray
    draws: list
    ubo: abi.TriGlobalUbo
    materials: list = field(default_factory=list)  # [(base_rgba, (metallic, roughness, 1, 0))]
    textures: list = field(default_factory=list)  # [(slot, rgba8 HxWx4)]
    clear: tuple = (0.005, 0.005, 0.005, 1.0)
    bones: np.ndarray = None
    skybox: np.ndarray = None  # uint8 [6, n, n, 4] sRGB cubemap (+X,-X,+Y,-Y,+Z,-Z), None = no skybox pass
    shadow: abi.TriShadowConfig = None  # shadow-map pre-pass (tri_set_shadow), None = off
    ai_frame: np.ndarray = None  # uint8 [h, w, 4] R8G8B8A8_UNORM AI frame (tri_upload_ai_frame), None = none

    @property
    def triangles(self):
        return int(sum(int(self.meshes[d.mesh_index]["index_count"]) // 3 for d in self.draws))

    def algorithmic_bytes(self, rows=None):
        """12*T + 44*V + 4*W*H colour + 4*W*H depth (+ texture footprint)."""
        rows = self.height if rows is None else rows
        V = int(self.vertices.shape[0])
        tex = sum(int(t.shape[0] * t.shape[1] * 4) for _, t in self.textures if t.size > 4)
        shadow = 0 if self.shadow is None else 8 * int(self.shadow.size) ** 2  # map write + read (§8(d) C5)
        return 12 * self.triangles + 44 * V + 8 * self.width * rows + tex + shadow


# CreateDefaultSkybox's last resort (Renderer.cpp:3925-3926): CreateSolidColor(0x808080) — bytes
# 80 80 80 00 on every face.
DEFAULT_SKYBOX = np.tile(np.array([0x80, 0x80, 0x80, 0x00], np.uint8), (6, 1, 1, 1))

# The cubemap a default Forge frame shows: the reference's Assets/Skyboxes PNG faces (committed as data
# under assets/), found and decoded by the shim's CreateSkyboxCubemap discovery (Renderer.cpp:3840-3915).
ASSETS_DIR = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "..", "assets"))
_REFERENCE_SKYBOX = None


def reference_skybox():
    """uint8 [6, 512, 512, 4]: the reference's default skybox, as the shim's discovery loads it."""
    global _REFERENCE_SKYBOX
    if _REFERENCE_SKYBOX is None:
        from . import app

        faces, source = app.load_default_skybox(ASSETS_DIR)
        if faces is None or source != "PNG fallback":
            raise FileNotFoundError(f"reference skybox faces not found under {ASSETS_DIR}/Skyboxes ({source!r})")
        _REFERENCE_SKYBOX = faces
    return _REFERENCE_SKYBOX


def _single_mesh_ranges(nidx, material=0):
    m = np.zeros(1, abi.MESH_RANGE_DTYPE)
    m[0] = (0, nidx, 0, material)
    return m


def scene_c1_cube(frame=0, width=640, height=480, skybox=None):
    """C1: Forge's default editor camera (0,3,8) and a cube primitive spawned 10 units ahead
    (ApplicationLayer.cpp:185-193, :677-718) spinning 30 deg/frame about Y; no lights -> fallback sun."""
    cam = (0.0, 3.0, 8.0)
    view, proj = editor_camera(cam, (0, 0, 0), 60.0, (width, height), 0.1, 1000.0)
    v, idx = cube_mesh()
    model = compose_transform((0.0, 3.0, -2.0), (0.0, 30.0 * frame, 0.0), (1, 1, 1))
    return Scene("c1_cube_640x480", width, height, v, idx, _single_mesh_ranges(idx.size),
                 [abi.make_draw(0, model, texture_slot=0, material_index=0)], pack_ubo(view, proj, cam),
                 materials=[((1, 1, 1, 1), (0.0, 1.0, 1.0, 0.0))], skybox=_sky(skybox))


def _sky(skybox):
    """Scene skybox argument: None = the reference's default (its PNG faces), "solid" = the 0x808080
    fallback, or explicit faces."""
    if skybox is None:
        return reference_skybox()
    if isinstance(skybox, str) and skybox == "solid":
        return DEFAULT_SKYBOX
    return skybox


def scene_c2_sphere(width=1920, height=1080, rings=125, segments=200, skybox=None):
    """C2 substitute (Assimp sample scene not in the snapshot): 50k-tri UV sphere, radius 3, 2 point lights."""
    rng = PCG32(0x5EED)
    cam = (0.0, 0.0, 9.0)
    view, proj = editor_camera(cam, (0, 0, 0), 60.0, (width, height), 0.1, 1000.0)
    v, idx = uv_sphere_mesh(rings, segments, 3.0)
    lights = [
        {"type": "point", "position": (4.0, 3.0, 5.0), "range": 15.0, "intensity": 6.0,
         "color": tuple(0.6 + 0.4 * rng.uniform(3))},
        {"type": "point", "position": (-4.0, -2.0, 4.0), "range": 15.0, "intensity": 4.0,
         "color": tuple(0.6 + 0.4 * rng.uniform(3))},
    ]
    return Scene(f"c2_sphere50k_{width}x{height}", width, height, v, idx, _single_mesh_ranges(idx.size),
                 [abi.make_draw(0, np.eye(4, dtype=F), material_index=0)], pack_ubo(view, proj, cam, lights),
                 materials=[((0.9, 0.75, 0.6, 1.0), (0.3, 0.45, 1.0, 0.0))], skybox=_sky(skybox))


def scene_c3_grid(width=3840, height=2160, n=708, skybox=None):
    """C3: 1M-triangle displaced grid at 4K, directional sun + 4 point lights, uv x4 (REPEAT)."""
    cam = (0.0, 0.0, 0.0)
    view, proj = editor_camera(cam, (0, 0, 0), 60.0, (width, height), 0.1, 1000.0)
    aspect = width / height
    half_h = 5.0 * np.tan(np.radians(30.0)) * 1.04
    v, idx = displaced_grid_mesh(n, extent=(half_h * aspect, half_h))
    lights = [{"type": "directional"}]
    for k, (px, py) in enumerate([(-3.0, 1.5), (3.0, 1.5), (-3.0, -1.5), (3.0, -1.5)]):
        lights.append({"type": "point", "position": (px, py, -2.5), "range": 8.0, "intensity": 3.0 + k,
                       "color": (1.0, 0.9 - 0.1 * k, 0.7 + 0.1 * k)})
    return Scene(f"c3_grid1m_{width}x{height}", width, height, v, idx, _single_mesh_ranges(idx.size),
                 [abi.make_draw(0, np.eye(4, dtype=F), material_index=0)], pack_ubo(view, proj, cam, lights),
                 materials=[((1.0, 1.0, 1.0, 1.0), (0.1, 0.6, 1.0, 0.0))], skybox=_sky(skybox))


# The C3 grid as a Forge entity would hand it over: a non-identity ComposeTransform (Renderer.cpp:417-427) —
# 20 deg of yaw and a uniform 0.95 scale, translated so that the grid's centre (0, 0, -5) stays in place.
C3_TRS_YAW, C3_TRS_SCALE = 20.0, 0.95


def c3_trs_model():
    th = np.radians(C3_TRS_YAW)
    s = C3_TRS_SCALE
    pos = (5.0 * s * np.sin(th), 0.0, -5.0 + 5.0 * s * np.cos(th))
    return compose_transform(pos, (0.0, C3_TRS_YAW, 0.0), (s, s, s))


def scene_c3_trs(width=3840, height=2160, n=708, skybox=None):
    """C3 under a translate + yaw + uniform-scale draw (the general object-space path: the fragment stage carries
    the interpolated position and normal through the model and normal matrices) instead of an identity model."""
    s = scene_c3_grid(width, height, n, skybox)
    s.draws = [abi.make_draw(0, c3_trs_model(), material_index=0)]
    s.name = f"c3trs_grid1m_{width}x{height}"
    return s


def procedural_texture(size, seed):
    """A seeded RGBA8 sRGB texture (bands + noise), opaque: every bilinear tap differs."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32) / size
    base = rng.uniform(40, 200, size=3)
    t = np.empty((size, size, 4), np.uint8)
    for c in range(3):
        wave = np.sin(2 * np.pi * ((c + 1) * 3 * xx + (3 - c) * 2 * yy + rng.uniform()))
        t[..., c] = np.clip(base[c] + 45 * wave + rng.integers(-20, 21, size=(size, size)), 0, 255)
    t[..., 3] = 255
    return t


def world_aabb(scene):
    """World-space box of every drawn vertex (the shim fits the shadow frustum to the same box)."""
    lo = np.full(3, np.inf, np.float32)
    hi = np.full(3, -np.inf, np.float32)
    for d in scene.draws:
        m = scene.meshes[d.mesh_index]
        idx = scene.indices[int(m["first_index"]):int(m["first_index"]) + int(m["index_count"])]
        if idx.size == 0:
            continue
        p = scene.vertices["position"][idx.astype(np.int64) + int(m["base_vertex"])].astype(np.float32)
        M = np.array(d.pc.model, np.float32).reshape(4, 4)  # [col][row]
        w = p @ M[:3, :3] + M[3, :3]
        lo, hi = np.minimum(lo, w.min(0)), np.maximum(hi, w.max(0))
    return lo, hi


def with_shadow(scene, size=2048, depth_bias=0.001, slope_bias=2.0):
    """Turn on the shadow pre-pass for the scene's directional light: the light transform is the one
    the shim fits (tri_shadow_fit_ortho over the world box of the draws)."""
    from . import raster

    lo, hi = world_aabb(scene)
    lvp = raster.shadow_fit_ortho(list(scene.ubo.directional_light_direction)[:3], lo, hi)
    scene.shadow = abi.make_shadow(lvp, size, depth_bias, slope_bias)
    return scene


def scene_c5_textured(width=3840, height=2160, n=708, tex_size=2048, shadow_size=2048, skybox=None):
    """C5: the C3 grid split into 4 meshes (row quarters), each drawn with its own tex_size^2 sRGB
    texture slot (4 bilinear textures, uv x4 REPEAT), plus the shadow_size^2 shadow-map pre-pass for the
    sun (tri_set_shadow; the reference only reserves LightComponent::m_ShadowCaster, so the pass follows
    DESIGN.md §5d). shadow_size 0 leaves the pre-pass off."""
    s = scene_c3_grid(width, height, n, skybox)
    tris = s.indices.size // 3
    q = [(k * tris) // 4 for k in range(5)]
    meshes = np.zeros(4, abi.MESH_RANGE_DTYPE)
    for k in range(4):
        meshes[k] = (3 * q[k], 3 * (q[k + 1] - q[k]), 0, 0)
    s.meshes = meshes
    s.textures = [(1 + k, procedural_texture(tex_size, 0xC5 + k)) for k in range(4)]
    s.draws = [abi.make_draw(k, np.eye(4, dtype=F), texture_slot=1 + k, material_index=0) for k in range(4)]
    s.name = f"c5_textured4x{tex_size}_{width}x{height}"
    if shadow_size:
        with_shadow(s, shadow_size)
        s.name = f"c5_textured4x{tex_size}_shadow{shadow_size}_{width}x{height}"
    return s


def load_scene(rast, scene, geometry=None):
    """Upload a Scene into a TriRaster or TriGroup (UploadMesh + materials + textures + frame + draws).
    geometry: a raster.TriGeometry already holding the scene's meshes, bound instead of uploading."""
    if geometry is not None:
        rast.bind_geometry(geometry)
    else:
        rast.upload_geometry(scene.vertices, scene.indices, scene.meshes)
    rast.upload_materials(scene.materials)
    for slot, tex in scene.textures:
        rast.upload_texture(slot, tex)
    if scene.bones is not None:
        rast.upload_bone_palette(scene.bones)
    if scene.skybox is not None:
        rast.upload_skybox(scene.skybox)
    rast.set_shadow(scene.shadow)
    if scene.ai_frame is not None:
        rast.upload_ai_frame(scene.ai_frame)
    rast.set_frame(scene.ubo, scene.clear)
    rast.set_draws(scene.draws)


def with_ai_blend(scene, strength=0.35, ai_frame=None, seed=0xA1):
    """Default.frag's AI frame blend (:182-191) on a scene: an R8G8B8A8_UNORM frame of the scene's extent (seeded
    noise unless given) and the UBO's AiBlendConfig as UpdateUniformBuffer packs it while the AI texture is ready,
    (strength, 1 / width, 1 / height, 1) (Renderer.cpp:5916-5921; SetAiBlendStrength's default 0.35, Renderer.h:508)."""
    if ai_frame is None:
        rng = np.random.default_rng(seed)
        ai_frame = rng.integers(0, 256, size=(scene.height, scene.width, 4), dtype=np.uint8)
    h, w = ai_frame.shape[:2]
    scene.ai_frame = ai_frame
    scene.ubo.ai_blend_config = (abi.C.c_float * 4)(strength, F(1) / F(max(w, 1)), F(1) / F(max(h, 1)), 1.0)
    return scene
