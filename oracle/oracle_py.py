"""TEST INFRASTRUCTURE: ctypes wrapper of the CPU parity oracle (oracle/build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
Parity status: see oracle/tri_oracle.h ("parity unpinned" vs the Vulkan driver; KAT-pinned).
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")
sys.path.insert(0, os.path.join(ORACLE_DIR, "..", "3d-renderer_amd", "python"))
from trident_raster import abi  # noqa: E402


class OracleTexture(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32), ("reserved", C.c_uint32),
                ("rgba8_srgb", C.c_void_p)]


class OracleScene(C.Structure):
    _fields_ = [
        ("vertices", C.c_void_p), ("vertex_count", C.c_uint64),
        ("indices", C.c_void_p), ("index_count", C.c_uint64),
        ("meshes", C.c_void_p), ("mesh_count", C.c_uint32), ("material_count", C.c_uint32),
        ("materials", C.c_void_p),
        ("textures", C.c_void_p), ("texture_count", C.c_uint32), ("bone_count", C.c_uint32),
        ("bones", C.c_void_p),
        ("draws", C.c_void_p), ("draw_count", C.c_uint32), ("reserved", C.c_uint32),
        ("ubo", C.POINTER(abi.TriGlobalUbo)),
        ("clear_rgba", C.c_float * 4),
        ("sky_faces", C.c_void_p), ("sky_size", C.c_uint32), ("sky_reserved", C.c_uint32),
        ("shadow", C.POINTER(abi.TriShadowConfig)), ("out_shadow_map", C.c_void_p),
        ("ai_frame", C.c_void_p), ("ai_width", C.c_uint32), ("ai_height", C.c_uint32),
    ]


class OracleStats(C.Structure):
    _fields_ = [("triangles_in", C.c_uint64), ("triangles_setup", C.c_uint64), ("triangles_clipped", C.c_uint64),
                ("fragments_tested", C.c_uint64)]


class OracleLight(C.Structure):
    _fields_ = [("type", C.c_uint32), ("enabled", C.c_uint32), ("color", C.c_float * 3), ("intensity", C.c_float),
                ("direction", C.c_float * 3), ("range", C.c_float), ("position", C.c_float * 3),
                ("has_transform", C.c_uint32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        lib.oracle_render.restype = C.c_int
        lib.oracle_render.argtypes = [C.POINTER(OracleScene), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                      C.c_void_p, C.c_void_p, C.POINTER(OracleStats)]
        lib.oracle_build_primitive.restype = C.c_int
        lib.oracle_build_primitive.argtypes = [C.c_int, C.c_void_p, C.POINTER(C.c_uint32), C.c_void_p,
                                               C.POINTER(C.c_uint32)]
        lib.oracle_build_uv_sphere.restype = C.c_int
        lib.oracle_build_uv_sphere.argtypes = [C.c_uint32, C.c_uint32, C.c_float, C.c_void_p, C.POINTER(C.c_uint32),
                                               C.c_void_p, C.POINTER(C.c_uint32)]
        fl3 = C.POINTER(C.c_float)
        lib.oracle_compose_transform.restype = None
        lib.oracle_compose_transform.argtypes = [fl3, fl3, fl3, fl3]
        lib.oracle_editor_camera.restype = None
        lib.oracle_editor_camera.argtypes = [fl3, fl3, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                             C.c_float, C.c_int, fl3, fl3, fl3]
        lib.oracle_runtime_camera.restype = None
        lib.oracle_runtime_camera.argtypes = [fl3, fl3, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                              C.c_float, C.c_int, fl3, fl3]
        lib.oracle_blit_linear.restype = None
        lib.oracle_blit_linear.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32]
        lib.oracle_shadow_fit_ortho.restype = None
        lib.oracle_shadow_fit_ortho.argtypes = [fl3, fl3, fl3, fl3]
        lib.oracle_pack_global_ubo.restype = None
        lib.oracle_pack_global_ubo.argtypes = [fl3, fl3, fl3, C.c_int, fl3, C.c_float, C.POINTER(OracleLight),
                                               C.c_uint32, C.POINTER(abi.TriGlobalUbo)]
        _lib = lib
    return _lib


def _f(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(C.POINTER(C.c_float))


def build_primitive(kind):
    lib = load()
    nv, ni = C.c_uint32(0), C.c_uint32(0)
    assert lib.oracle_build_primitive(kind, None, C.byref(nv), None, C.byref(ni)) == 0
    v = np.zeros(nv.value, abi.VERTEX_DTYPE)
    i = np.zeros(ni.value, np.uint32)
    assert lib.oracle_build_primitive(kind, v.ctypes.data, C.byref(nv), i.ctypes.data, C.byref(ni)) == 0
    return v, i


def build_uv_sphere(rings, segments, radius):
    lib = load()
    nv, ni = C.c_uint32(0), C.c_uint32(0)
    assert lib.oracle_build_uv_sphere(rings, segments, radius, None, C.byref(nv), None, C.byref(ni)) == 0
    v = np.zeros(nv.value, abi.VERTEX_DTYPE)
    i = np.zeros(ni.value, np.uint32)
    assert lib.oracle_build_uv_sphere(rings, segments, radius, v.ctypes.data, C.byref(nv), i.ctypes.data,
                                      C.byref(ni)) == 0
    return v, i


def compose_transform(pos, rot, scl=(1, 1, 1)):
    lib = load()
    p, pp = _f(pos); r, rp = _f(rot); s, sp = _f(scl)
    out = np.zeros(16, np.float32)
    lib.oracle_compose_transform(pp, rp, sp, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out.reshape(4, 4)


def editor_camera(pos, rot=(0, 0, 0), fov=60.0, viewport=(1280, 720), near=0.1, far=1000.0, ortho=20.0, ptype=0):
    lib = load()
    p, pp = _f(pos); r, rp = _f(rot)
    view = np.zeros(16, np.float32); proj = np.zeros(16, np.float32); fwd = np.zeros(3, np.float32)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    lib.oracle_editor_camera(pp, rp, fov, viewport[0], viewport[1], near, far, ortho, ptype, P(view), P(proj), P(fwd))
    return view.reshape(4, 4), proj.reshape(4, 4), fwd


def runtime_camera(pos, rot=(0, 0, 0), fov=60.0, viewport=(1280, 720), near=0.1, far=1000.0, ortho=20.0, ptype=0):
    lib = load()
    p, pp = _f(pos); r, rp = _f(rot)
    view = np.zeros(16, np.float32); proj = np.zeros(16, np.float32)
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    lib.oracle_runtime_camera(pp, rp, fov, viewport[0], viewport[1], near, far, ortho, ptype, P(view), P(proj))
    return view.reshape(4, 4), proj.reshape(4, 4)


def pack_ubo(view, proj, cam, lights=(), has_camera=True, ambient=(0.03, 0.03, 0.03), ambient_intensity=1.0):
    lib = load()
    arr = (OracleLight * max(len(lights), 1))()
    for k, L in enumerate(lights):
        o = arr[k]
        o.type = 0 if L["type"] == "directional" else 1
        o.enabled = 1 if L.get("enabled", True) else 0
        o.color = (C.c_float * 3)(*L.get("color", (1.0, 0.98, 0.92)))
        o.intensity = L.get("intensity", 5.0)
        o.direction = (C.c_float * 3)(*L.get("direction", (-0.5, -1.0, -0.3)))
        o.range = L.get("range", 10.0)
        o.position = (C.c_float * 3)(*L.get("position", (0, 0, 0)))
        o.has_transform = 1 if "position" in L else 0
    v, vp = _f(view); pr, pp = _f(proj); c, cp = _f(cam); a, ap = _f(ambient)
    u = abi.TriGlobalUbo()
    lib.oracle_pack_global_ubo(vp, pp, cp, 1 if has_camera else 0, ap, ambient_intensity, arr, len(lights), C.byref(u))
    return u


def shadow_fit_ortho(light_dir, aabb_min, aabb_max):
    lib = load()
    d, dp = _f(light_dir); a, ap = _f(aabb_min); b, bp = _f(aabb_max)
    out = np.zeros(16, np.float32)
    lib.oracle_shadow_fit_ortho(dp, ap, bp, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out.reshape(4, 4)


def render(scene, band=None, threads=None, shadow_map_out=None):
    """Render a trident_raster.scenes.Scene. Returns (bgra uint8 [rows,W,4], depth bits uint32 [rows,W], stats).
    shadow_map_out: optional uint32 [size, size] array that receives the shadow pre-pass's map."""
    lib = load()
    if threads is None:
        threads = min(os.cpu_count() or 1, 16)
    keep = []
    v = np.ascontiguousarray(scene.vertices, abi.VERTEX_DTYPE)
    i = np.ascontiguousarray(scene.indices, np.uint32)
    m = np.ascontiguousarray(scene.meshes, abi.MESH_RANGE_DTYPE)
    mats = (abi.TriMaterialRecord * max(len(scene.materials), 1))()
    for k, (base, fac) in enumerate(scene.materials):
        mats[k].base_color_factor = (C.c_float * 4)(*base)
        mats[k].material_factors = (C.c_float * 4)(*fac)
    texs = (OracleTexture * max(len(scene.textures), 1))()
    for k, (slot, t) in enumerate(scene.textures):
        t = np.ascontiguousarray(t, np.uint8)
        keep.append(t)
        texs[k].slot, texs[k].width, texs[k].height = slot, t.shape[1], t.shape[0]
        texs[k].rgba8_srgb = t.ctypes.data
    draws, nd = abi.draws_array(scene.draws)
    bones = None if scene.bones is None else np.ascontiguousarray(scene.bones, np.float32).reshape(-1, 16)
    sc = OracleScene()
    sc.vertices, sc.vertex_count = v.ctypes.data, v.size
    sc.indices, sc.index_count = i.ctypes.data, i.size
    sc.meshes, sc.mesh_count = m.ctypes.data, m.size
    sc.materials, sc.material_count = C.cast(mats, C.c_void_p), len(scene.materials)
    sc.textures, sc.texture_count = C.cast(texs, C.c_void_p), len(scene.textures)
    sc.bones, sc.bone_count = (bones.ctypes.data if bones is not None else None), (0 if bones is None else bones.shape[0])
    sc.draws, sc.draw_count = C.cast(draws, C.c_void_p), nd
    ubo = scene.ubo
    sc.ubo = C.pointer(ubo)
    sc.clear_rgba = (C.c_float * 4)(*scene.clear)
    sky = getattr(scene, "skybox", None)
    if sky is not None:
        sky = np.ascontiguousarray(sky, np.uint8)  # [6, n, n, 4]
        keep.append(sky)
        sc.sky_faces, sc.sky_size = sky.ctypes.data, sky.shape[1]
    ai = getattr(scene, "ai_frame", None)
    if ai is not None:  # the AI frame blend's R8G8B8A8_UNORM texture (Default.frag:182-191)
        ai = np.ascontiguousarray(ai, np.uint8)
        keep.append(ai)
        sc.ai_frame, sc.ai_width, sc.ai_height = ai.ctypes.data, ai.shape[1], ai.shape[0]
    shadow = getattr(scene, "shadow", None)
    if shadow is not None:
        sc.shadow = C.pointer(shadow)
        if shadow_map_out is not None:
            assert shadow_map_out.dtype == np.uint32 and shadow_map_out.size == shadow.size * shadow.size
            sc.out_shadow_map = shadow_map_out.ctypes.data
    y0, y1 = band if band is not None else (0, scene.height)
    rows = y1 - y0
    col = np.empty((rows, scene.width, 4), np.uint8)
    dep = np.empty((rows, scene.width), np.uint32)
    st = OracleStats()
    rc = lib.oracle_render(C.byref(sc), scene.width, scene.height, y0, y1, threads, col.ctypes.data, dep.ctypes.data,
                           C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return col, dep, {k: getattr(st, k) for k, _ in OracleStats._fields_}


def blit_linear(bgra, dw, dh):
    """vkCmdBlitImage with VK_FILTER_LINEAR (Renderer.cpp:5346-5361): uint8 [h, w, 4] -> [dh, dw, 4]."""
    lib = load()
    src = np.ascontiguousarray(bgra, np.uint8)
    h, w = src.shape[:2]
    out = np.zeros((dh, dw, 4), np.uint8)
    lib.oracle_blit_linear(src.ctypes.data, w, h, out.ctypes.data, dw, dh)
    return out

