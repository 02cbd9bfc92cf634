"""Python binding of the C++ Trident::Renderer shim (libtrident_renderer.so, host/include/trident_app.h).

The shim is the reference's renderer API (Renderer/RenderCommand over an ECS registry and the
editor/runtime cameras) restated in C++ on top of the HIP C-ABI. This binding drives it the way
Trident-Forge's ApplicationLayer does, for tests. No CPU fallback: the library must be built.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .raster import PKG_ROOT, TriError

LIB_PATH = os.path.join(PKG_ROOT, "lib", "libtrident_renderer.so")

PRIMITIVE = {"none": 0, "cube": 1, "sphere": 2, "quad": 3}
LIGHT = {"directional": 0, "point": 1}

_f3 = C.POINTER(C.c_float)
_APP_FUNCTIONS = [
    ("trident_app_create", C.c_int, [C.c_uint32, C.POINTER(C.c_void_p)]),
    ("trident_app_destroy", None, [C.c_void_p]),
    ("trident_app_append_mesh", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, _f3, C.c_float,
                                          C.c_float, C.c_char_p, C.POINTER(C.c_uint32)]),
    ("trident_app_upload_texture", C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("trident_app_add_mesh_entity", C.c_int, [C.c_void_p, C.c_int, C.c_uint32, _f3, _f3, _f3, C.POINTER(C.c_uint32)]),
    ("trident_app_set_entity_texture", C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p]),
    ("trident_app_set_entity_transform", C.c_int, [C.c_void_p, C.c_uint32, _f3, _f3, _f3]),
    ("trident_app_set_entity_visible", C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    ("trident_app_set_entity_bones", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    ("trident_app_set_assets_dir", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_uint32]),
    ("trident_app_viewport_texture", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(abi.TriImage)]),
    ("trident_app_set_light_shadow_caster", C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    ("trident_app_set_shadow_map_size", C.c_int, [C.c_void_p, C.c_uint32]),
    ("trident_app_set_device_count", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    ("trident_app_add_sprite_entity", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                C.c_void_p, C.c_float, C.POINTER(C.c_uint32)]),
    ("trident_app_set_sprite_visible", C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    ("trident_app_entity_sprite", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_float * 10)]),
    ("trident_app_shadow_config", C.c_int, [C.c_void_p, C.POINTER(abi.TriShadowConfig), C.POINTER(C.c_int)]),
    ("trident_app_geometry_uploads", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    ("trident_load_image", C.c_int, [C.c_char_p, C.c_int, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32)]),
    ("trident_load_default_skybox", C.c_int, [C.c_char_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_char_p,
                                              C.c_uint32]),
    ("trident_app_add_light", C.c_int, [C.c_void_p, C.c_int, _f3, _f3, _f3, C.c_float, C.c_float, C.c_int,
                                        C.POINTER(C.c_uint32)]),
    ("trident_app_set_camera", C.c_int, [C.c_void_p, C.c_int, _f3, _f3, C.c_float, C.c_float, C.c_float, C.c_int]),
    ("trident_app_set_viewport", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("trident_app_set_clear_color", C.c_int, [C.c_void_p, _f3]),
    ("trident_app_set_skybox", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("trident_app_draw_frame", C.c_int, [C.c_void_p]),
    ("trident_app_finish_frame", C.c_int, [C.c_void_p]),
    ("trident_app_set_frames_in_flight", C.c_int, [C.c_void_p, C.c_uint32]),
    ("trident_app_read_pixels", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("trident_app_frame_inputs", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(abi.TriGlobalUbo), C.c_void_p, C.c_uint32,
                                           C.POINTER(C.c_uint32)]),
    ("trident_app_geometry", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_size_t), C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("trident_app_materials", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("trident_app_frame_timing", C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    ("trident_app_import_model", C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("trident_app_save_scene", C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p]),
    ("trident_app_load_scene", C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint32)]),
    ("trident_app_use_scene_camera", C.c_int, [C.c_void_p]),
    ("trident_app_entity_transform", C.c_int, [C.c_void_p, C.c_uint32, _f3]),
    ("trident_app_entity_mesh", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]),
    ("trident_app_entity_count", C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    ("trident_app_set_present_extent", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    ("trident_app_set_ai_blend_strength", C.c_int, [C.c_void_p, C.c_float]),
    ("trident_app_submit_ai_frame", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("trident_app_read_present", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]),
]

_lib = None


def load_library(path=LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"Trident renderer shim not built: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, res, args in _APP_FUNCTIONS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc, what):
    if rc != abi.TRI_OK:
        raise TriError(rc, what)


def _vec(v):
    return None if v is None else (C.c_float * len(v))(*[float(x) for x in v])


class TridentApp:
    """One Renderer + ECS registry + editor/runtime cameras (Forge's ApplicationLayer, reduced)."""

    def __init__(self, raster_flags=0):
        self._lib = load_library()
        h = C.c_void_p()
        _check(self._lib.trident_app_create(raster_flags, C.byref(h)), "trident_app_create")
        self._h = h

    def close(self):
        if self._h:
            self._lib.trident_app_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def append_mesh(self, vertices, indices, base_color=(1, 1, 1, 1), metallic=1.0, roughness=1.0, texture=None):
        v = np.ascontiguousarray(vertices, abi.VERTEX_DTYPE)
        i = np.ascontiguousarray(indices, np.uint32)
        out = C.c_uint32()
        _check(self._lib.trident_app_append_mesh(self._h, v.ctypes.data, v.shape[0], i.ctypes.data, i.size,
                                                 _vec(base_color), metallic, roughness,
                                                 texture.encode() if texture else None, C.byref(out)),
               "append_mesh")
        return out.value

    def upload_texture(self, path, rgba):
        rgba = np.ascontiguousarray(rgba, np.uint8)
        _check(self._lib.trident_app_upload_texture(self._h, path.encode(), rgba.ctypes.data, rgba.shape[1],
                                                    rgba.shape[0]), "upload_texture")

    def add_mesh_entity(self, primitive="none", mesh_index=0, position=(0, 0, 0), rotation=(0, 0, 0), scale=(1, 1, 1)):
        e = C.c_uint32()
        _check(self._lib.trident_app_add_mesh_entity(self._h, PRIMITIVE[primitive], mesh_index, _vec(position),
                                                     _vec(rotation), _vec(scale), C.byref(e)), "add_mesh_entity")
        return e.value

    def add_sprite_entity(self, position=(0, 0, 0), rotation=(0, 0, 0), scale=(1, 1, 1), tint=(1, 1, 1, 1),
                          uv_scale=(1, 1), uv_offset=(0, 0), tiling=1.0):
        """Transform + SpriteComponent (drawn after the meshes, Renderer.cpp:2996-3089)."""
        f = lambda v: (C.c_float * len(v))(*[float(x) for x in v])  # noqa: E731
        e = C.c_uint32()
        _check(self._lib.trident_app_add_sprite_entity(self._h, f(position), f(rotation), f(scale), f(tint), f(uv_scale),
                                                       f(uv_offset), float(tiling), C.byref(e)), "add_sprite_entity")
        return e.value

    def set_sprite_visible(self, entity, visible):
        _check(self._lib.trident_app_set_sprite_visible(self._h, entity, 1 if visible else 0), "set_sprite_visible")

    def entity_sprite(self, entity):
        """SpriteComponent: {tint, uv_scale, uv_offset, tiling, visible}, or None."""
        out = (C.c_float * 10)()
        if self._lib.trident_app_entity_sprite(self._h, entity, C.byref(out)) != 0:
            return None
        v = list(out)
        return {"tint": tuple(v[0:4]), "uv_scale": tuple(v[4:6]), "uv_offset": tuple(v[6:8]), "tiling": v[8],
                "visible": bool(v[9])}

    def set_entity_texture(self, entity, path):
        _check(self._lib.trident_app_set_entity_texture(self._h, entity, path.encode()), "set_entity_texture")

    def set_entity_transform(self, entity, position=None, rotation=None, scale=None):
        _check(self._lib.trident_app_set_entity_transform(self._h, entity, _vec(position), _vec(rotation), _vec(scale)),
               "set_entity_transform")

    def set_entity_visible(self, entity, visible):
        _check(self._lib.trident_app_set_entity_visible(self._h, entity, 1 if visible else 0), "set_entity_visible")

    def set_assets_dir(self, directory):
        """Renderer::SetAssetsDirectory (skybox discovery under directory/Skyboxes); returns the source."""
        buf = C.create_string_buffer(64)
        _check(self._lib.trident_app_set_assets_dir(self._h, os.fsencode(directory), buf, 64), "set_assets_dir")
        return buf.value.decode()

    def set_light_shadow_caster(self, entity, caster=True):
        _check(self._lib.trident_app_set_light_shadow_caster(self._h, entity, 1 if caster else 0), "shadow caster")

    def set_shadow_map_size(self, size):
        _check(self._lib.trident_app_set_shadow_map_size(self._h, size), "shadow map size")

    def set_device_count(self, count, devices=None):
        """Renderer::SetDeviceCount: viewports as `count` row bands on `devices` (tri_group), count <= 1: one context."""
        arr = (C.c_int32 * len(devices))(*devices) if devices else None
        _check(self._lib.trident_app_set_device_count(self._h, count, arr), "device count")

    def shadow_config(self):
        """The pre-pass configuration DrawFrame would use now (abi.TriShadowConfig), or None."""
        cfg, on = abi.TriShadowConfig(), C.c_int()
        _check(self._lib.trident_app_shadow_config(self._h, C.byref(cfg), C.byref(on)), "shadow_config")
        return cfg if on.value else None

    def viewport_texture(self, viewport_id):
        """Renderer::GetViewportTexture: the viewport's abi.TriImage handle."""
        img = abi.TriImage()
        _check(self._lib.trident_app_viewport_texture(self._h, viewport_id, C.byref(img)), "viewport_texture")
        return img

    def geometry_uploads(self):
        n = C.c_uint64()
        _check(self._lib.trident_app_geometry_uploads(self._h, C.byref(n)), "geometry_uploads")
        return n.value

    def set_entity_bones(self, entity, matrices):
        """AnimationComponent::m_BoneMatrices: float32 [n, 4, 4] column-major mat4s (m[col][row])."""
        m = np.ascontiguousarray(matrices, dtype=np.float32).reshape(-1, 16)
        _check(self._lib.trident_app_set_entity_bones(self._h, entity, m.ctypes.data if m.size else None,
                                                      m.shape[0]), "set_entity_bones")

    def add_light(self, type, position=(0, 0, 0), direction=(-0.5, -1.0, -0.3), color=(1.0, 0.98, 0.92),
                  intensity=5.0, range=10.0, enabled=True):
        e = C.c_uint32()
        _check(self._lib.trident_app_add_light(self._h, LIGHT[type], _vec(position), _vec(direction), _vec(color),
                                               intensity, range, 1 if enabled else 0, C.byref(e)), "add_light")
        return e.value

    def set_camera(self, which, position, rotation=(0, 0, 0), fov=60.0, near=0.1, far=1000.0, ready=True):
        _check(self._lib.trident_app_set_camera(self._h, {"editor": 0, "runtime": 1}[which], _vec(position),
                                                _vec(rotation), fov, near, far, 1 if ready else 0), "set_camera")

    def set_viewport(self, viewport_id, width, height):
        _check(self._lib.trident_app_set_viewport(self._h, viewport_id, width, height), "set_viewport")

    def set_clear_color(self, rgba):
        _check(self._lib.trident_app_set_clear_color(self._h, _vec(rgba)), "set_clear_color")

    def set_skybox(self, faces):
        f = np.ascontiguousarray(faces, np.uint8)
        _check(self._lib.trident_app_set_skybox(self._h, f.ctypes.data, f.shape[1]), "set_skybox")

    def draw_frame(self):
        _check(self._lib.trident_app_draw_frame(self._h), "draw_frame")

    def set_frames_in_flight(self, n):
        """Renderer::SetFramesInFlight (1 = the reference's pacing: DrawFrame waits for the previous frame)."""
        _check(self._lib.trident_app_set_frames_in_flight(self._h, n), "set_frames_in_flight")

    def finish_frame(self):
        """Wait for the last draw_frame's frame (Renderer::FinishFrame; the next draw_frame does it first)."""
        _check(self._lib.trident_app_finish_frame(self._h), "finish_frame")

    def read_pixels(self, viewport_id, width, height, depth=True):
        rgba = np.zeros((height, width, 4), np.uint8)
        d = np.zeros((height, width), np.float32) if depth else None
        _check(self._lib.trident_app_read_pixels(self._h, viewport_id, rgba.ctypes.data,
                                                 d.ctypes.data if depth else None), "read_pixels")
        return rgba, d

    def frame_inputs(self, viewport_id, capacity=4096):
        ubo = abi.TriGlobalUbo()
        draws = (abi.TriDraw * capacity)()
        n = C.c_uint32()
        _check(self._lib.trident_app_frame_inputs(self._h, viewport_id, C.byref(ubo), draws, capacity, C.byref(n)),
               "frame_inputs")
        return ubo, list(draws[: n.value])

    def geometry(self, capacity=4096):
        vp, ip = C.c_void_p(), C.c_void_p()
        nv, ni = C.c_size_t(), C.c_size_t()
        ranges = np.zeros(capacity, abi.MESH_RANGE_DTYPE)
        nr = C.c_uint32()
        _check(self._lib.trident_app_geometry(self._h, C.byref(vp), C.byref(nv), C.byref(ip), C.byref(ni),
                                              ranges.ctypes.data, capacity, C.byref(nr)), "geometry")
        vb = np.frombuffer((C.c_uint8 * (nv.value * abi.VERTEX_DTYPE.itemsize)).from_address(vp.value),
                           abi.VERTEX_DTYPE).copy() if nv.value else np.zeros(0, abi.VERTEX_DTYPE)
        ib = np.ctypeslib.as_array((C.c_uint32 * ni.value).from_address(ip.value)).copy() if ni.value else \
            np.zeros(0, np.uint32)
        return vb, ib, ranges[: nr.value].copy()

    def materials(self, capacity=1024):
        recs = (abi.TriMaterialRecord * capacity)()
        n = C.c_uint32()
        _check(self._lib.trident_app_materials(self._h, recs, capacity, C.byref(n)), "materials")
        return [(tuple(r.base_color_factor), tuple(r.material_factors)) for r in recs[: n.value]]

    def frame_timing(self):
        out = (C.c_double * 7)()
        _check(self._lib.trident_app_frame_timing(self._h, out), "frame_timing")
        keys = ("min_ms", "max_ms", "avg_ms", "min_fps", "max_fps", "avg_fps", "samples")
        return dict(zip(keys, list(out)))

    # ---- ingestion: ModelLoader + .trident scenes ----
    def import_model(self, path, capacity=4096):
        ents = (C.c_uint32 * capacity)()
        n = C.c_uint32()
        _check(self._lib.trident_app_import_model(self._h, str(path).encode(), ents, capacity, C.byref(n)),
               f"import_model({path})")
        return list(ents[: min(n.value, capacity)])

    def save_scene(self, path, name="Untitled"):
        _check(self._lib.trident_app_save_scene(self._h, str(path).encode(), name.encode()), "save_scene")

    def load_scene(self, path):
        n = C.c_uint32()
        _check(self._lib.trident_app_load_scene(self._h, str(path).encode(), C.byref(n)), f"load_scene({path})")
        return n.value

    def use_scene_camera(self):
        _check(self._lib.trident_app_use_scene_camera(self._h), "use_scene_camera")

    def entity_transform(self, entity):
        out = (C.c_float * 9)()
        _check(self._lib.trident_app_entity_transform(self._h, entity, out), "entity_transform")
        v = list(out)
        return tuple(v[0:3]), tuple(v[3:6]), tuple(v[6:9])

    def entity_mesh(self, entity):
        out = (C.c_uint64 * 3)()
        _check(self._lib.trident_app_entity_mesh(self._h, entity, out), "entity_mesh")
        return {"mesh_index": out[0], "primitive": out[1], "source_mesh_index": out[2]}

    def entity_count(self):
        n = C.c_uint32()
        _check(self._lib.trident_app_entity_count(self._h, C.byref(n)), "entity_count")
        return n.value

    # ---- presentation: active viewport -> swapchain-sized image ----
    def set_present_extent(self, width, height):
        _check(self._lib.trident_app_set_present_extent(self._h, width, height), "set_present_extent")

    # ---- Default.frag's AI frame blend (SetAiBlendStrength / UploadAiInterpolationToGpu) ----
    def set_ai_blend_strength(self, strength):
        _check(self._lib.trident_app_set_ai_blend_strength(self._h, strength), "set_ai_blend_strength")

    def submit_ai_frame(self, pixels):
        """pixels: float32 [h, w, channels] in [0, 1] (the frame generator's output), or None to drop it."""
        if pixels is None:
            _check(self._lib.trident_app_submit_ai_frame(self._h, None, 0, 0, 0), "submit_ai_frame")
            return
        p = np.ascontiguousarray(pixels, np.float32)
        _check(self._lib.trident_app_submit_ai_frame(self._h, p.ctypes.data, p.shape[1], p.shape[0], p.shape[2]),
               "submit_ai_frame")

    def read_present(self, width, height):
        out = np.zeros((height, width, 4), np.uint8)
        _check(self._lib.trident_app_read_present(self._h, out.ctypes.data, width, height), "read_present")
        return out



def load_image(path, flip=True):
    """TextureLoader::Load (flip=True, 2D textures) or one cube face (flip=False): uint8 [h, w, 4] RGBA."""
    lib = load_library()
    w, h = C.c_uint32(), C.c_uint32()
    _check(lib.trident_load_image(os.fsencode(path), 1 if flip else 0, None, 0, C.byref(w), C.byref(h)), "load_image")
    out = np.empty((h.value, w.value, 4), np.uint8)
    _check(lib.trident_load_image(os.fsencode(path), 1 if flip else 0, out.ctypes.data, out.nbytes, C.byref(w),
                                  C.byref(h)), "load_image")
    return out


def load_default_skybox(assets_dir):
    """DiscoverDefaultSkybox (Renderer.cpp:3830-3927): (faces uint8 [6, n, n, 4] or None, source)."""
    lib = load_library()
    n = C.c_uint32()
    src = C.create_string_buffer(64)
    _check(lib.trident_load_default_skybox(os.fsencode(assets_dir), None, 0, C.byref(n), src, 64), "load_default_skybox")
    if n.value == 0:
        return None, src.value.decode()
    faces = np.empty((6, n.value, n.value, 4), np.uint8)
    _check(lib.trident_load_default_skybox(os.fsencode(assets_dir), faces.ctypes.data, faces.nbytes, C.byref(n), src, 64),
           "load_default_skybox")
    return faces, src.value.decode()
