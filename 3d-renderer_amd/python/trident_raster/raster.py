"""Python binding of the product C-ABI (libtri_raster.so, include/tri_raster.h).

This is plumbing for tests and bench.py: every call goes straight to the HIP library. There is no
CPU fallback — if the in-tree library is missing, import fails loudly.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.normpath(os.path.join(_HERE, "..", ".."))
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libtri_raster.so")

_lib = None


class TriError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"tri_raster error {code}: {msg}")
        self.code = code


def load_library(path=None):
    """Load the HIP rasterizer library (built by `make -C 3d-renderer_amd`). TRI_RASTER_LIB may name
    another in-tree build of the same library (kernel-variant experiments)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("TRI_RASTER_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"HIP rasterizer library not built: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    variant = os.path.abspath(path) != os.path.abspath(LIB_PATH)
    for name, res, args in abi.CABI_FUNCTIONS:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if not variant:  # the product library exports every entry point include/tri_raster.h declares
                raise
            continue  # an older A/B variant: entry points added since are absent there
        fn.restype = res
        fn.argtypes = args
    if lib.tri_abi_version() != abi.TRI_RASTER_ABI_VERSION:
        raise ImportError(f"tri_raster ABI version {lib.tri_abi_version()}, binding expects {abi.TRI_RASTER_ABI_VERSION}")
    _lib = lib
    return lib


def _check(rc):
    if rc != abi.TRI_OK:
        msg = _lib.tri_last_error().decode(errors="replace")
        raise TriError(rc, msg)


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


def shadow_fit_ortho(light_dir, aabb_min, aabb_max):
    """tri_shadow_fit_ortho (host-only): column-major light ortho * light view, as numpy [col][row]."""
    lib = load_library()
    f3 = lambda v: (C.c_float * 3)(*[float(x) for x in v])  # noqa: E731
    out = (C.c_float * 16)()
    _check(lib.tri_shadow_fit_ortho(C.byref(f3(light_dir)), C.byref(f3(aabb_min)), C.byref(f3(aabb_max)),
                                    C.byref(out)))
    return np.array(out[:], np.float32).reshape(4, 4)


class TriRaster:
    """One tri_ctx: a W x H framebuffer (optionally a row band) on one HIP device."""

    def __init__(self, width, height, band=None, device=-1, flags=0):
        lib = load_library()
        cfg = abi.TriConfig()
        cfg.width, cfg.height = width, height
        cfg.band_y0, cfg.band_y1 = band if band is not None else (0, 0)
        cfg.device = device
        cfg.flags = flags
        ctx = C.c_void_p()
        _check(lib.tri_create(C.byref(cfg), C.byref(ctx)))
        self._ctx = ctx
        self.width, self.height = width, height
        self.band = band if band is not None else (0, height)
        self.rows = self.band[1] - self.band[0]

    def close(self):
        if self._ctx:
            _lib.tri_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- uploads ----
    def upload_geometry(self, vertices, indices, meshes):
        v = np.ascontiguousarray(vertices, dtype=abi.VERTEX_DTYPE)
        i = np.ascontiguousarray(indices, dtype=np.uint32)
        m = np.ascontiguousarray(meshes, dtype=abi.MESH_RANGE_DTYPE)
        _check(_lib.tri_upload_geometry(self._ctx, _ptr(v), v.size, _ptr(i), i.size, _ptr(m), m.size))

    def upload_materials(self, records):
        n = len(records)
        arr = (abi.TriMaterialRecord * max(n, 1))()
        for k, (base, factors) in enumerate(records):
            arr[k].base_color_factor = (C.c_float * 4)(*base)
            arr[k].material_factors = (C.c_float * 4)(*factors)
        _check(_lib.tri_upload_materials(self._ctx, arr, n))

    def upload_texture(self, slot, rgba8):
        t = np.ascontiguousarray(rgba8, dtype=np.uint8)
        assert t.ndim == 3 and t.shape[2] == 4
        _check(_lib.tri_upload_texture(self._ctx, slot, _ptr(t), t.shape[1], t.shape[0]))

    def upload_bone_palette(self, mats):
        m = np.ascontiguousarray(mats, dtype=np.float32).reshape(-1, 16)
        _check(_lib.tri_upload_bone_palette(self._ctx, _ptr(m), m.shape[0]))

    def upload_ai_frame(self, rgba):
        """rgba: uint8 [h, w, 4] R8G8B8A8_UNORM AI frame (Default.frag's blend), or None to remove it."""
        if rgba is None:
            _check(_lib.tri_upload_ai_frame(self._ctx, None, 0, 0))
            return
        f = np.ascontiguousarray(rgba, dtype=np.uint8)
        if f.ndim != 3 or f.shape[2] != 4:
            raise ValueError("AI frame must be uint8 [h, w, 4]")
        _check(_lib.tri_upload_ai_frame(self._ctx, _ptr(f), f.shape[1], f.shape[0]))

    def upload_skybox(self, faces):
        """faces: uint8 [6, n, n, 4] sRGB (+X,-X,+Y,-Y,+Z,-Z), or None to remove the skybox."""
        if faces is None:
            _check(_lib.tri_upload_skybox(self._ctx, None, 0))
            return
        f = np.ascontiguousarray(faces, dtype=np.uint8)
        if f.ndim != 4 or f.shape[0] != 6 or f.shape[1] != f.shape[2] or f.shape[3] != 4:
            raise ValueError("skybox faces must be uint8 [6, n, n, 4]")
        _check(_lib.tri_upload_skybox(self._ctx, _ptr(f), f.shape[1]))

    def set_shadow(self, cfg):
        """tri_set_shadow: an abi.TriShadowConfig, or None to switch the shadow pre-pass off."""
        _check(_lib.tri_set_shadow(self._ctx, C.byref(cfg) if cfg is not None else None))
        self._shadow_size = int(cfg.size) if cfg is not None else 0

    def read_shadow_map(self):
        out = np.empty((self._shadow_size, self._shadow_size), np.uint32)
        _check(_lib.tri_read_shadow_map(self._ctx, _ptr(out)))
        return out

    # ---- frame ----
    def set_frame(self, ubo, clear=(0.005, 0.005, 0.005, 1.0)):
        cl = (C.c_float * 4)(*clear)
        _check(_lib.tri_set_frame(self._ctx, C.byref(ubo), C.byref(cl)))

    def set_draws(self, draws):
        arr, n = abi.draws_array(draws)
        _check(_lib.tri_set_draws(self._ctx, arr, n))

    def set_stream(self, stream_ptr):
        _check(_lib.tri_set_stream(self._ctx, C.c_void_p(stream_ptr) if stream_ptr else None))

    def frame_alpha(self):
        """tri_frame_alpha: the alpha byte every pixel of the next frame has, or -1 if not provably uniform."""
        a = C.c_int32()
        _check(_lib.tri_frame_alpha(self._ctx, C.byref(a)))
        return a.value

    def bind_geometry(self, geometry):
        """tri_bind_geometry: reference a shared TriGeometry (None: back to the context's own)."""
        _check(_lib.tri_bind_geometry(self._ctx, geometry._g if geometry is not None else None))

    def output_image(self):
        img = abi.TriImage()
        _check(_lib.tri_get_output(self._ctx, C.byref(img)))
        return img

    def bind_output(self, color_ptr, depth_ptr):
        _check(_lib.tri_bind_output(self._ctx, C.c_void_p(color_ptr) if color_ptr else None,
                                    C.c_void_p(depth_ptr) if depth_ptr else None))

    def render(self):
        _check(_lib.tri_render(self._ctx))

    def synchronize(self):
        _check(_lib.tri_synchronize(self._ctx))

    def readback(self, depth=True):
        """Returns (bgra uint8 [rows, W, 4], depth uint32 bits [rows, W] or None)."""
        col = np.empty((self.rows, self.width, 4), dtype=np.uint8)
        dep = np.empty((self.rows, self.width), dtype=np.uint32) if depth else None
        _check(_lib.tri_readback(self._ctx, _ptr(col), _ptr(dep) if depth else None))
        return col, dep

    def blit(self, width, height, dst_ptr=None):
        """tri_blit_linear: scale the frame to width x height (VK_FILTER_LINEAR presentation blit)."""
        _check(_lib.tri_blit_linear(self._ctx, C.c_void_p(dst_ptr) if dst_ptr else None, width, height))
        self._present = None if dst_ptr else (width, height)  # a caller-owned dst leaves the owned target stale

    def read_present(self):
        w, h = getattr(self, "_present", None) or (1, 1)  # nothing owned to read: the library reports TRI_E_STATE
        out = np.empty((h, w, 4), dtype=np.uint8)
        _check(_lib.tri_read_present(self._ctx, _ptr(out)))
        return out

    def render_frame(self, retries=2):
        """render + synchronize, re-rendering once after an internal-buffer overflow (buffers grow)."""
        for attempt in range(retries + 1):
            self.render()
            try:
                self.synchronize()
                return
            except TriError as e:
                if e.code != abi.TRI_E_OVERFLOW or attempt == retries:
                    raise

    def set_timing(self, enable, period=1):
        """Per-stage HIP-event timing of every `period`-th frame (enable=False: off)."""
        _check(_lib.tri_set_timing(self._ctx, int(period) if enable else 0))

    def timing(self):
        t = abi.TriTiming()
        _check(_lib.tri_get_timing(self._ctx, C.byref(t)))
        return {k: getattr(t, k) for k, _ in abi.TriTiming._fields_}

    def frame_stats(self):
        s = abi.TriFrameStats()
        _check(_lib.tri_get_frame_stats(self._ctx, C.byref(s)))
        return {k: getattr(s, k) for k, _ in abi.TriFrameStats._fields_}


class TriGeometry:
    """tri_geometry: meshes uploaded once on one device, bound by any number of contexts there."""

    def __init__(self, device=-1):
        lib = load_library()
        g = C.c_void_p()
        _check(lib.tri_geometry_create(device, C.byref(g)))
        self._g = g

    def upload(self, vertices, indices, meshes):
        v = np.ascontiguousarray(vertices, dtype=abi.VERTEX_DTYPE)
        i = np.ascontiguousarray(indices, dtype=np.uint32)
        m = np.ascontiguousarray(meshes, dtype=abi.MESH_RANGE_DTYPE)
        _check(_lib.tri_geometry_upload(self._g, _ptr(v), v.size, _ptr(i), i.size, _ptr(m), m.size))

    def close(self):
        if self._g:
            _lib.tri_geometry_destroy(self._g)
            self._g = None


def pack_bgr24(src_ptr, dst_ptr, pixels, alpha, flag_ptr=None, stream_ptr=None):
    """tri_pack_bgr24: B8G8R8A8 -> 3-byte BGR on the device, stream-ordered (flag: device uint32 set when an
    alpha byte differs from `alpha`)."""
    load_library()
    _check(_lib.tri_pack_bgr24(C.c_void_p(src_ptr), C.c_void_p(dst_ptr), pixels, alpha,
                               C.c_void_p(flag_ptr) if flag_ptr else None, C.c_void_p(stream_ptr) if stream_ptr else None))


def unpack_bgr24(src_ptr, dst_ptr, pixels, alpha, stream_ptr=None):
    """tri_unpack_bgr24: 3-byte BGR -> B8G8R8A8 with the given alpha, stream-ordered."""
    load_library()
    _check(_lib.tri_unpack_bgr24(C.c_void_p(src_ptr), C.c_void_p(dst_ptr), pixels, alpha,
                                 C.c_void_p(stream_ptr) if stream_ptr else None))


def dbp_pack(src_ptr, pixels, alpha, dst_ptr, slot_bytes, flags_ptr=None, stream_ptr=None):
    """tri_dbp_pack: B8G8R8A8 -> the delta bit-plane stream (slots of slot_bytes), stream-ordered; flags: device
    uint32[2] (bit 1 alpha mismatch, bit 2 slot overflow; the largest slot's bytes)."""
    load_library()
    _check(_lib.tri_dbp_pack(C.c_void_p(src_ptr), pixels, alpha, C.c_void_p(dst_ptr), slot_bytes,
                             C.c_void_p(flags_ptr) if flags_ptr else None, C.c_void_p(stream_ptr) if stream_ptr else None))


def dbp_unpack(src_ptr, pixels, alpha, slot_bytes, dst_ptr, stream_ptr=None):
    """tri_dbp_unpack: the delta bit-plane stream -> B8G8R8A8 with the given alpha, stream-ordered."""
    load_library()
    _check(_lib.tri_dbp_unpack(C.c_void_p(src_ptr), pixels, alpha, slot_bytes, C.c_void_p(dst_ptr),
                               C.c_void_p(stream_ptr) if stream_ptr else None))


def dbp_unpack_bands(src_ptrs, dst_ptrs, pixels, alpha, slot_bytes, stream_ptr=None):
    """tri_dbp_unpack_bands: several delta bit-plane streams (one slot size) -> their B8G8R8A8 bands, one launch."""
    load_library()
    k = len(src_ptrs)
    srcs = (C.c_void_p * max(k, 1))(*src_ptrs)
    dsts = (C.c_void_p * max(k, 1))(*dst_ptrs)
    npx = (C.c_uint64 * max(k, 1))(*pixels)
    _check(_lib.tri_dbp_unpack_bands(srcs, dsts, npx, k, alpha, slot_bytes, C.c_void_p(stream_ptr) if stream_ptr else None))


def dbp_bytes(pixels, slot_bytes):
    load_library()
    return int(_lib.tri_dbp_bytes(pixels, slot_bytes))


def copy_device_to_host(ptr, nbytes, device=0):
    """hipMemcpy of `nbytes` at a device pointer (a tri_image handle) into a numpy byte array."""
    hip = C.CDLL("libamdhip64.so")
    hip.hipSetDevice.argtypes = [C.c_int]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    out = np.empty(nbytes, np.uint8)
    assert hip.hipSetDevice(device) == 0
    assert hip.hipMemcpy(out.ctypes.data, C.c_void_p(ptr), nbytes, 2) == 0  # hipMemcpyDeviceToHost
    return out


class TriGroup:
    """tri_group: one frame over N row-band contexts on the given devices (RCCL gather onto the display
    band's device; bands sharing that device render in place)."""

    def __init__(self, width, height, devices, display=0, flags=0, group_flags=0):
        lib = load_library()
        n = len(devices)
        self._devs = (C.c_int32 * n)(*devices)
        cfg = abi.TriGroupConfig(width, height, n, display, self._devs, flags, group_flags)
        g = C.c_void_p()
        _check(lib.tri_group_create(C.byref(cfg), C.byref(g)))
        self._g = g
        self.width, self.height, self.n = width, height, n

    def close(self):
        if self._g:
            _lib.tri_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def upload_geometry(self, vertices, indices, meshes):
        v = np.ascontiguousarray(vertices, dtype=abi.VERTEX_DTYPE)
        i = np.ascontiguousarray(indices, dtype=np.uint32)
        m = np.ascontiguousarray(meshes, dtype=abi.MESH_RANGE_DTYPE)
        _check(_lib.tri_group_upload_geometry(self._g, _ptr(v), v.size, _ptr(i), i.size, _ptr(m), m.size))

    def upload_materials(self, records):
        n = len(records)
        arr = (abi.TriMaterialRecord * max(n, 1))()
        for k, (base, factors) in enumerate(records):
            arr[k].base_color_factor = (C.c_float * 4)(*base)
            arr[k].material_factors = (C.c_float * 4)(*factors)
        _check(_lib.tri_group_upload_materials(self._g, arr, n))

    def upload_texture(self, slot, rgba8):
        t = np.ascontiguousarray(rgba8, dtype=np.uint8)
        _check(_lib.tri_group_upload_texture(self._g, slot, _ptr(t), t.shape[1], t.shape[0]))

    def upload_bone_palette(self, mats):
        m = np.ascontiguousarray(mats, dtype=np.float32).reshape(-1, 16)
        _check(_lib.tri_group_upload_bone_palette(self._g, _ptr(m), m.shape[0]))

    def upload_ai_frame(self, rgba):
        if rgba is None:
            _check(_lib.tri_group_upload_ai_frame(self._g, None, 0, 0))
            return
        f = np.ascontiguousarray(rgba, dtype=np.uint8)
        _check(_lib.tri_group_upload_ai_frame(self._g, _ptr(f), f.shape[1], f.shape[0]))

    def upload_skybox(self, faces):
        if faces is None:
            _check(_lib.tri_group_upload_skybox(self._g, None, 0))
            return
        f = np.ascontiguousarray(faces, dtype=np.uint8)
        _check(_lib.tri_group_upload_skybox(self._g, _ptr(f), f.shape[1]))

    def set_shadow(self, cfg):
        _check(_lib.tri_group_set_shadow(self._g, C.byref(cfg) if cfg is not None else None))

    def set_frame(self, ubo, clear=(0.005, 0.005, 0.005, 1.0)):
        cl = (C.c_float * 4)(*clear)
        _check(_lib.tri_group_set_frame(self._g, C.byref(ubo), C.byref(cl)))

    def set_draws(self, draws):
        arr, n = abi.draws_array(draws)
        _check(_lib.tri_group_set_draws(self._g, arr, n))

    def render(self):
        _check(_lib.tri_group_render(self._g))

    def synchronize(self):
        _check(_lib.tri_group_synchronize(self._g))

    def render_frame(self, retries=2):
        for attempt in range(retries + 1):
            self.render()
            try:
                self.synchronize()
                return
            except TriError as e:
                if e.code != abi.TRI_E_OVERFLOW or attempt == retries:
                    raise

    def readback(self, depth=True):
        col = np.empty((self.height, self.width, 4), dtype=np.uint8)
        dep = np.empty((self.height, self.width), dtype=np.uint32) if depth else None
        _check(_lib.tri_group_readback(self._g, _ptr(col), _ptr(dep) if depth else None))
        return col, dep

    def frame_pointer(self):
        p, d = C.c_void_p(), C.c_int32()
        _check(_lib.tri_group_frame(self._g, C.byref(p), C.byref(d)))
        return p.value, d.value

    def output_image(self):
        img = abi.TriImage()
        _check(_lib.tri_group_get_output(self._g, C.byref(img)))
        return img

    def present(self, stream_ptr=None):
        """tri_group_present: the consumer fence on the most recent frame (after `stream_ptr`'s work, or now)."""
        _check(_lib.tri_group_present(self._g, C.c_void_p(stream_ptr) if stream_ptr else None))

    def bind_geometry(self, geometries):
        """tri_group_bind_geometry: caller-owned TriGeometry objects (one per device); [] = the group's own."""
        arr = (C.c_void_p * max(len(geometries), 1))(*[g._g.value for g in geometries])
        _check(_lib.tri_group_bind_geometry(self._g, len(geometries), arr))

    def context(self, band):
        """The band's tri_ctx handle (tri_group_context)."""
        c = C.c_void_p()
        _check(_lib.tri_group_context(self._g, band, C.byref(c)))
        return c

    def blit(self, width, height, dst_ptr=None):
        _check(_lib.tri_group_blit_linear(self._g, C.c_void_p(dst_ptr) if dst_ptr else None, width, height))
        self._present = None if dst_ptr else (width, height)

    def read_present(self):
        w, h = getattr(self, "_present", None) or (1, 1)  # nothing owned to read: the library reports TRI_E_STATE
        out = np.empty((h, w, 4), dtype=np.uint8)
        _check(_lib.tri_group_read_present(self._g, _ptr(out)))
        return out

    def transfer_info(self):
        """tri_group_transfer_info: (bytes per pixel on the links, inbound RCCL bytes) of the last frame."""
        bpp, inbound = C.c_uint32(), C.c_uint64()
        _check(_lib.tri_group_transfer_info(self._g, C.byref(bpp), C.byref(inbound)))
        return bpp.value, inbound.value

    def transfer_format(self):
        """tri_group_transfer_format: (TRI_GROUP_FMT_*, dbp slot bytes or 0) of the last frame."""
        fmt, slot = C.c_uint32(), C.c_uint32()
        _check(_lib.tri_group_transfer_format(self._g, C.byref(fmt), C.byref(slot)))
        return fmt.value, slot.value
