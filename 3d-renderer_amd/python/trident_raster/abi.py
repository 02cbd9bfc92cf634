"""ctypes / numpy mirrors of include/tri_raster.h (the C-ABI boundary).

Struct layouts are byte-identical to the reference's GPU ABI structs:
Vertex (Trident/src/Renderer/Vertex.h:9-78, 100 B), RenderablePushConstant (RenderData.h:14-30,
128 B), GlobalUniformBuffer (UniformBuffer.h:17-28, 480 B), MaterialUniformBuffer (32 B),
MeshDrawInfo (Renderer.h:293-299).
"""
import ctypes as C

import numpy as np

TRI_RASTER_ABI_VERSION = 2  # include/tri_raster.h

TRI_OK = 0
TRI_E_INVALID = -1
TRI_E_HIP = -2
TRI_E_OOM = -3
TRI_E_OVERFLOW = -4
TRI_E_UNSUPPORTED = -5
TRI_E_STATE = -6
TRI_E_TIMEOUT = -7

TRI_MAX_POINT_LIGHTS = 8
TRI_MAX_TEXTURE_SLOTS = 256
TRI_FLAG_NO_DEPTH_OUTPUT = 0x1
TRI_FLAG_EXACT_SHADING = 0x2
TRI_FLAG_CLUSTER_CULL = 0x4

VERTEX_DTYPE = np.dtype(
    [
        ("position", "<f4", 3),
        ("normal", "<f4", 3),
        ("tangent", "<f4", 3),
        ("bitangent", "<f4", 3),
        ("color", "<f4", 3),
        ("texcoord", "<f4", 2),
        ("bone_indices", "<i4", 4),
        ("bone_weights", "<f4", 4),
    ]
)
assert VERTEX_DTYPE.itemsize == 100

MESH_RANGE_DTYPE = np.dtype(
    [("first_index", "<u4"), ("index_count", "<u4"), ("base_vertex", "<i4"), ("material_index", "<i4")]
)


class TriVertex(C.Structure):
    _fields_ = [
        ("position", C.c_float * 3),
        ("normal", C.c_float * 3),
        ("tangent", C.c_float * 3),
        ("bitangent", C.c_float * 3),
        ("color", C.c_float * 3),
        ("texcoord", C.c_float * 2),
        ("bone_indices", C.c_int32 * 4),
        ("bone_weights", C.c_float * 4),
    ]


class TriMeshRange(C.Structure):
    _fields_ = [
        ("first_index", C.c_uint32),
        ("index_count", C.c_uint32),
        ("base_vertex", C.c_int32),
        ("material_index", C.c_int32),
    ]


class TriPushConstant(C.Structure):
    _fields_ = [
        ("model", C.c_float * 16),
        ("tint", C.c_float * 4),
        ("texture_scale", C.c_float * 2),
        ("texture_offset", C.c_float * 2),
        ("tiling_factor", C.c_float),
        ("texture_slot", C.c_int32),
        ("use_material_override", C.c_int32),
        ("sort_bias", C.c_float),
        ("material_index", C.c_int32),
        ("padding0", C.c_int32),
        ("bone_offset", C.c_int32),
        ("bone_count", C.c_int32),
    ]


class TriDraw(C.Structure):
    _fields_ = [("mesh_index", C.c_uint32), ("reserved", C.c_uint32 * 3), ("pc", TriPushConstant)]


class TriPointLight(C.Structure):
    _fields_ = [("position_range", C.c_float * 4), ("color_intensity", C.c_float * 4)]


class TriGlobalUbo(C.Structure):
    _fields_ = [
        ("view", C.c_float * 16),
        ("projection", C.c_float * 16),
        ("camera_position", C.c_float * 4),
        ("ambient_color_intensity", C.c_float * 4),
        ("directional_light_direction", C.c_float * 4),
        ("directional_light_color", C.c_float * 4),
        ("light_counts", C.c_uint32 * 4),
        ("ai_blend_config", C.c_float * 4),
        ("point_lights", TriPointLight * TRI_MAX_POINT_LIGHTS),
    ]


class TriMaterialRecord(C.Structure):
    _fields_ = [("base_color_factor", C.c_float * 4), ("material_factors", C.c_float * 4)]


class TriConfig(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("band_y0", C.c_uint32),
        ("band_y1", C.c_uint32),
        ("device", C.c_int32),
        ("flags", C.c_uint32),
    ]


class TriTiming(C.Structure):
    _fields_ = [
        ("frames", C.c_uint64),
        ("ms_vertex", C.c_double),
        ("ms_setup", C.c_double),
        ("ms_shadow", C.c_double),
        ("ms_raster", C.c_double),
        ("ms_frame", C.c_double),
        ("reserved", C.c_double),
    ]


class TriFrameStats(C.Structure):
    _fields_ = [
        ("triangles_in", C.c_uint64),
        ("triangles_setup", C.c_uint64),
        ("triangles_clipped", C.c_uint64),
        ("bin_entries", C.c_uint64),
        ("vertices_shaded", C.c_uint64),
        ("bins_x", C.c_uint32),
        ("bins_y", C.c_uint32),
        ("bin_size", C.c_uint32),
        ("path", C.c_uint32),
    ]


# tri_frame_stats.path bits (include/tri_raster.h)
TRI_PATH_ONE_DRAW, TRI_PATH_VARY_OBJ, TRI_PATH_OBJ_XFORM, TRI_PATH_OBJ_UCOL, TRI_PATH_SHADOW = 0x1, 0x2, 0x4, 0x8, 0x10
TRI_PATH_OBJ48 = 0x20
TRI_PATH_IDX_ROUTE = 0x40

# the delta bit-plane band format (include/tri_raster.h)
TRI_DBP_SLOT_PIXELS, TRI_DBP_MIN_SLOT, TRI_DBP_MAX_SLOT, TRI_DBP_MAX_BANDS = 4096, 176, 12448, 16


class TriShadowConfig(C.Structure):
    _fields_ = [
        ("size", C.c_uint32),
        ("flags", C.c_uint32),
        ("depth_bias", C.c_float),
        ("slope_bias", C.c_float),
        ("light_view_proj", C.c_float * 16),
    ]


def make_shadow(light_view_proj, size=2048, depth_bias=0.001, slope_bias=2.0):
    s = TriShadowConfig()
    s.size, s.flags, s.depth_bias, s.slope_bias = size, 0, depth_bias, slope_bias
    s.light_view_proj = mat_to_c(light_view_proj)
    return s


TRI_FORMAT_B8G8R8A8_UNORM = 44


class TriImage(C.Structure):
    _fields_ = [
        ("device_ptr", C.c_void_p),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("pitch_bytes", C.c_uint32),
        ("format", C.c_uint32),
        ("device", C.c_int32),
        ("reserved", C.c_uint32),
    ]


class TriGroupConfig(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("device_count", C.c_uint32),
        ("display", C.c_uint32),
        ("devices", C.POINTER(C.c_int32)),
        ("flags", C.c_uint32),
        ("group_flags", C.c_uint32),
    ]


TRI_GROUP_NO_PACK = 0x1
TRI_GROUP_STAGE_BANDS = 0x2
TRI_GROUP_PACK_BGR24 = 0x4
TRI_XFER_ID_BYTES = 128


class TriXferConfig(C.Structure):
    _fields_ = [("width", C.c_uint32), ("band_y", C.POINTER(C.c_uint32)), ("display", C.c_uint32),
                ("format", C.c_uint32), ("slot_bytes", C.c_uint32), ("alpha", C.c_uint32), ("nbuf", C.c_uint32)]
TRI_GROUP_FMT_BGRA32, TRI_GROUP_FMT_BGR24, TRI_GROUP_FMT_DBP = 0, 1, 2

for _s, _n in ((TriImage, 32), (TriGroupConfig, 32), (TriVertex, 100), (TriPushConstant, 128), (TriDraw, 144), (TriGlobalUbo, 480), (TriMaterialRecord, 32),
               (TriShadowConfig, 80)):
    assert C.sizeof(_s) == _n, (_s, C.sizeof(_s))

# every entry point include/tri_raster.h declares: (name, restype, argtypes)
CABI_FUNCTIONS = [
    ("tri_create", C.c_int, [C.POINTER(TriConfig), C.POINTER(C.c_void_p)]),
    ("tri_destroy", C.c_int, [C.c_void_p]),
    ("tri_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("tri_last_error", C.c_char_p, []),
    ("tri_abi_version", C.c_int, []),
    ("tri_upload_geometry", C.c_int,
     [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32]),
    ("tri_upload_materials", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_upload_texture", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("tri_upload_bone_palette", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_upload_skybox", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_upload_ai_frame", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("tri_set_frame", C.c_int, [C.c_void_p, C.POINTER(TriGlobalUbo), C.POINTER(C.c_float * 4)]),
    ("tri_set_draws", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_bind_output", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("tri_render", C.c_int, [C.c_void_p]),
    ("tri_synchronize", C.c_int, [C.c_void_p]),
    ("tri_readback", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("tri_blit_linear", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("tri_read_present", C.c_int, [C.c_void_p, C.c_void_p]),
    ("tri_frame_alpha", C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    ("tri_pack_bgr24", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("tri_unpack_bgr24", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]),
    ("tri_dbp_pack", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("tri_dbp_unpack", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("tri_dbp_bytes", C.c_uint64, [C.c_uint64, C.c_uint32]),
    ("tri_xfer_unique_id", C.c_int, [C.c_void_p]),
    ("tri_xfer_comm_create", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int32, C.POINTER(C.c_void_p)]),
    ("tri_xfer_comm_destroy", C.c_int, [C.c_void_p]),
    ("tri_xfer_create", C.c_int, [C.POINTER(C.c_void_p), C.c_uint32, C.c_void_p, C.POINTER(C.c_void_p)]),
    ("tri_xfer_destroy", C.c_int, [C.c_void_p]),
    ("tri_xfer_bind_slot", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    ("tri_xfer_frame", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_uint32, C.c_uint32]),
    ("tri_xfer_synchronize", C.c_int, [C.c_void_p]),
    ("tri_xfer_wait", C.c_int, [C.c_void_p]),
    ("tri_xfer_set_timeout", C.c_int, [C.c_void_p, C.c_uint32]),
    ("tri_xfer_comm_count", C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    ("tri_xfer_info", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    ("tri_xfer_loopback_create", C.c_int, [C.c_uint32, C.POINTER(C.c_void_p)]),
    ("tri_xfer_loopback_destroy", C.c_int, [C.c_void_p]),
    ("tri_xfer_comm_create_loopback", C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.POINTER(C.c_void_p)]),
    ("tri_dbp_unpack_bands", C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_uint32,
                                       C.c_uint32, C.c_uint32, C.c_void_p]),
    ("tri_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("tri_get_timing", C.c_int, [C.c_void_p, C.POINTER(TriTiming)]),
    ("tri_get_frame_stats", C.c_int, [C.c_void_p, C.POINTER(TriFrameStats)]),
    ("tri_set_shadow", C.c_int, [C.c_void_p, C.POINTER(TriShadowConfig)]),
    ("tri_shadow_fit_ortho", C.c_int, [C.POINTER(C.c_float * 3), C.POINTER(C.c_float * 3), C.POINTER(C.c_float * 3),
                                       C.POINTER(C.c_float * 16)]),
    ("tri_read_shadow_map", C.c_int, [C.c_void_p, C.c_void_p]),
    ("tri_get_output", C.c_int, [C.c_void_p, C.POINTER(TriImage)]),
    ("tri_geometry_create", C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    ("tri_geometry_upload", C.c_int,
     [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32]),
    ("tri_geometry_destroy", C.c_int, [C.c_void_p]),
    ("tri_bind_geometry", C.c_int, [C.c_void_p, C.c_void_p]),
    ("tri_group_create", C.c_int, [C.POINTER(TriGroupConfig), C.POINTER(C.c_void_p)]),
    ("tri_group_destroy", C.c_int, [C.c_void_p]),
    ("tri_group_context", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("tri_group_upload_geometry", C.c_int,
     [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32]),
    ("tri_group_upload_materials", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_group_upload_texture", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("tri_group_upload_bone_palette", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_group_upload_skybox", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_group_upload_ai_frame", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("tri_group_set_shadow", C.c_int, [C.c_void_p, C.POINTER(TriShadowConfig)]),
    ("tri_group_set_frame", C.c_int, [C.c_void_p, C.POINTER(TriGlobalUbo), C.POINTER(C.c_float * 4)]),
    ("tri_group_set_draws", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    ("tri_group_render", C.c_int, [C.c_void_p]),
    ("tri_group_synchronize", C.c_int, [C.c_void_p]),
    ("tri_group_readback", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("tri_group_frame", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int32)]),
    ("tri_group_get_output", C.c_int, [C.c_void_p, C.POINTER(TriImage)]),
    ("tri_group_present", C.c_int, [C.c_void_p, C.c_void_p]),
    ("tri_group_bind_geometry", C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("tri_group_blit_linear", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]),
    ("tri_group_read_present", C.c_int, [C.c_void_p, C.c_void_p]),
    ("tri_group_transfer_info", C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    ("tri_group_transfer_format", C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
]


def mat_to_c(m):
    """Column-major 4x4 (numpy [col][row] or flat 16) -> c_float*16."""
    a = np.ascontiguousarray(np.asarray(m, dtype=np.float32).reshape(16))
    return (C.c_float * 16)(*a.tolist())


def make_draw(mesh_index, model, texture_slot=0, material_index=-1, tint=(1, 1, 1, 1), bone_offset=0, bone_count=0,
              texture_scale=(1, 1), texture_offset=(0, 0), tiling=1.0):
    """One MeshDrawCommand -> push constant, as RecordCommandBuffer fills it (Renderer.cpp:5129-5146)."""
    d = TriDraw()
    d.mesh_index = mesh_index
    pc = d.pc
    pc.model = mat_to_c(model)
    pc.tint = (C.c_float * 4)(*tint)
    pc.texture_scale = (C.c_float * 2)(*texture_scale)
    pc.texture_offset = (C.c_float * 2)(*texture_offset)
    pc.tiling_factor = tiling
    pc.texture_slot = texture_slot
    pc.use_material_override = 0
    pc.sort_bias = 0.0
    pc.material_index = material_index
    pc.bone_offset = bone_offset
    pc.bone_count = bone_count
    return d


def draws_array(draws):
    arr = (TriDraw * max(len(draws), 1))()
    for i, d in enumerate(draws):
        arr[i] = d
    return arr, len(draws)
