"""CPU tests of the drop-in boundary: struct layouts, exported symbols, loud failure without a GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

from trident_raster import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tri_raster.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*|uint64_t)\s+(tri_\w+)\(", text, flags=re.M)))


def test_header_declares_exactly_the_python_mirror():
    assert header_functions() == sorted(n for n, _, _ in abi.CABI_FUNCTIONS)


def test_struct_layout_matches_c_compiler(tmp_path):
    """sizeof/offsetof from gcc on the real header == the ctypes mirror == the reference's GPU ABI."""
    structs = {
        "tri_vertex": abi.TriVertex, "tri_mesh_range": abi.TriMeshRange, "tri_push_constant": abi.TriPushConstant,
        "tri_draw": abi.TriDraw, "tri_point_light": abi.TriPointLight, "tri_global_ubo": abi.TriGlobalUbo,
        "tri_material_record": abi.TriMaterialRecord, "tri_config": abi.TriConfig, "tri_timing": abi.TriTiming,
        "tri_frame_stats": abi.TriFrameStats, "tri_shadow_config": abi.TriShadowConfig,
        "tri_group_config": abi.TriGroupConfig, "tri_image": abi.TriImage,
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                              check=True).stdout.strip().splitlines())
    for cname, py in structs.items():
        assert int(out[f"{cname} size"]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(out[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)
    # the reference's byte layouts (Vertex.h:9-78, RenderData.h:14-30, UniformBuffer.h:17-35)
    assert C.sizeof(abi.TriVertex) == 100 and abi.TriVertex.texcoord.offset == 60
    assert abi.TriVertex.bone_indices.offset == 68 and abi.TriVertex.bone_weights.offset == 84
    assert C.sizeof(abi.TriPushConstant) == 128 and abi.TriPushConstant.texture_slot.offset == 100
    assert abi.TriPushConstant.material_index.offset == 112 and abi.TriPushConstant.bone_count.offset == 124
    assert C.sizeof(abi.TriGlobalUbo) == 480 and abi.TriGlobalUbo.light_counts.offset == 192
    assert abi.TriGlobalUbo.ai_blend_config.offset == 208 and abi.TriGlobalUbo.point_lights.offset == 224


def test_library_exports_every_declared_symbol(hiplib):
    out = subprocess.run(["nm", "-D", "--defined-only", hiplib._name], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (tri_\w+)", out))
    missing = set(header_functions()) - exported
    assert not missing, missing
    assert hiplib.tri_abi_version() == abi.TRI_RASTER_ABI_VERSION == 2


def test_fails_loudly_without_gpu(hiplib):
    """On a host without a HIP device the product returns TRI_E_HIP with a message: no CPU fallback."""
    from tests_gpu_probe import gpu_present  # noqa: F401  (helper below)

    if gpu_present():
        pytest.skip("a GPU is present")
    cfg = abi.TriConfig(64, 64, 0, 0, -1, 0)
    ctx = C.c_void_p()
    rc = hiplib.tri_create(C.byref(cfg), C.byref(ctx))
    assert rc == abi.TRI_E_HIP
    assert b"device" in hiplib.tri_last_error()
    assert not ctx.value


def test_invalid_arguments_are_rejected(hiplib):
    cfg = abi.TriConfig(0, 64, 0, 0, -1, 0)
    ctx = C.c_void_p()
    assert hiplib.tri_create(C.byref(cfg), C.byref(ctx)) == abi.TRI_E_INVALID
    cfg = abi.TriConfig(64, 64, 40, 20, -1, 0)  # empty band
    assert hiplib.tri_create(C.byref(cfg), C.byref(ctx)) == abi.TRI_E_INVALID
    cfg = abi.TriConfig(9000, 64, 0, 0, -1, 0)  # beyond TRI_MAX_DIM
    assert hiplib.tri_create(C.byref(cfg), C.byref(ctx)) == abi.TRI_E_INVALID
    assert hiplib.tri_create(None, C.byref(ctx)) == abi.TRI_E_INVALID
    assert hiplib.tri_destroy(None) == abi.TRI_OK
    assert hiplib.tri_render(None) == abi.TRI_E_INVALID
