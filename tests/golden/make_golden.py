#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz: small parity scenes with their full inputs (vertex/index/mesh/draw/
UBO/material/texture/bone bytes) and the CPU oracle's outputs (B8G8R8A8 bytes + D32 depth bits).

The reference cannot be built or run in this environment, so the fixtures pin
the oracle (whose arithmetic is itself pinned by tests/test_oracle_kat.py) and, through
tests/test_golden.py, the HIP path. Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "3d-renderer_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_py  # noqa: E402
import scene_cases as sc  # noqa: E402
from trident_raster import abi  # noqa: E402


def cases():
    o = oracle_py
    yield "c1_cube_f0", sc.c1_cube(0)
    yield "c1_cube_f1", sc.c1_cube(1)
    yield "c1_cube_f3", sc.c1_cube(3)
    yield "primitives", sc.primitives_row(o)
    yield "textured_grid", sc.textured_grid(256, 144, 24)
    yield "near_clip", sc.near_clip_grid(320, 240, 40)
    yield "depth_ties", sc.depth_ties()
    yield "skinned", sc.skinned_quad(o)
    yield "invalid", sc.invalid_inputs(o)
    yield "sphere_360p", sc.sphere_c2(640, 360, 40, 64, oracle=o)
    yield "skybox_only", sc.skybox_only(192, 144, fov=110.0)
    yield "c1_cube_skybox", sc.c1_cube_skybox(1, 320, 240)


def pack(scene):
    draws, n = abi.draws_array(scene.draws)
    mats = np.array([list(b) + list(f) for b, f in scene.materials], np.float32).reshape(-1, 8)
    d = dict(width=scene.width, height=scene.height, vertices=scene.vertices.view(np.uint8),
             indices=scene.indices, meshes=scene.meshes.view(np.uint8),
             draws=np.frombuffer(bytes(draws), np.uint8)[: n * abi.C.sizeof(abi.TriDraw)],
             ubo=np.frombuffer(bytes(scene.ubo), np.uint8), materials=mats,
             clear=np.array(scene.clear, np.float32),
             bones=np.zeros((0, 16), np.float32) if scene.bones is None else np.asarray(scene.bones, np.float32))
    for k, (slot, t) in enumerate(scene.textures):
        d[f"tex{k}_slot"] = np.array(slot)
        d[f"tex{k}"] = t
    if scene.skybox is not None:
        d["skybox"] = np.asarray(scene.skybox, np.uint8)
    return d


def unpack(z):
    from trident_raster import scenes

    draws_raw = z["draws"].tobytes()
    size = abi.C.sizeof(abi.TriDraw)
    draws = [abi.TriDraw.from_buffer_copy(draws_raw[i:i + size]) for i in range(0, len(draws_raw), size)]
    mats = [(tuple(m[:4]), tuple(m[4:])) for m in z["materials"]]
    texs = []
    k = 0
    while f"tex{k}" in z:
        texs.append((int(z[f"tex{k}_slot"]), z[f"tex{k}"]))
        k += 1
    bones = z["bones"] if z["bones"].size else None
    return scenes.Scene("golden", int(z["width"]), int(z["height"]),
                        z["vertices"].view(abi.VERTEX_DTYPE), z["indices"], z["meshes"].view(abi.MESH_RANGE_DTYPE),
                        draws, abi.TriGlobalUbo.from_buffer_copy(z["ubo"].tobytes()), materials=mats, textures=texs,
                        clear=tuple(float(c) for c in z["clear"]), bones=bones,
                        skybox=z["skybox"] if "skybox" in z else None)


def main(only=()):
    oracle_py.build()
    for name, scene in cases():
        if only and name not in only:
            continue
        if scene.skybox is not None and scene.skybox.shape[1] > 64:
            # keep fixtures small: the 512^2 reference cubemap (6 MB) is covered by the skybox GPU tests
            scene.skybox = sc.SOLID_0x808080
        col, dep, st = oracle_py.render(scene)
        d = pack(scene)
        d["out_bgra"], d["out_depth"] = col, dep
        d["stats"] = np.array([st["triangles_in"], st["triangles_setup"], st["triangles_clipped"]], np.int64)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"{name:16s} {scene.width}x{scene.height} covered={(dep != 0x3F800000).sum():7d} "
              f"{os.path.getsize(path) / 1024:.0f} KiB")


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))  # optional fixture names: regenerate only those
