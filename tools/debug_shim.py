"""GPU debug: the two-viewport shim scene rendered through the shim, through the C-ABI directly, and
by the oracle; prints where they differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3d-renderer_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle_py  # noqa: E402
from trident_raster import app, raster, scenes  # noqa: E402

import test_host_shim as t  # noqa: E402

a = app.TridentApp()
a.set_camera("editor", (0, 1, 6))
a.set_camera("runtime", (3, 2, 5), (-10, 30, 0), fov=55.0, ready=True)
a.set_viewport(1, 480, 320)
a.set_viewport(2, 256, 200)
yy, xx = np.mgrid[0:8, 0:8]
checker = np.where(((xx + yy) % 2)[..., None] == 0, 230, 25).astype(np.uint8).repeat(4, -1)
checker[..., 3] = 255
a.upload_texture("checker.png", checker)
v, i = scenes.uv_sphere_mesh(24, 32, 1.0)
m = a.append_mesh(v, i, base_color=(0.9, 0.8, 0.7, 1), metallic=0.2, roughness=0.5, texture="checker.png")
a.add_mesh_entity("none", m, position=(0, 0.5, 0))
a.add_mesh_entity("cube", position=(-1.5, 0, 0), rotation=(10, 20, 30))
q = a.add_mesh_entity("quad", position=(1.5, 0, 0), scale=(1.5, 1.5, 1))
a.set_entity_texture(q, "checker.png")
a.add_light("point", position=(0, 2, 2), color=(1, 0.9, 0.8), intensity=8.0, range=6.0)
a.draw_frame()
for vp, (w, h) in ((1, (480, 320)), (2, (256, 200))):
    rgba, depth = a.read_pixels(vp, w, h)
    sc = t.shim_scene(a, vp, w, h, [(1, checker)])
    oc, od, ost = oracle_py.render(sc)
    with raster.TriRaster(w, h) as r:
        scenes.load_scene(r, sc)
        r.render_frame()
        gc, gd = r.readback()
        gst = r.frame_stats()
    sd = depth.view(np.uint32)
    print(f"vp{vp}: draws={[d.mesh_index for d in sc.draws]} ranges={sc.meshes.tolist()} nverts={len(sc.vertices)}")
    print(f"  oracle covered={int((od != 0x3F800000).sum())} stats={ost}")
    print(f"  capi   covered={int((gd != 0x3F800000).sum())} depth_mismatch={int((gd != od).sum())} stats={gst}")
    print(f"  shim   covered={int((sd != 0x3F800000).sum())} depth_mismatch={int((sd != od).sum())}")
    print(f"  shim vs capi depth mismatch={int((sd != gd).sum())}")
    bad = np.argwhere(sd != od)
    if len(bad):
        y, x = bad[0]
        print(f"  first bad px ({x},{y}) shim={sd[y, x]:#x} oracle={od[y, x]:#x} capi={gd[y, x]:#x}")
        print(f"  bad rows {bad[:, 0].min()}..{bad[:, 0].max()} cols {bad[:, 1].min()}..{bad[:, 1].max()}")
