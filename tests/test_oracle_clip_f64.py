"""The oracle's clipping, raster and depth, checked against an independent float64 restatement written from the
Vulkan rules rather than from either implementation ("the oracle moved toward the kernels").

Vulkan (and Pipeline.cpp's state: depth clamp off, cull back, CCW front with the projection's Y flip) clips a
primitive to 0 <= z_c <= w_c and the frustum's sides, rasterizes the clipped polygon with its pixel centres,
interpolates z_ndc linearly in screen space and keeps the LEQUAL minimum in primitive order. The float64 version
below does exactly that with no sub-pixel snap, no guard band and no fan order: it shares no code or
formulation with the oracle (which clips in float32 with barycentric weights, fans the polygon, snaps to 8
sub-pixel bits). Where a pixel centre lies at least half a pixel inside the winning float64 polygon, the two
must agree on coverage and on depth within the error the 1/256-px snap and float32 can introduce.
"""
import numpy as np

import scene_cases as sc

WMIN = 1e-5  # the oracle's w clip plane; Vulkan's z >= 0 plane is the one that cuts here


def _clip_polygon(poly, plane):
    out = []
    n = len(poly)
    for i in range(n):
        a, b = poly[i], poly[(i + 1) % n]
        da, db = plane(a), plane(b)
        if da >= 0:
            out.append(a)
        if (da >= 0) != (db >= 0):
            t = da / (da - db)
            out.append(a + t * (b - a))
    return out


def f64_depth(scene):
    """Depth buffer of the scene's mesh draws, float64 Vulkan rules; also the per-pixel distance (px) from the
    winning polygon's boundary, the winner's depth gradient magnitude, and whether the winner was clipped."""
    W, H = scene.width, scene.height
    view = np.array(scene.ubo.view, np.float64).reshape(4, 4).T
    proj = np.array(scene.ubo.projection, np.float64).reshape(4, 4).T
    depth = np.ones((H, W))
    margin = np.full((H, W), -1.0)
    grad = np.zeros((H, W))
    clipped = np.zeros((H, W), bool)
    ys, xs = np.mgrid[0:H, 0:W] + 0.5
    for d in scene.draws:
        m = scene.meshes[d.mesh_index]
        model = np.array(d.pc.model, np.float64).reshape(4, 4).T
        mvp = proj @ view @ model
        first, count, base = int(m["first_index"]), int(m["index_count"]), int(m["base_vertex"])
        tris = scene.indices[first:first + count - count % 3].reshape(-1, 3).astype(np.int64) + base
        pos = scene.vertices["position"].astype(np.float64)
        for t in tris:
            c = [mvp @ np.append(pos[i], 1.0) for i in t]
            poly = _clip_polygon(c, lambda v: v[3] - WMIN)
            poly = _clip_polygon(poly, lambda v: v[2])  # 0 <= z_c
            if len(poly) < 3:
                continue
            was_clipped = not all(any(np.array_equal(p, q) for q in c) for p in poly)
            sx = np.array([p[0] / p[3] * W / 2 + W / 2 for p in poly])
            sy = np.array([p[1] / p[3] * H / 2 + H / 2 for p in poly])
            sz = np.array([p[2] / p[3] for p in poly])
            area = 0.5 * np.sum(sx * np.roll(sy, -1) - np.roll(sx, -1) * sy)
            if area >= 0:  # back face (front = clockwise in this y-down screen space after the flip)
                continue
            x0, x1 = max(int(np.floor(sx.min())), 0), min(int(np.ceil(sx.max())), W - 1)
            y0, y1 = max(int(np.floor(sy.min())), 0), min(int(np.ceil(sy.max())), H - 1)
            if x0 > x1 or y0 > y1:
                continue
            px, py = xs[y0:y1 + 1, x0:x1 + 1], ys[y0:y1 + 1, x0:x1 + 1]
            inside = np.full(px.shape, np.inf)
            n = len(poly)
            for k in range(n):  # signed distance to each edge, positive inside (the polygon is convex)
                ax, ay, bx, by = sx[k], sy[k], sx[(k + 1) % n], sy[(k + 1) % n]
                ln = np.hypot(bx - ax, by - ay)
                if ln == 0:
                    continue
                dist = -((bx - ax) * (py - ay) - (by - ay) * (px - ax)) / ln
                inside = np.minimum(inside, dist)
            # z plane through the first three (non-collinear) polygon vertices: exact for a planar polygon
            A = np.array([[sx[0], sy[0], 1], [sx[1], sy[1], 1], [sx[2], sy[2], 1]])
            if abs(np.linalg.det(A)) < 1e-12:
                continue
            a, b, cz = np.linalg.solve(A, sz[:3])
            z = a * px + b * py + cz
            cov = (inside >= 0) & (z <= 1.0)
            zc = np.maximum(z, 0.0)
            win = cov & (zc <= depth[y0:y1 + 1, x0:x1 + 1])
            depth[y0:y1 + 1, x0:x1 + 1][win] = zc[win]
            margin[y0:y1 + 1, x0:x1 + 1][win] = inside[win]
            grad[y0:y1 + 1, x0:x1 + 1][win] = np.hypot(a, b)
            clipped[y0:y1 + 1, x0:x1 + 1][win] = was_clipped
    return depth, margin, grad, clipped


def test_oracle_clipping_and_depth_match_float64_vulkan_rules(oracle):
    s = sc.near_clip_grid(320, 240, 24)
    _, od_bits, stats = oracle.render(s)
    assert stats["triangles_clipped"] > 0
    od = od_bits.view(np.float32).astype(np.float64)
    fd, margin, grad, clipped = f64_depth(s)
    interior = margin >= 0.5
    assert interior.sum() > 20000
    # coverage: every pixel centre half a pixel inside a float64 polygon is covered by the oracle too
    assert (od[interior] < 1.0).all()
    # and the oracle covers nothing the float64 raster leaves as background, away from polygon edges
    bg = (margin < 0) & (fd >= 1.0)
    near_edge = np.zeros_like(bg)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            near_edge |= np.roll(np.roll(margin >= 0, dy, 0), dx, 1)
    assert (od[bg & ~near_edge] >= 1.0).all()
    # depth: the 1/256-px vertex snap moves the plane by at most about |grad z| * 2/256 per pixel, plus float32
    tol = grad * (2.0 / 256.0) + 4e-7 + 2e-6 * np.abs(fd)
    err = np.abs(od - fd)
    assert (err[interior] <= tol[interior]).all(), float((err - tol)[interior].max())
    # the comparison includes pixels of clipped primitives
    assert (interior & clipped).sum() > 1000
