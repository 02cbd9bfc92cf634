"""The oracle's clipping, raster and depth, checked against an independent float64 restatement written from the
Vulkan rules rather than from either implementation ("the oracle moved toward the kernels").

Vulkan (and Pipeline.cpp's state: depth clamp off, cull back, CCW front with the projection's Y flip) clips a
primitive to 0 <= z_c <= w_c and the frustum's sides, rasterizes the clipped polygon with its pixel centres,
interpolates z_ndc linearly in screen space and keeps the LEQUAL minimum in primitive order. The float64 version
below does exactly that with no sub-pixel snap, no guard band and no fan order: it shares no code or
formulation with the oracle (which clips in float32 with barycentric weights, fans the polygon, snaps to 8
sub-pixel bits). Where a pixel centre lies at least half a pixel inside the winning float64 polygon, the two
must agree on coverage and on depth within the error the 1/256-px snap and float32 can introduce, and (second
half of the file) on the stored colour within 1 LSB, with Default.vert/Default.frag evaluated in float64.
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


# ---- the whole fragment path in float64 -----------------------------------------------------------------------
# Default.vert (world position, normal through transpose(inverse(mat3(model))), colour, uv * scale * tiling +
# offset) and Default.frag (PBR, Reinhard, 1/2.2 gamma) evaluated in float64 at each pixel centre, with the
# perspective-correct weights solved from the ORIGINAL triangle's clip-space vertices (homogeneous
# rasterisation: the weights b with sum b_i (x_i - x w_i) = sum b_i (y_i - y w_i) = 0, sum b_i = 1), so clipping
# only limits where a triangle is visible, never what it interpolates. Texture taps: sRGB decoded in float64,
# bilinear, REPEAT, level 0. Nothing here follows the oracle's (or the kernels') operation order.
def _srgb_to_linear(c):
    c = c / 255.0
    return np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)


def _sample(tex, u, v):
    h, w = tex.shape[:2]
    x, y = u * w - 0.5, v * h - 0.5
    x0, y0 = np.floor(x), np.floor(y)
    a, b = (x - x0)[..., None], (y - y0)[..., None]
    x0, y0 = x0.astype(np.int64) % w, y0.astype(np.int64) % h
    x1, y1 = (x0 + 1) % w, (y0 + 1) % h
    lin = np.concatenate([_srgb_to_linear(tex[..., :3].astype(np.float64)), tex[..., 3:4] / 255.0], -1)
    t00, t10, t01, t11 = lin[y0, x0], lin[y0, x1], lin[y1, x0], lin[y1, x1]
    return (t00 * (1 - a) + t10 * a) * (1 - b) + (t01 * (1 - a) + t11 * a) * b


def _shade(scene, draw, P, N, col, uv):
    """Default.frag:123-180 in float64 for arrays of fragments of one draw."""
    g = scene.ubo
    base, fac = scene.materials[0] if scene.materials else ((1, 1, 1, 1), (0, 1, 1, 0))  # record-0 quirk
    slot = draw.pc.texture_slot
    tex = next((t for s, t in scene.textures if s == slot), None)
    smp = _sample(tex, uv[:, 0], uv[:, 1]) if tex is not None else np.ones((len(P), 4))
    tint = np.array(draw.pc.tint, np.float64)
    alb = smp[:, :3] * np.array(base[:3]) * tint[:3] * col
    met = min(max(fac[0], 0.0), 1.0)
    rough = min(max(fac[1], 0.045), 1.0)
    amb_s = min(max(fac[2], 0.0), 1.0)
    F0 = 0.04 * (1 - met) + alb * met
    Nn = N / np.linalg.norm(N, axis=1, keepdims=True)
    V = np.array(g.camera_position[:3], np.float64) - P
    V /= np.linalg.norm(V, axis=1, keepdims=True)
    dot = lambda a, b: np.sum(a * b, axis=1)

    def pbr(L, rad):
        H = V + L
        H /= np.linalg.norm(H, axis=1, keepdims=True)
        a2 = (rough * rough) ** 2
        nh = np.maximum(dot(Nn, H), 0)
        ndf = a2 / (np.pi * (nh * nh * (a2 - 1) + 1) ** 2)
        k = (rough + 1) ** 2 / 8
        nv, nl = np.maximum(dot(Nn, V), 0), np.maximum(dot(Nn, L), 0)
        geo = nv / np.maximum(nv * (1 - k) + k, 1e-4) * (nl / np.maximum(nl * (1 - k) + k, 1e-4))
        Fr = F0 + (1 - F0) * (np.clip(1 - np.maximum(dot(H, V), 0), 0, 1) ** 5)[:, None]
        spec = (ndf * geo)[:, None] * Fr / np.maximum(4 * nv * nl, 1e-4)[:, None]
        kD = (1 - Fr) * (1 - met)
        return (kD * alb / np.pi + spec) * rad * nl[:, None]

    direct = np.zeros_like(P)
    if g.light_counts[0] > 0:
        d = -np.array(g.directional_light_direction[:3], np.float64)
        L = np.broadcast_to(d / np.linalg.norm(d), P.shape)
        direct += pbr(L, np.array(g.directional_light_color[:3]) * g.directional_light_color[3])
    for i in range(min(g.light_counts[1], 8)):
        pl = g.point_lights[i]
        to = np.array(pl.position_range[:3], np.float64) - P
        dist = np.linalg.norm(to, axis=1)
        ok = dist > 1e-4
        att = (1 - np.clip(dist / max(pl.position_range[3], 1e-4), 0, 1)) ** 2
        rad = np.array(pl.color_intensity[:3]) * pl.color_intensity[3] * att[:, None]
        contrib = pbr(to / np.where(ok, dist, 1)[:, None], rad)
        direct += np.where(ok[:, None], contrib, 0)
    amb = np.array(g.ambient_color_intensity[:3]) * g.ambient_color_intensity[3] * alb * amb_s
    c = amb + direct
    c = (c / (c + 1)) ** (1 / 2.2)
    alpha = base[3] * tint[3] * smp[:, 3]
    return np.concatenate([c, alpha[:, None]], 1)


def f64_colour(scene, fd, margin):
    """Colour (float64, before the UNORM store) of every pixel with margin >= 0.5 whose winning triangle is
    found again by depth; returns (colour [H, W, 4], mask)."""
    W, H = scene.width, scene.height
    view = np.array(scene.ubo.view, np.float64).reshape(4, 4).T
    proj = np.array(scene.ubo.projection, np.float64).reshape(4, 4).T
    out = np.zeros((H, W, 4))
    done = np.zeros((H, W), bool)
    ys, xs = np.mgrid[0:H, 0:W] + 0.5
    xn, yn = (xs - W / 2) / (W / 2), (ys - H / 2) / (H / 2)
    want = margin >= 0.5
    vx = scene.vertices
    for d in scene.draws:
        m = scene.meshes[d.mesh_index]
        model = np.array(d.pc.model, np.float64).reshape(4, 4).T
        nmat = np.linalg.inv(model[:3, :3]).T
        first, count, base = int(m["first_index"]), int(m["index_count"]), int(m["base_vertex"])
        tris = scene.indices[first:first + count - count % 3].reshape(-1, 3).astype(np.int64) + base
        pos = np.c_[vx["position"].astype(np.float64), np.ones(len(vx))]
        world = (model @ pos.T).T
        clip = (proj @ view @ world.T).T
        nrm = (nmat @ vx["normal"].astype(np.float64).T).T
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        uvt = vx["texcoord"].astype(np.float64) * np.array(d.pc.texture_scale) * d.pc.tiling_factor + np.array(d.pc.texture_offset)
        colv = vx["color"].astype(np.float64)
        for t in tris:
            C = clip[t]
            sxv = C[:, 0] / np.where(C[:, 3] > 0, C[:, 3], np.nan) * W / 2 + W / 2
            syv = C[:, 1] / np.where(C[:, 3] > 0, C[:, 3], np.nan) * H / 2 + H / 2
            if np.all(C[:, 3] > 0):  # a bbox for the common case; a clipped triangle tests the whole frame
                x0, x1 = max(int(np.floor(sxv.min())), 0), min(int(np.ceil(sxv.max())), W - 1)
                y0, y1 = max(int(np.floor(syv.min())), 0), min(int(np.ceil(syv.max())), H - 1)
            else:
                x0, x1, y0, y1 = 0, W - 1, 0, H - 1
            if x0 > x1 or y0 > y1:
                continue
            sl = (slice(y0, y1 + 1), slice(x0, x1 + 1))
            cand = want[sl] & ~done[sl]
            if not cand.any():
                continue
            px, py = xn[sl][cand], yn[sl][cand]
            a = C[None, :, 0] - px[:, None] * C[None, :, 3]
            c = C[None, :, 1] - py[:, None] * C[None, :, 3]
            b = np.cross(a, c)
            bs = b.sum(1, keepdims=True)
            ok = np.abs(bs[:, 0]) > 1e-300  # a degenerate (zero-area) triangle has no weights
            b = b / np.where(ok[:, None], bs, 1.0)
            inside = ok & np.all(b >= 0, axis=1)
            bw = b @ C[:, 3]
            z = (b @ C[:, 2]) / np.where(inside, bw, 1.0)
            hit = inside & (np.abs(z - fd[sl][cand]) <= 1e-9)
            if not hit.any():
                continue
            bh = b[hit]
            P = bh @ world[t, :3]
            rgba = _shade(scene, d, P, bh @ nrm[t], bh @ colv[t], bh @ uvt[t])
            iy, ix = np.nonzero(cand)
            iy, ix = iy[hit] + y0, ix[hit] + x0
            out[iy, ix] = rgba
            done[iy, ix] = True
    return out, done


def _check_colour(oracle, s, min_pixels):
    bgra, od_bits, _ = oracle.render(s)
    fd, margin, _, _ = f64_depth(s)
    ref, mask = f64_colour(s, fd, margin)
    assert mask.sum() >= min_pixels
    want = np.rint(np.clip(ref, 0, 1) * 255.0)
    got = bgra[..., [2, 1, 0, 3]].astype(np.float64)
    diff = np.abs(got - want)[mask]
    # float32 against float64 differs by 1 LSB where a value sits on a rounding boundary, never more
    assert diff.max() <= 1, (diff.max(), np.argwhere(np.abs(got - want).max(-1) * mask > 1)[:5])
    return diff


def test_oracle_colour_matches_float64_shading_textured(oracle):
    # sun + 4 point lights, an sRGB texture with alpha under REPEAT, tint, uv scale/offset/tiling, vertex colours
    diff = _check_colour(oracle, sc.textured_grid(320, 180, 30), 30000)
    assert (diff == 0).mean() > 0.9


def test_oracle_colour_matches_float64_shading_sphere(oracle):
    # curved normals out to grazing view angles (N.V -> 0: the 1e-4 clamps of Default.frag), two point lights
    s = sc.sphere_c2(320, 240, 40, 60)
    s.skybox = None
    _check_colour(oracle, s, 6000)


def test_oracle_colour_matches_float64_shading_clipped(oracle):
    # a point light over a ground plane cut by the near plane: the visible parts of clipped triangles shaded
    _check_colour(oracle, sc.near_clip_grid(320, 240, 24), 40000)


# ---- the skybox pass in float64 -------------------------------------------------------------------------------
# Skybox.cpp:13-36's cube (scaled by 20, Skybox.cpp:74) through Skybox.vert (gl_Position = (P mat4(mat3(View))
# world).xyww, outDirection = mat3(View) world) rasterised homogeneously: at each pixel the direction is the
# clip-space convex combination of a triangle's view-space vertices with positive w — the ray's exit point, as a
# rasteriser interpolating outDirection over the visible face produces it. Skybox.frag samples the cube map at
# normalize(direction): Vulkan's major-axis face table, sRGB decoded in float64, bilinear within the face.
# Pixels whose direction lies near a face edge (where seamless filtering takes taps from two faces) are skipped.
_SKY_POS = np.array([[-1, -1, 1], [1, -1, 1], [1, 1, 1], [-1, 1, 1],
                     [-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1]], np.float64) * 20.0
_SKY_IDX = np.array([0, 1, 2, 2, 3, 0, 1, 5, 6, 6, 2, 1, 5, 4, 7, 7, 6, 5,
                     4, 0, 3, 3, 7, 4, 3, 2, 6, 6, 7, 3, 4, 5, 1, 1, 0, 4]).reshape(-1, 3)


def f64_sky(scene):
    W, H = scene.width, scene.height
    view = np.array(scene.ubo.view, np.float64).reshape(4, 4).T
    proj = np.array(scene.ubo.projection, np.float64).reshape(4, 4).T
    R = view[:3, :3]
    vpos = _SKY_POS @ R.T  # outDirection at the cube's corners
    clip = np.c_[vpos, np.ones(8)] @ proj.T
    ys, xs = np.mgrid[0:H, 0:W] + 0.5
    xn, yn = ((xs - W / 2) / (W / 2)).ravel(), ((ys - H / 2) / (H / 2)).ravel()
    dirs = np.full((H * W, 3), np.nan)
    for t in _SKY_IDX:
        C = clip[t]
        a = C[None, :, 0] - xn[:, None] * C[None, :, 3]
        c = C[None, :, 1] - yn[:, None] * C[None, :, 3]
        b = np.cross(a, c)
        s = b.sum(1, keepdims=True)
        ok = np.abs(s[:, 0]) > 1e-12
        b = b / np.where(ok[:, None], s, 1)
        hit = ok & np.all(b >= 0, axis=1) & (b @ C[:, 3] > 0)
        dirs[hit] = b[hit] @ vpos[t]
    faces = scene.skybox
    n = faces.shape[1]
    lin = _srgb_to_linear(faces[..., :3].astype(np.float64))
    out = np.full((H * W, 3), np.nan)
    good = ~np.isnan(dirs[:, 0])
    d = dirs[good] / np.linalg.norm(dirs[good], axis=1, keepdims=True)
    ax = np.abs(d)
    major = np.argmax(ax, axis=1)
    srt = np.sort(ax, axis=1)
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    # Vulkan's cube map face selection table: (face, sc, tc, ma)
    face = np.where(major == 0, np.where(x >= 0, 0, 1), np.where(major == 1, np.where(y >= 0, 2, 3), np.where(z >= 0, 4, 5)))
    sc_ = np.select([face == 0, face == 1, face == 2, face == 3, face == 4], [-z, z, x, x, x], -x)
    tc_ = np.select([face == 0, face == 1, face == 2, face == 3, face == 4], [-y, -y, z, -z, -y], -y)
    ma = srt[:, 2]
    u = (0.5 * sc_ / ma + 0.5) * n - 0.5
    v = (0.5 * tc_ / ma + 0.5) * n - 0.5
    i0, j0 = np.floor(u).astype(np.int64), np.floor(v).astype(np.int64)
    inner = (i0 >= 0) & (i0 + 1 <= n - 1) & (j0 >= 0) & (j0 + 1 <= n - 1) & (srt[:, 2] - srt[:, 1] > 1e-6)
    a_, b_ = (u - i0)[:, None], (v - j0)[:, None]
    i0c, j0c = np.clip(i0, 0, n - 2), np.clip(j0, 0, n - 2)
    t00, t10 = lin[face, j0c, i0c], lin[face, j0c, i0c + 1]
    t01, t11 = lin[face, j0c + 1, i0c], lin[face, j0c + 1, i0c + 1]
    col = (t00 * (1 - a_) + t10 * a_) * (1 - b_) + (t01 * (1 - a_) + t11 * a_) * b_
    idx = np.nonzero(good)[0]
    out[idx[inner]] = col[inner]
    return out.reshape(H, W, 3)


def test_oracle_skybox_matches_float64_cube_pass(oracle):
    for rot, fov in (((0.0, 0.0, 0.0), 100.0), ((25.0, 140.0, 10.0), 70.0), ((-80.0, 30.0, 0.0), 90.0)):
        s = sc.skybox_only(160, 120, fov, rot, sc.cubemap_faces(32, seed=5))
        bgra, _, _ = oracle.render(s)
        ref = f64_sky(s)
        mask = ~np.isnan(ref[..., 0])
        assert mask.mean() > 0.6, mask.mean()
        want = np.rint(np.clip(ref, 0, 1) * 255.0)
        got = bgra[..., [2, 1, 0]].astype(np.float64)
        diff = np.abs(got - want)[mask]
        assert diff.max() <= 1, (rot, diff.max())
        assert (bgra[..., 3] == 255).all()
