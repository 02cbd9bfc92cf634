// tri_oracle.cpp — TEST INFRASTRUCTURE: CPU restatement of the reference's graphics-pipeline stage,
// used only as the parity checker (tests/, __graft_entry__.smoke()) and as bench.py's cpu_baseline
// ("port"). Never linked into the product. Header comment of tri_oracle.h states the parity status
// ("parity unpinned" against the Vulkan driver; pinned by KATs + committed fixtures, and cross-checked
// against an independent float64 restatement in tests/test_oracle_clip_f64.py).
//
// It restates, in this order:
//   * Default.vert main() (Trident-Forge/Assets/Shaders/Default.vert:60-105)
//   * Vulkan fixed-function state from Pipeline.cpp:611-666 (TRIANGLE_LIST, cull BACK, front CCW,
//     no depth clamp/bias, 1 sample, no blend, depth test+write LESS_OR_EQUAL), the viewport of
//     Renderer.cpp:5062-5069 and the depth clear 1.0 of Renderer.cpp:5037
//   * Default.frag main() (Default.frag:67-192), sampler state of Renderer.cpp:3592-3607
//     (R8G8B8A8_SRGB, LINEAR, REPEAT, maxLod 0) and B8G8R8A8_UNORM output (Swapchain.cpp:161-172).
//
// The raster rules below are the precise restatement both this oracle and the HIP kernels follow
// (DESIGN.md §3 "Raster rules"): 8 sub-pixel bits, pixel-centre sampling, top-left fill rule,
// homogeneous clipping against w >= 1e-5, z >= 0 and a guard band, per-pixel far-plane discard,
// screen-linear depth from a plane equation, in-order LEQUAL. Evaluation order is fixed and no FMA
// contraction is used (build with -ffp-contract=off), so depth is reproducible bit-for-bit.
#include "tri_oracle.h"
#include "oracle_glm.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

using namespace oracle;

namespace {

constexpr float kWMin = 1e-5f;         // clip plane w >= kWMin (protects the divide)
constexpr float kGuardBandPx = 16000.f; // |framebuffer coordinate| bound for unclipped triangles
constexpr uint32_t kPrimMax = (1u << 29) - 1u;
constexpr float kPi = 3.14159265359f;   // Default.frag:65

struct VsOut {
    vec4 clip;
    vec3 world;
    vec3 normal;
    vec2 uv;
    vec3 color;
    vec3 lpos;  // light-space (shadow-map NDC) position: light_view_proj * world (shadow pass only)
};

mat4 load_mat4(const float* p) {
    mat4 m;
    std::memcpy(m.m, p, 64);
    return m;
}

// GLSL mat4 * vec4 in the kernel order: ((c0*x + c1*y) + c2*z) + c3*w, no FMA.
inline vec4 mat_vec_seq(const mat4& m, vec4 v) {
    vec4 r;
    float* rp = &r.x;
    for (int i = 0; i < 4; ++i) {
        float s = m.m[0][i] * v.x;
        s = s + m.m[1][i] * v.y;
        s = s + m.m[2][i] * v.z;
        s = s + m.m[3][i] * v.w;
        rp[i] = s;
    }
    return r;
}

// Default.vert:60-105 for one vertex of one draw.
VsOut vertex_shader(const tri_vertex& in, const tri_push_constant& pc, const mat4& pv,
                    const float* bones, uint32_t bone_count, const mat4* lvp) {
    const mat4 model = load_mat4(pc.model);
    vec4 sp{in.position[0], in.position[1], in.position[2], 1.0f};
    vec3 sn{in.normal[0], in.normal[1], in.normal[2]};
    if (pc.bone_count > 0) {  // Default.vert:64-85
        mat4 skin = mat4_zero();
        for (int k = 0; k < TRI_MAX_BONE_INFLUENCES; ++k) {
            const float w = in.bone_weights[k];
            if (w <= 0.0f) continue;
            const int32_t bi = in.bone_indices[k];
            if (bi < 0 || bi >= pc.bone_count) continue;
            const uint32_t buf = (uint32_t)(pc.bone_offset + bi);
            if (buf >= bone_count) continue;  // robust access: out-of-palette reads contribute 0
            const float* b = bones + 16ull * buf;
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) skin.m[c][r] = skin.m[c][r] + w * b[c * 4 + r];
        }
        sp = mat_vec_seq(skin, sp);
        vec3 n;
        n.x = (skin.m[0][0] * sn.x + skin.m[1][0] * sn.y) + skin.m[2][0] * sn.z;
        n.y = (skin.m[0][1] * sn.x + skin.m[1][1] * sn.y) + skin.m[2][1] * sn.z;
        n.z = (skin.m[0][2] * sn.x + skin.m[1][2] * sn.y) + skin.m[2][2] * sn.z;
        sn = n;
    }
    const vec4 world = mat_vec_seq(model, sp);

    // transpose(inverse(mat3(M))) — glm mat3 inverse (cofactors * 1/det)
    const float (*m)[4] = model.m;
    const float det = (m[0][0] * (m[1][1] * m[2][2] - m[2][1] * m[1][2]) -
                       m[1][0] * (m[0][1] * m[2][2] - m[2][1] * m[0][2])) +
                      m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2]);
    const float od = 1.0f / det;
    float inv[3][3];
    inv[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]) * od;
    inv[1][0] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]) * od;
    inv[2][0] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]) * od;
    inv[0][1] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]) * od;
    inv[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]) * od;
    inv[2][1] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]) * od;
    inv[0][2] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]) * od;
    inv[1][2] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]) * od;
    inv[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]) * od;
    // normal matrix NM = transpose(inv): NM[c][r] = inv[r][c]; N' = NM * n
    vec3 nn;
    nn.x = (inv[0][0] * sn.x + inv[0][1] * sn.y) + inv[0][2] * sn.z;
    nn.y = (inv[1][0] * sn.x + inv[1][1] * sn.y) + inv[1][2] * sn.z;
    nn.z = (inv[2][0] * sn.x + inv[2][1] * sn.y) + inv[2][2] * sn.z;

    VsOut o;
    o.world = {world.x, world.y, world.z};
    o.normal = normalize(nn);
    o.uv.x = (in.texcoord[0] * pc.texture_scale[0]) * pc.tiling_factor + pc.texture_offset[0];
    o.uv.y = (in.texcoord[1] * pc.texture_scale[1]) * pc.tiling_factor + pc.texture_offset[1];
    o.color = {in.color[0], in.color[1], in.color[2]};
    o.clip = mat_vec_seq(pv, world);  // (P*V)*world, Default.vert:104
    o.lpos = {0.0f, 0.0f, 0.0f};
    if (lvp) {  // shadow pre-pass (tri_shadow_config): the affine light transform of the same world point
        const vec4 l = mat_vec_seq(*lvp, world);
        o.lpos = {l.x, l.y, l.z};
    }
    return o;
}

struct RTri {
    int32_t X[3], Y[3];
    float z[3], iw[3];
    uint32_t v[3];  // indices into the VsOut pool
    uint32_t prim, sub, draw;
    int64_t S;  // 2x area in 1/256-px units, > 0 after orientation normalisation
    bool far_clip;
    int32_t px0, px1, py0, py1;
    int64_t a[3], b[3], c[3], D[3];
    float dzdX, dzdY;
};

struct Setup {
    uint32_t W, H, y0, y1;
    float hw, hh, gx, gy;
};

inline int32_t floor_shift8(int32_t v) { return v >> 8; }  // arithmetic shift == floor(v/256)

// Direct (unclipped) triangle setup. Returns false if culled / empty.
bool setup_triangle(const Setup& su, const VsOut* const vs[3], const uint32_t vid[3], uint32_t prim,
                    uint32_t sub, uint32_t draw, RTri& t) {
    int32_t X[3], Y[3];
    float z[3], iw[3];
    bool far = false;
    for (int k = 0; k < 3; ++k) {
        // perspective divide as x * (1/w) with a correctly rounded 1/w (one divide per vertex)
        const vec4 c = vs[k]->clip;
        iw[k] = 1.0f / c.w;
        const float xd = c.x * iw[k], yd = c.y * iw[k], zd = c.z * iw[k];
        const float xf = xd * su.hw + su.hw;
        const float yf = yd * su.hh + su.hh;
        X[k] = (int32_t)std::rint(xf * 256.0f);
        Y[k] = (int32_t)std::rint(yf * 256.0f);
        z[k] = zd;
        far = far || (zd > 1.0f);
    }
    const int64_t S = (int64_t)(X[1] - X[0]) * (int64_t)(Y[2] - Y[0]) -
                      (int64_t)(Y[1] - Y[0]) * (int64_t)(X[2] - X[0]);
    // Vulkan a = -S/2; front-facing (CCW) iff a > 0 iff S < 0; cullMode BACK drops S > 0.
    if (S >= 0) return false;
    int o[3] = {0, 2, 1};  // swap v1<->v2 so the edge functions see S' = -S > 0
    for (int k = 0; k < 3; ++k) {
        t.X[k] = X[o[k]];
        t.Y[k] = Y[o[k]];
        t.z[k] = z[o[k]];
        t.iw[k] = iw[o[k]];
        t.v[k] = vid[o[k]];
    }
    t.S = -S;
    const int32_t xmin = std::min(t.X[0], std::min(t.X[1], t.X[2]));
    const int32_t xmax = std::max(t.X[0], std::max(t.X[1], t.X[2]));
    const int32_t ymin = std::min(t.Y[0], std::min(t.Y[1], t.Y[2]));
    const int32_t ymax = std::max(t.Y[0], std::max(t.Y[1], t.Y[2]));
    // pixel centres 256*p+128 inside [min,max]
    int32_t px0 = -floor_shift8(128 - xmin), px1 = floor_shift8(xmax - 128);
    int32_t py0 = -floor_shift8(128 - ymin), py1 = floor_shift8(ymax - 128);
    px0 = std::max(px0, 0);
    px1 = std::min(px1, (int32_t)su.W - 1);
    py0 = std::max(py0, (int32_t)su.y0);
    py1 = std::min(py1, (int32_t)su.y1 - 1);
    if (px0 > px1 || py0 > py1) return false;
    t.px0 = px0; t.px1 = px1; t.py0 = py0; t.py1 = py1;
    for (int e = 0; e < 3; ++e) {
        const int i = e, j = (e + 1) % 3;
        const int64_t a = (int64_t)t.Y[i] - t.Y[j];
        const int64_t b = (int64_t)t.X[j] - t.X[i];
        const int64_t c = -(a * t.X[i] + b * t.Y[i]);
        const bool top_left = (a > 0) || (a == 0 && b > 0);
        const int64_t cp = c + 128 * a + 128 * b - (top_left ? 0 : 1);
        t.a[e] = a; t.b[e] = b; t.c[e] = c;
        t.D[e] = cp >> 8;  // floor
    }
    const float fX1 = (float)(t.X[1] - t.X[0]), fY1 = (float)(t.Y[1] - t.Y[0]);
    const float fX2 = (float)(t.X[2] - t.X[0]), fY2 = (float)(t.Y[2] - t.Y[0]);
    const float fS = (float)t.S;
    const float dz1 = t.z[1] - t.z[0], dz2 = t.z[2] - t.z[0];
    t.dzdX = (dz1 * fY2 - dz2 * fY1) / fS;
    t.dzdY = (dz2 * fX1 - dz1 * fX2) / fS;
    t.far_clip = far;
    t.prim = prim; t.sub = sub; t.draw = draw;
    return true;
}

// Homogeneous Sutherland-Hodgman against w>=kWMin, z>=0 and the guard-band x/y planes, then a fan.
// A polygon vertex carries its clip position and its barycentric weights on the source triangle, both
// interpolated along the clipped edges (x + t * (y - x)); its varyings are then the weighted sums
// (b0 * a0 + b1 * a1) + b2 * a2 of the source vertices' varyings. Vulkan leaves the precision of
// clipped attributes to the implementation; this is the formulation the kernels use too.
struct ClipV {
    vec4 c;
    float b0, b1, b2;
};

int clip_polygon(const Setup& su, const VsOut in[3], VsOut* out /* >= 9 */) {
    ClipV bufA[12], bufB[12];
    int n = 3;
    for (int k = 0; k < 3; ++k) bufA[k] = {in[k].clip, k == 0 ? 1.0f : 0.0f, k == 1 ? 1.0f : 0.0f, k == 2 ? 1.0f : 0.0f};
    ClipV* src = bufA;
    ClipV* dst = bufB;
    for (int plane = 0; plane < 6 && n > 0; ++plane) {
        auto dist = [&](const ClipV& v) -> float {
            const vec4 c = v.c;
            switch (plane) {
                case 0: return c.w - kWMin;
                case 1: return c.z;
                case 2: return c.x + su.gx * c.w;
                case 3: return su.gx * c.w - c.x;
                case 4: return c.y + su.gy * c.w;
                default: return su.gy * c.w - c.y;
            }
        };
        int m = 0;
        for (int i = 0; i < n; ++i) {
            const ClipV& a = src[i];
            const ClipV& b = src[(i + 1) % n];
            const float da = dist(a), db = dist(b);
            if (da >= 0.0f && m < 12) dst[m++] = a;
            if ((da >= 0.0f) != (db >= 0.0f) && m < 12) {
                const float t = da / (da - db);
                auto l = [t](float x, float y) { return x + t * (y - x); };
                dst[m++] = {{l(a.c.x, b.c.x), l(a.c.y, b.c.y), l(a.c.z, b.c.z), l(a.c.w, b.c.w)},
                            l(a.b0, b.b0), l(a.b1, b.b1), l(a.b2, b.b2)};
            }
        }
        n = m;
        std::swap(src, dst);
    }
    // a triangle clipped by 6 planes has at most 9 vertices; a numerically non-convex polygon is cut
    // to its first 9 (fan sub-triangle indices 0..6, as the kernels' 3-bit key field requires)
    n = std::min(n, 9);
    for (int k = 0; k < n; ++k) {
        const ClipV& v = src[k];
        auto w = [&](float x0, float x1, float x2) { return (v.b0 * x0 + v.b1 * x1) + v.b2 * x2; };
        VsOut& o = out[k];
        o.clip = v.c;
        o.world = {w(in[0].world.x, in[1].world.x, in[2].world.x), w(in[0].world.y, in[1].world.y, in[2].world.y),
                   w(in[0].world.z, in[1].world.z, in[2].world.z)};
        o.normal = {w(in[0].normal.x, in[1].normal.x, in[2].normal.x), w(in[0].normal.y, in[1].normal.y, in[2].normal.y),
                    w(in[0].normal.z, in[1].normal.z, in[2].normal.z)};
        o.uv = {w(in[0].uv.x, in[1].uv.x, in[2].uv.x), w(in[0].uv.y, in[1].uv.y, in[2].uv.y)};
        o.color = {w(in[0].color.x, in[1].color.x, in[2].color.x), w(in[0].color.y, in[1].color.y, in[2].color.y),
                   w(in[0].color.z, in[1].color.z, in[2].color.z)};
        o.lpos = {w(in[0].lpos.x, in[1].lpos.x, in[2].lpos.x), w(in[0].lpos.y, in[1].lpos.y, in[2].lpos.y),
                  w(in[0].lpos.z, in[1].lpos.z, in[2].lpos.z)};
    }
    return n;
}

// ---- fragment stage (Default.frag) -----------------------------------------------------------
struct Texture {
    uint32_t w = 1, h = 1;
    std::vector<uint8_t> rgba{255, 255, 255, 255};  // slot 0 default white (Renderer.cpp:3415-3430)
};

float g_srgb_lut[256];
void init_srgb_lut() {
    static bool done = false;
    if (done) return;
    for (int i = 0; i < 256; ++i) {
        const double c = i / 255.0;
        const double l = c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4);
        g_srgb_lut[i] = (float)l;
    }
    done = true;
}

inline float lerpf(float x, float y, float t) { return x + t * (y - x); }

// texture(sampler2D[slot], uv): SRGB decode before LINEAR filtering, REPEAT, level 0 only.
vec4 sample_texture(const Texture& tx, vec2 uv) {
    const float u = uv.x * (float)tx.w - 0.5f;
    const float v = uv.y * (float)tx.h - 0.5f;
    const float fu = std::floor(u), fv = std::floor(v);
    const float a = u - fu, b = v - fv;
    auto wrap = [](int64_t i, uint32_t n) -> uint32_t {
        int64_t r = i % (int64_t)n;
        if (r < 0) r += n;
        return (uint32_t)r;
    };
    const int64_t i0 = (int64_t)fu, j0 = (int64_t)fv;
    const uint32_t x0 = wrap(i0, tx.w), x1 = wrap(i0 + 1, tx.w);
    const uint32_t y0 = wrap(j0, tx.h), y1 = wrap(j0 + 1, tx.h);
    auto texel = [&](uint32_t x, uint32_t y) -> vec4 {
        const uint8_t* p = &tx.rgba[4ull * ((uint64_t)y * tx.w + x)];
        return {g_srgb_lut[p[0]], g_srgb_lut[p[1]], g_srgb_lut[p[2]], (float)p[3] / 255.0f};
    };
    const vec4 t00 = texel(x0, y0), t10 = texel(x1, y0), t01 = texel(x0, y1), t11 = texel(x1, y1);
    vec4 r;
    r.x = lerpf(lerpf(t00.x, t10.x, a), lerpf(t01.x, t11.x, a), b);
    r.y = lerpf(lerpf(t00.y, t10.y, a), lerpf(t01.y, t11.y, a), b);
    r.z = lerpf(lerpf(t00.z, t10.z, a), lerpf(t01.z, t11.z, a), b);
    r.w = lerpf(lerpf(t00.w, t10.w, a), lerpf(t01.w, t11.w, a), b);
    return r;
}

inline float clampf(float x, float lo, float hi) { return std::min(std::max(x, lo), hi); }
inline float maxf(float a, float b) { return std::max(a, b); }

float distribution_ggx(vec3 N, vec3 H, float roughness) {  // Default.frag:69-78
    const float a = roughness * roughness;
    const float a2 = a * a;
    const float NdotH = maxf(dot(N, H), 0.0f);
    const float NdotH2 = NdotH * NdotH;
    const float denom = (NdotH2 * (a2 - 1.0f) + 1.0f);
    return a2 / ((kPi * denom) * denom);
}
float geometry_schlick_ggx(float NdotV, float roughness) {  // :80-87
    const float r = roughness + 1.0f;
    const float k = (r * r) / 8.0f;
    const float denom = NdotV * (1.0f - k) + k;
    return NdotV / maxf(denom, 1e-4f);
}
float geometry_smith(vec3 N, vec3 V, vec3 L, float roughness) {  // :89-97
    const float NdotV = maxf(dot(N, V), 0.0f);
    const float NdotL = maxf(dot(N, L), 0.0f);
    const float ggx2 = geometry_schlick_ggx(NdotV, roughness);
    const float ggx1 = geometry_schlick_ggx(NdotL, roughness);
    return ggx1 * ggx2;
}
vec3 fresnel_schlick(float cosTheta, vec3 F0) {  // :99-102
    const float p = std::pow(clampf(1.0f - cosTheta, 0.0f, 1.0f), 5.0f);
    return {F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p};
}
vec3 evaluate_pbr(vec3 L, vec3 radiance, vec3 N, vec3 V, vec3 albedo, float metallic,
                  float roughness, vec3 F0) {  // :104-121
    const vec3 H = normalize(V + L);
    const float NDF = distribution_ggx(N, H, roughness);
    const float G = geometry_smith(N, V, L, roughness);
    const vec3 F = fresnel_schlick(maxf(dot(H, V), 0.0f), F0);
    const vec3 num = F * (NDF * G);
    const float den = maxf((4.0f * maxf(dot(N, V), 0.0f)) * maxf(dot(N, L), 0.0f), 1e-4f);
    const vec3 spec = {num.x / den, num.y / den, num.z / den};
    const vec3 kD = vec3{1.0f - F.x, 1.0f - F.y, 1.0f - F.z} * (1.0f - metallic);
    const float NdotL = maxf(dot(N, L), 0.0f);
    const vec3 diff = {(kD.x * albedo.x) / kPi, (kD.y * albedo.y) / kPi, (kD.z * albedo.z) / kPi};
    return ((diff + spec) * radiance) * NdotL;
}

struct FragIn {
    vec3 world, normal;
    vec2 uv;
    vec3 color;
};

// Default.frag:123-180 (AiBlendConfig.w == 0 path). Returns linear RGBA before UNORM conversion.
vec4 fragment_shader(const FragIn& f, const tri_push_constant& pc, const tri_global_ubo& g,
                     const tri_material_record& mat, const Texture& tex, float sun_vis) {
    const vec3 Nn = normalize(f.normal);
    const vec3 N = normalize(Nn);  // normalize(TBN * (0,0,1)) == normalize(N): T/B are dead
    const vec3 cam{g.camera_position[0], g.camera_position[1], g.camera_position[2]};
    const vec3 V = normalize(cam - f.world);
    const vec4 s = sample_texture(tex, f.uv);
    const vec3 base{mat.base_color_factor[0], mat.base_color_factor[1], mat.base_color_factor[2]};
    const vec3 tint{pc.tint[0], pc.tint[1], pc.tint[2]};
    const vec3 albedo = ((vec3{s.x, s.y, s.z} * base) * tint) * f.color;
    const float metallic = clampf(mat.material_factors[0], 0.0f, 1.0f);
    const float roughness = clampf(mat.material_factors[1], 0.045f, 1.0f);
    const float ambient_strength = clampf(mat.material_factors[2], 0.0f, 1.0f);
    // mix(vec3(0.04), albedo, metallic) = x*(1-a) + y*a
    const vec3 F0 = {0.04f * (1.0f - metallic) + albedo.x * metallic,
                     0.04f * (1.0f - metallic) + albedo.y * metallic,
                     0.04f * (1.0f - metallic) + albedo.z * metallic};
    vec3 direct{0.0f, 0.0f, 0.0f};
    if (g.light_counts[0] > 0u) {
        const vec3 L = normalize(vec3{-g.directional_light_direction[0], -g.directional_light_direction[1],
                                      -g.directional_light_direction[2]});
        // sun_vis: the shadow pre-pass's visibility (1 without it, so the product is exact)
        const vec3 rad = (vec3{g.directional_light_color[0], g.directional_light_color[1],
                               g.directional_light_color[2]} * g.directional_light_color[3]) * sun_vis;
        direct = direct + evaluate_pbr(L, rad, N, V, albedo, metallic, roughness, F0);
    }
    const uint32_t pcount = std::min(g.light_counts[1], 8u);
    for (uint32_t i = 0; i < pcount; ++i) {
        const tri_point_light& pl = g.point_lights[i];
        const vec3 to = vec3{pl.position_range[0], pl.position_range[1], pl.position_range[2]} - f.world;
        const float dist = length(to);
        if (dist <= 1e-4f) continue;
        const vec3 L = {to.x / dist, to.y / dist, to.z / dist};
        const float radius = maxf(pl.position_range[3], 1e-4f);
        const float nd = clampf(dist / radius, 0.0f, 1.0f);
        float att = 1.0f - nd;
        att = att * att;
        const vec3 rad = (vec3{pl.color_intensity[0], pl.color_intensity[1], pl.color_intensity[2]} *
                          pl.color_intensity[3]) * att;
        direct = direct + evaluate_pbr(L, rad, N, V, albedo, metallic, roughness, F0);
    }
    const vec3 amb = ((vec3{g.ambient_color_intensity[0], g.ambient_color_intensity[1],
                            g.ambient_color_intensity[2]} * g.ambient_color_intensity[3]) * albedo) *
                     ambient_strength;
    vec3 c = amb + direct;
    c = {c.x / (c.x + 1.0f), c.y / (c.y + 1.0f), c.z / (c.z + 1.0f)};
    const float gamma = 1.0f / 2.2f;
    c = {std::pow(c.x, gamma), std::pow(c.y, gamma), std::pow(c.z, gamma)};
    const float alpha = (mat.base_color_factor[3] * pc.tint[3]) * s.w;
    return {c.x, c.y, c.z, alpha};
}

// ---- skybox pass ---------------------------------------------------------------------------------
// Skybox.cpp:13-79 (cube of half-size 1 scaled by 20, pushed as the model matrix), Skybox.vert:30-41
// (gl_Position = (P * mat4(mat3(View)) * world).xyww, outDirection = mat3(View) * world),
// Skybox.frag:28-35 (texture(samplerCube, normalize(dir)).rgb, alpha 1), pipeline
// Pipeline.cpp:727-880 (cull FRONT, depth LEQUAL, no depth write), recorded before the meshes
// (Renderer.cpp:5076-5082). Every pixel whose ray leaves the cube in front of the camera gets the
// sky; the interpolated direction at a pixel is the view-space exit point of that pixel's ray, which
// is computed here analytically. Cube sampling is Vulkan's: major-axis face selection, LINEAR
// within the face (sRGB decoded before filtering, one level), seamless edges (texels across an
// edge come from the adjacent face; a corner texel is the mean of the three that meet there).
struct SkyConst {
    float ip[16];  // inverse(Projection), column-major (computed in double, rounded)
    float R[9];    // mat3(View), column-major
    float pw[4];   // Projection row 3 (clip w of a view-space point)
};

// 4x4 inverse by cofactors in double (column-major in/out).
void invert4(const float* m, float* out) {
    double a[16], inv[16];
    for (int i = 0; i < 16; ++i) a[i] = m[i];
    inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] + a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
    inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] - a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
    inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] + a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
    inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] - a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
    inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] - a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
    inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] + a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
    inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] - a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
    inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] + a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
    inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] + a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
    inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] - a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
    inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] + a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
    inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] - a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
    inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] - a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
    inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] + a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
    inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] - a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
    inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] + a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
    const double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
    const double id = det != 0.0 ? 1.0 / det : 0.0;
    for (int i = 0; i < 16; ++i) out[i] = (float)(inv[i] * id);
}

SkyConst sky_constants(const tri_global_ubo& g) {
    SkyConst k;
    invert4(g.projection, k.ip);
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) k.R[c * 3 + r] = g.view[c * 4 + r];
    for (int c = 0; c < 4; ++c) k.pw[c] = g.projection[c * 4 + 3];
    return k;
}

// Vulkan cube face selection: face 0..5 = +X,-X,+Y,-Y,+Z,-Z; (s, t) in [0, 1] on that face.
int cube_face(vec3 d, float& s, float& t) {
    const float ax = std::fabs(d.x), ay = std::fabs(d.y), az = std::fabs(d.z);
    int face;
    float ma, sc, tc;
    if (ax >= ay && ax >= az) {
        face = d.x >= 0.0f ? 0 : 1; ma = ax; sc = d.x >= 0.0f ? -d.z : d.z; tc = -d.y;
    } else if (ay >= az) {
        face = d.y >= 0.0f ? 2 : 3; ma = ay; sc = d.x; tc = d.y >= 0.0f ? d.z : -d.z;
    } else {
        face = d.z >= 0.0f ? 4 : 5; ma = az; sc = d.z >= 0.0f ? d.x : -d.x; tc = -d.y;
    }
    if (!(ma > 0.0f)) { s = 0.5f; t = 0.5f; return face; }
    s = 0.5f * (sc / ma) + 0.5f;
    t = 0.5f * (tc / ma) + 0.5f;
    return face;
}

// Direction through face-local (sc, tc) in [-1, 1]^2 (major axis component 1).
vec3 face_dir(int face, float sc, float tc) {
    switch (face) {
        case 0: return {1.0f, -tc, -sc};
        case 1: return {-1.0f, -tc, sc};
        case 2: return {sc, 1.0f, tc};
        case 3: return {sc, -1.0f, -tc};
        case 4: return {sc, -tc, 1.0f};
        default: return {-sc, -tc, -1.0f};
    }
}

struct Sky {
    const uint8_t* faces;
    int32_t n;
    vec3 texel(int face, int32_t i, int32_t j) const {  // decoded linear rgb
        const uint8_t* p = faces + 4ull * (((uint64_t)face * n + (uint64_t)j) * n + (uint64_t)i);
        return {g_srgb_lut[p[0]], g_srgb_lut[p[1]], g_srgb_lut[p[2]]};
    }
    // texel (i, j) of `face` with exactly one coordinate outside [0, n): from the adjacent face
    vec3 across(int face, int32_t i, int32_t j) const {
        const float sc = 2.0f * (((float)i + 0.5f) / (float)n) - 1.0f;
        const float tc = 2.0f * (((float)j + 0.5f) / (float)n) - 1.0f;
        float s, t;
        const int f2 = cube_face(face_dir(face, sc, tc), s, t);
        const int32_t i2 = std::min(std::max((int32_t)std::floor(s * (float)n), 0), n - 1);
        const int32_t j2 = std::min(std::max((int32_t)std::floor(t * (float)n), 0), n - 1);
        return texel(f2, i2, j2);
    }
    vec3 fetch(int face, int32_t i, int32_t j) const {
        const bool in_i = i >= 0 && i < n, in_j = j >= 0 && j < n;
        if (in_i && in_j) return texel(face, i, j);
        if (in_i || in_j) return across(face, i, j);
        const int32_t ci = std::min(std::max(i, 0), n - 1), cj = std::min(std::max(j, 0), n - 1);
        const vec3 a = texel(face, ci, cj), b = across(face, i, cj), c = across(face, ci, j);
        return {((a.x + b.x) + c.x) / 3.0f, ((a.y + b.y) + c.y) / 3.0f, ((a.z + b.z) + c.z) / 3.0f};
    }
    vec3 sample(vec3 d) const {
        float s, t;
        const int face = cube_face(d, s, t);
        const float u = s * (float)n - 0.5f, v = t * (float)n - 0.5f;
        const float fu = std::floor(u), fv = std::floor(v);
        const float a = u - fu, b = v - fv;
        const int32_t i0 = (int32_t)fu, j0 = (int32_t)fv;
        const vec3 t00 = fetch(face, i0, j0), t10 = fetch(face, i0 + 1, j0);
        const vec3 t01 = fetch(face, i0, j0 + 1), t11 = fetch(face, i0 + 1, j0 + 1);
        return {lerpf(lerpf(t00.x, t10.x, a), lerpf(t01.x, t11.x, a), b),
                lerpf(lerpf(t00.y, t10.y, a), lerpf(t01.y, t11.y, a), b),
                lerpf(lerpf(t00.z, t10.z, a), lerpf(t01.z, t11.z, a), b)};
    }
};

// Sky colour of pixel (px, py); false where the skybox cube does not cover the pixel.
bool sky_pixel(const SkyConst& k, const Sky& sky, uint32_t W, uint32_t H, int32_t px, int32_t py, vec3& out) {
    const float xn = (float)(2 * px + 1) / (float)W - 1.0f;
    const float yn = (float)(2 * py + 1) / (float)H - 1.0f;
    auto unproject = [&](float zn, vec3& p) {
        const float* m = k.ip;
        const float x = ((m[0] * xn + m[4] * yn) + m[8] * zn) + m[12];
        const float y = ((m[1] * xn + m[5] * yn) + m[9] * zn) + m[13];
        const float z = ((m[2] * xn + m[6] * yn) + m[10] * zn) + m[14];
        const float w = ((m[3] * xn + m[7] * yn) + m[11] * zn) + m[15];
        p = {x / w, y / w, z / w};
    };
    vec3 o, o1;
    unproject(0.0f, o);
    unproject(1.0f, o1);
    const vec3 r = o1 - o;
    // into cube space (inverse of the rotation mat3(View) = its transpose)
    const float* R = k.R;
    const vec3 oc = {(R[0] * o.x + R[1] * o.y) + R[2] * o.z, (R[3] * o.x + R[4] * o.y) + R[5] * o.z,
                     (R[6] * o.x + R[7] * o.y) + R[8] * o.z};
    const vec3 rc = {(R[0] * r.x + R[1] * r.y) + R[2] * r.z, (R[3] * r.x + R[4] * r.y) + R[5] * r.z,
                     (R[6] * r.x + R[7] * r.y) + R[8] * r.z};
    const float half = 20.0f;
    float t_in = -INFINITY, t_out = INFINITY;
    const float oa[3] = {oc.x, oc.y, oc.z}, ra[3] = {rc.x, rc.y, rc.z};
    for (int a = 0; a < 3; ++a) {
        if (ra[a] != 0.0f) {
            const float t0 = (-half - oa[a]) / ra[a], t1 = (half - oa[a]) / ra[a];
            t_in = std::max(t_in, std::min(t0, t1));
            t_out = std::min(t_out, std::max(t0, t1));
        } else if (oa[a] < -half || oa[a] > half) {
            return false;
        }
    }
    if (!(t_out >= t_in)) return false;
    const vec3 h = o + r * t_out;  // view-space exit point == interpolated outDirection
    const float w = ((k.pw[0] * h.x + k.pw[1] * h.y) + k.pw[2] * h.z) + k.pw[3];
    if (!(w > 0.0f)) return false;  // behind the camera: clipped
    out = sky.sample(normalize(h));
    return true;
}

// ---- shadow-map pre-pass (tri_shadow_config) ---------------------------------
// Depth-only raster of every triangle by the affine light transform into a size x size map: the main
// pass's snap / fill / plane-depth rules with the light NDC as window coordinates (w = 1), no culling
// (a clockwise triangle is set up with its own orientation), depth clamped to [0, 1] instead of
// near/far clipping, a slope-scaled depth bias (Vulkan depthBiasSlopeFactor: + slope * the triangle's
// largest depth change per texel) before the clamp, guard-band violators dropped; each texel keeps the
// minimum depth (LEQUAL with writes: the result does not depend on primitive order).
struct ShadowMap {
    uint32_t S = 0;
    float bias = 0.0f;   // lookup: subtracted from the receiver's depth
    float slope = 0.0f;  // raster: depthBiasSlopeFactor
    std::vector<float> d;
};

void shadow_raster_triangle(ShadowMap& sm, const vec3& a, const vec3& b, const vec3& c, int32_t row0, int32_t row1) {
    const float hs = (float)sm.S * 0.5f;
    const float g = (2.0f * kGuardBandPx) / (float)sm.S - 1.0f;
    const vec3 v[3] = {a, b, c};
    int32_t X[3], Y[3];
    float z[3];
    for (int k = 0; k < 3; ++k) {
        // the main pass's snap with w = 1: iw = 1 / 1, xd = x * 1
        if (v[k].x < -g || v[k].x > g || v[k].y < -g || v[k].y > g) return;  // beyond the guard band
        X[k] = (int32_t)std::rint((v[k].x * hs + hs) * 256.0f);
        Y[k] = (int32_t)std::rint((v[k].y * hs + hs) * 256.0f);
        z[k] = v[k].z;
    }
    auto all = [&](auto f) { return f(v[0]) && f(v[1]) && f(v[2]); };
    if (all([](vec3 p) { return p.x + 1.0f < 0.0f; }) || all([](vec3 p) { return 1.0f - p.x < 0.0f; }) ||
        all([](vec3 p) { return p.y + 1.0f < 0.0f; }) || all([](vec3 p) { return 1.0f - p.y < 0.0f; }))
        return;  // trivially outside the map (covers no texel centre)
    int64_t S = (int64_t)(X[1] - X[0]) * (int64_t)(Y[2] - Y[0]) - (int64_t)(Y[1] - Y[0]) * (int64_t)(X[2] - X[0]);
    if (S == 0) return;
    int o[3] = {0, 1, 2};
    if (S < 0) { o[1] = 2; o[2] = 1; S = -S; }  // same v1 <-> v2 normalisation as the main pass
    int32_t tX[3], tY[3];
    float tz[3];
    for (int k = 0; k < 3; ++k) { tX[k] = X[o[k]]; tY[k] = Y[o[k]]; tz[k] = z[o[k]]; }
    const int32_t xmin = std::min(tX[0], std::min(tX[1], tX[2])), xmax = std::max(tX[0], std::max(tX[1], tX[2]));
    const int32_t ymin = std::min(tY[0], std::min(tY[1], tY[2])), ymax = std::max(tY[0], std::max(tY[1], tY[2]));
    const int32_t px0 = std::max(-floor_shift8(128 - xmin), 0), px1 = std::min(floor_shift8(xmax - 128), (int32_t)sm.S - 1);
    const int32_t py0 = std::max(-floor_shift8(128 - ymin), row0), py1 = std::min(floor_shift8(ymax - 128), row1);
    if (px0 > px1 || py0 > py1) return;
    int64_t ea[3], eb[3], eD[3];
    for (int e = 0; e < 3; ++e) {
        const int i = e, j = (e + 1) % 3;
        const int64_t aa = (int64_t)tY[i] - tY[j];
        const int64_t bb = (int64_t)tX[j] - tX[i];
        const int64_t cc = -(aa * tX[i] + bb * tY[i]);
        const bool top_left = (aa > 0) || (aa == 0 && bb > 0);
        ea[e] = aa; eb[e] = bb;
        eD[e] = (cc + 128 * aa + 128 * bb - (top_left ? 0 : 1)) >> 8;
    }
    const float fX1 = (float)(tX[1] - tX[0]), fY1 = (float)(tY[1] - tY[0]);
    const float fX2 = (float)(tX[2] - tX[0]), fY2 = (float)(tY[2] - tY[0]);
    const float fS = (float)S;
    const float dz1 = tz[1] - tz[0], dz2 = tz[2] - tz[0];
    const float dzdX = (dz1 * fY2 - dz2 * fY1) / fS;
    const float dzdY = (dz2 * fX1 - dz1 * fX2) / fS;
    // slope-scaled bias: slope * the largest depth change per texel (the plane's per-1/256 slopes * 256)
    const float off = sm.slope * (std::max(std::fabs(dzdX), std::fabs(dzdY)) * 256.0f);
    for (int32_t py = py0; py <= py1; ++py)
        for (int32_t px = px0; px <= px1; ++px) {
            bool inside = true;
            for (int e = 0; e < 3; ++e) inside = inside && (ea[e] * px + eb[e] * py + eD[e] >= 0);
            if (!inside) continue;
            const float t1 = dzdX * (float)(256 * px + 128 - tX[0]);
            const float t2 = dzdY * (float)(256 * py + 128 - tY[0]);
            float zz = ((tz[0] + t1) + t2) + off;
            if (!(zz > 0.0f)) zz = 0.0f;  // depth clamp (also canonicalises -0)
            if (zz > 1.0f) zz = 1.0f;
            float& d = sm.d[(size_t)py * sm.S + px];
            if (zz <= d) d = zz;
        }
}

// Fraction of the 2x2 bilinear depth compare that passes at light-NDC point l (1 outside the map).
float shadow_visibility(const ShadowMap& sm, vec3 l) {
    const float u = l.x * 0.5f + 0.5f, v = l.y * 0.5f + 0.5f;
    if (!(u >= 0.0f && u <= 1.0f && v >= 0.0f && v <= 1.0f)) return 1.0f;
    const float fx = u * (float)sm.S - 0.5f, fy = v * (float)sm.S - 0.5f;
    const float x0 = std::floor(fx), y0 = std::floor(fy);
    const float a = fx - x0, b = fy - y0;
    const int32_t i0 = (int32_t)x0, j0 = (int32_t)y0;
    const float zref = l.z - sm.bias;
    auto tap = [&](int32_t i, int32_t j) -> float {
        i = std::min(std::max(i, 0), (int32_t)sm.S - 1);
        j = std::min(std::max(j, 0), (int32_t)sm.S - 1);
        return zref <= sm.d[(size_t)j * sm.S + i] ? 1.0f : 0.0f;
    };
    const float c00 = tap(i0, j0), c10 = tap(i0 + 1, j0), c01 = tap(i0, j0 + 1), c11 = tap(i0 + 1, j0 + 1);
    return lerpf(lerpf(c00, c10, a), lerpf(c01, c11, a), b);
}

// Default.frag:186-188: texture(AiBlendTexture, gl_FragCoord.xy * AiBlendConfig.yz) on the AI texture of
// EnsureAiTextureResources (Renderer.cpp:1406-1470): R8G8B8A8_UNORM (decode b / 255), LINEAR, CLAMP_TO_EDGE, level 0,
// Vulkan's unnormalized coordinates u * width - 0.5, floor and fraction.
vec4 ai_sample(const uint8_t* tex, int32_t tw, int32_t th, float sx, float sy, int32_t px, int32_t py) {
    const float u = ((float)px + 0.5f) * sx, v = ((float)py + 0.5f) * sy;
    const float x = u * (float)tw - 0.5f, y = v * (float)th - 0.5f;
    const float fx = std::floor(x), fy = std::floor(y);
    const float a = x - fx, b = y - fy;
    const int32_t i0 = (int32_t)std::fmin(std::fmax(fx, -1.0f), 1.0e9f), j0 = (int32_t)std::fmin(std::fmax(fy, -1.0f), 1.0e9f);
    const int32_t xa = std::min(std::max(i0, 0), tw - 1), xb = std::min(std::max(i0 + 1, 0), tw - 1);
    const int32_t ya = std::min(std::max(j0, 0), th - 1), yb = std::min(std::max(j0 + 1, 0), th - 1);
    float r[4];
    for (int c = 0; c < 4; ++c) {
        auto t = [&](int32_t i, int32_t j) { return (float)tex[((size_t)j * tw + i) * 4 + c] / 255.0f; };
        r[c] = lerpf(lerpf(t(xa, ya), t(xb, ya), a), lerpf(t(xa, yb), t(xb, yb), a), b);
    }
    return {r[0], r[1], r[2], r[3]};
}
// GLSL mix(x, y, a) = x * (1 - a) + y * a
inline float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }

inline uint32_t unorm8(float c) {
    const float cc = std::fmin(std::fmax(c, 0.0f), 1.0f);  // NaN -> 0
    return (uint32_t)(int)(cc * 255.0f + 0.5f);
}
inline uint32_t pack_bgra(vec4 c) {
    return unorm8(c.z) | (unorm8(c.y) << 8) | (unorm8(c.x) << 16) | (unorm8(c.w) << 24);
}

}  // namespace

extern "C" int oracle_render(const oracle_scene* sc, uint32_t W, uint32_t H, uint32_t band_y0,
                             uint32_t band_y1, int threads, uint32_t* out_bgra, uint32_t* out_depth,
                             oracle_stats* stats) {
    if (!sc || !sc->ubo || W == 0 || H == 0 || W > TRI_MAX_DIM || H > TRI_MAX_DIM) return TRI_E_INVALID;
    if (band_y0 == 0 && band_y1 == 0) band_y1 = H;
    if (band_y0 >= band_y1 || band_y1 > H) return TRI_E_INVALID;
    init_srgb_lut();
    const tri_global_ubo& g = *sc->ubo;
    const mat4 pv = mul(load_mat4(g.projection), load_mat4(g.view));

    Setup su;
    su.W = W; su.H = H; su.y0 = band_y0; su.y1 = band_y1;
    su.hw = (float)W * 0.5f;
    su.hh = (float)H * 0.5f;
    su.gx = (2.0f * kGuardBandPx) / (float)W - 1.0f;
    su.gy = (2.0f * kGuardBandPx) / (float)H - 1.0f;

    // textures: unused slots alias slot 0 (Renderer.cpp:3645-3656)
    std::vector<Texture> texs(1);
    std::vector<int> slot_map(TRI_MAX_TEXTURE_SLOTS, 0);
    for (uint32_t i = 0; i < sc->texture_count; ++i) {
        const oracle_texture& t = sc->textures[i];
        if (t.slot >= TRI_MAX_TEXTURE_SLOTS || t.width == 0 || t.height == 0 || !t.rgba8_srgb) continue;
        Texture tx;
        tx.w = t.width; tx.h = t.height;
        tx.rgba.assign(t.rgba8_srgb, t.rgba8_srgb + 4ull * t.width * t.height);
        if (t.slot == 0) { texs[0] = tx; continue; }
        slot_map[t.slot] = (int)texs.size();
        texs.push_back(std::move(tx));
    }
    tri_material_record mat0{{1, 1, 1, 1}, {1, 1, 1, 0}};  // BuildMaterialPayload default
    if (sc->material_count > 0 && sc->materials) mat0 = sc->materials[0];

    const bool shadow_on = sc->shadow && sc->shadow->size > 0;
    if (shadow_on) {
        const float* m = sc->shadow->light_view_proj;
        if (sc->shadow->size > TRI_MAX_DIM || m[3] != 0.0f || m[7] != 0.0f || m[11] != 0.0f || m[15] != 1.0f)
            return TRI_E_INVALID;  // the light transform must be affine (orthographic)
    }
    const mat4 lvp = shadow_on ? load_mat4(sc->shadow->light_view_proj) : mat4_identity();
    std::vector<uint32_t> shadow_prims;  // (pool index of vertex 0, 1, 2) of every valid primitive, in order

    // ---- vertex stage + primitive assembly, in submission order ----
    std::vector<VsOut> pool;
    std::vector<RTri> tris;
    uint64_t tri_in = 0, clipped = 0;
    uint32_t prim_base = 0;
    for (uint32_t d = 0; d < sc->draw_count; ++d) {
        const tri_draw& dr = sc->draws[d];
        if (dr.mesh_index >= sc->mesh_count) continue;
        const tri_mesh_range& mr = sc->meshes[dr.mesh_index];
        if (mr.index_count < 3 || (uint64_t)mr.first_index + mr.index_count > sc->index_count) continue;
        const uint32_t nprim = mr.index_count / 3;
        uint32_t mn = 0xFFFFFFFFu, mx = 0;
        for (uint32_t i = 0; i < nprim * 3; ++i) {
            const uint32_t v = sc->indices[mr.first_index + i];
            mn = std::min(mn, v);
            mx = std::max(mx, v);
        }
        const uint32_t pool_base = (uint32_t)pool.size();
        std::vector<uint8_t> valid(mx - mn + 1);
        pool.resize(pool.size() + (mx - mn + 1));
        for (uint32_t v = mn; v <= mx; ++v) {
            const int64_t gi = (int64_t)mr.base_vertex + v;
            valid[v - mn] = (gi >= 0 && (uint64_t)gi < sc->vertex_count);
            if (valid[v - mn])
                pool[pool_base + (v - mn)] =
                    vertex_shader(sc->vertices[gi], dr.pc, pv, sc->bones, sc->bone_count, shadow_on ? &lvp : nullptr);
            if (v == 0xFFFFFFFFu) break;
        }
        for (uint32_t t = 0; t < nprim; ++t) {
            const uint32_t prim = prim_base + t;
            ++tri_in;
            uint32_t vid[3];
            bool ok = true;
            for (int k = 0; k < 3; ++k) {
                const uint32_t v = sc->indices[mr.first_index + 3 * t + k];
                ok = ok && valid[v - mn];
                vid[k] = pool_base + (v - mn);
            }
            if (!ok) continue;
            if (shadow_on) shadow_prims.insert(shadow_prims.end(), {vid[0], vid[1], vid[2]});
            const VsOut* vs[3] = {&pool[vid[0]], &pool[vid[1]], &pool[vid[2]]};
            // trivial reject: all three outside one clip half-space (0<=z<=w, -w<=x,y<=w)
            auto all_neg = [&](auto f) { return f(vs[0]->clip) < 0.0f && f(vs[1]->clip) < 0.0f && f(vs[2]->clip) < 0.0f; };
            if (all_neg([](vec4 c) { return c.z; }) || all_neg([](vec4 c) { return c.w - c.z; }) ||
                all_neg([](vec4 c) { return c.x + c.w; }) || all_neg([](vec4 c) { return c.w - c.x; }) ||
                all_neg([](vec4 c) { return c.y + c.w; }) || all_neg([](vec4 c) { return c.w - c.y; }))
                continue;
            bool need_clip = false;
            for (int k = 0; k < 3; ++k) {
                const vec4 c = vs[k]->clip;
                need_clip = need_clip || (c.w < kWMin) || (c.z < 0.0f) || (c.x < -su.gx * c.w) ||
                            (c.x > su.gx * c.w) || (c.y < -su.gy * c.w) || (c.y > su.gy * c.w);
            }
            if (!need_clip) {
                RTri rt;
                if (setup_triangle(su, vs, vid, prim, 0, d, rt)) tris.push_back(rt);
                continue;
            }
            ++clipped;
            VsOut in[3] = {*vs[0], *vs[1], *vs[2]};
            VsOut poly[12];
            const int n = clip_polygon(su, in, poly);
            if (n < 3) continue;
            const uint32_t cbase = (uint32_t)pool.size();
            for (int k = 0; k < n; ++k) pool.push_back(poly[k]);
            for (int k = 1; k + 1 < n; ++k) {
                const uint32_t sv[3] = {cbase, cbase + (uint32_t)k, cbase + (uint32_t)k + 1};
                const VsOut* svs[3] = {&pool[sv[0]], &pool[sv[1]], &pool[sv[2]]};
                RTri rt;
                if (setup_triangle(su, svs, sv, prim, (uint32_t)(k - 1), d, rt)) tris.push_back(rt);
            }
        }
        prim_base += nprim;
        if (prim_base > kPrimMax) return TRI_E_INVALID;
    }

    if (threads <= 0) threads = 1;
    // ---- shadow-map pre-pass: rows of the map in parallel blocks, each walking every caster ----
    ShadowMap sm;
    if (shadow_on) {
        sm.S = sc->shadow->size;
        sm.bias = sc->shadow->depth_bias;
        sm.slope = sc->shadow->slope_bias;
        sm.d.assign((size_t)sm.S * sm.S, 1.0f);
        constexpr int32_t kRows = 64;
        const int32_t nb = ((int32_t)sm.S + kRows - 1) / kRows;
        std::atomic<int32_t> next{0};
        auto worker = [&]() {
            for (;;) {
                const int32_t blk = next.fetch_add(1);
                if (blk >= nb) break;
                const int32_t r0 = blk * kRows, r1 = std::min(r0 + kRows, (int32_t)sm.S) - 1;
                for (size_t t = 0; t < shadow_prims.size(); t += 3)
                    shadow_raster_triangle(sm, pool[shadow_prims[t]].lpos, pool[shadow_prims[t + 1]].lpos,
                                           pool[shadow_prims[t + 2]].lpos, r0, r1);
            }
        };
        std::vector<std::thread> ts;
        for (int i = 1; i < threads; ++i) ts.emplace_back(worker);
        worker();
        for (auto& th : ts) th.join();
        if (sc->out_shadow_map) std::memcpy(sc->out_shadow_map, sm.d.data(), sm.d.size() * 4);
    }

    // ---- rasterization: in-order LEQUAL depth test (Pipeline.cpp:655-658) ----
    const uint32_t rows = band_y1 - band_y0;
    std::vector<float> depth((size_t)rows * W, 1.0f);  // depth clear 1.0 (Renderer.cpp:5037)
    std::vector<int32_t> vis((size_t)rows * W, -1);
    constexpr uint32_t kBlock = 16;
    const uint32_t nblocks = (rows + kBlock - 1) / kBlock;
    std::vector<std::vector<uint32_t>> lists(nblocks);
    for (uint32_t i = 0; i < tris.size(); ++i) {
        const RTri& t = tris[i];
        const uint32_t b0 = ((uint32_t)t.py0 - band_y0) / kBlock, b1 = ((uint32_t)t.py1 - band_y0) / kBlock;
        for (uint32_t b = b0; b <= b1; ++b) lists[b].push_back(i);
    }
    std::atomic<uint32_t> next_block{0};
    std::atomic<uint64_t> frags{0};
    auto raster_worker = [&]() {
        uint64_t local_frags = 0;
        for (;;) {
            const uint32_t b = next_block.fetch_add(1);
            if (b >= nblocks) break;
            const int32_t ylo = (int32_t)(band_y0 + b * kBlock);
            const int32_t yhi = std::min((int32_t)band_y1 - 1, ylo + (int32_t)kBlock - 1);
            for (uint32_t ti : lists[b]) {
                const RTri& t = tris[ti];
                const int32_t ya = std::max(t.py0, ylo), yb = std::min(t.py1, yhi);
                for (int32_t py = ya; py <= yb; ++py) {
                    const int32_t Yp = 256 * py + 128;
                    for (int32_t px = t.px0; px <= t.px1; ++px) {
                        bool inside = true;
                        for (int e = 0; e < 3; ++e)
                            inside = inside && (t.a[e] * px + t.b[e] * py + t.D[e] >= 0);
                        if (!inside) continue;
                        ++local_frags;
                        const int32_t Xp = 256 * px + 128;
                        const float fdx = (float)(Xp - t.X[0]);
                        const float fdy = (float)(Yp - t.Y[0]);
                        const float t1 = t.dzdX * fdx;
                        const float t2 = t.dzdY * fdy;
                        float z = (t.z[0] + t1) + t2;
                        if (t.far_clip && z > 1.0f) continue;  // far plane (z <= w) clip
                        if (!(z > 0.0f)) z = 0.0f;               // also canonicalises -0
                        if (z > 1.0f) z = 1.0f;
                        const size_t idx = (size_t)(py - band_y0) * W + px;
                        if (z <= depth[idx]) {  // VK_COMPARE_OP_LESS_OR_EQUAL, write enabled
                            depth[idx] = z;
                            vis[idx] = (int32_t)ti;
                        }
                    }
                }
            }
        }
        frags += local_frags;
    };
    {
        std::vector<std::thread> pool_t;
        for (int i = 1; i < threads; ++i) pool_t.emplace_back(raster_worker);
        raster_worker();
        for (auto& th : pool_t) th.join();
    }

    // ---- fragment shading of the surviving fragment (no blending, no discard: the last passing
    //      fragment's colour is the pixel colour) ----
    const uint32_t clear = pack_bgra({sc->clear_rgba[0], sc->clear_rgba[1], sc->clear_rgba[2], sc->clear_rgba[3]});
    const bool has_sky = sc->sky_faces != nullptr && sc->sky_size > 0;
    // AiBlendConfig: w > 0 switches the blend on; the weight is clamp(x, 0, 1) and must be positive (Default.frag:182-185)
    const float ai_w = std::fmin(std::fmax(g.ai_blend_config[0], 0.0f), 1.0f);
    const bool ai_on = g.ai_blend_config[3] > 0.0f && ai_w > 0.0f && sc->ai_frame && sc->ai_width && sc->ai_height;
    const SkyConst skk = sky_constants(g);
    const Sky sky{sc->sky_faces, (int32_t)sc->sky_size};
    std::atomic<uint32_t> next_row{0};
    auto shade_worker = [&]() {
        for (;;) {
            const uint32_t r = next_row.fetch_add(1);
            if (r >= rows) break;
            const int32_t py = (int32_t)(band_y0 + r);
            for (uint32_t px = 0; px < W; ++px) {
                const size_t idx = (size_t)r * W + px;
                uint32_t dbits;
                std::memcpy(&dbits, &depth[idx], 4);
                if (out_depth) out_depth[idx] = dbits;
                const int32_t ti = vis[idx];
                if (ti < 0) {
                    vec3 skc;
                    if (out_bgra)
                        out_bgra[idx] = (has_sky && sky_pixel(skk, sky, W, H, (int32_t)px, py, skc))
                                            ? pack_bgra({skc.x, skc.y, skc.z, 1.0f})
                                            : clear;
                    continue;
                }
                const RTri& t = tris[ti];
                const int64_t Xp = 256 * (int64_t)px + 128, Yp = 256 * (int64_t)py + 128;
                const int64_t e01 = t.a[0] * Xp + t.b[0] * Yp + t.c[0];
                const int64_t e12 = t.a[1] * Xp + t.b[1] * Yp + t.c[1];
                const int64_t e20 = t.a[2] * Xp + t.b[2] * Yp + t.c[2];
                const float fS = (float)t.S;
                const float l0 = (float)e12 / fS, l1 = (float)e20 / fS, l2 = (float)e01 / fS;
                const float q0 = l0 * t.iw[0], q1 = l1 * t.iw[1], q2 = l2 * t.iw[2];
                const float qs = (q0 + q1) + q2;
                const float b0 = q0 / qs, b1 = q1 / qs, b2 = q2 / qs;
                const VsOut& v0 = pool[t.v[0]];
                const VsOut& v1 = pool[t.v[1]];
                const VsOut& v2 = pool[t.v[2]];
                auto ip = [&](float x0, float x1, float x2) { return (b0 * x0 + b1 * x1) + b2 * x2; };
                FragIn f;
                f.world = {ip(v0.world.x, v1.world.x, v2.world.x), ip(v0.world.y, v1.world.y, v2.world.y),
                           ip(v0.world.z, v1.world.z, v2.world.z)};
                f.normal = {ip(v0.normal.x, v1.normal.x, v2.normal.x), ip(v0.normal.y, v1.normal.y, v2.normal.y),
                            ip(v0.normal.z, v1.normal.z, v2.normal.z)};
                f.uv = {ip(v0.uv.x, v1.uv.x, v2.uv.x), ip(v0.uv.y, v1.uv.y, v2.uv.y)};
                f.color = {ip(v0.color.x, v1.color.x, v2.color.x), ip(v0.color.y, v1.color.y, v2.color.y),
                           ip(v0.color.z, v1.color.z, v2.color.z)};
                const tri_push_constant& pc = sc->draws[t.draw].pc;
                int slot = pc.texture_slot;
                const int tidx = (slot >= 0 && slot < TRI_MAX_TEXTURE_SLOTS) ? slot_map[slot] : 0;
                float vis = 1.0f;
                if (shadow_on && g.light_counts[0] > 0u)
                    vis = shadow_visibility(sm, {ip(v0.lpos.x, v1.lpos.x, v2.lpos.x), ip(v0.lpos.y, v1.lpos.y, v2.lpos.y),
                                                 ip(v0.lpos.z, v1.lpos.z, v2.lpos.z)});
                vec4 c = fragment_shader(f, pc, g, mat0, texs[tidx], vis);
                if (ai_on) {  // Default.frag:182-191
                    const vec4 ai = ai_sample(sc->ai_frame, (int32_t)sc->ai_width, (int32_t)sc->ai_height,
                                              g.ai_blend_config[1], g.ai_blend_config[2], (int32_t)px, py);
                    c = {mixf(c.x, ai.x, ai_w), mixf(c.y, ai.y, ai_w), mixf(c.z, ai.z, ai_w), mixf(c.w, ai.w, ai_w)};
                }
                if (out_bgra) out_bgra[idx] = pack_bgra(c);
            }
        }
    };
    {
        std::vector<std::thread> pool_t;
        for (int i = 1; i < threads; ++i) pool_t.emplace_back(shade_worker);
        shade_worker();
        for (auto& th : pool_t) th.join();
    }
    if (stats) {
        stats->triangles_in = tri_in;
        stats->triangles_setup = tris.size();
        stats->triangles_clipped = clipped;
        stats->fragments_tested = frags.load();
    }
    return TRI_OK;
}

// ---- host-side restatements ----------------------------------------------------------------

namespace {
void put(tri_vertex& v, vec3 p, vec3 n, vec3 t, vec3 b, vec2 uv) {
    std::memset(&v, 0, sizeof v);
    v.position[0] = p.x; v.position[1] = p.y; v.position[2] = p.z;
    v.normal[0] = n.x; v.normal[1] = n.y; v.normal[2] = n.z;
    v.tangent[0] = t.x; v.tangent[1] = t.y; v.tangent[2] = t.z;
    v.bitangent[0] = b.x; v.bitangent[1] = b.y; v.bitangent[2] = b.z;
    v.color[0] = v.color[1] = v.color[2] = 1.0f;
    v.texcoord[0] = uv.x; v.texcoord[1] = uv.y;
}

void build_sphere(uint32_t rings, uint32_t segs, float radius, std::vector<tri_vertex>& vs,
                  std::vector<uint32_t>& is) {  // BuildPrimitiveSphereMesh, Renderer.cpp:175-246
    const float pi = 3.14159265358979323846264338327950288f;  // glm::pi<float>()
    const float two_pi = 6.28318530717958647692528676655900576f;  // glm::two_pi<float>()
    for (uint32_t r = 0; r <= rings; ++r) {
        const float V = (float)r / (float)rings;
        const float phi = V * pi;
        for (uint32_t s = 0; s <= segs; ++s) {
            const float U = (float)s / (float)segs;
            const float theta = U * two_pi;
            const float sp = std::sin(phi), cp = std::cos(phi), st = std::sin(theta), ct = std::cos(theta);
            const vec3 p{radius * sp * ct, radius * cp, radius * sp * st};
            const vec3 n = normalize(p);
            vec3 t{-st, 0.0f, ct};
            if (length(t) < 0.0001f) t = {1.0f, 0.0f, 0.0f};
            t = normalize(t);
            vec3 b = normalize(cross(n, t));
            if (length(b) < 0.0001f) b = {0.0f, 1.0f, 0.0f};
            tri_vertex v;
            put(v, p, n, t, b, {U, 1.0f - V});
            vs.push_back(v);
        }
    }
    const uint32_t row = segs + 1;
    for (uint32_t r = 0; r < rings; ++r)
        for (uint32_t s = 0; s < segs; ++s) {
            const uint32_t i0 = r * row + s, i1 = (r + 1) * row + s, i2 = (r + 1) * row + s + 1, i3 = r * row + s + 1;
            is.insert(is.end(), {i0, i2, i1, i0, i3, i2});
        }
}

int emit(const std::vector<tri_vertex>& vs, const std::vector<uint32_t>& is, tri_vertex* ov,
         uint32_t* nv, uint32_t* oi, uint32_t* ni) {
    if (!nv || !ni) return TRI_E_INVALID;
    if (ov) {
        if (*nv < vs.size()) return TRI_E_INVALID;
        std::memcpy(ov, vs.data(), vs.size() * sizeof(tri_vertex));
    }
    if (oi) {
        if (*ni < is.size()) return TRI_E_INVALID;
        std::memcpy(oi, is.data(), is.size() * 4);
    }
    *nv = (uint32_t)vs.size();
    *ni = (uint32_t)is.size();
    return TRI_OK;
}

void store(const mat4& m, float* out) { std::memcpy(out, m.m, 64); }
}  // namespace

extern "C" int oracle_build_primitive(int kind, tri_vertex* ov, uint32_t* nv, uint32_t* oi, uint32_t* ni) {
    std::vector<tri_vertex> vs;
    std::vector<uint32_t> is;
    if (kind == 1) {  // BuildPrimitiveCubeMesh, Renderer.cpp:106-173
        struct Face { vec3 n, t, b; vec3 p[4]; };
        const Face faces[6] = {
            {{0, 0, 1}, {1, 0, 0}, {0, 1, 0}, {{-0.5f, -0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f}}},
            {{0, 0, -1}, {-1, 0, 0}, {0, 1, 0}, {{0.5f, -0.5f, -0.5f}, {-0.5f, -0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}}},
            {{1, 0, 0}, {0, 0, -1}, {0, 1, 0}, {{0.5f, -0.5f, 0.5f}, {0.5f, -0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}, {0.5f, 0.5f, 0.5f}}},
            {{-1, 0, 0}, {0, 0, 1}, {0, 1, 0}, {{-0.5f, -0.5f, -0.5f}, {-0.5f, -0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f}, {-0.5f, 0.5f, -0.5f}}},
            {{0, 1, 0}, {1, 0, 0}, {0, 0, -1}, {{-0.5f, 0.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {0.5f, 0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f}}},
            {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}, {{-0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, 0.5f}, {-0.5f, -0.5f, 0.5f}}},
        };
        const vec2 uvs[4] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
        uint32_t off = 0;
        for (const Face& f : faces) {
            for (int k = 0; k < 4; ++k) {
                tri_vertex v;
                put(v, f.p[k], f.n, f.t, f.b, uvs[k]);
                vs.push_back(v);
            }
            is.insert(is.end(), {off + 0, off + 2, off + 1, off + 0, off + 3, off + 2});
            off += 4;
        }
    } else if (kind == 2) {
        build_sphere(16, 24, 0.5f, vs, is);
    } else if (kind == 3) {  // BuildPrimitiveQuadMesh, Renderer.cpp:72-104
        const vec3 p[4] = {{-0.5f, -0.5f, 0}, {0.5f, -0.5f, 0}, {0.5f, 0.5f, 0}, {-0.5f, 0.5f, 0}};
        const vec2 uvs[4] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
        for (int k = 0; k < 4; ++k) {
            tri_vertex v;
            put(v, p[k], {0, 0, 1}, {1, 0, 0}, {0, 1, 0}, uvs[k]);
            vs.push_back(v);
        }
        is = {0, 1, 2, 0, 2, 3};
    } else {
        return TRI_E_INVALID;
    }
    return emit(vs, is, ov, nv, oi, ni);
}

extern "C" int oracle_build_uv_sphere(uint32_t rings, uint32_t segs, float radius, tri_vertex* ov,
                                      uint32_t* nv, uint32_t* oi, uint32_t* ni) {
    if (rings == 0 || segs == 0) return TRI_E_INVALID;
    std::vector<tri_vertex> vs;
    std::vector<uint32_t> is;
    build_sphere(rings, segs, radius, vs, is);
    return emit(vs, is, ov, nv, oi, ni);
}

extern "C" void oracle_compose_transform(const float p[3], const float r[3], const float s[3], float out[16]) {
    mat4 m = mat4_identity();
    m = translate(m, {p[0], p[1], p[2]});
    m = rotate(m, radians(r[0]), {1.0f, 0.0f, 0.0f});
    m = rotate(m, radians(r[1]), {0.0f, 1.0f, 0.0f});
    m = rotate(m, radians(r[2]), {0.0f, 0.0f, 1.0f});
    m = scale(m, {s[0], s[1], s[2]});
    store(m, out);
}

extern "C" void oracle_editor_camera(const float pos[3], const float rot[3], float fov, float vw, float vh,
                                     float n, float f, float ortho, int ptype, float out_view[16],
                                     float out_proj[16], float out_fwd[3]) {
    // EditorCamera::RecalculateOrientation / ViewMatrix / ProjectionMatrix (EditorCamera.cpp:126-160)
    const quat q = quat_from_euler(radians(vec3{rot[0], rot[1], rot[2]}));
    const mat4 R = mat4_cast(conjugate(q));
    const mat4 T = translate(mat4_identity(), {-pos[0], -pos[1], -pos[2]});
    store(mul(R, T), out_view);
    const float aspect = std::max(vw / std::max(vh, 0.0001f), 0.0001f);
    mat4 P;
    if (ptype == 1) {
        const float hh = ortho * 0.5f, hw = hh * aspect;
        P = orthoRH_ZO(-hw, hw, -hh, hh, n, f);
    } else {
        P = perspectiveRH_ZO(radians(fov), aspect, n, f);
    }
    P.m[1][1] *= -1.0f;  // Vulkan Y flip (EditorCamera.cpp:159)
    store(P, out_proj);
    if (out_fwd) {
        const vec3 fw = rotate(q, vec3{0.0f, 0.0f, -1.0f});  // GetForwardDirection
        out_fwd[0] = fw.x; out_fwd[1] = fw.y; out_fwd[2] = fw.z;
    }
}

extern "C" void oracle_runtime_camera(const float pos[3], const float rot[3], float fov, float vw, float vh,
                                      float n, float f, float ortho, int ptype, float out_view[16],
                                      float out_proj[16]) {
    const quat q = normalize(quat_from_euler(radians(vec3{rot[0], rot[1], rot[2]})));
    const vec3 p{pos[0], pos[1], pos[2]};
    const vec3 fwd = rotate(q, vec3{0.0f, 0.0f, -1.0f});
    const vec3 up = rotate(q, vec3{0.0f, 1.0f, 0.0f});
    store(lookAtRH(p, p + fwd, up), out_view);  // RuntimeCamera.cpp:166-175
    const float aspect = (vh > 0.0f) ? (vw / vh) : 1.0f;
    mat4 P;
    if (ptype == 0) {
        P = perspectiveRH_NO(radians(fov), aspect, n, f);  // glm::perspective, RuntimeCamera.cpp:183
        P.m[1][1] *= -1.0f;
    } else {
        const float oh = ortho, ow = oh * aspect;
        P = orthoRH_NO(-ow, ow, -oh, oh, n, f);  // glm::ortho, no Y flip (RuntimeCamera.cpp:190)
    }
    store(P, out_proj);
}

extern "C" void oracle_pack_global_ubo(const float view[16], const float proj[16], const float cam[3],
                                       int has_camera, const float amb[3], float amb_i,
                                       const oracle_light* lights, uint32_t nl, tri_global_ubo* out) {
    std::memset(out, 0, sizeof *out);
    if (has_camera) {
        std::memcpy(out->view, view, 64);
        std::memcpy(out->projection, proj, 64);
        out->camera_position[0] = cam[0]; out->camera_position[1] = cam[1]; out->camera_position[2] = cam[2];
    } else {
        const mat4 I = mat4_identity();
        std::memcpy(out->view, I.m, 64);
        std::memcpy(out->projection, I.m, 64);
    }
    out->camera_position[3] = 1.0f;
    out->ambient_color_intensity[0] = amb[0]; out->ambient_color_intensity[1] = amb[1];
    out->ambient_color_intensity[2] = amb[2]; out->ambient_color_intensity[3] = amb_i;
    vec3 dir = normalize(vec3{-0.5f, -1.0f, -0.3f});  // s_DefaultDirectionalDirection (Renderer.h:464)
    vec3 col{1.0f, 0.98f, 0.92f};
    float inten = 5.0f;
    uint32_t ndir = 0, npt = 0;
    for (uint32_t i = 0; i < nl; ++i) {
        const oracle_light& L = lights[i];
        if (!L.enabled) continue;
        if (L.type == 0) {
            if (ndir == 0) {
                const vec3 d{L.direction[0], L.direction[1], L.direction[2]};
                if (dot(d, d) > 0.0001f) dir = normalize(d);
                col = {L.color[0], L.color[1], L.color[2]};
                inten = std::max(L.intensity, 0.0f);
            }
            ++ndir;
            continue;
        }
        if (L.type == 1) {
            if (npt >= TRI_MAX_POINT_LIGHTS) continue;
            const float rng = std::max(L.range, 0.0f), it = std::max(L.intensity, 0.0f);
            tri_point_light& pl = out->point_lights[npt];
            pl.position_range[0] = L.has_transform ? L.position[0] : 0.0f;
            pl.position_range[1] = L.has_transform ? L.position[1] : 0.0f;
            pl.position_range[2] = L.has_transform ? L.position[2] : 0.0f;
            pl.position_range[3] = rng;
            pl.color_intensity[0] = L.color[0]; pl.color_intensity[1] = L.color[1];
            pl.color_intensity[2] = L.color[2]; pl.color_intensity[3] = it;
            ++npt;
        }
    }
    const bool fallback = (ndir == 0 && npt == 0);
    out->directional_light_direction[0] = dir.x; out->directional_light_direction[1] = dir.y;
    out->directional_light_direction[2] = dir.z; out->directional_light_direction[3] = 0.0f;
    out->directional_light_color[0] = col.x; out->directional_light_color[1] = col.y;
    out->directional_light_color[2] = col.z; out->directional_light_color[3] = inten;
    out->light_counts[0] = (ndir > 0 || fallback) ? 1u : 0u;
    out->light_counts[1] = npt;
}

// vkCmdBlitImage(primary offscreen target -> swapchain image, VK_FILTER_LINEAR), Renderer.cpp:5346-5361.
// Vulkan "Image Blits": destination texel centre (x + 0.5) scaled by src/dst extent into the source,
// bilinear filtering of UNORM values over clamp-to-edge taps, UNORM8 round-to-nearest on the write.
extern "C" void oracle_blit_linear(const uint32_t* src, uint32_t w, uint32_t h, uint32_t* dst, uint32_t dw,
                                   uint32_t dh) {
    const float sx = (float)w / (float)dw, sy = (float)h / (float)dh;
    for (uint32_t y = 0; y < dh; ++y)
        for (uint32_t x = 0; x < dw; ++x) {
            const float u = ((float)x + 0.5f) * sx - 0.5f;
            const float v = ((float)y + 0.5f) * sy - 0.5f;
            const float fu = std::floor(u), fv = std::floor(v);
            const float a = u - fu, b = v - fv;
            const int32_t i0 = (int32_t)fu, j0 = (int32_t)fv;
            auto cl = [](int32_t i, uint32_t n) { return (uint32_t)std::min(std::max(i, 0), (int32_t)n - 1); };
            const uint32_t xa = cl(i0, w), xb = cl(i0 + 1, w), ya = cl(j0, h), yb = cl(j0 + 1, h);
            const uint32_t p00 = src[(size_t)ya * w + xa], p10 = src[(size_t)ya * w + xb];
            const uint32_t p01 = src[(size_t)yb * w + xa], p11 = src[(size_t)yb * w + xb];
            uint32_t out = 0;
            for (int c = 0; c < 4; ++c) {
                auto un = [c](uint32_t p) { return (float)((p >> (8 * c)) & 0xFFu) / 255.0f; };
                const float t00 = un(p00), t10 = un(p10), t01 = un(p01), t11 = un(p11);
                const float l0 = t00 + a * (t10 - t00);
                const float l1 = t01 + a * (t11 - t01);
                out |= unorm8(l0 + b * (l1 - l0)) << (8 * c);
            }
            dst[(size_t)y * dw + x] = out;
        }
}

// tri_shadow_fit_ortho (include/tri_raster.h): the light transform the shim fits for a shadow-casting
// directional light. glm::lookAtRH from 2 * radius behind the box centre along the light's direction,
// then glm::orthoRH_ZO over the 8 box corners in light view space, widened by 1 % (+1e-4) per axis.
extern "C" void oracle_shadow_fit_ortho(const float dir[3], const float mn[3], const float mx[3], float out[16]) {
    vec3 d{dir[0], dir[1], dir[2]};
    if (!(dot(d, d) > 1e-12f)) d = {-0.5f, -1.0f, -0.3f};
    d = normalize(d);
    const vec3 lo{mn[0], mn[1], mn[2]}, hi{mx[0], mx[1], mx[2]};
    const vec3 c = (lo + hi) * 0.5f;
    const float r = std::max(length(hi - lo) * 0.5f, 1e-3f);
    const vec3 eye = c - d * (2.0f * r);
    const vec3 up = std::fabs(d.y) > 0.99f ? vec3{0.0f, 0.0f, 1.0f} : vec3{0.0f, 1.0f, 0.0f};
    const mat4 V = lookAtRH(eye, c, up);
    float b0[3] = {INFINITY, INFINITY, INFINITY}, b1[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 8; ++k) {
        const vec4 p = mul(V, vec4{(k & 1) ? hi.x : lo.x, (k & 2) ? hi.y : lo.y, (k & 4) ? hi.z : lo.z, 1.0f});
        const float q[3] = {p.x, p.y, p.z};
        for (int a = 0; a < 3; ++a) {
            b0[a] = std::min(b0[a], q[a]);
            b1[a] = std::max(b1[a], q[a]);
        }
    }
    float m[3];
    for (int a = 0; a < 3; ++a) m[a] = (b1[a] - b0[a]) * 0.01f + 1e-4f;
    // view space looks down -z: near = -(max z) - margin, far = -(min z) + margin
    const mat4 P = orthoRH_ZO(b0[0] - m[0], b1[0] + m[0], b0[1] - m[1], b1[1] + m[1], -b1[2] - m[2], -b0[2] + m[2]);
    store(mul(P, V), out);
}
