// tri_raster_capi.hip — the C-ABI (include/tri_raster.h) over the gfx950 kernels.
// Owns device memory, the stream and timing events; mirrors Trident::Renderer's upload / frame
// semantics (Renderer.cpp:1784-2116 geometry, :3404-3656 texture slots, :5822-6051 uniforms,
// :5110-5151 draws, :5297-5338 readback).
#include "raster_launch.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <chrono>

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return fail(_e == hipErrorOutOfMemory ? TRI_E_OOM : TRI_E_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(_e), __FILE__, __LINE__);                   \
    } while (0)

template <typename T>
int grow(T*& p, size_t& cap, size_t need) {
    if (need <= cap && p) return TRI_OK;
    if (p) HIP_TRY(hipFree(p));
    p = nullptr;
    cap = std::max<size_t>(need, 1);
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p), cap * sizeof(T)));
    return TRI_OK;
}

uint32_t unorm8_host(float c) {
    const float cc = std::fmin(std::fmax(c, 0.0f), 1.0f);
    return (uint32_t)(int)(cc * 255.0f + 0.5f);
}

// R8G8B8A8_SRGB decode of one channel byte (sRGB EOTF in double, rounded): the kernels' LUT.
float srgb_decode(int i) {
    const double v = i / 255.0;
    return (float)(v <= 0.04045 ? v / 12.92 : std::pow((v + 0.055) / 1.055, 2.4));
}

struct TimingSet {
    hipEvent_t ev[kStageCount + 1];
    bool shadow = false;  // the frame ran the shadow pre-pass (ev[kStageShadow] was recorded)
};

}  // namespace

// Geometry (UploadMeshFromCache, Renderer.cpp:1965-2116): one concatenated vertex buffer, one index
// buffer, the per-mesh ranges and the cluster-culling tables. A context owns one; a tri_geometry made
// with tri_geometry_create is the same object shared by several contexts of one device (the editor's
// Scene and Game viewports read one vertex/index buffer, as the reference's do).
struct tri_geometry {
    int device = 0;
    bool shared = false;
    uint64_t version = 0;  // bumped by every upload (contexts re-resolve their draws)
    TriVsIn* d_vin = nullptr; size_t cap_vin = 0;
    float* d_pos = nullptr; size_t cap_pos = 0;  // 3 floats per vertex (k_vertex's stream with vary_obj)
    float* d_attr = nullptr; size_t cap_attr = 0;  // 9 floats per vertex {pos, normal, colour} (k_raster's, vary_obj)
    TriVsSkin* d_skin = nullptr; size_t cap_skin = 0;
    bool has_skin_data = false;
    // every vertex has a finite position and a unit normal (|n|^2 within 1e-5 of 1): a draw over it may keep
    // its varyings in object space (TriFrameParams::vary_obj)
    bool obj_ok = false;
    bool uni_col = false;  // every vertex has the colour ucol (TriFrameParams::obj_ucol)
    float ucol[3] = {0.0f, 0.0f, 0.0f};
    uint64_t nverts = 0;
    uint32_t* d_idx = nullptr; size_t cap_idx = 0;
    uint64_t nidx = 0;
    std::vector<tri_mesh_range> meshes;
    std::vector<uint32_t> mesh_min, mesh_max;
    std::vector<uint32_t> mesh_cl_first, mesh_ncl, mesh_vblk_first;  // cluster culling tables per mesh
    TriCluster* d_clusters = nullptr; size_t cap_clusters = 0;
    TriCluster* d_vbox = nullptr; size_t cap_vbox = 0;  // per vertex block: union box of its clusters
    bool geometry_set = false;
};

struct tri_ctx {
    tri_config cfg{};
    int device = 0;
    int32_t W = 0, H = 0, y0 = 0, y1 = 0, nbx = 0, nby = 0, nbins = 0;
    int cu_count = 256;  // compute units of the device (k_setup's grid sizing)
    uint32_t last_path = 0;  // tri_frame_stats.path of the last frame built
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    tri_geometry own_geom;
    tri_geometry* geom = &own_geom;  // own_geom, or a shared tri_geometry (tri_bind_geometry)
    uint64_t geom_seen = 0;          // geom->version the resolved draws were built against

    tri_material_record mat0{{1, 1, 1, 1}, {1, 1, 1, 0}};

    // texture slots; slot 0 = default 1x1 white
    uint32_t* d_tex[TRI_MAX_TEXTURE_SLOTS] = {};
    uint32_t tex_w[TRI_MAX_TEXTURE_SLOTS] = {}, tex_h[TRI_MAX_TEXTURE_SLOTS] = {};
    uint32_t tex_solid[TRI_MAX_TEXTURE_SLOTS] = {};  // texel of a 1x1 slot (RGBA8)
    int16_t tex_alpha[TRI_MAX_TEXTURE_SLOTS] = {};    // the alpha byte every texel of the slot has, or -1
    TriTexDesc texdesc[TRI_MAX_TEXTURE_SLOTS] = {};  // per-slot descriptors, aliases resolved
    bool tex_dirty = true;
    float* d_lut = nullptr;

    float* d_bones = nullptr; size_t cap_bones = 0;
    uint32_t* d_sky = nullptr; size_t cap_sky = 0;
    uint32_t* d_ai = nullptr; size_t cap_ai = 0;  // the AI blend's RGBA8 UNORM frame (tri_upload_ai_frame)
    uint32_t ai_w = 0, ai_h = 0;
    uint32_t sky_size = 0;
    bool sky_uniform = false;  // every texel of the cubemap equal (e.g. the solid fallback)
    uint32_t sky_uniform_bgra = 0;
    uint32_t nbones = 0;

    // per frame
    tri_global_ubo ubo{};
    float pv[16] = {};
    uint32_t clear_bgra = 0;
    bool frame_set = false;
    std::vector<tri_draw> draws;
    bool draws_dirty = true;

    // resolved draws
    TriDrawDev* d_draws = nullptr; size_t cap_draws = 0;
    TriDrawShade* d_draw_shade = nullptr; size_t cap_draw_shade = 0;
    TriDrawShade shade0{};  // the shade record of a single-draw frame
    uint32_t* d_vbase = nullptr; size_t cap_vbase = 0;
    uint32_t* d_pbase = nullptr; size_t cap_pbase = 0;
    uint32_t* d_cbase = nullptr; size_t cap_cbase = 0;
    uint32_t* d_cvis = nullptr; size_t cap_cvis = 0;
    uint32_t ncl_total = 0;
    void* h_stage = nullptr; size_t cap_stage = 0;  // pinned upload staging
    TriCounters* h_ctr = nullptr;  // pinned: the frame's counters, copied on the stream by tri_synchronize
    hipEvent_t stage_free = nullptr;
    uint32_t ndraws = 0, nslots = 0, nprims = 0;
    bool any_skin = false;
    TriDrawDev draw0{};  // the resolved draw when there is exactly one (passed by value to the kernels)
    bool draw0_obj = false;    // draw0 may keep object-space varyings (draw_obj_ok)
    bool draw0_xform = false;  // ... and its model matrix is not the identity
    bool draw0_ucol = false;   // ... and every vertex of its geometry has one colour
    bool obj48 = false;        // every active draw may keep object-space varyings (TriFrameParams::obj48)
    bool obj48_xform = false;  // ... and some draw's model matrix is not the identity
    uint32_t vdelta[TRI_OBJ48_DRAWS] = {};  // per draw: base_vertex + min_index - first slot
    bool idx_route = false;                   // TriFrameParams::idx_route and its tables
    uint32_t idx_k = 0, pbase[TRI_OBJ48_DRAWS] = {}, vbd[TRI_OBJ48_DRAWS] = {};

    // work buffers
    float4* d_clip = nullptr; size_t cap_clip = 0;
    TriSnap* d_snap = nullptr; size_t cap_snap = 0;
    uint8_t* d_oc = nullptr; size_t cap_oc = 0;
    int32_t bin_log2 = 6;
    float4* d_vary = nullptr; size_t cap_vary = 0;
    TriRec* d_recs = nullptr; size_t cap_recs = 0;
    uint32_t* d_clip_slot = nullptr; size_t cap_clip_slot = 0;
    uint4* d_prim_vs = nullptr; size_t cap_prim_vs = 0;
    uint2* d_setup_stats = nullptr; size_t cap_setup_stats = 0;
    uint32_t last_nchunks = 0;
    uint32_t* d_bin_count = nullptr; size_t cap_bin_count = 0;
    uint32_t* d_bin_list = nullptr; size_t cap_bin_list = 0;
    TriCounters* d_ctr = nullptr;
    uint32_t ovf_rec_cap = 1u << 16, ovf_vert_cap = 1u << 17;
    uint32_t bin_cap = 0;

    // shadow-map pre-pass (tri_set_shadow)
    tri_shadow_config shadow{};
    float4* d_lpos = nullptr; size_t cap_lpos = 0;
    TriSnap* d_lsnap = nullptr; size_t cap_lsnap = 0;
    uint32_t* d_sbin_count = nullptr; size_t cap_sbin_count = 0;
    uint32_t* d_sbin_list = nullptr; size_t cap_sbin_list = 0;
    uint32_t* d_shadow = nullptr; size_t cap_shadow = 0;
    uint32_t s_nbx = 0, s_nbins = 0, s_bin_cap = 0;
    bool shadow_rendered = false;  // a frame with the current map size has been enqueued

    uint32_t* d_color_own = nullptr;
    float* d_depth_own = nullptr;
    uint32_t* d_present = nullptr; size_t cap_present = 0;  // tri_blit_linear's owned target
    uint32_t present_w = 0, present_h = 0;
    uint32_t* d_color = nullptr;
    float* d_depth = nullptr;

    // the frame's arguments: built here by tri_render, passed by value to the frame's first kernel, which
    // publishes them to d_args for the later kernels (raster_launch.h)
    TriLaunchArgs args{};
    TriLaunchArgs* d_args = nullptr;
    bool launched = false;  // a frame was enqueued (tri_set_stream orders the next one behind it)
#ifdef TRI_DIAG_FRONT
    uint32_t diag_frames = 0;  // diagnostics build: frames rendered (the first one runs the whole plan)
#endif

    bool timing = false;
    uint32_t timing_period = 1, timing_counter = 0;  // time every timing_period-th frame
    std::vector<TimingSet> pending;
    std::vector<TimingSet> free_sets;
    tri_timing acc{};
};

namespace {

int make_current(tri_ctx* c) {
    HIP_TRY(hipSetDevice(c->device));
    return TRI_OK;
}


// transpose(inverse(mat3(M))) exactly as Default.vert:95 evaluates it per vertex (glm cofactor
// form, same float operation order as the oracle); out[c*3+r] = NM[c][r] = inverse[r][c].
void normal_matrix(const float* M, float* out) {
    auto m = [M](int c, int r) { return M[c * 4 + r]; };
    const float det = (m(0, 0) * (m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) -
                       m(1, 0) * (m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2))) +
                      m(2, 0) * (m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2));
    const float od = 1.0f / det;
    float inv[3][3];
    inv[0][0] = +(m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) * od;
    inv[1][0] = -(m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2)) * od;
    inv[2][0] = +(m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1)) * od;
    inv[0][1] = -(m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2)) * od;
    inv[1][1] = +(m(0, 0) * m(2, 2) - m(2, 0) * m(0, 2)) * od;
    inv[2][1] = -(m(0, 0) * m(2, 1) - m(2, 0) * m(0, 1)) * od;
    inv[0][2] = +(m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)) * od;
    inv[1][2] = -(m(0, 0) * m(1, 2) - m(1, 0) * m(0, 2)) * od;
    inv[2][2] = +(m(0, 0) * m(1, 1) - m(1, 0) * m(0, 1)) * od;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) out[c * 3 + r] = inv[r][c];
}

float clamp01(float x) { return std::fmin(std::fmax(x, 0.0f), 1.0f); }

bool identity_model(const float* m) {
    for (int i = 0; i < 16; ++i)
        if (m[i] != ((i % 5 == 0) ? 1.0f : 0.0f)) return false;
    return true;
}

// Object-space varyings (TriFrameParams::vary_obj) are the world-space ones up to rounding when the draw is
// affine and unskinned (clip_from_world: world = A p + t, a linear map of the interpolated position), its normal
// matrix is conformal (orthogonal columns of one length s, so normalize(NM n) = NM n / s for every unit n and the
// fragment's normalize sees the same direction) and every object normal is unit, with all its vertex records
// in the vertex buffer.
bool draw_obj_ok(const tri_geometry& g, const TriDrawDev& d) {
    if (!g.obj_ok || !d.clip_from_world || d.vert_count == 0) return false;
    const int64_t first = (int64_t)d.base_vertex + (int64_t)d.min_index;
    if (first < 0 || (uint64_t)first + d.vert_count > g.nverts) return false;
    double c[3][3];
    for (int k = 0; k < 3; ++k)
        for (int r = 0; r < 3; ++r) c[k][r] = d.nm[k * 3 + r];
    auto dot = [&](int a, int b) { return c[a][0] * c[b][0] + c[a][1] * c[b][1] + c[a][2] * c[b][2]; };
    const double s2 = (dot(0, 0) + dot(1, 1) + dot(2, 2)) / 3.0;
    if (!(s2 > 0.0) || !std::isfinite(s2)) return false;
    const double tol = 1e-5 * s2;
    return std::fabs(dot(0, 0) - s2) <= tol && std::fabs(dot(1, 1) - s2) <= tol && std::fabs(dot(2, 2) - s2) <= tol &&
           std::fabs(dot(0, 1)) <= tol && std::fabs(dot(0, 2)) <= tol && std::fabs(dot(1, 2)) <= tol;
}

// Default.frag frame constants hoisted for the fast shading build (Default.frag:131-174).
void shade_constants(const tri_global_ubo& g, const tri_material_record& m, TriShadeConst& sc) {
    std::memset(&sc, 0, sizeof sc);
    std::memcpy(sc.cam, g.camera_position, 16);
    std::memcpy(sc.base, m.base_color_factor, 16);
    sc.metallic = clamp01(m.material_factors[0]);
    sc.roughness = std::fmin(std::fmax(m.material_factors[1], 0.045f), 1.0f);
    sc.amb_strength = clamp01(m.material_factors[2]);
    const float a = sc.roughness * sc.roughness, a2 = a * a, rr = sc.roughness + 1.0f;
    sc.a2m1 = a2 - 1.0f;
    sc.a2pi = a2 / 3.14159265359f;
    sc.kg = rr * rr * 0.125f;
    sc.omkg = 1.0f - sc.kg;
    sc.kgo = sc.kg / sc.omkg;     // omkg >= 0.5 (k <= 0.5 for roughness <= 1)
    sc.a2pio = sc.a2pi / sc.omkg;
    sc.spAk = 0.25f * sc.a2pio;
    sc.spBk = 1e4f * sc.a2pio;
    sc.om = 0.04f * (1.0f - sc.metallic);
    sc.kd = (1.0f - sc.metallic) * (1.0f / 3.14159265359f);
    for (int i = 0; i < 3; ++i) sc.amb[i] = g.ambient_color_intensity[i] * g.ambient_color_intensity[3];
    sc.has_sun = g.light_counts[0] > 0u ? 1u : 0u;
    const float lx = -g.directional_light_direction[0], ly = -g.directional_light_direction[1],
                lz = -g.directional_light_direction[2];
    const float il = 1.0f / std::sqrt((lx * lx + ly * ly) + lz * lz);
    sc.sun_l[0] = lx * il; sc.sun_l[1] = ly * il; sc.sun_l[2] = lz * il;
    for (int i = 0; i < 3; ++i) sc.sun_rad[i] = g.directional_light_color[i] * g.directional_light_color[3];
    sc.npt = std::min<uint32_t>(g.light_counts[1], TRI_MAX_POINT_LIGHTS);
    for (uint32_t i = 0; i < sc.npt; ++i) {
        const tri_point_light& pl = g.point_lights[i];
        for (int k = 0; k < 3; ++k) {
            sc.pl[i].pos[k] = pl.position_range[k];
            sc.pl[i].rad[k] = pl.color_intensity[k] * pl.color_intensity[3];
        }
        sc.pl[i].pos[3] = 1.0f / std::fmax(pl.position_range[3], 1e-4f);
    }
}

// Skybox constants: inverse(Projection) by cofactors in double (rounded to float), mat3(View) and
// the projection's w row (same arithmetic as the oracle's sky_constants()).
void sky_constants(const tri_global_ubo& g, float* ip, float* R, float* pw) {
    double a[16], inv[16];
    for (int i = 0; i < 16; ++i) a[i] = g.projection[i];
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
    for (int i = 0; i < 16; ++i) ip[i] = (float)(inv[i] * id);
    for (int col = 0; col < 3; ++col)
        for (int r = 0; r < 3; ++r) R[col * 3 + r] = g.view[col * 4 + r];
    for (int col = 0; col < 4; ++col) pw[col] = g.projection[col * 4 + 3];
}

// glm mat4 * mat4 (column j = ((A0*B[j][0] + A1*B[j][1]) + A2*B[j][2]) + A3*B[j][3])
void mat4_mul(const float* a, const float* b, float* r) {
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            float s = a[0 * 4 + i] * b[j * 4 + 0];
            s = s + a[1 * 4 + i] * b[j * 4 + 1];
            s = s + a[2 * 4 + i] * b[j * 4 + 2];
            s = s + a[3 * 4 + i] * b[j * 4 + 3];
            r[j * 4 + i] = s;
        }
}

// ---- tri_shadow_fit_ortho: glm::lookAtRH + glm::orthoRH_ZO (same operation order as the oracle's
// restatement, oracle_shadow_fit_ortho; CPU test compares them bit for bit) ----------------------
struct V3 { float x, y, z; };
V3 v3sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 v3mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float v3dot(V3 a, V3 b) {  // glm compute_dot: (x + y) + z
    const float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return (tx + ty) + tz;
}
V3 v3cross(V3 x, V3 y) { return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
V3 v3norm(V3 v) { return v3mul(v, 1.0f / std::sqrt(v3dot(v, v))); }

void shadow_fit_ortho(const float dir[3], const float mn[3], const float mx[3], float out[16]) {
    V3 d{dir[0], dir[1], dir[2]};
    if (!(v3dot(d, d) > 1e-12f)) d = {-0.5f, -1.0f, -0.3f};
    d = v3norm(d);
    const V3 lo{mn[0], mn[1], mn[2]}, hi{mx[0], mx[1], mx[2]};
    const V3 c{(lo.x + hi.x) * 0.5f, (lo.y + hi.y) * 0.5f, (lo.z + hi.z) * 0.5f};
    const float r = std::max(std::sqrt(v3dot(v3sub(hi, lo), v3sub(hi, lo))) * 0.5f, 1e-3f);
    const V3 eye = v3sub(c, v3mul(d, 2.0f * r));
    const V3 up = std::fabs(d.y) > 0.99f ? V3{0.0f, 0.0f, 1.0f} : V3{0.0f, 1.0f, 0.0f};
    // glm::lookAtRH(eye, c, up), column-major V[col*4 + row]
    const V3 f = v3norm(v3sub(c, eye));
    const V3 sv = v3norm(v3cross(f, up));
    const V3 u = v3cross(sv, f);
    float V[16] = {sv.x, u.x, -f.x, 0.0f, sv.y, u.y, -f.y, 0.0f, sv.z, u.z, -f.z, 0.0f,
                   -v3dot(sv, eye), -v3dot(u, eye), v3dot(f, eye), 1.0f};
    float b0[3] = {INFINITY, INFINITY, INFINITY}, b1[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 8; ++k) {
        const float p[4] = {(k & 1) ? hi.x : lo.x, (k & 2) ? hi.y : lo.y, (k & 4) ? hi.z : lo.z, 1.0f};
        for (int a = 0; a < 3; ++a) {  // glm mat4 * vec4: (m0 v0 + m1 v1) + (m2 v2 + m3 v3)
            const float add0 = V[0 * 4 + a] * p[0] + V[1 * 4 + a] * p[1];
            const float add1 = V[2 * 4 + a] * p[2] + V[3 * 4 + a] * p[3];
            const float q = add0 + add1;
            b0[a] = std::min(b0[a], q);
            b1[a] = std::max(b1[a], q);
        }
    }
    float m[3];
    for (int a = 0; a < 3; ++a) m[a] = (b1[a] - b0[a]) * 0.01f + 1e-4f;
    // glm::orthoRH_ZO(l, r, b, t, n, f); view space looks down -z
    const float l = b0[0] - m[0], rr = b1[0] + m[0], bt = b0[1] - m[1], tp = b1[1] + m[1];
    const float n = -b1[2] - m[2], fr = -b0[2] + m[2];
    float P[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    P[0] = 2.0f / (rr - l);
    P[5] = 2.0f / (tp - bt);
    P[10] = -1.0f / (fr - n);
    P[12] = -(rr + l) / (rr - l);
    P[13] = -(tp + bt) / (tp - bt);
    P[14] = -n / (fr - n);
    mat4_mul(P, V, out);
}

int upload_texture_table(tri_ctx* c) {
    if (!c->tex_dirty) return TRI_OK;
    TriTexDesc* h = c->texdesc;
    for (int s = 0; s < TRI_MAX_TEXTURE_SLOTS; ++s) {
        const int src = c->d_tex[s] ? s : 0;  // unused slots alias slot 0 (Renderer.cpp:3645-3656)
        h[s].texels = c->d_tex[src];
        h[s].w = c->tex_w[src];
        h[s].h = c->tex_h[src];
        const uint32_t p = c->tex_solid[src];
        for (int k = 0; k < 3; ++k) h[s].solid[k] = srgb_decode((p >> (8 * k)) & 0xFF);
        h[s].solid[3] = (float)(p >> 24) / 255.0f;  // alpha: linear UNORM decode
    }
    c->tex_dirty = false;
    c->draws_dirty = true;  // the per-draw shade records carry the slot descriptors
    return TRI_OK;
}

// Resolve the draw list against the uploaded meshes (GatherMeshDraws + the draw loop's skips).
int resolve_draws(tri_ctx* c) {
    if (!c->draws_dirty) return TRI_OK;
    const uint32_t n = (uint32_t)c->draws.size();
    std::vector<TriDrawDev> dd(n);
    std::vector<TriDrawShade> ds(n);
    std::vector<uint32_t> vb(n + 1), pb(n + 1), cbase(n + 1);
    uint64_t vslots = 0, prims = 0, ncl = 0;
    bool skin = false;
    for (uint32_t d = 0; d < n; ++d) {
        const tri_draw& src = c->draws[d];
        TriDrawDev& o = dd[d];
        std::memset(&o, 0, sizeof o);
        std::memcpy(o.model, src.pc.model, 64);
        normal_matrix(src.pc.model, o.nm);
        TriDrawShade& sh = ds[d];
        std::memset(&sh, 0, sizeof sh);
        std::memcpy(sh.tint, src.pc.tint, 16);
        const int32_t slot = src.pc.texture_slot;
        sh.tex = c->texdesc[(slot >= 0 && slot < TRI_MAX_TEXTURE_SLOTS) ? slot : 0];
        o.tex_scale[0] = src.pc.texture_scale[0];
        o.tex_scale[1] = src.pc.texture_scale[1];
        o.tex_offset[0] = src.pc.texture_offset[0];
        o.tex_offset[1] = src.pc.texture_offset[1];
        o.tiling = src.pc.tiling_factor;
        o.bone_offset = src.pc.bone_offset;
        o.bone_count = src.pc.bone_count;
        o.clip_from_world = (o.bone_count <= 0 && o.model[3] == 0.0f && o.model[7] == 0.0f && o.model[11] == 0.0f &&
                             o.model[15] == 1.0f) ? 1u : 0u;
        vb[d] = (uint32_t)vslots;
        pb[d] = (uint32_t)prims;
        cbase[d] = (uint32_t)ncl;
        if (src.mesh_index >= c->geom->meshes.size()) continue;  // Renderer.cpp:5118-5127 skip
        const tri_mesh_range& mr = c->geom->meshes[src.mesh_index];
        if (mr.index_count < 3 || (uint64_t)mr.first_index + mr.index_count > c->geom->nidx) continue;
        o.first_index = (int32_t)mr.first_index;
        o.base_vertex = mr.base_vertex;
        o.min_index = c->geom->mesh_min[src.mesh_index];
        o.vert_count = c->geom->mesh_max[src.mesh_index] - o.min_index + 1;
        o.cl_first = c->geom->mesh_cl_first[src.mesh_index];
        o.vblk_first = c->geom->mesh_vblk_first[src.mesh_index];
        o.ncl = c->geom->mesh_ncl[src.mesh_index];
        vslots += o.vert_count;
        prims += mr.index_count / 3;
        ncl += o.ncl;
        skin = skin || (o.bone_count > 0);
    }
    vb[n] = (uint32_t)vslots;
    pb[n] = (uint32_t)prims;
    cbase[n] = (uint32_t)ncl;
    if (vslots > 0xFFFFFFF0ull) return fail(TRI_E_INVALID, "too many vertex-shader invocations (%llu)", (unsigned long long)vslots);
    if (prims > TRI_PRIM_MAX) return fail(TRI_E_INVALID, "too many primitives (%llu > %u)", (unsigned long long)prims, TRI_PRIM_MAX);
    int rc;
    if ((rc = grow(c->d_draws, c->cap_draws, std::max<size_t>(n, 1)))) return rc;
    if ((rc = grow(c->d_draw_shade, c->cap_draw_shade, std::max<size_t>(n, 1)))) return rc;
    if ((rc = grow(c->d_vbase, c->cap_vbase, n + 1))) return rc;
    if ((rc = grow(c->d_pbase, c->cap_pbase, n + 1))) return rc;
    if ((rc = grow(c->d_cbase, c->cap_cbase, n + 1))) return rc;
    if ((rc = grow(c->d_cvis, c->cap_cvis, std::max<size_t>(ncl, 1)))) return rc;
    const size_t o_shade = n * sizeof(TriDrawDev);
    const size_t o_vb = o_shade + n * sizeof(TriDrawShade);
    const size_t o_pb = o_vb + (n + 1) * 4;
    const size_t o_cb = o_pb + (n + 1) * 4;
    const size_t bytes = o_cb + (n + 1) * 4;
    if (c->stage_free) HIP_TRY(hipEventSynchronize(c->stage_free));
    if (bytes > c->cap_stage) {
        if (c->h_stage) HIP_TRY(hipHostFree(c->h_stage));
        c->h_stage = nullptr;
        c->cap_stage = bytes * 2;
        HIP_TRY(hipHostMalloc(&c->h_stage, c->cap_stage, hipHostMallocDefault));
    }
    char* st = static_cast<char*>(c->h_stage);
    std::memcpy(st, dd.data(), n * sizeof(TriDrawDev));
    std::memcpy(st + o_shade, ds.data(), n * sizeof(TriDrawShade));
    std::memcpy(st + o_vb, vb.data(), (n + 1) * 4);
    std::memcpy(st + o_pb, pb.data(), (n + 1) * 4);
    std::memcpy(st + o_cb, cbase.data(), (n + 1) * 4);
    if (n) {
        HIP_TRY(hipMemcpyAsync(c->d_draws, st, n * sizeof(TriDrawDev), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->d_draw_shade, st + o_shade, n * sizeof(TriDrawShade), hipMemcpyHostToDevice,
                               c->stream));
    }
    HIP_TRY(hipMemcpyAsync(c->d_vbase, st + o_vb, (n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_pbase, st + o_pb, (n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_cbase, st + o_cb, (n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    if (!c->stage_free) HIP_TRY(hipEventCreateWithFlags(&c->stage_free, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->stage_free, c->stream));
    c->ndraws = n;
    if (n == 1) {
        c->draw0 = dd[0];
        c->shade0 = ds[0];
    }
    c->draw0_obj = n == 1 && draw_obj_ok(*c->geom, dd[0]);
    c->draw0_xform = c->draw0_obj && !identity_model(dd[0].model);
    c->draw0_ucol = c->draw0_obj && c->geom->uni_col;
    // object-space varyings for any draw list (obj48): every active draw affine, unskinned, conformal, with an
    // identity texture transform (uv * scale * tiling + offset == uv bit for bit), at most TRI_OBJ48_DRAWS of them
    c->obj48 = n >= 1 && n <= TRI_OBJ48_DRAWS && !skin;
    c->obj48_xform = false;
    for (uint32_t d = 0; d < n && c->obj48; ++d) {
        const TriDrawDev& o = dd[d];
        c->vdelta[d] = (uint32_t)((int64_t)o.base_vertex + (int64_t)o.min_index - (int64_t)vb[d]);
        if (o.vert_count == 0) continue;  // inactive: no slots, no primitives
        const bool uv_id = o.tex_scale[0] == 1.0f && o.tex_scale[1] == 1.0f && o.tiling == 1.0f &&
                           o.tex_offset[0] == 0.0f && o.tex_offset[1] == 0.0f;
        c->obj48 = uv_id && draw_obj_ok(*c->geom, o);
        c->obj48_xform = c->obj48_xform || !identity_model(o.model);
    }
    // the index route (TriFrameParams::idx_route): every active draw's index rows start at idx_k + 3 * its first
    // primitive (one K for all)
    c->idx_route = n >= 2 && n <= TRI_OBJ48_DRAWS;
    bool have_k = false;
    for (uint32_t d = 0; d < n && c->idx_route; ++d) {
        const TriDrawDev& o = dd[d];
        c->vbd[d] = (uint32_t)((int64_t)vb[d] - (int64_t)o.min_index);
        c->pbase[d] = pb[d];
        if (pb[d + 1] == pb[d]) continue;  // no primitives (inactive or skipped)
        const int64_t k = (int64_t)o.first_index - 3 * (int64_t)pb[d];
        if (k < 0 || (have_k && (uint32_t)k != c->idx_k)) c->idx_route = false;
        c->idx_k = (uint32_t)k;
        have_k = true;
    }
    c->nslots = (uint32_t)vslots;
    c->nprims = (uint32_t)prims;
    c->ncl_total = (uint32_t)ncl;
    c->any_skin = skin;
    c->draws_dirty = false;
    return TRI_OK;
}

// A stride near nchunks / golden ratio, coprime to nchunks.
uint32_t chunk_stride(uint32_t n) {
    if (n <= 2) return 1;
    uint32_t s = (uint32_t)((double)n * 0.6180339887) | 1u;
    auto gcd = [](uint32_t a, uint32_t b) { while (b) { const uint32_t t = a % b; a = b; b = t; } return a; };
    while (gcd(s, n) != 1) ++s;
    return s % n ? s % n : 1u;
}

int ensure_work_buffers(tri_ctx* c) {
    int rc;
    const size_t nrec = c->ovf_rec_cap;
    const size_t nvary = 3ull * ((size_t)c->nslots + c->ovf_vert_cap);
    // per-bin queue capacity: ~8x the mean entries per bin (1.3 bins per triangle), >= 256,
    // grown from the observed maximum after an overflow (check_overflow)
    const uint64_t mean = ((uint64_t)c->nprims * 13 / 10) / (uint64_t)std::max(c->nbins, 1);
    c->bin_cap = std::max<uint32_t>(c->bin_cap, (uint32_t)std::min<uint64_t>(((8 * mean + 64 + 63) / 64) * 64, 1u << 30));
    c->bin_cap = std::max<uint32_t>(c->bin_cap, 256u);
    const size_t nlist = (size_t)c->nbins * c->bin_cap;
    if (nlist * 4 > (8ull << 30)) return fail(TRI_E_OOM, "bin queues would need %zu MB", nlist * 4 >> 20);
    // k_raster gathers varyings, snapped vertices and prim_vs records through raw buffer loads with
    // 32-bit byte offsets
    if (nvary * 16 > 0xFFFFFFFFull || (uint64_t)c->nprims * 16 > 0xFFFFFFFFull)
        return fail(TRI_E_INVALID, "too many vertex invocations or primitives (%zu varyings, %u primitives)", nvary,
                    c->nprims);
    bool realloc = c->cap_clip < std::max<size_t>(c->nslots, 1) || c->cap_vary < nvary || c->cap_recs < nrec ||
                   c->cap_clip_slot < std::max<size_t>(c->nprims, 1) || c->cap_prim_vs < std::max<size_t>(c->nprims, 1) ||
                   c->cap_bin_list < nlist;
    if (realloc) HIP_TRY(hipStreamSynchronize(c->stream));
    if ((rc = grow(c->d_clip, c->cap_clip, std::max<size_t>(c->nslots, 1)))) return rc;
    if ((rc = grow(c->d_snap, c->cap_snap, std::max<size_t>(c->nslots, 1)))) return rc;
    if ((rc = grow(c->d_oc, c->cap_oc, std::max<size_t>(c->nslots, 1)))) return rc;
    if ((rc = grow(c->d_vary, c->cap_vary, nvary))) return rc;
    if ((rc = grow(c->d_recs, c->cap_recs, nrec))) return rc;
    if ((rc = grow(c->d_clip_slot, c->cap_clip_slot, std::max<size_t>(c->nprims, 1)))) return rc;
    if ((rc = grow(c->d_prim_vs, c->cap_prim_vs, std::max<size_t>(c->nprims, 1)))) return rc;
    if ((rc = grow(c->d_setup_stats, c->cap_setup_stats, (size_t)c->nprims / TRI_BLOCK + 1))) return rc;
    if ((rc = grow(c->d_bin_list, c->cap_bin_list, nlist))) return rc;
    if (c->shadow.size) {
        // map queues: ~8x the mean entries per map bin (a triangle covers ~1.3 bins), >= 256
        const uint64_t smean = ((uint64_t)c->nprims * 13 / 10) / (uint64_t)std::max<uint32_t>(c->s_nbins, 1);
        c->s_bin_cap = std::max<uint32_t>(c->s_bin_cap, (uint32_t)std::min<uint64_t>(((8 * smean + 64 + 63) / 64) * 64, 1u << 30));
        c->s_bin_cap = std::max<uint32_t>(c->s_bin_cap, 256u);
        const size_t slist = (size_t)c->s_nbins * c->s_bin_cap;
        if (slist * 4 > (8ull << 30)) return fail(TRI_E_OOM, "shadow-map bin queues would need %zu MB", slist * 4 >> 20);
        const size_t smap = (size_t)c->shadow.size * c->shadow.size;
        if (c->cap_lpos < nvary / 3 || c->cap_lsnap < std::max<size_t>(c->nslots, 1) || c->cap_sbin_list < slist ||
            c->cap_sbin_count < c->s_nbins || c->cap_shadow < smap)
            HIP_TRY(hipStreamSynchronize(c->stream));
        if ((rc = grow(c->d_lpos, c->cap_lpos, nvary / 3))) return rc;
        if ((rc = grow(c->d_lsnap, c->cap_lsnap, std::max<size_t>(c->nslots, 1)))) return rc;
        if ((rc = grow(c->d_sbin_list, c->cap_sbin_list, slist))) return rc;
        if ((rc = grow(c->d_shadow, c->cap_shadow, smap))) return rc;
    }
    return TRI_OK;
}

int collect_timing(tri_ctx* c) {
    if (c->pending.empty()) return TRI_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (TimingSet& t : c->pending) {
        float ms[kStageCount] = {}, tot;
        // stamps: vertex | setup (+ the map's binning) | shadow-map raster (only with the pre-pass) | raster
        HIP_TRY(hipEventElapsedTime(&ms[kStageVertex], t.ev[kStageVertex], t.ev[kStageSetup]));
        HIP_TRY(hipEventElapsedTime(&ms[kStageSetup], t.ev[kStageSetup], t.ev[t.shadow ? kStageShadow : kStageRaster]));
        if (t.shadow) HIP_TRY(hipEventElapsedTime(&ms[kStageShadow], t.ev[kStageShadow], t.ev[kStageRaster]));
        HIP_TRY(hipEventElapsedTime(&ms[kStageRaster], t.ev[kStageRaster], t.ev[kStageCount]));
        HIP_TRY(hipEventElapsedTime(&tot, t.ev[0], t.ev[kStageCount]));
        c->acc.ms_vertex += ms[kStageVertex];
        c->acc.ms_setup += ms[kStageSetup];
        c->acc.ms_shadow += ms[kStageShadow];
        c->acc.ms_raster += ms[kStageRaster];
        c->acc.ms_frame += tot;
        c->acc.frames += 1;
        c->free_sets.push_back(t);
    }
    c->pending.clear();
    return TRI_OK;
}

int check_overflow(tri_ctx* c, const TriCounters* pinned = nullptr) {
    TriCounters h;
    if (pinned) h = *pinned;  // (copied on the context's stream before the wait)
    else HIP_TRY(hipMemcpy(&h, c->d_ctr, sizeof h, hipMemcpyDeviceToHost));
    if (!h.flags) return TRI_OK;
    // the resets are stream-ordered before the next frame's kernels (the context's stream is non-blocking:
    // work on the null stream is not ordered with it)
    HIP_TRY(hipMemsetAsync(&c->d_ctr->flags, 0, 4, c->stream));
    if (h.flags & TRI_OVF_CLIP_RECORDS) c->ovf_rec_cap *= 4;
    if (h.flags & TRI_OVF_CLIP_VERTS) c->ovf_vert_cap *= 4;
    if (h.flags & TRI_OVF_BIN_LIST) {
        c->bin_cap = std::max<uint32_t>(c->bin_cap * 2, h.bin_max + h.bin_max / 4);
        c->bin_cap = (c->bin_cap + 63) & ~63u;
        HIP_TRY(hipMemsetAsync(&c->d_ctr->bin_max, 0, 4, c->stream));
    }
    if (h.flags & TRI_OVF_SHADOW_BIN_LIST) {
        c->s_bin_cap = std::max<uint32_t>(c->s_bin_cap * 2, h.sbin_max + h.sbin_max / 4);
        c->s_bin_cap = (c->s_bin_cap + 63) & ~63u;
        HIP_TRY(hipMemsetAsync(&c->d_ctr->sbin_max, 0, 4, c->stream));
    }
    int rc = ensure_work_buffers(c);
    if (rc) return rc;
    return fail(TRI_E_OVERFLOW, "frame overflowed an internal buffer (flags 0x%x); capacities grown, re-render",
                h.flags);
}

// Bin grid: 32x32-pixel bins while the grid stays under 16384 bins (else 64x64). Sparse frames
// (fewer than 0.05 triangles per pixel, e.g. C2's 50k-triangle sphere at 1080p) on small grids use
// 16x16 bins: more workgroups to balance, and few triangles span several bins. Dense bands keep 32x32
// (16x16 measured 10-25 % slower there: more bin entries, each paying its edge set-up).
// -DTRI_FORCE_BIN_LOG2=4..6 forces a size (diagnostics builds only, tools/build_variant.sh).
#ifndef TRI_FORCE_BIN_LOG2
#define TRI_FORCE_BIN_LOG2 0
#endif
int choose_bin_grid(tri_ctx* c) {
    constexpr int forced = TRI_FORCE_BIN_LOG2;
    static_assert(forced == 0 || (forced >= 4 && forced <= 6), "TRI_FORCE_BIN_LOG2: 4, 5 or 6");
    auto bins = [c](int bl) {
        const int32_t bs = 1 << bl;
        return ((c->W + bs - 1) / bs) * ((c->y1 - c->y0 + bs - 1) / bs);
    };
    int bl = forced;
    if (!bl) {
        const double density = (double)c->nprims / ((double)c->W * (double)c->H);
        const int32_t n32 = bins(5);
        bl = n32 > 16384 ? 6 : ((n32 < 4096 && density < 0.05) ? 4 : 5);
    }
    if (bl == c->bin_log2) return TRI_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));  // queued frames still use the old grid
    int rc;
    const int32_t bs = 1 << bl;
    c->bin_log2 = bl;
    c->nbx = (c->W + bs - 1) / bs;
    c->nby = (c->y1 - c->y0 + bs - 1) / bs;
    c->nbins = c->nbx * c->nby;
    c->bin_cap = 0;  // re-derived for the new grid by ensure_work_buffers
    if ((rc = grow(c->d_bin_count, c->cap_bin_count, (size_t)c->nbins))) return rc;
    HIP_TRY(hipMemsetAsync(c->d_bin_count, 0, (size_t)c->nbins * 4, c->stream));  // before this frame's k_setup
    return TRI_OK;
}

// UploadMeshFromCache into a geometry object: the caller has made its device current and drained the
// streams that read it.
int geometry_upload(tri_geometry* g, const tri_vertex* v, uint64_t nv, const uint32_t* idx, uint64_t ni,
                    const tri_mesh_range* meshes, uint32_t nm) {
    if ((nv && !v) || (ni && !idx) || (nm && !meshes)) return fail(TRI_E_INVALID, "tri_upload_geometry: null array");
    if (nv * sizeof(TriVsIn) > 0xFFFFFFFFull)  // k_vertex reads the records with 32-bit byte offsets
        return fail(TRI_E_INVALID, "tri_upload_geometry: %llu vertices exceed the 4 GiB vertex-record buffer",
                    (unsigned long long)nv);
    int rc;
    // AoS 100-byte Vertex -> 48-byte shading records (+ 32-byte skin records when weights exist)
    std::vector<TriVsIn> vin(nv);
    std::vector<TriVsSkin> skin;
    bool has_skin = false, obj_ok = true;
    for (uint64_t i = 0; i < nv; ++i) {
        const tri_vertex& s = v[i];
        TriVsIn& o = vin[i];
        o.px = s.position[0]; o.py = s.position[1]; o.pz = s.position[2];
        o.nx = s.normal[0]; o.ny = s.normal[1]; o.nz = s.normal[2];
        const double n2 = (double)o.nx * o.nx + (double)o.ny * o.ny + (double)o.nz * o.nz;
        obj_ok = obj_ok && std::fabs(n2 - 1.0) <= 1e-5 && std::isfinite(o.px) && std::isfinite(o.py) &&
                 std::isfinite(o.pz);
        o.cr = s.color[0]; o.cg = s.color[1]; o.cb = s.color[2];
        o.u = s.texcoord[0]; o.v = s.texcoord[1]; o.pad = 0.0f;
        has_skin = has_skin || s.bone_weights[0] > 0.f || s.bone_weights[1] > 0.f || s.bone_weights[2] > 0.f ||
                   s.bone_weights[3] > 0.f;
    }
    if (has_skin) {
        skin.resize(nv);
        for (uint64_t i = 0; i < nv; ++i) {
            std::memcpy(skin[i].idx, v[i].bone_indices, 16);
            std::memcpy(skin[i].w, v[i].bone_weights, 16);
        }
        if ((rc = grow(g->d_skin, g->cap_skin, nv))) return rc;
        HIP_TRY(hipMemcpy(g->d_skin, skin.data(), nv * sizeof(TriVsSkin), hipMemcpyHostToDevice));
    }
    g->has_skin_data = has_skin;
    g->obj_ok = obj_ok;
    g->uni_col = nv > 0;
    for (uint64_t i = 0; i < nv && g->uni_col; ++i)
        g->uni_col = vin[i].cr == vin[0].cr && vin[i].cg == vin[0].cg && vin[i].cb == vin[0].cb;
    if (g->uni_col) { g->ucol[0] = vin[0].cr; g->ucol[1] = vin[0].cg; g->ucol[2] = vin[0].cb; }
    if ((rc = grow(g->d_vin, g->cap_vin, std::max<uint64_t>(nv, 1)))) return rc;
    if (nv) HIP_TRY(hipMemcpy(g->d_vin, vin.data(), nv * sizeof(TriVsIn), hipMemcpyHostToDevice));
    {  // the object-space streams of vary_obj frames: positions (k_vertex) and 36-B attribute records (k_raster)
        std::vector<float> pos(3 * nv), attr(9 * nv);
        for (uint64_t i = 0; i < nv; ++i) {
            const TriVsIn& o = vin[i];
            pos[3 * i] = o.px; pos[3 * i + 1] = o.py; pos[3 * i + 2] = o.pz;
            const float a[9] = {o.px, o.py, o.pz, o.nx, o.ny, o.nz, o.cr, o.cg, o.cb};
            std::memcpy(&attr[9 * i], a, sizeof a);
        }
        if ((rc = grow(g->d_pos, g->cap_pos, std::max<uint64_t>(3 * nv, 3)))) return rc;
        if ((rc = grow(g->d_attr, g->cap_attr, std::max<uint64_t>(9 * nv, 9)))) return rc;
        if (nv) HIP_TRY(hipMemcpy(g->d_pos, pos.data(), nv * 12, hipMemcpyHostToDevice));
        if (nv) HIP_TRY(hipMemcpy(g->d_attr, attr.data(), nv * 36, hipMemcpyHostToDevice));
    }
    if ((rc = grow(g->d_idx, g->cap_idx, std::max<uint64_t>(ni, 1)))) return rc;
    if (ni) HIP_TRY(hipMemcpy(g->d_idx, idx, ni * 4, hipMemcpyHostToDevice));
    g->nverts = nv;
    g->nidx = ni;
    g->meshes.assign(meshes, meshes + nm);
    g->mesh_min.assign(nm, 0);
    g->mesh_max.assign(nm, 0);
    for (uint32_t m = 0; m < nm; ++m) {  // referenced vertex range per mesh (VS invocation range)
        const tri_mesh_range& mr = meshes[m];
        if (mr.index_count < 3 || (uint64_t)mr.first_index + mr.index_count > ni) continue;
        const uint32_t cnt = (mr.index_count / 3) * 3;
        uint32_t mn = 0xFFFFFFFFu, mx = 0;
        for (uint32_t i = 0; i < cnt; ++i) {
            mn = std::min(mn, idx[mr.first_index + i]);
            mx = std::max(mx, idx[mr.first_index + i]);
        }
        if (mx - mn >= 0x7FFFFFFFu) return fail(TRI_E_INVALID, "mesh %u: index range too large", m);
        g->mesh_min[m] = mn;
        g->mesh_max[m] = mx;
    }
    // cluster tables (row-band culling): runs of TRI_CLUSTER_PRIMS primitives with their object-space
    // boxes and index ranges; per 256-slot vertex block the interval of clusters whose range meets it
    std::vector<TriCluster> cl;
    std::vector<uint2> vblk;
    std::vector<TriCluster> vbox;  // parallel to vblk
    g->mesh_cl_first.assign(nm, 0);
    g->mesh_ncl.assign(nm, 0);
    g->mesh_vblk_first.assign(nm, 0);
    for (uint32_t m = 0; m < nm; ++m) {
        const tri_mesh_range& mr = meshes[m];
        if (mr.index_count < 3 || (uint64_t)mr.first_index + mr.index_count > ni) continue;
        const uint32_t ntri = mr.index_count / 3;
        const uint32_t ncl = (ntri + TRI_CLUSTER_PRIMS - 1) / TRI_CLUSTER_PRIMS;
        const uint32_t mn = g->mesh_min[m];
        const uint32_t nblk = (g->mesh_max[m] - mn) / TRI_VBLOCK + 1;
        g->mesh_cl_first[m] = (uint32_t)cl.size();
        g->mesh_ncl[m] = ncl;
        g->mesh_vblk_first[m] = (uint32_t)vblk.size();
        vblk.resize(vblk.size() + nblk, make_uint2(0xFFFFFFFFu, 0u));
        uint2* iv = vblk.data() + g->mesh_vblk_first[m];
        for (uint32_t k = 0; k < ncl; ++k) {
            TriCluster t;
            for (int a = 0; a < 3; ++a) { t.lo[a] = INFINITY; t.hi[a] = -INFINITY; }
            t.vmin = 0xFFFFFFFFu;
            t.vmax = 0;
            const uint32_t i0 = mr.first_index + 3 * k * TRI_CLUSTER_PRIMS;
            const uint32_t i1 = mr.first_index + 3 * std::min(ntri, (k + 1) * TRI_CLUSTER_PRIMS);
            for (uint32_t i = i0; i < i1; ++i) {
                const uint32_t x = idx[i];
                t.vmin = std::min(t.vmin, x);
                t.vmax = std::max(t.vmax, x);
                const int64_t gi = (int64_t)mr.base_vertex + x;
                if (gi < 0 || (uint64_t)gi >= nv) continue;
                for (int a = 0; a < 3; ++a) {
                    t.lo[a] = std::fmin(t.lo[a], v[gi].position[a]);
                    t.hi[a] = std::fmax(t.hi[a], v[gi].position[a]);
                }
            }
            for (uint32_t bk = (t.vmin - mn) / TRI_VBLOCK; bk <= (t.vmax - mn) / TRI_VBLOCK; ++bk) {
                iv[bk].x = std::min(iv[bk].x, k);
                iv[bk].y = std::max(iv[bk].y, k);
            }
            cl.push_back(t);
        }
        // per vertex block: the union of the boxes of every cluster whose index range meets it (empty when
        // none does): k_vertex keeps the block iff that box can reach the rows, one load and one test per wave
        for (uint32_t bk = 0; bk < nblk; ++bk) {
            TriCluster u;
            for (int a = 0; a < 3; ++a) { u.lo[a] = INFINITY; u.hi[a] = -INFINITY; }
            u.vmin = u.vmax = 0;
            for (uint32_t k = iv[bk].x; iv[bk].x <= iv[bk].y && k <= iv[bk].y; ++k) {
                const TriCluster& t = cl[g->mesh_cl_first[m] + k];
                for (int a = 0; a < 3; ++a) { u.lo[a] = std::fmin(u.lo[a], t.lo[a]); u.hi[a] = std::fmax(u.hi[a], t.hi[a]); }
            }
            vbox.push_back(u);
        }
    }
    if ((rc = grow(g->d_clusters, g->cap_clusters, std::max<size_t>(cl.size(), 1)))) return rc;
    if (!cl.empty()) HIP_TRY(hipMemcpy(g->d_clusters, cl.data(), cl.size() * sizeof(TriCluster), hipMemcpyHostToDevice));
    if ((rc = grow(g->d_vbox, g->cap_vbox, std::max<size_t>(vbox.size(), 1)))) return rc;
    if (!vbox.empty()) HIP_TRY(hipMemcpy(g->d_vbox, vbox.data(), vbox.size() * sizeof(TriCluster), hipMemcpyHostToDevice));
    // null-stream copies are not ordered with the contexts' non-blocking streams: complete them before any
    // context can launch a frame that reads this geometry
    HIP_TRY(hipStreamSynchronize(nullptr));
    g->geometry_set = true;
    // versions come from one process-wide counter: a context that switches between geometry objects
    // (tri_bind_geometry, tri_upload_geometry) can never see an equal version on a different object
    static std::atomic<uint64_t> g_geometry_version{0};
    g->version = ++g_geometry_version;
    return TRI_OK;
}

void free_geometry(tri_geometry& g) {
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    f(g.d_vin); f(g.d_pos); f(g.d_attr); f(g.d_skin); f(g.d_idx); f(g.d_clusters); f(g.d_vbox);
    g.d_vin = nullptr; g.d_pos = nullptr; g.d_attr = nullptr; g.d_skin = nullptr; g.d_idx = nullptr;
    g.d_clusters = nullptr; g.d_vbox = nullptr;
    g.cap_vin = g.cap_pos = g.cap_attr = g.cap_skin = g.cap_idx = g.cap_clusters = g.cap_vbox = 0;
}

}  // namespace

hipStream_t tri_internal_stream(tri_ctx* c) { return c->stream; }
int tri_internal_device(tri_ctx* c) { return c->device; }
int tri_internal_fail(int code, const char* msg) { return fail(code, "%s", msg); }
int tri_internal_geometry_device(const tri_geometry* g) { return g->device; }
const float* tri_internal_unorm_lut(tri_ctx* c) { return c->d_lut + 256; }

extern "C" {

const char* tri_last_error(void) { return g_last_error.c_str(); }
int tri_abi_version(void) { return TRI_RASTER_ABI_VERSION; }

int tri_create(const tri_config* cfg, tri_ctx** out) {
    if (!cfg || !out) return fail(TRI_E_INVALID, "tri_create: null argument");
    *out = nullptr;
    if (cfg->width == 0 || cfg->height == 0 || cfg->width > TRI_MAX_DIM || cfg->height > TRI_MAX_DIM)
        return fail(TRI_E_INVALID, "tri_create: framebuffer %ux%u outside 1..%d", cfg->width, cfg->height, TRI_MAX_DIM);
    uint32_t y0 = cfg->band_y0, y1 = cfg->band_y1;
    if (y0 == 0 && y1 == 0) y1 = cfg->height;
    if (y0 >= y1 || y1 > cfg->height) return fail(TRI_E_INVALID, "tri_create: bad row band [%u,%u)", y0, y1);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(TRI_E_HIP, "tri_create: no HIP device available");
    tri_ctx* c = new tri_ctx();
    c->cfg = *cfg;
    if (cfg->device >= 0) {
        if (cfg->device >= ndev) { delete c; return fail(TRI_E_INVALID, "tri_create: device %d of %d", cfg->device, ndev); }
        c->device = cfg->device;
    } else if (hipGetDevice(&c->device) != hipSuccess) {
        delete c;
        return fail(TRI_E_HIP, "tri_create: hipGetDevice failed");
    }
    c->W = (int32_t)cfg->width;
    c->H = (int32_t)cfg->height;
    c->y0 = (int32_t)y0;
    c->y1 = (int32_t)y1;
    c->bin_log2 = 0;  // the bin grid is chosen at the first tri_render (choose_bin_grid)
    auto bail = [&](int rc) { tri_destroy(c); return rc; };
    int rc = make_current(c);
    if (rc) return bail(rc);
    if (tri_kernels_init() != hipSuccess) return bail(fail(TRI_E_HIP, "tri_create: kernel attribute setup failed"));
    if (hipDeviceGetAttribute(&c->cu_count, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
        c->cu_count <= 0)
        c->cu_count = 256;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(TRI_E_HIP, "tri_create: stream creation failed"));
    c->stream = c->own_stream;
    const size_t px = (size_t)c->W * (size_t)(c->y1 - c->y0);
    if (hipMalloc(&c->d_color_own, px * 4) != hipSuccess || hipMalloc(&c->d_depth_own, px * 4) != hipSuccess ||
        hipMalloc(&c->d_ctr, sizeof(TriCounters)) != hipSuccess ||
        hipMalloc(&c->d_lut, 512 * sizeof(float)) != hipSuccess)
        return bail(fail(TRI_E_OOM, "tri_create: target allocation failed"));
    c->d_color = c->d_color_own;
    c->d_depth = c->d_depth_own;
    if (hipMemset(c->d_ctr, 0, sizeof(TriCounters)) != hipSuccess)
        return bail(fail(TRI_E_HIP, "tri_create: memset failed"));
    if (hipMalloc(&c->d_args, sizeof(TriLaunchArgs)) != hipSuccess)
        return bail(fail(TRI_E_OOM, "tri_create: argument copy allocation failed"));
    float lut[512];
    for (int i = 0; i < 256; ++i) {  // R8G8B8A8_SRGB decode (sRGB EOTF), evaluated in double
        lut[i] = srgb_decode(i);
        lut[256 + i] = (float)i / 255.0f;  // alpha: linear UNORM decode (IEEE float division)
    }
    if (hipMemcpy(c->d_lut, lut, sizeof lut, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(TRI_E_HIP, "tri_create: LUT upload failed"));
    const uint8_t white[4] = {0xFF, 0xFF, 0xFF, 0xFF};  // CreateDefaultTexture (Renderer.cpp:3404-3436)
    if ((rc = tri_upload_texture(c, 0, white, 1, 1))) return bail(rc);
    const float clear[4] = {0.005f, 0.005f, 0.005f, 1.0f};  // m_ClearColor default (Renderer.h:469)
    c->clear_bgra = unorm8_host(clear[2]) | (unorm8_host(clear[1]) << 8) | (unorm8_host(clear[0]) << 16) |
                    (unorm8_host(clear[3]) << 24);
    // the counters, LUT and default texture above went through null-stream copies: complete them before
    // any kernel on the context's non-blocking stream can read them
    if (hipDeviceSynchronize() != hipSuccess) return bail(fail(TRI_E_HIP, "tri_create: device synchronisation failed"));
    *out = c;
    return TRI_OK;
}

int tri_destroy(tri_ctx* c) {
    if (!c) return TRI_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    auto f = [](void* p) { if (p) (void)hipFree(p); };
    free_geometry(c->own_geom);
    f(c->d_lut); f(c->d_bones); f(c->d_sky); f(c->d_ai);
    for (auto& t : c->d_tex) f(t);
    f(c->d_draws); f(c->d_draw_shade); f(c->d_vbase); f(c->d_pbase); f(c->d_cbase); f(c->d_cvis);
    f(c->d_clip); f(c->d_snap); f(c->d_oc); f(c->d_vary); f(c->d_recs); f(c->d_clip_slot); f(c->d_prim_vs); f(c->d_setup_stats);
    f(c->d_bin_count); f(c->d_bin_list); f(c->d_ctr);
    f(c->d_color_own); f(c->d_depth_own); f(c->d_present);
    f(c->d_lpos); f(c->d_lsnap); f(c->d_sbin_count); f(c->d_sbin_list); f(c->d_shadow);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_ctr) (void)hipHostFree(c->h_ctr);
    f(c->d_args);
    if (c->stage_free) (void)hipEventDestroy(c->stage_free);
    for (auto& v : {std::cref(c->pending), std::cref(c->free_sets)})
        for (const TimingSet& t : v.get())
            for (auto e : t.ev) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return TRI_OK;
}

int tri_set_stream(tri_ctx* c, void* s) {
    if (!c) return fail(TRI_E_INVALID, "tri_set_stream: null context");
    hipStream_t next = s ? static_cast<hipStream_t>(s) : c->own_stream;
    if (next != c->stream && c->launched) {
        // the next frame's argument copy must not overtake the previous frame's kernels on the old stream
        int rc = make_current(c);
        if (rc) return rc;
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(e, c->stream));
        HIP_TRY(hipStreamWaitEvent(next, e, 0));
        HIP_TRY(hipEventDestroy(e));
    }
    c->stream = next;
    return TRI_OK;
}

int tri_upload_geometry(tri_ctx* c, const tri_vertex* v, uint64_t nv, const uint32_t* idx, uint64_t ni,
                        const tri_mesh_range* meshes, uint32_t nm) {
    if (!c) return fail(TRI_E_INVALID, "tri_upload_geometry: null context");
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->geom = &c->own_geom;
    c->own_geom.device = c->device;
    c->geom_seen = 0;  // re-resolve the draws against the new buffers even if the draw list is unchanged
    c->draws_dirty = true;
    return geometry_upload(&c->own_geom, v, nv, idx, ni, meshes, nm);
}

int tri_geometry_create(int32_t device, tri_geometry** out) {
    if (!out) return fail(TRI_E_INVALID, "tri_geometry_create: null argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(TRI_E_HIP, "tri_geometry_create: no HIP device available");
    int d = device;
    if (d < 0 && hipGetDevice(&d) != hipSuccess) return fail(TRI_E_HIP, "tri_geometry_create: hipGetDevice failed");
    if (d >= ndev) return fail(TRI_E_INVALID, "tri_geometry_create: device %d of %d", d, ndev);
    tri_geometry* g = new tri_geometry();
    g->device = d;
    g->shared = true;
    *out = g;
    return TRI_OK;
}

int tri_geometry_upload(tri_geometry* g, const tri_vertex* v, uint64_t nv, const uint32_t* idx, uint64_t ni,
                        const tri_mesh_range* meshes, uint32_t nm) {
    if (!g) return fail(TRI_E_INVALID, "tri_geometry_upload: null geometry");
    HIP_TRY(hipSetDevice(g->device));
    HIP_TRY(hipDeviceSynchronize());  // any context's stream may be reading the old buffers
    return geometry_upload(g, v, nv, idx, ni, meshes, nm);
}

int tri_geometry_destroy(tri_geometry* g) {
    if (!g) return TRI_OK;
    (void)hipSetDevice(g->device);
    (void)hipDeviceSynchronize();
    free_geometry(*g);
    delete g;
    return TRI_OK;
}

int tri_bind_geometry(tri_ctx* c, tri_geometry* g) {
    if (!c) return fail(TRI_E_INVALID, "tri_bind_geometry: null context");
    if (g && g->device != c->device)
        return fail(TRI_E_INVALID, "tri_bind_geometry: geometry on device %d, context on device %d", g->device, c->device);
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->geom = g ? g : &c->own_geom;
    c->geom_seen = 0;
    c->draws_dirty = true;
    return TRI_OK;
}

int tri_upload_materials(tri_ctx* c, const tri_material_record* r, uint32_t n) {
    if (!c) return fail(TRI_E_INVALID, "tri_upload_materials: null context");
    if (n && !r) return fail(TRI_E_INVALID, "tri_upload_materials: null records");
    c->mat0 = n ? r[0] : tri_material_record{{1, 1, 1, 1}, {1, 1, 1, 0}};
    return TRI_OK;
}

int tri_upload_texture(tri_ctx* c, uint32_t slot, const uint8_t* rgba, uint32_t w, uint32_t h) {
    if (!c) return fail(TRI_E_INVALID, "tri_upload_texture: null context");
    if (slot >= TRI_MAX_TEXTURE_SLOTS) return fail(TRI_E_INVALID, "tri_upload_texture: slot %u >= %d", slot, TRI_MAX_TEXTURE_SLOTS);
    if (!rgba || w == 0 || h == 0 || (uint64_t)w * h > (1ull << 28))
        return fail(TRI_E_INVALID, "tri_upload_texture: bad texture %ux%u", w, h);
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->d_tex[slot]) HIP_TRY(hipFree(c->d_tex[slot]));
    c->d_tex[slot] = nullptr;
    HIP_TRY(hipMalloc(&c->d_tex[slot], (size_t)w * h * 4));
    HIP_TRY(hipMemcpy(c->d_tex[slot], rgba, (size_t)w * h * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipStreamSynchronize(nullptr));  // complete before the next frame on the non-blocking stream
    c->tex_w[slot] = w;
    c->tex_h[slot] = h;
    std::memcpy(&c->tex_solid[slot], rgba, 4);
    c->tex_alpha[slot] = rgba[3];
    for (size_t i = 1, n = (size_t)w * h; i < n; ++i)
        if (rgba[4 * i + 3] != rgba[3]) {
            c->tex_alpha[slot] = -1;
            break;
        }
    c->tex_dirty = true;
    return TRI_OK;
}

int tri_upload_bone_palette(tri_ctx* c, const float* m, uint32_t n) {
    if (!c) return fail(TRI_E_INVALID, "tri_upload_bone_palette: null context");
    if (n && !m) return fail(TRI_E_INVALID, "tri_upload_bone_palette: null matrices");
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if ((rc = grow(c->d_bones, c->cap_bones, std::max<size_t>(16ull * n, 16)))) return rc;
    if (n) HIP_TRY(hipMemcpy(c->d_bones, m, 64ull * n, hipMemcpyHostToDevice));
    HIP_TRY(hipStreamSynchronize(nullptr));  // complete before the next frame on the non-blocking stream
    c->nbones = n;
    return TRI_OK;
}

int tri_upload_skybox(tri_ctx* c, const uint8_t* faces, uint32_t n) {
    if (!c) return fail(TRI_E_INVALID, "tri_upload_skybox: null context");
    if (!faces || n == 0) {
        c->sky_size = 0;
        return TRI_OK;
    }
    if (n > 16384) return fail(TRI_E_INVALID, "tri_upload_skybox: face size %u too large", n);
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    const size_t texels = 6ull * n * n;
    if ((rc = grow(c->d_sky, c->cap_sky, texels))) return rc;
    HIP_TRY(hipMemcpy(c->d_sky, faces, texels * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipStreamSynchronize(nullptr));  // complete before the next frame on the non-blocking stream
    c->sky_size = n;
    const uint32_t* t = reinterpret_cast<const uint32_t*>(faces);
    uint32_t t0;
    std::memcpy(&t0, faces, 4);
    c->sky_uniform = true;
    for (size_t i = 1; i < texels && c->sky_uniform; ++i) {
        uint32_t ti;
        std::memcpy(&ti, t + i, 4);
        c->sky_uniform = ti == t0;
    }
    // Skybox.frag writes the decoded linear colour, alpha 1, to the UNORM target
    c->sky_uniform_bgra = unorm8_host(srgb_decode((t0 >> 16) & 0xFF)) | (unorm8_host(srgb_decode((t0 >> 8) & 0xFF)) << 8) |
                          (unorm8_host(srgb_decode(t0 & 0xFF)) << 16) | (255u << 24);
    return TRI_OK;
}

// The AI frame-generation texture (EnsureAiTextureResources, Renderer.cpp:1390-1500; UploadAiInterpolationToGpu,
// :1560-1700): R8G8B8A8_UNORM, the extent of the frame it was generated for.
int tri_upload_ai_frame(tri_ctx* c, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    if (!c) return fail(TRI_E_INVALID, "tri_upload_ai_frame: null context");
    if (!rgba8 || w == 0 || h == 0) {  // DestroyAiResources: no texture, no blend
        c->ai_w = c->ai_h = 0;
        return TRI_OK;
    }
    if (w > TRI_MAX_DIM || h > TRI_MAX_DIM)
        return fail(TRI_E_INVALID, "tri_upload_ai_frame: extent %ux%u outside 1..%d", w, h, TRI_MAX_DIM);
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));  // no queued frame still samples the previous texture
    if ((rc = grow(c->d_ai, c->cap_ai, (size_t)w * h))) return rc;
    HIP_TRY(hipMemcpy(c->d_ai, rgba8, (size_t)w * h * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipStreamSynchronize(nullptr));  // complete before the next frame on the non-blocking stream
    c->ai_w = w;
    c->ai_h = h;
    return TRI_OK;
}

int tri_set_shadow(tri_ctx* c, const tri_shadow_config* cfg) {
    if (!c) return fail(TRI_E_INVALID, "tri_set_shadow: null context");
    if (!cfg || cfg->size == 0) {
        c->shadow = tri_shadow_config{};
        c->shadow_rendered = false;
        return TRI_OK;
    }
    if (cfg->size > TRI_MAX_DIM) return fail(TRI_E_INVALID, "tri_set_shadow: map size %u > %d", cfg->size, TRI_MAX_DIM);
    const float* m = cfg->light_view_proj;
    if (m[3] != 0.0f || m[7] != 0.0f || m[11] != 0.0f || m[15] != 1.0f)
        return fail(TRI_E_INVALID, "tri_set_shadow: light_view_proj must be affine (an orthographic light)");
    for (int i = 0; i < 16; ++i)
        if (!std::isfinite(m[i])) return fail(TRI_E_INVALID, "tri_set_shadow: non-finite light transform");
    if (!std::isfinite(cfg->depth_bias) || !std::isfinite(cfg->slope_bias))
        return fail(TRI_E_INVALID, "tri_set_shadow: non-finite depth bias");
    int rc = make_current(c);
    if (rc) return rc;
    const uint32_t nbx = (cfg->size + 31) / 32;
    if (cfg->size != c->shadow.size) {  // new map grid: fresh (zeroed) queue counters
        HIP_TRY(hipStreamSynchronize(c->stream));
        if ((rc = grow(c->d_sbin_count, c->cap_sbin_count, (size_t)nbx * nbx))) return rc;
        HIP_TRY(hipMemsetAsync(c->d_sbin_count, 0, (size_t)nbx * nbx * 4, c->stream));
        c->s_bin_cap = 0;
        c->shadow_rendered = false;
    }
    c->shadow = *cfg;
    c->s_nbx = nbx;
    c->s_nbins = nbx * nbx;
    return TRI_OK;
}

int tri_shadow_fit_ortho(const float dir[3], const float mn[3], const float mx[3], float out[16]) {
    if (!dir || !mn || !mx || !out) return fail(TRI_E_INVALID, "tri_shadow_fit_ortho: null argument");
    for (int a = 0; a < 3; ++a)
        if (!std::isfinite(mn[a]) || !std::isfinite(mx[a]) || mn[a] > mx[a])
            return fail(TRI_E_INVALID, "tri_shadow_fit_ortho: bad box");
    shadow_fit_ortho(dir, mn, mx, out);
    return TRI_OK;
}

int tri_read_shadow_map(tri_ctx* c, uint32_t* out) {
    if (!c || !out) return fail(TRI_E_INVALID, "tri_read_shadow_map: null argument");
    if (!c->shadow.size || !c->shadow_rendered) return fail(TRI_E_STATE, "tri_read_shadow_map: no shadow pass rendered");
    int rc = tri_synchronize(c);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(out, c->d_shadow, (size_t)c->shadow.size * c->shadow.size * 4, hipMemcpyDeviceToHost));
    return TRI_OK;
}

int tri_set_frame(tri_ctx* c, const tri_global_ubo* ubo, const float clear[4]) {
    if (!c || !ubo) return fail(TRI_E_INVALID, "tri_set_frame: null argument");
    c->ubo = *ubo;
    mat4_mul(ubo->projection, ubo->view, c->pv);  // (P*V), Default.vert:104
    if (clear)
        c->clear_bgra = unorm8_host(clear[2]) | (unorm8_host(clear[1]) << 8) | (unorm8_host(clear[0]) << 16) |
                        (unorm8_host(clear[3]) << 24);
    c->frame_set = true;
    return TRI_OK;
}

// Default.frag's alpha is (base.a * tint.a) * texture.a (the UNORM decode b / 255, bilinear taps of one value
// return it exactly), stored as unorm8 by both shading builds; background pixels hold the clear colour's alpha,
// or 1 where Skybox.frag writes. The same float operations here give the byte each draw can produce.
int tri_frame_alpha(tri_ctx* c, int32_t* alpha) {
    if (!c || !alpha) return fail(TRI_E_INVALID, "tri_frame_alpha: null argument");
    int32_t a = (int32_t)(c->clear_bgra >> 24);
    bool uniform = !c->sky_size || a == 255;
    // the AI frame blend mixes every mesh fragment's alpha with the AI frame's (not proven uniform here)
    if (c->ubo.ai_blend_config[3] > 0.0f && c->ubo.ai_blend_config[0] > 0.0f && !c->draws.empty()) uniform = false;
    for (const tri_draw& d : c->draws) {
        if (!uniform) break;
        int32_t slot = d.pc.texture_slot;
        if (slot < 0 || slot >= TRI_MAX_TEXTURE_SLOTS || !c->d_tex[slot]) slot = 0;  // unused slots alias slot 0
        const int16_t ta = c->tex_alpha[slot];
        if (ta < 0) {
            uniform = false;
            break;
        }
        const float t = (float)ta / 255.0f;
        uniform = (int32_t)unorm8_host((c->mat0.base_color_factor[3] * d.pc.tint[3]) * t) == a;
    }
    *alpha = uniform ? a : -1;
    return TRI_OK;
}

int tri_set_draws(tri_ctx* c, const tri_draw* d, uint32_t n) {
    if (!c) return fail(TRI_E_INVALID, "tri_set_draws: null context");
    if (n && !d) return fail(TRI_E_INVALID, "tri_set_draws: null draws");
    if (n == c->draws.size() && (n == 0 || std::memcmp(c->draws.data(), d, n * sizeof(tri_draw)) == 0))
        return TRI_OK;  // unchanged draw list: keep the device copy (no per-frame upload)
    c->draws.assign(d, d + n);
    c->draws_dirty = true;
    return TRI_OK;
}

int tri_bind_output(tri_ctx* c, void* color, void* depth) {
    if (!c) return fail(TRI_E_INVALID, "tri_bind_output: null context");
    c->d_color = color ? static_cast<uint32_t*>(color) : c->d_color_own;
    c->d_depth = depth ? static_cast<float*>(depth) : c->d_depth_own;
    return TRI_OK;
}

// Diagnostics builds only (-DTRI_HOST_TIMING): tri_render's host time split at its phase boundaries (entry,
// current device, state checks and buffers, frame arguments, launches), read by tools/host_breakdown.py.
#ifdef TRI_HOST_TIMING
static double g_host_ns[5];
static uint64_t g_host_calls;
#define TRI_HSTAMP(k) const auto hs##k = std::chrono::steady_clock::now()
extern "C" void tri_debug_host_times(double* out, int reset) {
    for (int i = 0; i < 5; ++i) out[i] = g_host_calls ? g_host_ns[i] / (double)g_host_calls : 0.0;
    if (reset) { for (double& x : g_host_ns) x = 0.0; g_host_calls = 0; }
}
#else
#define TRI_HSTAMP(k) do { } while (0)
#endif

int tri_render(tri_ctx* c) {
    TRI_HSTAMP(0);
    if (!c) return fail(TRI_E_INVALID, "tri_render: null context");
    if (!c->frame_set) return fail(TRI_E_STATE, "tri_render: tri_set_frame was not called");
    if (!c->draws.empty() && !c->geom->geometry_set) return fail(TRI_E_STATE, "tri_render: draws without geometry");
    int rc = make_current(c);
    if (rc) return rc;
    TRI_HSTAMP(1);
    if ((rc = upload_texture_table(c))) return rc;
    if (c->geom->version != c->geom_seen) {  // (shared) geometry changed since the draws were resolved
        c->draws_dirty = true;
        c->geom_seen = c->geom->version;
    }
    if ((rc = resolve_draws(c))) return rc;
    if (c->any_skin && !c->geom->has_skin_data) {
        // a skinned draw over vertices without weights: skin matrix = 0 -> everything collapses
        // to the origin, exactly like the shader with all-zero weights; give the kernel zeros. The
        // geometry may be shared with contexts on other streams, so the zeros are in place (device
        // synchronised) before the shared flag says so.
        if ((rc = grow(c->geom->d_skin, c->geom->cap_skin, std::max<uint64_t>(c->geom->nverts, 1)))) return rc;
        HIP_TRY(hipMemset(c->geom->d_skin, 0, std::max<uint64_t>(c->geom->nverts, 1) * sizeof(TriVsSkin)));
        HIP_TRY(hipDeviceSynchronize());
        c->geom->has_skin_data = true;
    }
    if ((rc = choose_bin_grid(c))) return rc;
    if ((rc = ensure_work_buffers(c))) return rc;

    TRI_HSTAMP(2);
    TriLaunchArgs& ha = c->args;  // passed by value at launch: free to rewrite for the next frame
    TriFrameParams& fp = ha.fp;
    std::memset(&fp, 0, sizeof fp);
    fp.W = c->W; fp.H = c->H; fp.y0 = c->y0; fp.y1 = c->y1;
    fp.nbx = c->nbx; fp.nby = c->nby; fp.nbins = c->nbins;
    fp.bin_log2 = c->bin_log2;
    // k_setup grid: a shadow frame takes at most one resident round of workgroups (6 per CU at its
    // occupancy): a workgroup's fetch -> set-up -> reservation -> store chain is latency, and a partial
    // second round doubles the kernel (C3: 1953 chunks of 512 -> 977 of 1024, set-up 33 -> 30 us). Other
    // frames take 2 per CU with more primitives each, leaving wave slots to the raster of the frame in
    // flight beside them (TRI_SETUP_WGS_PER_CU_OVERLAP, raster_launch.h). A band (cluster culling) keeps
    // 512-primitive chunks: most of them exit at once, and the visible ones keep one chain each.
    const bool culling = (c->y0 != 0 || c->y1 != c->H || (c->cfg.flags & TRI_FLAG_CLUSTER_CULL)) && c->ncl_total > 0;
    const uint32_t target_chunks = culling ? (uint32_t)TRI_SETUP_BAND_CHUNKS
                                           : (uint32_t)c->cu_count * (c->shadow.size ? TRI_SETUP_WGS_PER_CU
                                                                                      : TRI_SETUP_WGS_PER_CU_OVERLAP);
    uint32_t ppt = (c->nprims + target_chunks * TRI_BLOCK - 1) / (target_chunks * TRI_BLOCK);
    // k_setup sets up and bins pairs: an odd count leaves half of its last round idle, which costs more
    // than the extra chunks save (C3: 3 per lane 29.2 us, 4 per lane 28.3 us), except on a frame whose
    // primitives fit one primitive per lane in one round (C2: 14.2 -> 12.9 us)
    ppt = ppt <= 1 && !culling ? 1u : std::min<uint32_t>(std::max<uint32_t>((ppt + 1) & ~1u, 2), TRI_MAX_PPT);
    fp.ppt = (int32_t)ppt;
    fp.nchunks = (c->nprims + ppt * TRI_BLOCK - 1) / (ppt * TRI_BLOCK);
    fp.chunk_stride = chunk_stride(fp.nchunks);
    c->last_nchunks = fp.nchunks;
    fp.hw = (float)c->W * 0.5f;
    fp.hh = (float)c->H * 0.5f;
    fp.gx = (2.0f * TRI_GUARD_BAND_PX) / (float)c->W - 1.0f;
    fp.gy = (2.0f * TRI_GUARD_BAND_PX) / (float)c->H - 1.0f;
    fp.nprims = c->nprims;
    fp.nslots = c->nslots;
    fp.ndraws = c->ndraws;
    fp.one_draw = c->ndraws == 1 ? 1u : 0u;
    if (fp.one_draw) fp.draw0 = c->draw0;
    fp.shade_solid = (fp.one_draw && c->shade0.tex.w == 1 && c->shade0.tex.h == 1) ? 1u : 0u;
    // the frames k_raster_plain<.., ONE> shades keep 36-B varyings (no texture coordinates)
    // Default.frag's AI frame blend (:182-191): on when AiBlendConfig.w > 0 and its clamped weight is positive; its
    // frames take k_raster_ai (the general instantiation: world-space or obj48 varyings, never the ONE 36-B records)
    const float ai_wgt = std::fmin(std::fmax(c->ubo.ai_blend_config[0], 0.0f), 1.0f);
    fp.ai_on = (c->ubo.ai_blend_config[3] > 0.0f && ai_wgt > 0.0f) ? 1u : 0u;
    if (fp.ai_on) {
        if (!c->ai_w) return fail(TRI_E_STATE, "tri_render: AiBlendConfig.w > 0 but no AI frame uploaded (tri_upload_ai_frame)");
        if (c->shadow.size)
            return fail(TRI_E_UNSUPPORTED, "tri_render: the AI frame blend with the shadow pre-pass (the reference has no shadow pass)");
        fp.ai_wgt = ai_wgt;
        fp.ai_sx = c->ubo.ai_blend_config[1];
        fp.ai_sy = c->ubo.ai_blend_config[2];
        fp.ai_tw = c->ai_w;
        fp.ai_th = c->ai_h;
    }
    fp.vary36 = (fp.shade_solid && !c->shadow.size && !fp.ai_on) ? 1u : 0u;
    fp.vary_obj = fp.vary36 && c->draw0_obj ? 1u : 0u;
    fp.obj_xform = fp.vary_obj && c->draw0_xform ? 1u : 0u;
    fp.vin_base = fp.vary_obj ? (uint32_t)((int64_t)c->draw0.base_vertex + (int64_t)c->draw0.min_index) : 0u;
    fp.obj_ucol = TRI_UCOL && fp.vary_obj && c->draw0_ucol ? 1u : 0u;
    if (fp.obj_ucol) std::memcpy(fp.ucol, c->geom->ucol, sizeof fp.ucol);
    // object-space varyings for the other instantiations (the ONE frames keep vary_obj's 36-B records)
    // (not with the pre-pass over a transformed draw: the shadow instantiation carries no per-draw transform)
    fp.obj48 = (TRI_OBJ48 && !fp.vary36 && c->obj48 && !(c->shadow.size && c->obj48_xform)) ? 1u : 0u;
    fp.obj48_xform = fp.obj48 && c->obj48_xform ? 1u : 0u;
    // (with the pre-pass only under TRI_IDX_ROUTE_SHADOW: the shadow kernels carry the draw search only then)
    fp.idx_route = (TRI_IDX_ROUTE && c->idx_route && (!c->shadow.size || TRI_IDX_ROUTE_SHADOW)) ? 1u : 0u;
    if (fp.idx_route) {
        fp.idx_k = c->idx_k;
        std::memcpy(fp.pbase, c->pbase, sizeof fp.pbase);
        std::memcpy(fp.vbd, c->vbd, sizeof fp.vbd);
    }
    if (fp.obj48) std::memcpy(fp.vdelta, c->vdelta, sizeof fp.vdelta);  // (zero otherwise: world-space records
                                                                          // at the slots themselves)
    c->last_path = (fp.obj48 ? TRI_PATH_OBJ48 : 0u) | (fp.shade_solid ? TRI_PATH_ONE_DRAW : 0u) | (fp.vary_obj ? TRI_PATH_VARY_OBJ : 0u) |
                   (fp.obj_xform ? TRI_PATH_OBJ_XFORM : 0u) | (fp.obj_ucol ? TRI_PATH_OBJ_UCOL : 0u) |
                   (c->shadow.size ? TRI_PATH_SHADOW : 0u) | (fp.idx_route ? TRI_PATH_IDX_ROUTE : 0u);
    fp.ovf_rec_cap = c->ovf_rec_cap;
    fp.ovf_vert_cap = c->ovf_vert_cap;
    fp.bin_cap = c->bin_cap;
    fp.bone_count = c->nbones;
    fp.clear_bgra = c->clear_bgra;
    fp.write_depth = (c->cfg.flags & TRI_FLAG_NO_DEPTH_OUTPUT) ? 0u : 1u;
    fp.exact_shading = (c->cfg.flags & TRI_FLAG_EXACT_SHADING) ? 1u : 0u;
    fp.sky_size = c->sky_size;
    if (c->sky_size) {
        sky_constants(c->ubo, fp.sky_ip, fp.sky_R, fp.sky_pw);
        // the projection's centre is the view origin when its w row has no constant term
        const bool persp = fp.sky_pw[3] == 0.0f;
        fp.sky_mode = !persp ? TRI_SKY_RAY : (c->sky_uniform ? TRI_SKY_UNIFORM : TRI_SKY_PERSP);
        fp.sky_bgra = c->sky_uniform_bgra;
        fp.sky_lut = fp.sky_mode != TRI_SKY_UNIFORM || fp.exact_shading ? 1u : 0u;
        for (int r = 0; r < 4; ++r) {  // inverse(P) * (xn, yn, 1, 1), row r
            fp.sky_far[4 * r + 0] = fp.sky_ip[0 * 4 + r];
            fp.sky_far[4 * r + 1] = fp.sky_ip[1 * 4 + r];
            fp.sky_far[4 * r + 2] = fp.sky_ip[2 * 4 + r] + fp.sky_ip[3 * 4 + r];
        }
    }
    for (int t = 0; t < TRI_MAX_TEXTURE_SLOTS && !fp.need_lut; ++t)
        fp.need_lut = c->d_tex[t] && (c->tex_w[t] != 1 || c->tex_h[t] != 1);
    fp.cull_on = culling ? 1u : 0u;
    fp.cull_vertex = fp.cull_on && !c->shadow.size ? 1u : 0u;  // the pre-pass needs every caster
    fp.ncl_total = c->ncl_total;
    fp.setup_multi = fp.cull_on && fp.one_draw && !c->shadow.size ? 1u : 0u;
    if (fp.setup_multi) c->last_nchunks = (fp.nchunks + 3u) / 4u;  // the launch's statistics slots
    if (c->shadow.size) {
        fp.shadow_on = 1u;
        fp.s_size = c->shadow.size;
        fp.s_nbx = c->s_nbx;
        fp.s_nbins = c->s_nbins;
        fp.s_bin_cap = c->s_bin_cap;
        fp.s_hw = (float)c->shadow.size * 0.5f;
        fp.s_g = (2.0f * TRI_GUARD_BAND_PX) / (float)c->shadow.size - 1.0f;
        fp.s_bias = c->shadow.depth_bias;
        fp.s_slope = c->shadow.slope_bias;
        std::memcpy(fp.lvp, c->shadow.light_view_proj, 64);
    }
    std::memcpy(fp.pv, c->pv, 64);
    fp.ubo = c->ubo;
    fp.mat0 = c->mat0;
    shade_constants(c->ubo, c->mat0, fp.sc);
    if (fp.shade_solid) {  // (after shade_constants, which clears fp.sc)
        std::memcpy(fp.sc.solid, c->shade0.tex.solid, 16);
        std::memcpy(fp.sc.tint, c->shade0.tint, 16);
        for (int i = 0; i < 3; ++i) fp.sc.sbt[i] = (fp.sc.solid[i] * fp.sc.base[i]) * fp.sc.tint[i];
        fp.sc.sbt[3] = (fp.sc.base[3] * fp.sc.tint[3]) * fp.sc.solid[3];
        fp.sc.a8 = (uint32_t)(int)(std::fmin(std::fmax(fp.sc.sbt[3], 0.0f), 1.0f) * 255.0f + 0.5f);  // unorm8
        const float kd = fp.sc.kd;
        for (int i = 0; i < 3; ++i) {
            fp.sc.sbtm[i] = fp.sc.sbt[i] * fp.sc.metallic;
            fp.sc.sbtkd[i] = fp.sc.sbt[i] * kd;
            fp.sc.sbtamb[i] = (fp.sc.amb[i] * fp.sc.sbt[i]) * fp.sc.amb_strength;
        }
    }

    TriDeviceBuffers& b = ha.b;
    b.vin = c->geom->d_vin;
    b.vpos = c->geom->d_pos;
    b.vattr = c->geom->d_attr;
    b.vskin = c->any_skin ? c->geom->d_skin : nullptr;
    b.bones = c->d_bones;
    b.vertex_count = c->geom->nverts;
    b.indices = c->geom->d_idx;
    b.draws = c->d_draws;
    b.draw_shade = c->d_draw_shade;
    b.draw_vbase = c->d_vbase;
    b.draw_pbase = c->d_pbase;
    b.srgb_lut = c->d_lut;
    b.sky = c->d_sky;
    b.ai_frame = fp.ai_on ? c->d_ai : nullptr;
    b.clip = c->d_clip;
    b.snap = c->d_snap;
    b.oc = c->d_oc;
    b.vary = c->d_vary;
    b.recs = c->d_recs;
    b.clip_slot = c->d_clip_slot;
    b.prim_vs = c->d_prim_vs;
    b.setup_stats = c->d_setup_stats;
    b.bin_count = c->d_bin_count;
    b.bin_list = c->d_bin_list;
    b.counters = c->d_ctr;
    b.color = c->d_color;
    b.depth = c->d_depth;
    b.clusters = c->geom->d_clusters;
    b.vbox = c->geom->d_vbox;
    b.draw_cbase = c->d_cbase;
    b.cvis = c->d_cvis;
    b.lpos = c->d_lpos;
    b.lsnap = c->d_lsnap;
    b.sbin_count = c->d_sbin_count;
    b.sbin_list = c->d_sbin_list;
    b.shadow_map = c->d_shadow;

    hipEvent_t* ev = nullptr;
    TimingSet ts{};
    const bool timed = c->timing && (c->timing_counter++ % c->timing_period) == 0;
    if (timed) {
        if (!c->free_sets.empty()) {
            ts = c->free_sets.back();
            c->free_sets.pop_back();
        } else {
            for (auto& e : ts.ev) HIP_TRY(hipEventCreate(&e));
        }
        ev = ts.ev;
    }
    ts.shadow = fp.shadow_on != 0;
    TriFramePlan plan;
    tri_plan_frame(fp, plan);
#ifdef TRI_DIAG_FRONT
    if (c->diag_frames++ > 0) tri_diag_front_plan(plan);
#endif
    TRI_HSTAMP(3);
    HIP_TRY(tri_run_plan(plan, ha, c->d_args, c->stream, ev));
    c->launched = true;
    if (timed) c->pending.push_back(ts);
    if (fp.shadow_on) c->shadow_rendered = true;
#ifdef TRI_HOST_TIMING
    const auto hs4 = std::chrono::steady_clock::now();
    const std::chrono::steady_clock::time_point t[5] = {hs0, hs1, hs2, hs3, hs4};
    for (int i = 0; i < 4; ++i) g_host_ns[i] += (double)std::chrono::duration_cast<std::chrono::nanoseconds>(t[i + 1] - t[i]).count();
    g_host_ns[4] += (double)std::chrono::duration_cast<std::chrono::nanoseconds>(hs4 - hs0).count();
    ++g_host_calls;
#endif
    return TRI_OK;
}

int tri_synchronize(tri_ctx* c) {
    if (!c) return fail(TRI_E_INVALID, "tri_synchronize: null context");
    int rc = make_current(c);
    if (rc) return rc;
    // the counters ride the stream into pinned memory, so one wait covers the frame and its flags (a blocking
    // hipMemcpy after the wait cost the engine's per-frame fence another round trip)
    if (!c->h_ctr) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_ctr), sizeof(TriCounters), hipHostMallocDefault));
    HIP_TRY(hipMemcpyAsync(c->h_ctr, c->d_ctr, sizeof(TriCounters), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return check_overflow(c, c->h_ctr);
}

int tri_readback(tri_ctx* c, uint8_t* bgra, uint32_t* depth) {
    if (!c) return fail(TRI_E_INVALID, "tri_readback: null context");
    int rc = tri_synchronize(c);
    if (rc) return rc;
    const size_t px = (size_t)c->W * (size_t)(c->y1 - c->y0);
    if (bgra) HIP_TRY(hipMemcpy(bgra, c->d_color, px * 4, hipMemcpyDeviceToHost));
    if (depth) {
        if (c->cfg.flags & TRI_FLAG_NO_DEPTH_OUTPUT)
            return fail(TRI_E_STATE, "tri_readback: depth output disabled by TRI_FLAG_NO_DEPTH_OUTPUT");
        HIP_TRY(hipMemcpy(depth, c->d_depth, px * 4, hipMemcpyDeviceToHost));
    }
    return TRI_OK;
}

int tri_get_output(tri_ctx* c, tri_image* out) {
    if (!c || !out) return fail(TRI_E_INVALID, "tri_get_output: null argument");
    out->device_ptr = c->d_color;
    out->width = (uint32_t)c->W;
    out->height = (uint32_t)(c->y1 - c->y0);
    out->pitch_bytes = (uint32_t)c->W * 4u;
    out->format = TRI_FORMAT_B8G8R8A8_UNORM;
    out->device = c->device;
    out->reserved = 0;
    return TRI_OK;
}

int tri_blit_linear(tri_ctx* c, void* dst, uint32_t width, uint32_t height) {
    if (!c) return fail(TRI_E_INVALID, "tri_blit_linear: null context");
    if (width == 0 || height == 0 || width > TRI_MAX_DIM || height > TRI_MAX_DIM)
        return fail(TRI_E_INVALID, "tri_blit_linear: destination %ux%u outside 1..%d", width, height, TRI_MAX_DIM);
    if (c->y0 != 0 || c->y1 != c->H) return fail(TRI_E_STATE, "tri_blit_linear: a row-band context has no whole frame");
    int rc = make_current(c);
    if (rc) return rc;
    uint32_t* out = static_cast<uint32_t*>(dst);
    if (!out) {
        if ((size_t)width * height > c->cap_present) {
            HIP_TRY(hipStreamSynchronize(c->stream));
        }
        if ((rc = grow(c->d_present, c->cap_present, (size_t)width * height))) return rc;
        out = c->d_present;
        c->present_w = width;
        c->present_h = height;
    } else {
        c->present_w = c->present_h = 0;  // the owned target no longer holds the latest blit: read_present fails
    }
    // the alpha half of the decode LUT is the UNORM8 decode b / 255 (IEEE float division)
    HIP_TRY(tri_launch_blit(c->d_color, c->W, c->H, out, (int32_t)width, (int32_t)height, c->d_lut + 256, c->stream));
    return TRI_OK;
}

int tri_read_present(tri_ctx* c, uint8_t* bgra) {
    if (!c || !bgra) return fail(TRI_E_INVALID, "tri_read_present: null argument");
    if (!c->d_present || !c->present_w) return fail(TRI_E_STATE, "tri_read_present: nothing was blitted");
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(bgra, c->d_present, (size_t)c->present_w * c->present_h * 4, hipMemcpyDeviceToHost));
    return TRI_OK;
}

int tri_set_timing(tri_ctx* c, int enable) {
    if (!c) return fail(TRI_E_INVALID, "tri_set_timing: null context");
    int rc = collect_timing(c);
    if (rc) return rc;
    if (enable < 0) return fail(TRI_E_INVALID, "tri_set_timing: negative period %d", enable);
    c->timing = enable != 0;
    c->timing_period = enable > 0 ? (uint32_t)enable : 1u;
    c->timing_counter = 0;
    c->acc = tri_timing{};
    return TRI_OK;
}

int tri_get_timing(tri_ctx* c, tri_timing* out) {
    if (!c || !out) return fail(TRI_E_INVALID, "tri_get_timing: null argument");
    int rc = collect_timing(c);
    if (rc) return rc;
    *out = c->acc;
    return TRI_OK;
}

int tri_get_frame_stats(tri_ctx* c, tri_frame_stats* out) {
    if (!c || !out) return fail(TRI_E_INVALID, "tri_get_frame_stats: null argument");
    int rc = make_current(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    TriCounters h;
    HIP_TRY(hipMemcpy(&h, c->d_ctr, sizeof h, hipMemcpyDeviceToHost));
    std::memset(out, 0, sizeof *out);
    out->triangles_in = c->nprims;
    std::vector<uint2> ws(c->last_nchunks);
    if (!ws.empty()) HIP_TRY(hipMemcpy(ws.data(), c->d_setup_stats, ws.size() * sizeof(uint2), hipMemcpyDeviceToHost));
    uint64_t setup = h.tris_setup, entries = h.bin_entries;  // per-frame counters (0 unless a kernel adds)
    for (const uint2& w : ws) {
        setup += w.x;
        entries += w.y;
    }
    out->triangles_setup = setup;
    out->triangles_clipped = h.tris_clipped;
    out->bin_entries = entries;
    out->vertices_shaded = c->nslots;
    out->bins_x = (uint32_t)c->nbx;
    out->bins_y = (uint32_t)c->nby;
    out->bin_size = 1u << c->bin_log2;
    out->path = c->last_path;
    return TRI_OK;
}

}  // extern "C"
