// raster_common.h — device-side data layout shared by the HIP kernels and the C-ABI host code.
// HBM layout:
//   VsIn      48 B/vertex  {pos.xyz, uv.x}, {normal.xyz, uv.y}, {color.xyz, pad} (the 44 B of the 100-byte
//                          Trident Vertex that reach the output, Vertex.h:9-78, in the 48-B varying record's layout)
//   vpos      12 B/vertex  position stream, vattr 36 B/vertex {pos, normal, colour}: the same vertices split for
//                          vary_obj frames (k_vertex reads only vpos; the fragment stage gathers vattr records)
//   VsSkin    32 B/vertex  {bone indices, bone weights}, only when any draw has BoneCount > 0
//   clip      16 B/slot    float4 clip-space position per (draw, vertex) VS invocation; written only for
//                          vertices with an outcode on draws with clip_from_world (the clipper recomputes the rest)
//   snap      16 B/slot    {X (24-bit 8.8 fixed) | outcode << 24, Y, 1/w, z_ndc} (the fragment stage
//                          loads the first 12 bytes: it needs no depth)
//   vary      48 B/slot    {world.xyz, uv.x}, {normal.xyz, uv.y}, {color.xyz, 0} (VsIn's layout: obj48 frames read
//                          the object-space input records with the same code); 36 B/slot {world.xyz},
//                          {normal.xyz}, {color.xyz} on single-draw solid frames (TriFrameParams::vary36);
//                          none but the clipper's polygon vertices (object space, 36 B) with vary_obj
//   prim_vs   16 B/prim    {vertex slots 0..2, draw | clipped flag}, written by k_setup for the
//                          primitives it bins or clips on frames with several draws: k_raster's one-load
//                          route from a primitive id to its vertices and draw (instead of a draw search);
//                          a single-draw frame reads the 12 index bytes instead and writes none
//   bin_list   4 B/entry   primitive ids per bin (order-free: visibility is resolved by a 64-bit key)
//   TriRec    64 B/record  clipped sub-triangles only: snapped vertices, z, 1/w, prim<<3|sub, slots
//   colour     4 B/pixel   B8G8R8A8_UNORM;  depth 4 B/pixel D32_SFLOAT bits
#pragma once

#include <stdint.h>
#include "../../include/tri_raster.h"

#define TRI_BIN_LOG2 6
#define TRI_BIN (1 << TRI_BIN_LOG2)
#define TRI_BLOCK 256
#define TRI_PRIM_MAX ((1u << 29) - 1u)
// bin-queue entry: a primitive id, or TRI_ENTRY_CLIPPED | index of a clipped sub-triangle's record
#define TRI_ENTRY_CLIPPED 0x80000000u
// prim_vs[p].w flag: primitive p was clipped (its fragments come from TriRec sub-triangles)
#define TRI_PRIM_CLIPPED 0x80000000u
#define TRI_MAX_CLIP_VERTS 12
// Clipping a triangle by 6 planes yields at most 3 + 6 = 9 vertices; a numerically non-convex
// polygon can come out longer and is cut to its first 9 (oracle clip_polygon does the same). The fan
// then has at most 7 sub-triangles k = 1..7, stored in the 3-bit `sub` field of a visibility key as k
// (sub = 0: the primitive was not clipped). The background key has depth bits just above 1.0, which no
// fragment reaches (the [0, 1] clamp), so it never equals a fragment's key.
#define TRI_MAX_CLIP_POLY 9
static_assert(TRI_MAX_CLIP_POLY - 2 <= 7, "clipped sub-triangle number k = 1..nsub must fit 3 bits");
static_assert(TRI_MAX_CLIP_POLY <= TRI_MAX_CLIP_VERTS, "clip polygon buffers");
#define TRI_WMIN 1e-5f
#define TRI_GUARD_BAND_PX 16000.0f
#ifndef TRI_MAX_PPT
#define TRI_MAX_PPT 16  // primitives per k_setup thread
#endif
#define TRI_OBJ48_DRAWS 16  // draws a frame may hold for object-space varyings outside the ONE instantiation

#ifndef TRI_SNAP_F
#define TRI_SNAP_F 1
#endif

#define TRI_SKY_RAY 0u
#define TRI_SKY_PERSP 1u
#define TRI_SKY_UNIFORM 2u

// overflow flag bits (TriCounters.flags)
#define TRI_OVF_CLIP_RECORDS 0x1u
#define TRI_OVF_CLIP_VERTS 0x2u
#define TRI_OVF_BIN_LIST 0x4u
#define TRI_OVF_SHADOW_BIN_LIST 0x8u

struct __attribute__((aligned(16))) TriVsIn {
    float px, py, pz, u;
    float nx, ny, nz, v;
    float cr, cg, cb, pad;
};

struct __attribute__((aligned(16))) TriVsSkin {
    int32_t idx[4];
    float w[4];
};

// Per-vertex window-space record written by k_vertex (the perspective divide + viewport transform
// + 8-bit snap are done once per vertex): X (signed 24 bits) | outcode << 24, Y, 1/w, z_ndc. With TRI_SNAP_F
// (the main pass; the shadow map's lsnap keeps the packed form) X and Y are stored as floats — they are
// integers below 2^22 in magnitude, so exactly — and the outcode goes to its own byte per slot: the fragment
// stage's weights then start from float differences (no per-pixel sign extension and conversions).
struct __attribute__((aligned(16))) TriSnap {
    int32_t xo;
    int32_t y;
    float iw;
    float z;
};
// outcode bits: one per Vulkan clip half-space a vertex is outside of, + "needs geometric clip"
#define TRI_OC_ZNEG 0x01u   /* z < 0     */
#define TRI_OC_ZFAR 0x02u   /* z > w     */
#define TRI_OC_XNEG 0x04u   /* x < -w    */
#define TRI_OC_XPOS 0x08u   /* x > w     */
#define TRI_OC_YNEG 0x10u   /* y < -w    */
#define TRI_OC_YPOS 0x20u   /* y > w     */
#define TRI_OC_CLIP 0x40u   /* w < WMIN, z < 0 or outside the guard band */
#define TRI_OC_BAD 0x80u    /* vertex index out of range */
#define TRI_OC_REJECT 0x3Fu

struct __attribute__((aligned(16))) TriRec {
    int32_t X[3];
    int32_t Y[3];
    float z[3];
    float iw[3];
    uint32_t prim_sub;  // prim << 3 | sub (sub = fan index of a clipped sub-triangle)
    uint32_t v[3];      // vary slots (post orientation swap)
};
// A set-up triangle. Unclipped triangles are rebuilt in registers from their snapped vertices
// wherever they are needed; only clipped sub-triangles are stored (TriDeviceBuffers::recs).
static_assert(sizeof(TriRec) == 64, "TriRec must be one 64-byte line");

// Per-draw vertex-stage constants (push constant + hoisted normal matrix).
struct __attribute__((aligned(16))) TriDrawDev {
    float model[16];
    float nm[9];         // transpose(inverse(mat3(model))), glm cofactor form, computed on the host
    float tex_scale[2];
    float tex_offset[2];
    float tiling;
    int32_t bone_offset;
    int32_t bone_count;
    int32_t first_index;
    int32_t base_vertex;
    uint32_t min_index;
    uint32_t vert_count; // VS invocations for this draw (max-min+1), 0 = inactive
    uint32_t cl_first;   // the mesh's first cluster (TriCluster) and first vertex-block interval
    uint32_t vblk_first;
    uint32_t ncl;        // the mesh's cluster count (0 for an inactive draw)
    // 1: unskinned with an affine model matrix (last row 0, 0, 0, 1), so world.w == 1 for every finite
    // vertex and its clip position is pv * (world.xyz, 1): k_vertex stores clip only for vertices with an
    // outcode, k_setup's clipper recomputes the others from the world position in `vary`
    uint32_t clip_from_world;
};
static_assert(sizeof(TriDrawDev) == 160, "TriDrawDev: 40 words");

// Cluster culling (row bands): a mesh's primitives in runs of TRI_CLUSTER_PRIMS, each with the object-
// space box of the vertices it references and their mesh-local index range, computed once at upload.
// Per frame the k_vertex waves mark the (draw, cluster) pairs whose projected box can reach the rows;
// k_setup skips primitives of unmarked clusters before their index fetch, and k_vertex skips each 256-
// slot vertex block none of whose referencing clusters is marked (TriVertexBlock interval).
#define TRI_CLUSTER_PRIMS 512
#define TRI_VBLOCK 256
struct __attribute__((aligned(16))) TriCluster {
    float lo[3];
    uint32_t vmin;  // mesh-local index range of every referenced vertex (valid or not)
    float hi[3];    // box of the valid referenced vertices; lo > hi: none is valid
    uint32_t vmax;
};

struct __attribute__((aligned(16))) TriTexDesc {
    const uint32_t* texels;  // RGBA8 sRGB, row-major
    uint32_t w, h;
    float solid[4];          // 1x1 textures: the decoded texel (every bilinear tap is that texel)
};

// Per-draw fragment-stage constants: the push constant's tint and the descriptor of the draw's texture
// slot (unused slots alias slot 0), copied in on the host so a fragment reads its texture after one
// load that depends only on the draw, not after a second, dependent descriptor load.
struct __attribute__((aligned(16))) TriDrawShade {
    float tint[4];
    TriTexDesc tex;
};
static_assert(sizeof(TriDrawShade) == 48, "TriDrawShade: tint + texture descriptor");

struct TriCounters {  // per-frame fields are zeroed before every frame; `flags`/`bin_max` are sticky
    uint32_t ovf_records;
    uint32_t ovf_verts;
    uint32_t tris_setup;
    uint32_t tris_clipped;
    uint32_t bin_entries;
    uint32_t sbin_max;  // largest shadow-map bin entry count seen (sticky, like bin_max)
    uint32_t bin_max;  // largest per-bin entry count seen (sizes the bin queues after an overflow)
    uint32_t flags;
};

// Frame constants of Default.frag hoisted on the host (fast shading path).
struct TriShadeConst {
    float cam[4];
    float base[4];        // MaterialUniformBuffer[0].BaseColorFactor
    float metallic, roughness, amb_strength;
    float om;             // the fast build's 0.04 (1 - metallic), F0's dielectric term
    float amb[4];         // AmbientColorIntensity.rgb * .w
    uint32_t has_sun, npt;
    uint32_t a8;          // ONE frames: the fragment alpha sbt[3] as its UNORM8 byte (uniform)
    float kd;             // (1 - metallic) / pi, the diffuse factor
    float sun_l[4];       // normalize(-DirectionalLightDirection)
    float sun_rad[4];     // DirectionalLightColor.rgb * .w
    // per point light, position and radiance side by side: the light loop reads one 32-B record per light
    // (one scalar load and one wait instead of two)
    struct {
        float pos[4];  // xyz, 1/max(radius, 1e-4)
        float rad[4];  // ColorIntensity.rgb * .w
    } pl[TRI_MAX_POINT_LIGHTS];
    // roughness terms of the fast BRDF: a2 - 1, a2 / pi, Schlick-GGX k and 1 - k (a = roughness^2)
    float a2m1, a2pi, kg, omkg;
    // single-draw frames whose texture slot is 1x1 (TriFrameParams::shade_solid): the draw's decoded texel
    // and tint, so no fragment gathers its shade record
    float solid[4], tint[4];
    // and the fast build's uniform albedo factor of such a draw: ((solid * base) * tint).rgb and the
    // fragment alpha (base.a * tint.a) * solid.a, in Default.frag's order of operations
    float sbt[4];
    // G_L's denominator divided through by 1 - k (the fast build's per-light v_fma becomes one add):
    // k / (1 - k) and a2 / pi / (1 - k), so NDF * G_L * G_V keeps its value
    // and spec_num's uniform factors 0.25 a2pio (spA / rgV) and 1e4 a2pio (spB / (NdotV rgV)); the host folds every
    // frame constant the fragment stage would otherwise form per pixel from scalars (no SALU float ops on gfx950)
    float kgo, a2pio, spAk, spBk;
    // the fast build's ONE frames (sbt uniform): albedo = sbt * vertex colour is never formed; F0, the diffuse
    // factor and the ambient term come straight from the colour with these folded factors: sbt * metallic,
    // sbt * (1 - metallic) / pi and (ambient * sbt) * ambient strength
    float sbtm[4], sbtkd[4], sbtamb[4];
};

struct TriFrameParams {
    int32_t W, H, y0, y1;
    int32_t nbx, nby, nbins, ppt;
    int32_t bin_log2;
    uint32_t sky_lut;   // the skybox pass samples the cubemap: workgroups with sky pixels stage the sRGB LUT
    uint32_t chunk_stride;  // k_setup visits chunks in the order (blockIdx * stride) mod nchunks
    uint32_t shade_solid;   // one draw with a 1x1 texture slot: sc.solid / sc.tint replace its shade record
    float hw, hh, gx, gy;
    uint32_t nprims, nslots, ndraws, nchunks;
    uint32_t ovf_rec_cap, ovf_vert_cap, bin_cap, bone_count;
    uint32_t clear_bgra;
    uint32_t write_depth;
    uint32_t exact_shading;
    uint32_t sky_size;  // skybox face size (0 = no skybox pass)
    // Skybox evaluation mode (fast build; the exact build always uses the oracle's ray/cube path):
    //  TRI_SKY_RAY     unproject both clip planes, intersect the 20-unit cube (oracle sky_pixel)
    //  TRI_SKY_PERSP   the projection's centre is the view origin (w row has no constant term), so
    //                  every ray leaves the eye-centred cube and the sampled direction is the far
    //                  point's homogeneous xyz: 3 dot products per pixel
    //  TRI_SKY_UNIFORM TRI_SKY_PERSP over a cubemap whose texels are all equal: LINEAR filtering of
    //                  equal taps returns that texel, so the sky is the constant sky_bgra
    uint32_t sky_mode;
    uint32_t sky_bgra;
    uint32_t need_lut;  // some texture larger than 1x1: every k_raster workgroup stages the sRGB LUT
    uint32_t one_draw;  // exactly one draw: draw0 / vbase0 / pbase0 carry it (kernel arguments, scalar loads)
    float sky_far[16];  // inverse(Projection) applied to (xn, yn, 1, 1): rows {x, y, z, w} as (a, b, c, 0)
    float pv[16];
    float sky_ip[16];   // inverse(Projection) (double on the host, rounded)
    float sky_R[9];     // mat3(View)
    float sky_pw[4];    // Projection row 3
    tri_global_ubo ubo;
    tri_material_record mat0;
    TriShadeConst sc;
    TriDrawDev draw0;  // the draw when one_draw (its vertex and primitive slots start at 0)
    // cluster culling (row bands): k_vertex marks ncl_total (draw, cluster) pairs; cull_vertex also lets
    // k_vertex skip vertex blocks (off while the shadow pre-pass needs every caster); setup_multi: k_setup
    // runs a quarter of the chunks' workgroups, four strided chunks each (single-draw bands, no pre-pass)
    uint32_t cull_on, cull_vertex, ncl_total, setup_multi;
    // vary36: single-draw solid frames without the pre-pass (k_raster_plain's ONE instantiation) store 36-B
    // varyings {world.xyz, N.xyz, colour.xyz} — no texture coordinates, which nothing samples — instead of 48 B.
    // vary_obj (such frames whose draw is affine, unskinned, with a conformal normal matrix, over unit object
    // normals): k_vertex writes no varyings at all; the fragment stage gathers the object-space position,
    // normal and colour from the 36-B object records (vattr + vin_base) and, when obj_xform, carries the interpolated
    // position and normal through the model and normal matrices (linear maps: the same values up to
    // rounding); the clipper writes object-space 36-B records for its polygon vertices.
    uint32_t vary36, vary_obj, obj_xform, vin_base;
    // obj_ucol (vary_obj frames whose vertices all carry one colour, ucol — meshes without vertex colours are
    // imported white): the fragment stage takes the colour from here instead of three gathers and an interpolation
    uint32_t obj_ucol;
    float ucol[3];
    // obj48 (frames outside the ONE instantiation — several draws, textures, the shadow pre-pass — whose every
    // active draw is affine, unskinned, with a conformal normal matrix and an identity texture transform, over unit
    // object normals, at most TRI_OBJ48_DRAWS draws): object-space varyings as well. k_vertex writes no varyings; the
    // fragment stage gathers each vertex's 48-B input record {pos, n.x}{n.yz, colour.rg}{colour.b, uv} (TriVsIn,
    // uploaded with the geometry) at slot + vdelta[draw] and, when obj48_xform (some draw has a non-identity model),
    // carries the interpolated position and normal through its draw's model and normal matrices; the clipper writes
    // its polygon vertices' records in the same layout.
    uint32_t obj48, obj48_xform;
    uint32_t vdelta[TRI_OBJ48_DRAWS];  // per draw: base_vertex + min_index - first slot (mod 2^32)
    // shadow-map pre-pass (tri_set_shadow): s_size x s_size map, 32x32 bins
    // Default.frag's AI frame blend (:182-191): on when AiBlendConfig.w > 0 and clamp(AiBlendConfig.x, 0, 1) > 0 (that
    // clamped weight is ai_wgt); the frame texture is ai_tw x ai_th RGBA8 UNORM (TriDeviceBuffers::ai_frame), sampled at
    // gl_FragCoord.xy * (ai_sx, ai_sy) = AiBlendConfig.yz
    uint32_t ai_on, ai_tw, ai_th;
    float ai_wgt, ai_sx, ai_sy;
    uint32_t shadow_on, s_size, s_nbx, s_nbins;
    uint32_t s_bin_cap;
    float s_hw;    // s_size / 2 (light NDC -> texel, the main pass's viewport transform)
    float s_g;     // guard band in light NDC: 2 * TRI_GUARD_BAND_PX / s_size - 1
    float s_bias;  // depth bias of the lookup compare
    float s_slope; // slope-scaled depth bias of the depth pass
    float lvp[16]; // light ortho * light view (affine)
    // idx_route (frames of 2..TRI_OBJ48_DRAWS draws whose index rows follow their primitive numbers: first_index =
    // idx_k + 3 * first primitive for every active draw, as meshes concatenated in draw order are): a primitive p's
    // vertex slots are its index triple at idx_k + 3 p plus its draw's slot offset vbd[d] (d: the last draw whose
    // first primitive pbase[d] <= p), as on single-draw frames, so k_setup writes no 16-B prim_vs record per
    // primitive and the fragment stage gathers 12 index bytes instead of it (C5: 16 MB of set-up writes per frame)
    uint32_t idx_route, idx_k;
    uint32_t pbase[TRI_OBJ48_DRAWS], vbd[TRI_OBJ48_DRAWS];
};
