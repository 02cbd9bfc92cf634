// raster_kernels.hip — hand-written gfx950 (CDNA4) kernels for Trident's graphics-pipeline stage.
//
//   k_vertex   vs_transform   Default.vert:60-105, one lane per (draw, referenced vertex)
//   k_setup    tri_setup_bin  primitive assembly + trivial reject + cull + bbox on the per-vertex
//                             snapped coordinates (Pipeline.cpp:611-643), binned into per-bin queues
//                             (wave-aggregated atomics: one per (wave, bin)); nothing else is stored
//                             per triangle. Triangles that need homogeneous clipping (rare) are
//                             clipped by their wave in place: Sutherland-Hodgman against w>=WMIN,
//                             z>=0 and the guard band + fan, one primitive per wave at a time
//   k_raster   tile_raster_shade: one workgroup per 32x32 (or 64x64) bin; coverage + early-Z in LDS
//              with 64-bit (depth, primitive-order) keys (== in-order LESS_OR_EQUAL,
//              Pipeline.cpp:655-658), then Default.frag:123-192 once per visible pixel, coalesced
//              B8G8R8A8 + D32 stores.
//
// Raster rules (shared with oracle/tri_oracle.cpp) are reproduced with the same
// float evaluation order; the file is compiled with -ffp-contract=off so depth is bit-exact. The
// fragment stage has two builds: EXACT (IEEE div/sqrt/powf, the oracle's operation order) and the
// default fast build (v_rcp/v_rsq/v_exp/v_log, hoisted frame constants), both within 1 LSB of the
// oracle's UNORM8 output.
#define TRI_KERNEL_TU 1  // device pointers in TriDeviceBuffers carry the global address space (raster_launch.h)
// This file is compiled three times: raster_plain.hip (TRI_RASTER_PLAIN_TU: k_raster_plain), vertex_stage.hip
// (TRI_VERTEX_TU: k_reset, k_vertex, k_vertex_band) and on its own (everything else, and the frame plan).
#if defined(TRI_RASTER_PLAIN_TU) || defined(TRI_VERTEX_TU)
#define TRI_MAIN_TU 0
#else
#define TRI_MAIN_TU 1
#endif
#include "raster_launch.h"

#include <hip/hip_runtime.h>
#include <math.h>

#include <type_traits>

namespace {

// Diagnostics builds only (tools/build_variant.sh NAME -DTRI_ABLATE=N): 1 = coverage without shading,
// 2 = shading without coverage, 4 = set-up without binning, 8 = one reservation round per batch,
// 16 = no reservation atomics, 32 = no queue stores, 64 = no lights, 128 = no texture sample, 256 = no varyings
// fetch, 1024 = no fragment colour gathers, 2048 = no shadow lookup (and the fast weights). The shipped library is
// built with 0, so none of these tests survives into its ISA.
#ifndef TRI_ABLATE
#define TRI_ABLATE 0
#endif
constexpr uint32_t kAblate = TRI_ABLATE;

// Diagnostics builds only (-DTRI_PHASE_TIMING): k_raster's wave 0 of every workgroup stamps s_memtime at
// its phase boundaries (start, init, coverage, large triangles, shading, end) for tools/phase_times.py.
// Diagnostics builds only (-DTRI_PRIM_GROUPS): the shading loop counts, per wave-iteration, the distinct primitives
// among its shaded lanes (tools/prim_groups.py): {iterations, distinct primitives, shaded lanes}.
#ifdef TRI_PRIM_GROUPS
__device__ unsigned long long g_tri_groups[3];
#endif
#ifdef TRI_PHASE_TIMING
constexpr int kPhaseSlots = 65536;
__device__ unsigned long long g_tri_phase[kPhaseSlots][6];
#define TRI_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < kPhaseSlots) g_tri_phase[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); } while (0)
// k_setup: start, primitives of the first round set up, first round binned, end
__device__ unsigned long long g_tri_setup_phase[kPhaseSlots][4];
#define TRI_SSTAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < kPhaseSlots) g_tri_setup_phase[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define TRI_STAMP(k) do { } while (0)
#define TRI_SSTAMP(k) do { } while (0)
#endif

// Launch arguments (raster_launch.h): the frame's first kernel takes TriLaunchArgs by value and publishes it
// (TRI_FIRST_KARGS / TRI_PUBLISH_ARGS); the later kernels read the published copy through a read-only,
// non-aliased pointer (TRI_KARGS / TRI_BIND_ARGS: scalar loads).
#define TRI_FIRST_KARGS TriLaunchArgs a_, TriLaunchArgs* __restrict__ pub_
#define TRI_BIND_FIRST_ARGS                   \
    const TriFrameParams& fp = a_.fp;         \
    const TriDeviceBuffers& b = a_.b
#define TRI_KARGS const TriLaunchArgs* __restrict__ args_
#define TRI_BIND_ARGS                         \
    const TriFrameParams& fp = args_->fp;     \
    const TriDeviceBuffers& b = args_->b
// Workgroup 0 of the first kernel copies its by-value arguments to the device copy, 16 B per lane.
__device__ __forceinline__ void publish_args(const TriLaunchArgs& a, TriLaunchArgs* dst) {
    if (blockIdx.x != 0) return;
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4* src = reinterpret_cast<const u4*>(&a);
    u4* d = reinterpret_cast<u4*>(dst);
    for (uint32_t i = threadIdx.x; i < sizeof(TriLaunchArgs) / 16; i += blockDim.x) d[i] = src[i];
}

constexpr uint64_t kBgKey = 0x3F800001ull << 32;  // above every fragment key (depth bits <= 1.0 after the clamp)
constexpr float kPi = 3.14159265359f;                                  // Default.frag:65

struct VsOut {
    float4 clip;
    float wx, wy, wz;
    float nx, ny, nz;
    float u, v;
    float cr, cg, cb;
};

constexpr int kLdsDraws = 64;  // k_setup stages up to this many draws' lookup data in LDS

__device__ __forceinline__ int find_range_lds(const uint32_t* base, int n, uint32_t x) {  // base in LDS
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (base[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ int find_range(const uint32_t* base, int n, uint32_t x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (base[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Raw buffer loads for k_raster's per-fragment gathers: a wave-uniform descriptor built from kernel
// arguments (SGPRs) and a 32-bit byte offset per lane, so a 16-byte record is ONE load instruction
// with no 64-bit address arithmetic (the compiler splits a plain struct load into per-field loads
// when fields are used on different paths, and serialises the prim_vs -> vertex chain on it).
// The host keeps every buffer read this way below 4 GiB (ensure_work_buffers).
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(uint32_t)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 ld128(Rsrc r, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
// Record gathers by index (TRI_IDXEN): a structured buffer resource carries the record stride, so a load names
// its record by index (buffer_load ... idxen) and the texture unit forms index * stride + offset; no VALU
// multiply per address (the per-pixel gathers of k_raster otherwise spend seven quarter-rate v_mul_lo_u32 on
// their x12 / x48 offsets). The LLVM intrinsic is bound by name: the compiler sees an ordinary buffer load.
#ifndef TRI_IDXEN
#define TRI_IDXEN 1
#endif
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3v __attribute__((ext_vector_type(3)));
__device__ u32x4v tri_sbuf_load_b128(Rsrc r, int vindex, int voffset, int soffset, int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");
__device__ u32x3v tri_sbuf_load_b96(Rsrc r, int vindex, int voffset, int soffset, int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v3i32");
// A buffer of `n` records of `stride` bytes (stride < 2^14): indexed loads when TRI_IDXEN, else byte offsets.
struct RecBuf {
    Rsrc r;
};
__device__ __forceinline__ RecBuf rec_buf(const void* p, uint32_t stride, uint64_t n) {
    if (TRI_IDXEN) return RecBuf{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)stride, (int)(uint32_t)n, 0x00020000)};
    return RecBuf{make_rsrc(p, (uint64_t)stride * n)};
}
template <uint32_t STRIDE>
__device__ __forceinline__ uint4 rec128(const RecBuf& b, uint32_t i, uint32_t off) {  // off: a constant < STRIDE
    if (TRI_IDXEN) {
        const u32x4v v = tri_sbuf_load_b128(b.r, (int)i, (int)off, 0, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
    }
    return ld128(b.r, i * STRIDE + off);
}
template <uint32_t STRIDE>
__device__ __forceinline__ u32x3v rec96(const RecBuf& b, uint32_t i, uint32_t off) {
    if (TRI_IDXEN) return tri_sbuf_load_b96(b.r, (int)i, (int)off, 0, 0);
    const auto q = __builtin_amdgcn_raw_buffer_load_b96(b.r, i * STRIDE + off, 0, 0);
    return u32x3v{q[0], q[1], q[2]};
}

// k_raster's gather sources: 16-B snaps, varyings, 48-B shade records. `src` holds an unclipped primitive's
// vertex attributes: the varyings, or with vary_obj the draw's own 36-B object-space records (vattr).
struct FetchBufs {
    RecBuf snap, vary, src, shade;
    const void* shade_base;  // the shade records for scalar loads (load_shade)
    uint32_t shade_bytes;
};
// The varying record: 48 B {world, u}{N, v}{colour, 0}, or 36 B {world}{N}{colour} on single-draw solid frames
// (TriFrameParams::vary36 — exactly the frames k_raster_plain<.., ONE> shades). TRI_VARY36 = 0 keeps 48 B.
// TRI_VARY_OBJ = 0 keeps world-space varyings on every frame (TriFrameParams::vary_obj).
#ifndef TRI_VARY36
#define TRI_VARY36 1
#endif
#ifndef TRI_VARY_OBJ
#define TRI_VARY_OBJ 1
#endif
__device__ __forceinline__ bool vary36_mode(const TriFrameParams& fp) { return TRI_VARY36 && fp.vary36; }
__device__ __forceinline__ bool obj_mode(const TriFrameParams& fp) { return TRI_VARY36 && TRI_VARY_OBJ && fp.vary_obj; }
struct F3 {
    float x, y, z;
};
__device__ __forceinline__ F3 ldF3(TRI_G const F3* p) { return F3{p->x, p->y, p->z}; }
__device__ __forceinline__ bool obj48_mode(const TriFrameParams& fp) { return TRI_OBJ48 && fp.obj48; }
// Attribute j (0 position, 1 normal, 2 colour) of geometry vertex gv's 36-B object record
__device__ __forceinline__ F3 vattr_at(const TriDeviceBuffers& b, uint32_t gv, int j) {
    TRI_G const float* q = b.vattr + 9u * gv + 3 * j;
    return F3{q[0], q[1], q[2]};
}
// ... of vertex record vin_base + slot, object space (vary_obj)
__device__ __forceinline__ F3 vin_attr(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t slot, int j) {
    return vattr_at(b, fp.vin_base + slot, j);
}
// obj48: the offset from draw d's vertex slots to its geometry vertices; a wave whose lanes share the draw (the
// common case) reads it with one scalar load
__device__ __forceinline__ uint32_t obj_delta(const TriFrameParams& fp, uint32_t d) {
    d = min(d, (uint32_t)TRI_OBJ48_DRAWS - 1u);
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
    if (__ballot(d != d0) == 0ull) return fp.vdelta[d0];
    return fp.vdelta[d];
}
template <bool ONE = false>
__device__ __forceinline__ FetchBufs fetch_bufs(const TriFrameParams& fp, const TriDeviceBuffers& b) {
    FetchBufs f;
    f.snap = rec_buf(b.snap, 16u, fp.nslots);
    f.vary = rec_buf(b.vary, (ONE && TRI_VARY36) ? 36u : 48u, (uint64_t)fp.nslots + fp.ovf_vert_cap);
    f.src = f.vary;
    if (ONE && obj_mode(fp)) f.src = rec_buf(b.vattr + 9u * fp.vin_base, 36u, fp.nslots);
    // obj48: an unclipped primitive's vertices are its geometry's own 48-B input records (index slot + vdelta)
    if (!ONE && obj48_mode(fp)) f.src = rec_buf(b.vin, 48u, b.vertex_count);
    f.shade = rec_buf(b.draw_shade, (uint32_t)sizeof(TriDrawShade), fp.ndraws);
    f.shade_base = (const void*)b.draw_shade;
    f.shade_bytes = (uint32_t)sizeof(TriDrawShade) * fp.ndraws;
    return f;
}
__device__ __forceinline__ TriSnap ld_snap(const FetchBufs& fb, uint32_t slot) {
    const uint4 q = rec128<16>(fb.snap, slot, 0u);
    return TriSnap{(int32_t)q.x, (int32_t)q.y, __uint_as_float(q.z), __uint_as_float(q.w)};
}
// The fragment stage's view of a snapped vertex: X, Y and 1/w (12 bytes, one load; z is not needed).
__device__ __forceinline__ TriSnap ld_snap_xyw(const FetchBufs& fb, uint32_t slot) {
    const u32x3v q = rec96<16>(fb.snap, slot, 0u);
    return TriSnap{(int32_t)q[0], (int32_t)q[1], __uint_as_float(q[2]), 0.0f};
}

// The main pass's snapped vertex fields (TRI_SNAP_F: exact floats + a separate outcode byte).
__device__ __forceinline__ int32_t snap_X(const TriSnap& s) {
    return TRI_SNAP_F ? (int32_t)__int_as_float(s.xo) : (s.xo << 8) >> 8;
}
__device__ __forceinline__ int32_t snap_Y(const TriSnap& s) { return TRI_SNAP_F ? (int32_t)__int_as_float(s.y) : s.y; }
__device__ __forceinline__ float snap_Xf(const TriSnap& s) { return TRI_SNAP_F ? __int_as_float(s.xo) : (float)snap_X(s); }
__device__ __forceinline__ float snap_Yf(const TriSnap& s) { return TRI_SNAP_F ? __int_as_float(s.y) : (float)s.y; }
// k_setup's gathers of a primitive's indices, snapped vertices and outcodes as buffer loads from wave-uniform
// descriptors (TRI_SETUP_RSRC): a record index per lane, no 64-bit address arithmetic, one 12-B index load.
#ifndef TRI_SETUP_RSRC
#define TRI_SETUP_RSRC 1
#endif
struct SetupBufs {
    RecBuf snap;
    Rsrc oc;
};
__device__ __forceinline__ TriSnap setup_snap(const SetupBufs& sb, const TriDeviceBuffers& b, uint32_t slot) {
    if (!TRI_SETUP_RSRC) return b.snap[slot];
    const uint4 q = rec128<16>(sb.snap, slot, 0u);
    return TriSnap{(int32_t)q.x, (int32_t)q.y, __uint_as_float(q.z), __uint_as_float(q.w)};
}
__device__ __forceinline__ uint32_t setup_oc(const SetupBufs& sb, const TriDeviceBuffers& b, const TriSnap& s,
                                             uint32_t slot) {
    if (!TRI_SNAP_F) return (uint32_t)s.xo >> 24;
    if (!TRI_SETUP_RSRC) return (uint32_t)b.oc[slot];
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(sb.oc, slot, 0, 0);
}
__device__ __forceinline__ uint32_t snap_oc(const TriDeviceBuffers& b, const TriSnap& s, uint32_t slot) {
    return TRI_SNAP_F ? (uint32_t)b.oc[slot] : (uint32_t)s.xo >> 24;
}

// ((c0*x + c1*y) + c2*z) + c3*w, column-major, no FMA (matches the oracle bit-for-bit)
__device__ __forceinline__ float4 mat_vec_seq(const float* m, float4 v) {
    float4 r;
    r.x = ((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * v.w;
    r.y = ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * v.w;
    r.z = ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * v.w;
    r.w = ((m[3] * v.x + m[7] * v.y) + m[11] * v.z) + m[15] * v.w;
    return r;
}

// IEEE a / b for several numerators over one denominator. This is the compiler's own f32 division
// sequence (v_rcp, one Newton step on the reciprocal, two FMA corrections of the quotient: LLVM's
// LowerFDIV32) without its v_div_scale / v_div_fixup range handling, which changes nothing for finite
// normal operands whose exponents are far from the format's limits -- exact integers below 2^48, their
// ratios, depth differences and perspective weights. The refined reciprocal is computed once per
// denominator, so each further quotient costs a multiply and four FMAs instead of a full division, with
// the same bits.
struct RcpRef {
    float b, y;
};
__device__ __forceinline__ RcpRef rcp_ref(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return RcpRef{b, __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0)};
}
__device__ __forceinline__ float div_rn(float a, const RcpRef& r) {
    const float q0 = a * r.y;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-r.b, q0, a), r.y, q0);
    return __builtin_fmaf(__builtin_fmaf(-r.b, q1, a), r.y, q1);
}

// ------------------------------------------------------------------------------------------
// vs_transform
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void snap_compute(const TriFrameParams& fp, float4 c, int32_t& X, int32_t& Y, float& z,
                                             float& iw);
__device__ __forceinline__ uint32_t outcode(const TriFrameParams& fp, float4 c);

// Shadow pre-pass, per vertex slot: the light-NDC position (light_view_proj is affine, so w = 1 and the
// main pass's perspective divide is the identity), kept for the fragment lookup, and its snap to the
// s_size x s_size map (oracle shadow_raster_triangle: X = rint((x * S/2 + S/2) * 256)) with outcode
// bits for the map's four sides and TRI_OC_CLIP beyond the guard band (such casters are dropped).
__device__ __forceinline__ void shadow_vertex(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t slot,
                                              float4 world) {
    const float4 l = mat_vec_seq(fp.lvp, world);
    b.lpos[slot] = make_float4(l.x, l.y, l.z, 0.0f);
    uint32_t oc = 0;
    if (l.x + 1.0f < 0.0f) oc |= TRI_OC_XNEG;
    if (1.0f - l.x < 0.0f) oc |= TRI_OC_XPOS;
    if (l.y + 1.0f < 0.0f) oc |= TRI_OC_YNEG;
    if (1.0f - l.y < 0.0f) oc |= TRI_OC_YPOS;
    if (l.x < -fp.s_g || l.x > fp.s_g || l.y < -fp.s_g || l.y > fp.s_g) oc |= TRI_OC_CLIP;
    TriSnap sn{(int32_t)(oc << 24), 0, 1.0f, l.z};
    if (!(oc & TRI_OC_CLIP)) {
        const int32_t X = (int32_t)rintf((l.x * fp.s_hw + fp.s_hw) * 256.0f);
        sn.xo = (X & 0x00FFFFFF) | (int32_t)(oc << 24);
        sn.y = (int32_t)rintf((l.y * fp.s_hw + fp.s_hw) * 256.0f);
    }
    b.lsnap[slot] = sn;
}

// Lanes of mask m below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void reset_counters(TriCounters* c) {
    c->ovf_records = 0; c->ovf_verts = 0; c->tris_setup = 0; c->tris_clipped = 0;
    c->bin_entries = 0;  // `flags` / `bin_max` are sticky (cleared by the host)
}

#ifdef TRI_VERTEX_TU
__global__ __launch_bounds__(TRI_BLOCK) void k_reset(TRI_FIRST_KARGS) {  // a frame with no vertex work
    if (threadIdx.x == 0) reset_counters(a_.b.counters);
    publish_args(a_, pub_);
}
#endif

// The clip position, outcode and snap of a vertex at `world` (its clip position kept when the clipper needs it).
__device__ __forceinline__ void store_snap(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t slot,
                                           const TriDrawDev& dr, float4 world) {
    const float4 clip = mat_vec_seq(fp.pv, world);
    uint32_t oc = outcode(fp, clip);
    // clip_from_world draws: a vertex without an outcode has world.w == 1 and its clip position is
    // recomputed by the clipper from `vary` (or its record); a non-finite position (w != 1) is marked for clipping
    if (dr.clip_from_world && oc == 0u && !(world.w == 1.0f)) oc = TRI_OC_CLIP;
    if (oc != 0u || !dr.clip_from_world) b.clip[slot] = clip;
    TriSnap sn{TRI_SNAP_F ? 0 : (int32_t)(oc << 24), 0, 0.0f, 0.0f};
    if (!(oc & TRI_OC_CLIP)) {
        int32_t X, Y;
        snap_compute(fp, clip, X, Y, sn.z, sn.iw);
        if (TRI_SNAP_F) {  // |X|, |Y| < 2^22 inside the guard band: exact as floats
            sn.xo = __float_as_int((float)X);
            sn.y = __float_as_int((float)Y);
        } else {
            sn.xo = (X & 0x00FFFFFF) | (int32_t)(oc << 24);
            sn.y = Y;
        }
    }
    b.snap[slot] = sn;
    if (TRI_SNAP_F) b.oc[slot] = (uint8_t)oc;
}

// Default.vert for vertex slot `slot` of draw `dr` (whose first slot is `vbase`).
__device__ __forceinline__ void vertex_slot(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t slot,
                                            const TriDrawDev& dr, uint32_t vbase) {
    const int64_t gi = (int64_t)dr.base_vertex + (int64_t)(dr.min_index + (slot - vbase));
    if (gi < 0 || (uint64_t)gi >= b.vertex_count) {
        b.snap[slot] = TriSnap{TRI_SNAP_F ? 0 : (int32_t)(TRI_OC_BAD << 24), 0, 0.0f, 0.0f};
        if (TRI_SNAP_F) b.oc[slot] = (uint8_t)TRI_OC_BAD;
        if (fp.shadow_on) b.lsnap[slot] = TriSnap{(int32_t)(TRI_OC_BAD << 24), 0, 0.0f, 0.0f};
        return;
    }
    if (obj_mode(fp) || obj48_mode(fp)) {  // no varyings to write: the position stream alone (12 B), then the snap
        const Rsrc pr = make_rsrc(b.vpos, 12ull * b.vertex_count);
        const auto q = __builtin_amdgcn_raw_buffer_load_b96(pr, (uint32_t)gi * 12u, 0, 0);
        const float4 world = mat_vec_seq(dr.model, make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]),
                                                               __uint_as_float(q[2]), 1.0f));
        store_snap(fp, b, slot, dr, world);
        // (obj48 with the pre-pass: the same world position as the input-record path below, so the same map)
        if (fp.shadow_on) shadow_vertex(fp, b, slot, world);
        return;
    }
    // three 16-byte loads (a plain struct load is split into overlapping per-field loads)
    const Rsrc vr = make_rsrc(b.vin, 48ull * b.vertex_count);
    const uint4 q0 = ld128(vr, (uint32_t)gi * 48u), q1 = ld128(vr, (uint32_t)gi * 48u + 16u),
                q2 = ld128(vr, (uint32_t)gi * 48u + 32u);
    TriVsIn in;  // {pos, u}{normal, v}{colour, 0}
    in.px = __uint_as_float(q0.x); in.py = __uint_as_float(q0.y); in.pz = __uint_as_float(q0.z);
    in.u = __uint_as_float(q0.w); in.nx = __uint_as_float(q1.x); in.ny = __uint_as_float(q1.y);
    in.nz = __uint_as_float(q1.z); in.v = __uint_as_float(q1.w); in.cr = __uint_as_float(q2.x);
    in.cg = __uint_as_float(q2.y); in.cb = __uint_as_float(q2.z);
    float4 sp = make_float4(in.px, in.py, in.pz, 1.0f);
    float snx = in.nx, sny = in.ny, snz = in.nz;
    if (dr.bone_count > 0 && b.vskin) {  // Default.vert:64-85
        const TriVsSkin sk = b.vskin[gi];
        float s[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float w = sk.w[k];
            if (w <= 0.0f) continue;
            const int bi = sk.idx[k];
            if (bi < 0 || bi >= dr.bone_count) continue;
            const uint32_t buf = (uint32_t)(dr.bone_offset + bi);
            if (buf >= fp.bone_count) continue;
            TRI_G const float* bm = b.bones + 16ull * buf;
#pragma unroll
            for (int i = 0; i < 16; ++i) s[i] = s[i] + w * bm[i];
        }
        sp = mat_vec_seq(s, sp);
        const float nx = (s[0] * snx + s[4] * sny) + s[8] * snz;
        const float ny = (s[1] * snx + s[5] * sny) + s[9] * snz;
        const float nz = (s[2] * snx + s[6] * sny) + s[10] * snz;
        snx = nx; sny = ny; snz = nz;
    }
    const float4 world = mat_vec_seq(dr.model, sp);
    const float* nm = dr.nm;  // NM[c*3+r]; N' = NM * n
    float nnx = (nm[0] * snx + nm[3] * sny) + nm[6] * snz;
    float nny = (nm[1] * snx + nm[4] * sny) + nm[7] * snz;
    float nnz = (nm[2] * snx + nm[5] * sny) + nm[8] * snz;
    const float inv = 1.0f / sqrtf((nnx * nnx + nny * nny) + nnz * nnz);
    nnx = nnx * inv; nny = nny * inv; nnz = nnz * inv;
    const float u = (in.u * dr.tex_scale[0]) * dr.tiling + dr.tex_offset[0];
    const float v = (in.v * dr.tex_scale[1]) * dr.tiling + dr.tex_offset[1];
    store_snap(fp, b, slot, dr, world);
    if (vary36_mode(fp)) {  // 36-B record: three 12-B stores (the slot's bytes are 4-B aligned)
        TRI_G F3* vo = reinterpret_cast<TRI_G F3*>(b.vary) + 3u * slot;
        vo[0] = F3{world.x, world.y, world.z};
        vo[1] = F3{nnx, nny, nnz};
        vo[2] = F3{in.cr, in.cg, in.cb};
    } else {  // the input records' layout (TriVsIn), so that obj48 frames read those records with the same code
        float4* vo = b.vary + 3u * slot;
        vo[0] = make_float4(world.x, world.y, world.z, u);
        vo[1] = make_float4(nnx, nny, nnz, v);
        vo[2] = make_float4(in.cr, in.cg, in.cb, 0.0f);
    }
    if (fp.shadow_on) shadow_vertex(fp, b, slot, world);
}

// Cluster culling (row bands). A cluster's object-space box goes through (P * V) * M; when every corner
// is in front of the eye (w > 0 over the whole box, w being affine) the box's image is bounded by its
// corners' images, and a cluster whose bound misses the context's rows or columns (2-pixel margin), or
// lies wholly before z = 0 or beyond z = w, has no fragment here: k_setup skips its primitives (exactly
// what their set-up would conclude). Skinned draws move their vertices off the boxes and are kept.
__device__ __forceinline__ bool cluster_visible(const TriFrameParams& fp, const TriDrawDev& dr, const TriCluster& c) {
    if (c.lo[0] > c.hi[0]) return false;  // no valid vertex: every primitive of the cluster is dropped anyway
    if (dr.bone_count > 0) return true;
    float m[16];  // (P * V) * M, column-major
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            m[4 * j + r] = fp.pv[r] * dr.model[4 * j] + fp.pv[4 + r] * dr.model[4 * j + 1] +
                           fp.pv[8 + r] * dr.model[4 * j + 2] + fp.pv[12 + r] * dr.model[4 * j + 3];
    float x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY, z0 = INFINITY, z1 = -INFINITY;
    bool front = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float px = (k & 1) ? c.hi[0] : c.lo[0], py = (k & 2) ? c.hi[1] : c.lo[1], pz = (k & 4) ? c.hi[2] : c.lo[2];
        const float cx = m[0] * px + m[4] * py + m[8] * pz + m[12];
        const float cy = m[1] * px + m[5] * py + m[9] * pz + m[13];
        const float cz = m[2] * px + m[6] * py + m[10] * pz + m[14];
        const float cw = m[3] * px + m[7] * py + m[11] * pz + m[15];
        front = front && cw > 1e-4f;
        const float iw = 1.0f / cw;
        x0 = fminf(x0, cx * iw); x1 = fmaxf(x1, cx * iw);
        y0 = fminf(y0, cy * iw); y1 = fmaxf(y1, cy * iw);
        z0 = fminf(z0, cz * iw); z1 = fmaxf(z1, cz * iw);
    }
    if (!front) return true;
    const float wx0 = x0 * fp.hw + fp.hw, wx1 = x1 * fp.hw + fp.hw;
    const float wy0 = y0 * fp.hh + fp.hh, wy1 = y1 * fp.hh + fp.hh;
    // the margins (2 px, 1e-4 in depth) cover the rounding difference between the box corners' (P V) M
    // product and the vertices' P V (M p): the test is never stricter than the vertices' own
    return !(wy1 < (float)fp.y0 - 2.0f || wy0 > (float)fp.y1 + 2.0f || wx1 < -2.0f || wx0 > (float)fp.W + 2.0f ||
             z1 < -1e-4f || z0 > 1.0f + 1e-4f);
}

// One lane per vertex slot. With cluster culling on: lanes 0 .. ncl_total-1 of the grid (the first few
// waves) test one (draw, cluster) box each and store its flag for k_setup; every wave then tests the union
// box of its 256-slot vertex block (the clusters referencing it, precomputed at upload: one load) and,
// unless the shadow pre-pass needs every caster, skips a block whose box misses the rows. A vertex of any
// visible primitive is always transformed: its cluster's box lies inside the block's union box.
#ifdef TRI_VERTEX_TU
__global__ __launch_bounds__(TRI_BLOCK) void k_vertex(TRI_FIRST_KARGS) {
    TRI_BIND_FIRST_ARGS;
    publish_args(a_, pub_);
    const uint32_t slot = blockIdx.x * TRI_BLOCK + threadIdx.x;
    if (slot == 0) reset_counters(b.counters);  // per-frame counters, consumed from k_setup on
    const bool valid = slot < fp.nslots;
    int d = 0;
    uint32_t vbase = 0;
    if (valid && !fp.one_draw) {
        d = find_range(b.draw_vbase, (int)fp.ndraws, slot);
        vbase = b.draw_vbase[d];
    }
    bool needed = true;
    if (fp.cull_on) {  // uniform
        if (slot < fp.ncl_total) {  // this lane's (draw, cluster) flag
            const int cd = fp.one_draw ? 0 : find_range(b.draw_cbase, (int)fp.ndraws, slot);
            const uint32_t lc = slot - (fp.one_draw ? 0u : b.draw_cbase[cd]);
            const bool vis = fp.one_draw ? cluster_visible(fp, fp.draw0, b.clusters[fp.draw0.cl_first + lc])
                                         : cluster_visible(fp, b.draws[cd], b.clusters[b.draws[cd].cl_first + lc]);
            b.cvis[slot] = vis ? 1u : 0u;
        }
        const uint32_t blk = (slot - vbase) / TRI_VBLOCK;
        uint64_t pending = __ballot(valid);
        while (pending) {  // the wave's distinct (draw, block) groups, usually one
            const int l = __builtin_ctzll(pending);
            const int gd = __builtin_amdgcn_readlane(d, l);
            const uint32_t gb = (uint32_t)__builtin_amdgcn_readlane((int)blk, l);
            const bool mine = valid && d == gd && blk == gb;
            pending &= ~__ballot(mine);
            const bool any = fp.one_draw ? cluster_visible(fp, fp.draw0, b.vbox[fp.draw0.vblk_first + gb])
                                         : cluster_visible(fp, b.draws[gd], b.vbox[b.draws[gd].vblk_first + gb]);
            if (mine) needed = any;
        }
    }
    if (!valid || (fp.cull_vertex && !needed)) return;
    // two calls, not one through a selected reference: each sees its draw's address space (kernel arguments or
    // global memory), so a single draw's constants are scalar loads
    if (fp.one_draw) vertex_slot(fp, b, slot, fp.draw0, vbase);
    else vertex_slot(fp, b, slot, b.draws[d], vbase);
}

// Row bands of single-draw frames (cull_vertex && one_draw): a quarter of k_vertex's workgroups, each owning
// the four 256-slot vertex blocks blockIdx.x + i * gridDim.x (i = 0..3). Wave i tests block i's union box
// (the four tests run side by side instead of four waves repeating one), the flags meet in LDS, and the
// whole workgroup transforms the visible blocks one after another. A band's visible blocks are contiguous
// in slot order (its rows' clusters), so the stride spreads them over different workgroups: at N = 8 a
// workgroup holds at most one, and 3/4 of the launch's dispatches (all empty) are gone. The cluster flags
// for k_setup are the same lanes' work as in k_vertex, grid-strided.
static_assert(TRI_VBLOCK == TRI_BLOCK, "k_vertex_band: one workgroup-wide pass per vertex block");
__global__ __launch_bounds__(TRI_BLOCK) void k_vertex_band(TRI_FIRST_KARGS) {
    TRI_BIND_FIRST_ARGS;
    publish_args(a_, pub_);
    __shared__ uint32_t blk_vis[TRI_BLOCK / 64];
    const uint32_t tid = threadIdx.x, G = gridDim.x;
    if (blockIdx.x == 0 && tid == 0) reset_counters(b.counters);
    const TriDrawDev& dr = fp.draw0;
    for (uint32_t c = blockIdx.x * TRI_BLOCK + tid; c < fp.ncl_total; c += G * TRI_BLOCK)
        b.cvis[c] = cluster_visible(fp, dr, b.clusters[dr.cl_first + c]) ? 1u : 0u;
    const uint32_t nblk = (fp.nslots + TRI_VBLOCK - 1) / TRI_VBLOCK;
    const uint32_t w = tid / 64u, blk = blockIdx.x + w * G;
    const bool vis = blk < nblk && cluster_visible(fp, dr, b.vbox[dr.vblk_first + blk]);
    if ((tid & 63u) == 0) blk_vis[w] = vis ? 1u : 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < TRI_BLOCK / 64; ++i) {
        if (!blk_vis[i]) continue;  // uniform
        const uint32_t slot = (blockIdx.x + i * G) * TRI_VBLOCK + tid;
        if (slot < fp.nslots) vertex_slot(fp, b, slot, dr, 0u);
    }
}
#endif

// ------------------------------------------------------------------------------------------
// tri_setup_bin
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int32_t floor_shift8(int32_t v) { return v >> 8; }

// Perspective divide (x * (1/w), one correctly rounded divide), viewport transform
// (Renderer.cpp:5062-5069) and 8-bit sub-pixel snap of one vertex. Mirrors oracle setup_triangle().
__device__ __forceinline__ void snap_compute(const TriFrameParams& fp, float4 c, int32_t& X, int32_t& Y, float& z,
                                             float& iw) {
    iw = 1.0f / c.w;
    const float xd = c.x * iw, yd = c.y * iw;
    z = c.z * iw;
    const float xf = xd * fp.hw + fp.hw;
    const float yf = yd * fp.hh + fp.hh;
    X = (int32_t)rintf(xf * 256.0f);
    Y = (int32_t)rintf(yf * 256.0f);
}

__device__ __forceinline__ uint32_t outcode(const TriFrameParams& fp, float4 c) {
    uint32_t oc = 0;
    if (c.z < 0.0f) oc |= TRI_OC_ZNEG;
    if (c.w - c.z < 0.0f) oc |= TRI_OC_ZFAR;
    if (c.x + c.w < 0.0f) oc |= TRI_OC_XNEG;
    if (c.w - c.x < 0.0f) oc |= TRI_OC_XPOS;
    if (c.y + c.w < 0.0f) oc |= TRI_OC_YNEG;
    if (c.w - c.y < 0.0f) oc |= TRI_OC_YPOS;
    if ((c.w < TRI_WMIN) || (c.z < 0.0f) || (c.x < -fp.gx * c.w) || (c.x > fp.gx * c.w) ||
        (c.y < -fp.gy * c.w) || (c.y > fp.gy * c.w))
        oc |= TRI_OC_CLIP;
    return oc;
}

// Setup of a triangle from snapped vertices (all inside w>=WMIN, z>=0 and the guard band).
// Mirrors oracle setup_triangle(). Returns false when culled or when its bbox is empty.
__device__ __forceinline__ bool setup_snapped(const TriFrameParams& fp, const int32_t X[3], const int32_t Y[3],
                                              const float z[3], const float iw[3], uint32_t s0, uint32_t s1,
                                              uint32_t s2, uint32_t prim_sub, TriRec& r, uint2& br) {
    const int64_t S = (int64_t)(X[1] - X[0]) * (int64_t)(Y[2] - Y[0]) -
                      (int64_t)(Y[1] - Y[0]) * (int64_t)(X[2] - X[0]);
    if (S >= 0) return false;  // zero area or back-facing (cull BACK, front CCW)
    const int32_t xmin = min(X[0], min(X[1], X[2])), xmax = max(X[0], max(X[1], X[2]));
    const int32_t ymin = min(Y[0], min(Y[1], Y[2])), ymax = max(Y[0], max(Y[1], Y[2]));
    int32_t px0 = -floor_shift8(128 - xmin), px1 = floor_shift8(xmax - 128);
    int32_t py0 = -floor_shift8(128 - ymin), py1 = floor_shift8(ymax - 128);
    px0 = max(px0, 0);
    px1 = min(px1, fp.W - 1);
    py0 = max(py0, fp.y0);
    py1 = min(py1, fp.y1 - 1);
    if (px0 > px1 || py0 > py1) return false;
    // swap v1 <-> v2 so the edge functions see S' = -S > 0
    r.X[0] = X[0]; r.X[1] = X[2]; r.X[2] = X[1];
    r.Y[0] = Y[0]; r.Y[1] = Y[2]; r.Y[2] = Y[1];
    r.z[0] = z[0]; r.z[1] = z[2]; r.z[2] = z[1];
    r.iw[0] = iw[0]; r.iw[1] = iw[2]; r.iw[2] = iw[1];
    r.v[0] = s0; r.v[1] = s2; r.v[2] = s1;
    r.prim_sub = prim_sub;
    const uint32_t bl = (uint32_t)fp.bin_log2;
    const uint32_t bx0 = (uint32_t)px0 >> bl, bx1 = (uint32_t)px1 >> bl;
    const uint32_t by0 = (uint32_t)(py0 - fp.y0) >> bl, by1 = (uint32_t)(py1 - fp.y0) >> bl;
    br = make_uint2(bx0 | (by0 << 16), bx1 | (by1 << 16));
    return true;
}

__device__ __forceinline__ bool setup_from_clip(const TriFrameParams& fp, float4 c0, float4 c1, float4 c2,
                                                uint32_t s0, uint32_t s1, uint32_t s2, uint32_t prim_sub, TriRec& r,
                                                uint2& br) {
    int32_t X[3], Y[3];
    float z[3], iw[3];
    snap_compute(fp, c0, X[0], Y[0], z[0], iw[0]);
    snap_compute(fp, c1, X[1], Y[1], z[1], iw[1]);
    snap_compute(fp, c2, X[2], Y[2], z[2], iw[2]);
    return setup_snapped(fp, X, Y, z, iw, s0, s1, s2, prim_sub, r, br);
}

template <typename F>
__device__ __forceinline__ void for_bins(uint2 br, int nbx, F&& f) {
    const uint32_t bx0 = br.x & 0xFFFFu, by0 = br.x >> 16, bx1 = br.y & 0xFFFFu, by1 = br.y >> 16;
    for (uint32_t by = by0; by <= by1; ++by)
        for (uint32_t bx = bx0; bx <= bx1; ++bx) f(by * (uint32_t)nbx + bx);
}

__device__ __forceinline__ void note_bin_overflow(const TriDeviceBuffers& b, uint32_t needed) {
    atomicOr(&b.counters->flags, TRI_OVF_BIN_LIST);
    atomicMax(&b.counters->bin_max, needed);
}

// Wave-aggregated queue reservation: every lane with `want` gets one slot in bin `bin`. Lanes of the
// wave that target the same bin form a group; each group's leader issues ONE atomicAdd for the whole
// group (all leaders at once, one round trip), and members take consecutive slots after it. Must be
// reached by the whole wave (uniform control flow).

// Reservation plan (ALU and ballots only): each wanting lane learns its group's leader lane and its
// rank in the group; a leader learns its group's size.
__device__ __forceinline__ void wave_reserve_plan(uint32_t bin, bool want, uint32_t& leader, uint32_t& rank,
                                                  uint32_t& cnt) {
    uint64_t pending = __ballot(want);
    const uint32_t lane = lanes_below(~0ull);
    leader = lane; rank = 0; cnt = 0;
    while (pending) {
        const uint32_t l = (uint32_t)__builtin_ctzll(pending);
        const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane((int)bin, (int)l);
        const uint64_t grp = __ballot(want && bin == lb) & pending;
        if (want && bin == lb) {
            leader = l;
            rank = lanes_below(grp);
        }
        if (lane == l) cnt = (uint32_t)__builtin_popcountll(grp);
        pending &= ~grp;
    }
}

// Binning rounds whose queue reservations k_setup keeps in flight together.
#ifndef TRI_RES_BATCH
#define TRI_RES_BATCH 4
#endif
constexpr int kResBatch = TRI_RES_BATCH;

// ------------------------------------------------------------------------------------------
// Homogeneous clipping (oracle clip_polygon: Sutherland-Hodgman against w >= WMIN, z >= 0 and the
// guard band, then a fan), done by the whole wave for one primitive at a time inside k_setup: lane i
// holds polygon vertex i, the output order of the sequential algorithm is rebuilt with ballots, and
// the two polygon buffers live in a per-wave LDS slice. No separate launch, no per-lane arrays.
// ------------------------------------------------------------------------------------------
struct ClipVert {
    float4 c;
    float b0, b1, b2;  // barycentric weights on the source triangle (for the varyings)
};
constexpr int kClipStride = 8;  // floats per LDS polygon vertex
constexpr int kWavesPerBlock = TRI_BLOCK / 64;

__device__ __forceinline__ ClipVert lerp_cv(const ClipVert& a, const ClipVert& b, float t) {
    ClipVert o;
#define L(f) o.f = a.f + t * (b.f - a.f)
    L(c.x); L(c.y); L(c.z); L(c.w); L(b0); L(b1); L(b2);
#undef L
    return o;
}

__device__ __forceinline__ float plane_dist(const TriFrameParams& fp, int plane, float4 c) {
    switch (plane) {
        case 0: return c.w - TRI_WMIN;
        case 1: return c.z;
        case 2: return c.x + fp.gx * c.w;
        case 3: return fp.gx * c.w - c.x;
        case 4: return c.y + fp.gy * c.w;
        default: return fp.gy * c.w - c.y;
    }
}

// The polygons live in LDS: the pointers say so (a generic pointer would make every access a flat instruction)
#if defined(__HIP_DEVICE_COMPILE__)
#define TRI_LDS __attribute__((address_space(3)))
#else
#define TRI_LDS
#endif
__device__ __forceinline__ void cv_store(TRI_LDS float* p, const ClipVert& v) {
    p[0] = v.c.x; p[1] = v.c.y; p[2] = v.c.z; p[3] = v.c.w; p[4] = v.b0; p[5] = v.b1; p[6] = v.b2;
}
__device__ __forceinline__ ClipVert cv_load(TRI_LDS const float* p) {
    ClipVert v;
    v.c = make_float4(p[0], p[1], p[2], p[3]);
    v.b0 = p[4]; v.b1 = p[5]; v.b2 = p[6];
    return v;
}
// Workgroup barrier ordering LDS only (s_waitcnt lgkmcnt(0) + s_barrier): global loads issued before it stay
// in flight (__syncthreads' fence would wait for them too).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// LDS traffic between lanes of one wave: DS instructions of a wave execute in order, so a
// compiler barrier is all that is needed between a lane's store and another lane's load.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Clip primitive `prim` (vertex slots sl[3]) with the whole wave; lanes that set up a fan
// sub-triangle bin it. Must be reached by the whole wave.
// `draw`: the primitive's draw (wave-uniform), for obj48 frames' object records and model matrix.
template <bool LPOS, bool ONE>
__device__ __forceinline__ void clip_prim_wave(const TriFrameParams& fp, const TriDeviceBuffers& b, TRI_LDS float* poly,
                                               uint32_t prim, uint32_t sl0, uint32_t sl1, uint32_t sl2, bool cfw,
                                               uint32_t draw, uint32_t& nsetup, uint32_t& nentries) {
    const uint32_t lane = lanes_below(~0ull);
    const uint64_t below = (lane == 63) ? 0x7FFFFFFFFFFFFFFFull : ((1ull << lane) - 1ull);
    TRI_LDS float* buf[2] = {poly, poly + TRI_MAX_CLIP_VERTS * kClipStride};
    // object-space records: the ONE frames' (vary_obj: 36-B records at vin_base + slot, never with the pre-pass),
    // or obj48's (the 48-B input records at slot + vdelta[draw]). ONE here is k_setup's single-draw instantiation, not
    // the raster's: a single draw may be an obj48 frame too (a textured draw, the pre-pass, the AI blend), and then
    // k_vertex wrote no varyings for the clipper to read (draw is 0 and fp.draw0 is that draw)
    const bool obj1 = !LPOS && obj_mode(fp), o48 = obj48_mode(fp);
    const bool one_draw = ONE || fp.one_draw;
    const uint32_t dl = o48 ? fp.vdelta[min(draw, (uint32_t)TRI_OBJ48_DRAWS - 1u)] : fp.vin_base;
    if (lane < 3) {
        ClipVert v;
        const uint32_t sl = lane == 0 ? sl0 : (lane == 1 ? sl1 : sl2);
        if (cfw && snap_oc(b, b.snap[sl], sl) == 0u) {  // not stored by k_vertex: world.w == 1
            F3 wv;
            if (obj1 || o48) {  // k_vertex's world position, from the record (same operations)
                const F3 p = vattr_at(b, dl + sl, 0);
                float m[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) m[i] = (o48 && !one_draw) ? b.draws[draw].model[i] : fp.draw0.model[i];
                const float4 w = mat_vec_seq(m, make_float4(p.x, p.y, p.z, 1.0f));
                wv = F3{w.x, w.y, w.z};
            } else {
                wv = vary36_mode(fp) ? ldF3(reinterpret_cast<TRI_G const F3*>(b.vary) + 3u * sl)
                                     : F3{b.vary[3u * sl].x, b.vary[3u * sl].y, b.vary[3u * sl].z};
            }
            v.c = mat_vec_seq(fp.pv, make_float4(wv.x, wv.y, wv.z, 1.0f));
        } else {
            v.c = b.clip[sl];
        }
        v.b0 = lane == 0 ? 1.0f : 0.0f;
        v.b1 = lane == 1 ? 1.0f : 0.0f;
        v.b2 = lane == 2 ? 1.0f : 0.0f;
        cv_store(buf[0] + lane * kClipStride, v);
    }
    int n = 3, cur = 0;
    for (int plane = 0; plane < 6 && n > 0; ++plane) {
        wave_lds_sync();
        const bool act = (int)lane < n;
        ClipVert a{}, nb{};
        float da = 0.0f, db = 0.0f;
        if (act) {
            a = cv_load(buf[cur] + lane * kClipStride);
            nb = cv_load(buf[cur] + ((int)lane + 1 < n ? lane + 1 : 0) * kClipStride);
            da = plane_dist(fp, plane, a.c);
            db = plane_dist(fp, plane, nb.c);
        }
        const bool in = act && da >= 0.0f;
        const bool cross = act && ((da >= 0.0f) != (db >= 0.0f));
        const uint64_t m_in = __ballot(in), m_cr = __ballot(cross);
        const int pos = __builtin_popcountll(m_in & below) + __builtin_popcountll(m_cr & below);
        wave_lds_sync();
        if (in && pos < TRI_MAX_CLIP_VERTS) cv_store(buf[cur ^ 1] + pos * kClipStride, a);
        const int pos2 = pos + (in ? 1 : 0);
        if (cross && pos2 < TRI_MAX_CLIP_VERTS) {
            const float t = da / (da - db);
            cv_store(buf[cur ^ 1] + pos2 * kClipStride, lerp_cv(a, nb, t));
        }
        n = min(__builtin_popcountll(m_in) + __builtin_popcountll(m_cr), TRI_MAX_CLIP_VERTS);
        cur ^= 1;
    }
    wave_lds_sync();
    if (n < 3) return;
    n = min(n, TRI_MAX_CLIP_POLY);
    const uint32_t nsub = (uint32_t)(n - 2);
    uint32_t rbase = 0, vbase = 0;
    if (lane == 0) {
        rbase = atomicAdd(&b.counters->ovf_records, nsub);
        vbase = atomicAdd(&b.counters->ovf_verts, (uint32_t)n);
    }
    rbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)rbase);
    vbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)vbase);
    if (rbase + nsub > fp.ovf_rec_cap || vbase + (uint32_t)n > fp.ovf_vert_cap) {
        if (lane == 0)
            atomicOr(&b.counters->flags, (rbase + nsub > fp.ovf_rec_cap) ? TRI_OVF_CLIP_RECORDS : TRI_OVF_CLIP_VERTS);
        return;
    }
    const uint32_t sbase = fp.nslots + vbase;
    TRI_LDS const float* src = buf[cur];
    if ((int)lane < n) {  // varyings of polygon vertex `lane` from the source triangle's barycentrics
        const ClipVert s = cv_load(src + lane * kClipStride);
        if (vary36_mode(fp)) {  // (object-space attributes from the vertex records with vary_obj)
            TRI_G const F3* v0 = reinterpret_cast<TRI_G const F3*>(b.vary) + 3u * sl0;
            TRI_G const F3* v1 = reinterpret_cast<TRI_G const F3*>(b.vary) + 3u * sl1;
            TRI_G const F3* v2 = reinterpret_cast<TRI_G const F3*>(b.vary) + 3u * sl2;
            TRI_G F3* vo = reinterpret_cast<TRI_G F3*>(b.vary) + 3u * (sbase + lane);
            const bool obj = !LPOS && obj_mode(fp);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const F3 x = obj ? vin_attr(fp, b, sl0, j) : ldF3(v0 + j), y = obj ? vin_attr(fp, b, sl1, j) : ldF3(v1 + j),
                         z = obj ? vin_attr(fp, b, sl2, j) : ldF3(v2 + j);
                vo[j] = F3{(s.b0 * x.x + s.b1 * y.x) + s.b2 * z.x, (s.b0 * x.y + s.b1 * y.y) + s.b2 * z.y,
                           (s.b0 * x.z + s.b1 * y.z) + s.b2 * z.z};
            }
        } else {  // 48-B records: the world-space varyings, or (obj48) the input records' own layout
            const float4* v0 = o48 ? reinterpret_cast<TRI_G const float4*>(b.vin + (dl + sl0)) : b.vary + 3u * sl0;
            const float4* v1 = o48 ? reinterpret_cast<TRI_G const float4*>(b.vin + (dl + sl1)) : b.vary + 3u * sl1;
            const float4* v2 = o48 ? reinterpret_cast<TRI_G const float4*>(b.vin + (dl + sl2)) : b.vary + 3u * sl2;
            float4* vo = b.vary + 3u * (sbase + lane);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const float4 x = v0[j], y = v1[j], z = v2[j];
                vo[j] = make_float4((s.b0 * x.x + s.b1 * y.x) + s.b2 * z.x, (s.b0 * x.y + s.b1 * y.y) + s.b2 * z.y,
                                    (s.b0 * x.z + s.b1 * y.z) + s.b2 * z.z, (s.b0 * x.w + s.b1 * y.w) + s.b2 * z.w);
            }
        }
        if constexpr (LPOS) {  // shadow pre-pass on: the polygon vertex's light-space position, same weights
            const float4 x = b.lpos[sl0], y = b.lpos[sl1], z = b.lpos[sl2];
            b.lpos[sbase + lane] = make_float4((s.b0 * x.x + s.b1 * y.x) + s.b2 * z.x,
                                               (s.b0 * x.y + s.b1 * y.y) + s.b2 * z.y,
                                               (s.b0 * x.z + s.b1 * y.z) + s.b2 * z.z, 0.0f);
        }
    }
    if (lane == 0) b.clip_slot[prim] = rbase;  // k_raster's fragment fetch finds sub-triangle `sub` at + sub - 1
    if (lane < nsub) {  // fan sub-triangle k = lane + 1: (v0, vk, vk+1)
        const uint32_t k = lane + 1;
        TriRec r;
        uint2 br;
        const uint32_t ps = (prim << 3) | k;  // sub = k >= 1 marks a clipped primitive's sub-triangle
        const uint32_t rid = rbase + k - 1;
        const float4 c0 = cv_load(src).c, ck = cv_load(src + k * kClipStride).c,
                     ck1 = cv_load(src + (k + 1) * kClipStride).c;
        if (setup_from_clip(fp, c0, ck, ck1, sbase, sbase + k, sbase + k + 1, ps, r, br)) {
            ++nsetup;
            b.recs[rid] = r;
            for_bins(br, fp.nbx, [&](uint32_t bi) {  // rare path: one global atomic per entry
                const uint32_t pos = atomicAdd(&b.bin_count[bi], 1u);
                if (pos < fp.bin_cap) b.bin_list[(size_t)bi * fp.bin_cap + pos] = TRI_ENTRY_CLIPPED | rid;
                else note_bin_overflow(b, pos + 1);
                ++nentries;
            });
        }
    }
}

// Shadow pre-pass set-up of a triangle from its map snaps (oracle shadow_raster_triangle): no culling,
// only zero-area triangles drop; the bbox of texel centres inside the map, as 32x32 bin ranges.
__device__ __forceinline__ bool shadow_bins(const TriFrameParams& fp, const int32_t X[3], const int32_t Y[3], uint2& br) {
    const int64_t S = (int64_t)(X[1] - X[0]) * (int64_t)(Y[2] - Y[0]) -
                      (int64_t)(Y[1] - Y[0]) * (int64_t)(X[2] - X[0]);
    if (S == 0) return false;
    const int32_t xmin = min(X[0], min(X[1], X[2])), xmax = max(X[0], max(X[1], X[2]));
    const int32_t ymin = min(Y[0], min(Y[1], Y[2])), ymax = max(Y[0], max(Y[1], Y[2]));
    const int32_t n1 = (int32_t)fp.s_size - 1;
    const int32_t px0 = max(-floor_shift8(128 - xmin), 0), px1 = min(floor_shift8(xmax - 128), n1);
    const int32_t py0 = max(-floor_shift8(128 - ymin), 0), py1 = min(floor_shift8(ymax - 128), n1);
    if (px0 > px1 || py0 > py1) return false;
    br = make_uint2((uint32_t)(px0 >> 5) | ((uint32_t)(py0 >> 5) << 16), (uint32_t)(px1 >> 5) | ((uint32_t)(py1 >> 5) << 16));
    return true;
}

__device__ __forceinline__ void note_shadow_bin_overflow(const TriDeviceBuffers& b, uint32_t needed) {
    atomicOr(&b.counters->flags, TRI_OVF_SHADOW_BIN_LIST);
    atomicMax(&b.counters->sbin_max, needed);
}

// One lane per primitive (ppt primitives per lane): assembly from the snapped vertices, trivial
// reject, cull, bbox, then one bin-queue entry per touched bin (batched wave reservations). Nothing else is
// written for a visible triangle: k_raster rebuilds it from `snap`. Triangles needing homogeneous
// clipping are clipped right here by their wave (clip_prim_wave). Entry order inside a bin is free:
// k_raster resolves visibility with (depth, primitive order) keys.

// Per-wave binning (the shadow and frame rounds whose workgroup bin box is too large for bin_pair_box's
// LDS grid): the lane's bin-queue entries, one per round: triangle 0's bbox bins, then triangle 1's. A batch of
// kResBatch rounds is planned with ballots and its reservations (one returning atomic per (wave, bin))
// are all issued before any result is used, so a wave waits for one atomic round trip per batch instead
// of one per round. Must be reached by the whole wave. Diagnostics: TRI_ABLATE=8 waits per round.
// Component-wise selects (a plain `c ? a : b` on uint4 became a dynamically indexed stack array).
__device__ __forceinline__ uint32_t pick(bool c, uint32_t a, uint32_t b) { return c ? a : b; }
__device__ __forceinline__ uint4 pick(bool c, uint4 a, uint4 b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

template <bool SHADOW_QUEUES, typename Q>
__device__ __forceinline__ void bin_pair(const TriDeviceBuffers& b, bool ok0, bool ok1, uint2 br0, uint2 br1, Q p0, Q p1,
                                         uint32_t nbx, uint32_t* bin_count, Q* bin_list, uint32_t cap, uint32_t lane,
                                         uint32_t& nentries) {
    bool has = (ok0 || ok1) && !(kAblate & 4);  // diagnostics: 4 = setup without binning
    bool second = !ok0;
    uint2 cur = second ? br1 : br0;
    uint32_t bx = cur.x & 0xFFFFu, by = cur.x >> 16;
    uint32_t bx0 = bx, bx1 = cur.y & 0xFFFFu, by1 = cur.y >> 16;
    const int batch = (kAblate & 8) ? 1 : kResBatch;
    while (__ballot(has)) {
        uint32_t rbin[kResBatch], rlr[kResBatch], rbase[kResBatch];  // rlr: group leader lane | rank << 8
        bool rwant[kResBatch], rsec[kResBatch];
#pragma unroll
        for (int r = 0; r < kResBatch; ++r) {
            rwant[r] = has && r < batch;
            rbin[r] = by * nbx + bx;
            rsec[r] = second;
            if (rwant[r]) {
                if (bx < bx1) {
                    ++bx;
                } else if (by < by1) {
                    bx = bx0;
                    ++by;
                } else if (!second && ok1) {
                    second = true;
                    bx = bx0 = br1.x & 0xFFFFu; by = br1.x >> 16;
                    bx1 = br1.y & 0xFFFFu; by1 = br1.y >> 16;
                } else {
                    has = false;
                }
            }
            uint32_t cnt, lead, rank;
            wave_reserve_plan(rbin[r], rwant[r], lead, rank, cnt);
            rlr[r] = lead | (rank << 8);
            rbase[r] = 0;
            if (rwant[r] && lane == lead && !(kAblate & 16))  // diagnostics: 16 = no atomics
                rbase[r] = atomicAdd(&bin_count[rbin[r]], cnt);
        }
#pragma unroll
        for (int r = 0; r < kResBatch; ++r) {
            const uint32_t pos = (uint32_t)__shfl((int)rbase[r], (int)(rlr[r] & 0xFFu)) + (rlr[r] >> 8);
            if (rwant[r]) {
                if (kAblate & 32) continue;  // diagnostics: 32 = no queue stores
                if (pos < cap) bin_list[(size_t)rbin[r] * cap + pos] = pick(rsec[r], p1, p0);
                else if (SHADOW_QUEUES) note_shadow_bin_overflow(b, pos + 1);
                else note_bin_overflow(b, pos + 1);
                ++nentries;
            }
        }
    }
}

// Workgroup-aggregated binning: a round's entries (two primitives per lane) are counted per bin in an
// LDS grid over the workgroup's union bin box (a wave min-reduction + one LDS atomicMin per wave and
// corner), one returning global atomic per (workgroup, bin) reserves the bin's run, and each entry takes
// its position in the run from a returning LDS atomic. The counts return to zero as positions are handed
// out, so the grid is never cleared. A round whose box exceeds kBinGrid cells bins with the per-wave
// reservations above (a uniform choice: every wave reads the same box). Must be reached by the whole
// workgroup. Rejected alternative: an LDS hash table keyed by bin (CAS probing): C3 set-up +2 us.
#ifndef TRI_BIN_GRID
#define TRI_BIN_GRID 1024
#endif
constexpr uint32_t kBinGrid = TRI_BIN_GRID;
struct BinBox {
    uint32_t cnt[kBinGrid];
    uint32_t base[kBinGrid];
    uint32_t box[2][2][4];  // per queue set and round parity: min bx, min by, ~max bx, ~max by (LDS atomicMin)
};

// The wave's minimum (uniform), as a DPP scan: row_shr 1/2/4/8 inside each row of 16, then row_bcast:15 / :31
// across rows; lane 63 ends with the minimum of all lanes. Lanes whose DPP source is out of range keep ~0 (the
// identity), so each step is one v_min with a DPP operand instead of a ds_bpermute round trip per step.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_max_id(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)~0u, (int)v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_zero_id(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
// Inclusive prefix sum over the wave's lanes, the same DPP scan (out-of-range sources add 0)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += dpp_zero_id<0x111>(v);
    v += dpp_zero_id<0x112>(v);
    v += dpp_zero_id<0x114>(v);
    v += dpp_zero_id<0x118>(v);
    v += dpp_zero_id<0x142, 0xa>(v);
    v += dpp_zero_id<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    v = min(v, dpp_max_id<0x111>(v));
    v = min(v, dpp_max_id<0x112>(v));
    v = min(v, dpp_max_id<0x114>(v));
    v = min(v, dpp_max_id<0x118>(v));
    v = min(v, dpp_max_id<0x142, 0xa>(v));
    v = min(v, dpp_max_id<0x143, 0xc>(v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

#ifndef TRI_SETUP_GROUP
#define TRI_SETUP_GROUP 2
#endif
constexpr int kSetupGroup = TRI_SETUP_GROUP;  // primitives per lane set up, then binned, together
static_assert(kSetupGroup == 2 || kSetupGroup == 4, "k_setup groups are one or two primitive pairs");

template <bool SHADOW_QUEUES>
__device__ __forceinline__ void bin_pair_box(const TriDeviceBuffers& b, BinBox& g, uint32_t round,
                                             const bool (&ok)[kSetupGroup], const uint2 (&br)[kSetupGroup],
                                             const uint32_t (&p)[kSetupGroup], uint32_t nbx, uint32_t* bin_count,
                                             uint32_t* bin_list, uint32_t cap, uint32_t lane, uint32_t& nentries) {
    if (kAblate & 4) return;  // diagnostics: 4 = setup without binning
#ifdef TRI_SETUP_WAVE_BINNING  // A/B: every round through the per-wave reservations (no LDS grid, no barriers)
#pragma unroll
    for (int t = 0; t < kSetupGroup; t += 2)
        bin_pair<SHADOW_QUEUES>(b, ok[t], ok[t + 1], br[t], br[t + 1], p[t], p[t + 1], nbx, bin_count, bin_list, cap,
                                lane, nentries);
    return;
#endif
    const uint32_t q = round & 1u;
    uint32_t (&box)[2][4] = g.box[SHADOW_QUEUES ? 1 : 0];
    uint32_t m[4] = {~0u, ~0u, ~0u, ~0u};
#pragma unroll
    for (int t = 0; t < kSetupGroup; ++t)
        if (ok[t]) {
            m[0] = min(m[0], br[t].x & 0xFFFFu); m[1] = min(m[1], br[t].x >> 16);
            m[2] = min(m[2], ~(br[t].y & 0xFFFFu)); m[3] = min(m[3], ~(br[t].y >> 16));
        }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        m[i] = wave_min(m[i]);
        if (lane == 0 && m[i] != ~0u) atomicMin(&box[q][i], m[i]);
    }
    __syncthreads();
    const uint32_t ox = box[q][0], oy = box[q][1], ex = ~box[q][2], ey = ~box[q][3];
    // the other parity's box was last read before this barrier; the next round accumulates into it only
    // after one more barrier (below, or on the early paths)
    if (threadIdx.x < 4) box[q ^ 1u][threadIdx.x] = ~0u;
    if (ox == ~0u) {  // no entry in the workgroup this round
        __syncthreads();
        return;
    }
    const uint32_t w = ex - ox + 1u, cells = w * (ey - oy + 1u);
    if (cells > kBinGrid) {
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kSetupGroup; t += 2)
            bin_pair<SHADOW_QUEUES>(b, ok[t], ok[t + 1], br[t], br[t + 1], p[t], p[t + 1], nbx, bin_count, bin_list,
                                    cap, lane, nentries);
        return;
    }
#pragma unroll
    for (int t = 0; t < kSetupGroup; ++t)
        if (ok[t])
            for (uint32_t by = br[t].x >> 16; by <= (br[t].y >> 16); ++by)
                for (uint32_t bx = br[t].x & 0xFFFFu; bx <= (br[t].y & 0xFFFFu); ++bx)
                    atomicAdd(&g.cnt[(by - oy) * w + bx - ox], 1u);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < cells; c += TRI_BLOCK) {
        const uint32_t n = g.cnt[c];
        if (n) {
            const uint32_t cy = c / w;
            const uint32_t base = atomicAdd(&bin_count[(oy + cy) * nbx + ox + (c - cy * w)], n);
            g.base[c] = base;
            if (base + n > cap) {
                if (SHADOW_QUEUES) note_shadow_bin_overflow(b, base + n);
                else note_bin_overflow(b, base + n);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kSetupGroup; ++t)
        if (ok[t])
            for (uint32_t by = br[t].x >> 16; by <= (br[t].y >> 16); ++by)
                for (uint32_t bx = br[t].x & 0xFFFFu; bx <= (br[t].y & 0xFFFFu); ++bx) {
                    const uint32_t c = (by - oy) * w + bx - ox;
                    const uint32_t pos = g.base[c] + atomicSub(&g.cnt[c], 1u) - 1u;
                    if (pos < cap) bin_list[(size_t)(by * nbx + bx) * cap + pos] = p[t];
                    ++nentries;
                }
}

// WITH_SHADOW (frames with the shadow pre-pass): the same index fetch also sets up every primitive
// for the map (oracle shadow_raster_triangle: light-NDC snaps, no culling, no clipping, guard-band
// violators dropped) and bins it into the map's own queues; clipped polygon vertices get light-space
// positions. A separate instantiation keeps that code, and its registers, out of other frames.
// ONE: a single-draw frame (fp.one_draw known set: the draw search, LDS staging and prim_vs records compile
// away)
// One set-up workgroup: chunk workgroup `bid` of `nblk`.
template <bool WITH_SHADOW, bool ONE>
__device__ __forceinline__ void setup_body(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t bid,
                                           uint32_t nblk) {
    if constexpr (WITH_SHADOW) {  // the map to 1.0 before k_shadow_raster's parts merge into it (coalesced stores)
        const uint32_t nt = fp.s_size * fp.s_size;
        for (uint32_t i = bid * TRI_BLOCK + threadIdx.x; i < nt; i += nblk * TRI_BLOCK) b.shadow_map[i] = 0x3F800000u;
    }
    __shared__ uint32_t red[2];
    __shared__ float clip_poly[kWavesPerBlock][2 * TRI_MAX_CLIP_VERTS * kClipStride];
    // Frames with a few draws: each draw's primitive base, first index, slot offset and cluster base
    // staged in LDS once per workgroup, so a primitive finds its draw and index row without the global
    // binary search -> draw record chain in front of its index fetch.
    __shared__ uint32_t dpb[kLdsDraws + 1], dfi[kLdsDraws], dvb[kLdsDraws], dcb[kLdsDraws];
    const bool lds_draws = !ONE && !fp.one_draw && fp.ndraws <= (uint32_t)kLdsDraws;
    __shared__ BinBox bin_box;
    // Row bands of single-draw frames (fp.setup_multi): a quarter of the chunks' workgroups, each owning the
    // four chunks bid + i * nblk. Wave i reads chunk i's cluster flags, and the workgroup sets up
    // and bins the visible ones in turn (a band's visible chunks are contiguous, so the stride gives each
    // workgroup at most one at N = 8, and 3/4 of the launch's mostly empty dispatches are gone).
    __shared__ uint32_t chunk_vis[TRI_BLOCK / 64];
    const bool multi = ONE && !WITH_SHADOW && fp.cull_on && fp.setup_multi;
    const auto chunk_visible = [&](uint32_t ck) {
        const uint32_t p0 = ck * (uint32_t)(TRI_BLOCK * fp.ppt);
        const uint32_t p1 = min(p0 + (uint32_t)(TRI_BLOCK * fp.ppt), fp.nprims);
        bool any = false;
        for (uint32_t c = p0 / TRI_CLUSTER_PRIMS; c <= (p1 - 1) / TRI_CLUSTER_PRIMS && !any; ++c) any = b.cvis[c] != 0u;
        return any;
    };
    if constexpr (ONE && !WITH_SHADOW) {
        if (multi) {
            const uint32_t w = threadIdx.x / 64u, ck = bid + w * nblk;
            const bool vis = ck < fp.nchunks && chunk_visible(ck);
            if ((threadIdx.x & 63u) == 0) chunk_vis[w] = vis ? 1u : 0u;
            __syncthreads();
            bool any = false;
#pragma unroll
            for (int i = 0; i < TRI_BLOCK / 64; ++i) any = any || chunk_vis[i] != 0u;
            if (!any) {
                if (threadIdx.x == 0) b.setup_stats[bid] = make_uint2(0u, 0u);
                return;
            }
        } else if (fp.cull_on) {
            // A row band's chunk whose clusters k_vertex culled (most chunks at N = 8): the whole workgroup
            // leaves before the LDS set-up and the binning barriers (its cluster flags: a few scalar loads)
            if (!chunk_visible((uint32_t)(((uint64_t)bid * fp.chunk_stride) % fp.nchunks))) {
                if (threadIdx.x == 0) b.setup_stats[bid] = make_uint2(0u, 0u);
                return;
            }
        }
    }
    for (uint32_t s = threadIdx.x; s < kBinGrid; s += TRI_BLOCK) bin_box.cnt[s] = 0;
    if (threadIdx.x < 16) bin_box.box[threadIdx.x >> 3][(threadIdx.x >> 2) & 1][threadIdx.x & 3] = ~0u;
    TRI_SSTAMP(0);
    if (threadIdx.x < 2) red[threadIdx.x] = 0;
    if (lds_draws) {
        for (uint32_t i = threadIdx.x; i <= fp.ndraws; i += TRI_BLOCK) dpb[i] = b.draw_pbase[i];
        for (uint32_t i = threadIdx.x; i < fp.ndraws; i += TRI_BLOCK) {
            dfi[i] = (uint32_t)b.draws[i].first_index;
            dvb[i] = b.draw_vbase[i] - b.draws[i].min_index;
            dcb[i] = fp.cull_on ? b.draw_cbase[i] : 0u;
        }
    }
    __syncthreads();
    uint32_t nsetup = 0, nentries = 0, sentries = 0;
    const uint32_t lane = lanes_below(~0ull);
    const SetupBufs sbuf{rec_buf(b.snap, 16u, fp.nslots), make_rsrc(b.oc, fp.nslots)};
    const RecBuf ibuf = rec_buf(b.indices + fp.draw0.first_index, 12u, fp.nprims);  // single-draw frames
    uint32_t round_base = 0;  // binning rounds so far (the bin box alternates its two halves per round)
    for (uint32_t ci = 0; ci < (multi ? (uint32_t)(TRI_BLOCK / 64) : 1u); ++ci) {
    if (multi && !chunk_vis[ci]) continue;  // uniform
    // Spread concurrently running workgroups over the primitive stream: meshes are usually
    // index-ordered in screen space, and neighbouring chunks hammering the same bin counters
    // serialise their atomics. The stride is coprime to nchunks, so the remap is a bijection.
    const uint32_t chunk = multi ? bid + ci * nblk : (uint32_t)(((uint64_t)bid * fp.chunk_stride) % fp.nchunks);
    const uint32_t chunk0 = chunk * (uint32_t)(TRI_BLOCK * fp.ppt);
    // Two primitives per lane, set up and binned together: both index/vertex fetch chains are in
    // flight at once, and the queue reservations of both are batched (one atomic round trip per
    // batch), so a wave's dependent latencies are paid once for two primitives.
    for (int k = 0; k < fp.ppt; k += kSetupGroup) {  // uniform trip count: binning needs the whole workgroup
        uint32_t p[kSetupGroup], sl0[kSetupGroup], sl1[kSetupGroup], sl2[kSetupGroup];
        bool ok[kSetupGroup], needs_clip[kSetupGroup], sok[kSetupGroup];
        int pd[kSetupGroup];  // the primitive's draw
        uint2 br[kSetupGroup], sbr[kSetupGroup];
#pragma unroll
        for (int t = 0; t < kSetupGroup; ++t) {
            const bool in_chunk = k + t < fp.ppt;  // ppt need not be a multiple of the group
            p[t] = in_chunk ? chunk0 + (k + t) * TRI_BLOCK + threadIdx.x : ~0u;
            ok[t] = false; needs_clip[t] = false; sok[t] = false;
            sl0[t] = sl1[t] = sl2[t] = 0;
            br[t] = make_uint2(0u, 0u);
            sbr[t] = make_uint2(0u, 0u);
            bool culled = false;
            int& d = pd[t];
            d = 0;
            uint32_t vb = 0, i0 = 0, i1 = 0, i2 = 0;
            if (p[t] < fp.nprims) {
                // the indices are fetched together with the cluster flag, not after it: a band's
                // visible primitives skip one dependent load (a culled one wastes 12 bytes)
                const uint32_t* ip;
                if (ONE || fp.one_draw) {  // kernel-argument constants: the index fetch starts at once
                    vb = 0u - fp.draw0.min_index;
                    if (TRI_SETUP_RSRC) {
                        const u32x3v q = rec96<12>(ibuf, p[t], 0u);
                        i0 = q[0]; i1 = q[1]; i2 = q[2];
                    } else {
                        ip = b.indices + fp.draw0.first_index + 3u * p[t];
                        i0 = ip[0]; i1 = ip[1]; i2 = ip[2];
                    }
                    if (fp.cull_on) culled = !b.cvis[p[t] / TRI_CLUSTER_PRIMS];
                } else if (lds_draws) {
                    d = find_range_lds(dpb, (int)fp.ndraws, p[t]);
                    const uint32_t lp = p[t] - dpb[d];
                    ip = b.indices + dfi[d] + 3u * lp;
                    vb = dvb[d];
                    i0 = ip[0]; i1 = ip[1]; i2 = ip[2];
                    if (fp.cull_on) culled = !b.cvis[dcb[d] + lp / TRI_CLUSTER_PRIMS];
                } else {
                    d = find_range(b.draw_pbase, (int)fp.ndraws, p[t]);
                    const TriDrawDev& dr = b.draws[d];
                    const uint32_t lp = p[t] - b.draw_pbase[d];
                    ip = b.indices + dr.first_index + 3u * lp;
                    vb = b.draw_vbase[d] - dr.min_index;
                    i0 = ip[0]; i1 = ip[1]; i2 = ip[2];
                    if (fp.cull_on) culled = !b.cvis[b.draw_cbase[d] + lp / TRI_CLUSTER_PRIMS];
                }
            }
            // a primitive culled for the context's rows may still cast a shadow into the map
            if (p[t] < fp.nprims && (!culled || WITH_SHADOW)) {
                sl0[t] = vb + i0; sl1[t] = vb + i1; sl2[t] = vb + i2;
                if (!culled) {
                    const TriSnap a0 = setup_snap(sbuf, b, sl0[t]), a1 = setup_snap(sbuf, b, sl1[t]),
                                  a2 = setup_snap(sbuf, b, sl2[t]);
                    const uint32_t oc0 = setup_oc(sbuf, b, a0, sl0[t]), oc1 = setup_oc(sbuf, b, a1, sl1[t]),
                                   oc2 = setup_oc(sbuf, b, a2, sl2[t]);
                    // invalid vertex, or trivial reject: all three vertices outside one clip half-space
                    if (!((oc0 | oc1 | oc2) & TRI_OC_BAD) && !(oc0 & oc1 & oc2 & TRI_OC_REJECT)) {
                        if ((oc0 | oc1 | oc2) & TRI_OC_CLIP) {
                            needs_clip[t] = true;
                        } else {
                            const int32_t X[3] = {snap_X(a0), snap_X(a1), snap_X(a2)};
                            const int32_t Y[3] = {snap_Y(a0), snap_Y(a1), snap_Y(a2)};
                            const float z[3] = {a0.z, a1.z, a2.z};
                            const float iw[3] = {a0.iw, a1.iw, a2.iw};
                            TriRec r;
                            ok[t] = setup_snapped(fp, X, Y, z, iw, sl0[t], sl1[t], sl2[t], p[t] << 3, r, br[t]);
                        }
                    }
                }
                if constexpr (WITH_SHADOW) {
                    const TriSnap l0 = b.lsnap[sl0[t]], l1 = b.lsnap[sl1[t]], l2 = b.lsnap[sl2[t]];
                    const uint32_t oc0 = (uint32_t)l0.xo >> 24, oc1 = (uint32_t)l1.xo >> 24, oc2 = (uint32_t)l2.xo >> 24;
                    if (!((oc0 | oc1 | oc2) & (TRI_OC_BAD | TRI_OC_CLIP)) && !(oc0 & oc1 & oc2 & TRI_OC_REJECT)) {
                        const int32_t X[3] = {(l0.xo << 8) >> 8, (l1.xo << 8) >> 8, (l2.xo << 8) >> 8};
                        const int32_t Y[3] = {l0.y, l1.y, l2.y};
                        sok[t] = shadow_bins(fp, X, Y, sbr[t]);
                    }
                }
                // k_raster's (and k_shadow_raster's) route from the primitive to its vertex slots and draw; a
                // single-draw frame finds the slots in the index buffer instead (prim_slots)
                if (!ONE && !fp.one_draw && !(TRI_IDX_ROUTE && fp.idx_route) && (ok[t] || needs_clip[t] || sok[t]))
                    b.prim_vs[p[t]] = make_uint4(sl0[t], sl1[t], sl2[t], (uint32_t)d | (needs_clip[t] ? TRI_PRIM_CLIPPED : 0u));
            }
            nsetup += ok[t] ? 1u : 0u;
        }
        if (k == 0) TRI_SSTAMP(1);
#pragma unroll
        for (int t = 0; t < kSetupGroup; ++t) {
            uint64_t cm = __ballot(needs_clip[t]);  // rare: the wave clips its primitives one at a time
            if (cm) {
                if (lane == 0) atomicAdd(&b.counters->tris_clipped, (uint32_t)__builtin_popcountll(cm));
                TRI_LDS float* poly = (TRI_LDS float*)clip_poly[threadIdx.x >> 6];
                while (cm) {
                    const int src = __builtin_ctzll(cm);
                    cm &= cm - 1;
                    clip_prim_wave<WITH_SHADOW, ONE>(fp, b, poly, (uint32_t)__builtin_amdgcn_readlane((int)p[t], src),
                                                (uint32_t)__builtin_amdgcn_readlane((int)sl0[t], src),
                                                (uint32_t)__builtin_amdgcn_readlane((int)sl1[t], src),
                                                (uint32_t)__builtin_amdgcn_readlane((int)sl2[t], src),
                                                (ONE || fp.one_draw) ? fp.draw0.clip_from_world != 0u
                                                            : b.draws[__builtin_amdgcn_readlane(pd[t], src)].clip_from_world != 0u,
                                                (ONE || fp.one_draw) ? 0u : (uint32_t)__builtin_amdgcn_readlane(pd[t], src),
                                                nsetup, nentries);
                }
            }
        }
        bin_pair_box<false>(b, bin_box, round_base + (uint32_t)(k / kSetupGroup), ok, br, p, (uint32_t)fp.nbx,
                            b.bin_count, b.bin_list, fp.bin_cap, lane, nentries);
        if constexpr (WITH_SHADOW)
            bin_pair_box<true>(b, bin_box, round_base + (uint32_t)(k / kSetupGroup), sok, sbr, p, fp.s_nbx,
                               b.sbin_count, b.sbin_list, fp.s_bin_cap, lane, sentries);
        if (k == 0) TRI_SSTAMP(2);
    }
    round_base += (uint32_t)((fp.ppt + kSetupGroup - 1) / kSetupGroup);
    }
    if (nsetup) atomicAdd(&red[0], nsetup);
    if (nentries) atomicAdd(&red[1], nentries);
    __syncthreads();
    // Statistics go to a per-workgroup slot with a plain store: same-address global atomics from
    // every workgroup serialise across the XCDs (measured: +34 us per frame at 4K/1M).
    if (threadIdx.x == 0) b.setup_stats[bid] = make_uint2(red[0], red[1]);
    TRI_SSTAMP(3);
}

// TRI_SETUP_WAVES_ONE: the single-draw instantiation without the pre-pass (C2, C3) within 64 VGPRs, so that each of its
// waves takes exactly one raster wave's registers from a concurrent frame's k_raster (8 waves x 64 fill a SIMD's
// register file) instead of 72 — with 3 of its workgroups per CU (TRI_SETUP_WGS_PER_CU_OVERLAP) C3 +0.6 % (round 6 A/B)
#ifndef TRI_SETUP_WAVES_ONE
#define TRI_SETUP_WAVES_ONE 8
#endif
template <bool WITH_SHADOW, bool ONE>
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu((ONE && !WITH_SHADOW) ? TRI_SETUP_WAVES_ONE : TRI_SETUP_WAVES))) void k_setup(TRI_KARGS) {
    TRI_BIND_ARGS;
    setup_body<WITH_SHADOW, ONE>(fp, b, blockIdx.x, gridDim.x);
}


// ------------------------------------------------------------------------------------------
// tile_raster_shade: coverage
// ------------------------------------------------------------------------------------------
struct EdgeSetup {
    int32_t A[3], B[3];
    int64_t D[3];
    float dzdX, dzdY;
};

// Mirrors oracle setup_triangle()'s edge / depth-plane derivation.
__device__ __forceinline__ void edge_setup(const TriRec& r, EdgeSetup& e) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int i = k, j = (k + 1) % 3;
        const int32_t a = r.Y[i] - r.Y[j];
        const int32_t bb = r.X[j] - r.X[i];
        const int64_t c = -((int64_t)a * r.X[i] + (int64_t)bb * r.Y[i]);
        const bool tl = (a > 0) || (a == 0 && bb > 0);
        const int64_t cp = c + 128 * (int64_t)a + 128 * (int64_t)bb - (tl ? 0 : 1);
        e.A[k] = a;
        e.B[k] = bb;
        e.D[k] = cp >> 8;
    }
    const int64_t S = (int64_t)(r.X[1] - r.X[0]) * (int64_t)(r.Y[2] - r.Y[0]) -
                      (int64_t)(r.Y[1] - r.Y[0]) * (int64_t)(r.X[2] - r.X[0]);
    const float fX1 = (float)(r.X[1] - r.X[0]), fY1 = (float)(r.Y[1] - r.Y[0]);
    const float fX2 = (float)(r.X[2] - r.X[0]), fY2 = (float)(r.Y[2] - r.Y[0]);
    const float fS = (float)S;
    const float dz1 = r.z[1] - r.z[0], dz2 = r.z[2] - r.z[0];
    const RcpRef rS = rcp_ref(fS);
    e.dzdX = div_rn(dz1 * fY2 - dz2 * fY1, rS);
    e.dzdY = div_rn(dz2 * fX1 - dz1 * fX2, rS);
}

__device__ __forceinline__ int32_t clamp_edge(int64_t f, bool& reject) {
    constexpr int64_t kLim = (1ll << 30) - 1;
    if (f < -kLim) { reject = true; return -1; }
    return (int32_t)(f > kLim ? kLim : f);
}

__device__ __forceinline__ TriRec load_rec(const TriRec* recs, uint32_t i) {
    const uint4* p = reinterpret_cast<const uint4*>(recs + i);
    const uint4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];  // field by field: stays in registers
    TriRec r;
    r.X[0] = (int32_t)q0.x; r.X[1] = (int32_t)q0.y; r.X[2] = (int32_t)q0.z;
    r.Y[0] = (int32_t)q0.w; r.Y[1] = (int32_t)q1.x; r.Y[2] = (int32_t)q1.y;
    r.z[0] = __uint_as_float(q1.z); r.z[1] = __uint_as_float(q1.w); r.z[2] = __uint_as_float(q2.x);
    r.iw[0] = __uint_as_float(q2.y); r.iw[1] = __uint_as_float(q2.z); r.iw[2] = __uint_as_float(q2.w);
    r.prim_sub = q3.x;
    r.v[0] = q3.y; r.v[1] = q3.z; r.v[2] = q3.w;
    return r;
}

// The record setup_snapped produced for an unclipped primitive (v1 <-> v2 swapped), rebuilt from
// its snapped vertices instead of being stored and re-read.
__device__ __forceinline__ TriRec rec_from_snaps(uint32_t p, const uint32_t sl[3], const TriSnap& a0,
                                                 const TriSnap& a1, const TriSnap& a2) {
    TriRec r;
    r.X[0] = snap_X(a0); r.X[1] = snap_X(a2); r.X[2] = snap_X(a1);
    r.Y[0] = snap_Y(a0); r.Y[1] = snap_Y(a2); r.Y[2] = snap_Y(a1);
    r.z[0] = a0.z; r.z[1] = a2.z; r.z[2] = a1.z;
    r.iw[0] = a0.iw; r.iw[1] = a2.iw; r.iw[2] = a1.iw;
    r.v[0] = sl[0]; r.v[1] = sl[2]; r.v[2] = sl[1];
    r.prim_sub = p << 3;
    return r;
}

// The vertex slots and draw of primitive p: on a single-draw frame straight from the index buffer (slot =
// index - min_index, as k_setup computed them; k_setup writes no prim_vs then), else its prim_vs record.
// ONE (k_raster_plain's single-draw, 1x1-texture instantiation): fp.one_draw and fp.shade_solid are known
// to be set, so the other paths and their uniform flags compile away.
// IDX: the instantiation may take the index route (not the shadow pre-pass's kernels: the draw search cost the C5
// fragment stage 4 spilled VGPRs and 1.3 % of C5's frame rate, more than the records' writes it saves; the host
// keeps idx_route off on shadow frames)
template <bool ONE = false, bool IDX = true>
__device__ __forceinline__ void prim_slots(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t p,
                                           uint32_t sl[3], uint32_t& d) {
    if (ONE || fp.one_draw) {
        const u32x3v q = rec96<12>(rec_buf(b.indices + fp.draw0.first_index, 12u, fp.nprims), p, 0u);
        sl[0] = q[0] - fp.draw0.min_index; sl[1] = q[1] - fp.draw0.min_index; sl[2] = q[2] - fp.draw0.min_index;
        d = 0;
    } else if (IDX && TRI_IDX_ROUTE && fp.idx_route) {  // (uniform) the index triple, the draw from the primitive bases
        const u32x3v q = rec96<12>(rec_buf(b.indices + fp.idx_k, 12u, fp.nprims), p, 0u);
        // the first active lane's draw by a scalar search; when every lane's primitive lies in it (a wave's pixels
        // are mostly one draw's) the draw and its slot offset stay scalar, else a compare-and-select per draw
        const uint32_t p0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p);
        uint32_t d0 = 0;
        while (d0 + 1 < fp.ndraws && p0 >= fp.pbase[d0 + 1]) ++d0;
        const uint32_t hi = d0 + 1 < fp.ndraws ? fp.pbase[d0 + 1] : ~0u;
        uint32_t dd = d0, v = fp.vbd[d0];
        if (__ballot(p < fp.pbase[d0] || p >= hi) != 0ull) {
            dd = 0;
            v = fp.vbd[0];
            for (uint32_t i = 1; i < fp.ndraws; ++i) {  // uniform trip count, scalar operands
                const bool ge = p >= fp.pbase[i];
                dd = ge ? i : dd;
                v = ge ? fp.vbd[i] : v;
            }
        }
        sl[0] = q[0] + v; sl[1] = q[1] + v; sl[2] = q[2] + v;
        d = dd;
    } else {
        const uint4 pv = rec128<16>(rec_buf(b.prim_vs, 16u, fp.nprims), p, 0u);
        sl[0] = pv.x; sl[1] = pv.y; sl[2] = pv.z;
        d = pv.w & ~TRI_PRIM_CLIPPED;
    }
}

// Whether an instantiation carries the index route's draw search (prim_slots' IDX): the shadow instantiations only with
// TRI_IDX_ROUTE_SHADOW (raster_launch.h; the host enables the route on shadow frames under the same switch)
template <bool SHADOW>
constexpr bool kIdxOk = !SHADOW || TRI_IDX_ROUTE_SHADOW;

// A bin-queue entry -> its triangle (and the primitive's draw: 0 for a clipped entry, whose record names its slots).
template <bool ONE = false, bool IDX = true>
__device__ __forceinline__ TriRec load_entry_d(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t e, uint32_t& d) {
    d = 0;
    if (e & TRI_ENTRY_CLIPPED) return load_rec(b.recs, e & ~TRI_ENTRY_CLIPPED);
    const FetchBufs fb = fetch_bufs(fp, b);
    uint32_t sl[3];
    prim_slots<ONE, IDX>(fp, b, e, sl, d);
    return rec_from_snaps(e, sl, ld_snap(fb, sl[0]), ld_snap(fb, sl[1]), ld_snap(fb, sl[2]));
}
template <bool ONE = false, bool IDX = true>
__device__ __forceinline__ TriRec load_entry(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t e) {
    uint32_t d;
    return load_entry_d<ONE, IDX>(fp, b, e, d);
}

// Fragment depth at pixel centre: plane through the snapped vertices, fixed evaluation order.
__device__ __forceinline__ float frag_depth(const TriRec& r, const EdgeSetup& e, int32_t px, int32_t py) {
    const float fdx = (float)(256 * px + 128 - r.X[0]);
    const float fdy = (float)(256 * py + 128 - r.Y[0]);
    const float t1 = e.dzdX * fdx;
    const float t2 = e.dzdY * fdy;
    return (r.z[0] + t1) + t2;
}

// The far-plane test and the [0, 1] depth clamp on the float's bit pattern. Depth is finite here (the
// plane comes from snapped vertices with w >= WMIN and S != 0); non-negative floats order like their
// bits, and a negative depth (sign bit set, -0.0 included) clamps to +0.0 exactly like
// `if (!(z > 0)) z = 0`. One v_med3_i32 instead of two float compares and selects.
__device__ __forceinline__ bool depth_key(float z, bool far_clip, uint32_t lowbits, uint64_t& key) {
    const int32_t zb = __float_as_int(z);
    if (far_clip && zb > 0x3F800000) return false;  // per-pixel far-plane (z <= w) clip: z > 1
    key = ((uint64_t)(uint32_t)min(max(zb, 0), 0x3F800000) << 32) | lowbits;
    return true;
}

__device__ __forceinline__ void rec_bbox(const TriRec& r, int32_t ox, int32_t oy, int32_t bw, int32_t bh, int32_t& cx0,
                                         int32_t& cx1, int32_t& cy0, int32_t& cy1) {
    const int32_t xmin = min(r.X[0], min(r.X[1], r.X[2])), xmax = max(r.X[0], max(r.X[1], r.X[2]));
    const int32_t ymin = min(r.Y[0], min(r.Y[1], r.Y[2])), ymax = max(r.Y[0], max(r.Y[1], r.Y[2]));
    cx0 = max(-floor_shift8(128 - xmin), ox);
    cx1 = min(floor_shift8(xmax - 128), ox + bw - 1);
    cy0 = max(-floor_shift8(128 - ymin), oy);
    cy1 = min(floor_shift8(ymax - 128), oy + bh - 1);
}

__device__ __forceinline__ uint32_t key_low(uint32_t prim_sub) {
    return ((TRI_PRIM_MAX - (prim_sub >> 3)) << 3) | (prim_sub & 7u);
}

// TRI_QTAB (A/B): in a bin of at most kQtab entries on a frame of at most 2^20 primitives, a key's low
// word carries the winning entry's queue position as a payload BELOW its primitive order:
//   low = (kQPrimMax - prim) << 11 | sub << 8 | queue position
// so the minimum still resolves depth ties by primitive order exactly as key_low does (the position only separates
// entries of one primitive, which never share a pixel), and the fragment finds the entry's vertex slots in an LDS
// table the coverage pass filled, instead of gathering its index triple. No hash and no sort. The coverage code takes
// the record's prim_sub re-encoded so that key_low() of it yields this word (qenc).
#ifndef TRI_QTAB
#define TRI_QTAB 1
#endif
// TRI_QTAB_SHADOW: the shadow instantiation keeps the table too, with each entry's draw as a fourth word (its
// fragments then gather no 16-B prim_vs record)
#ifndef TRI_QTAB_SHADOW
#define TRI_QTAB_SHADOW 1
#endif
constexpr uint32_t kQtab = 256, kQPrimMax = (1u << 20) - 1u;
__device__ __forceinline__ uint32_t qenc(uint32_t prim_sub, uint32_t qpos) {
    const uint32_t low = ((kQPrimMax - (prim_sub >> 3)) << 11) | ((prim_sub & 7u) << 8) | qpos;
    return (TRI_PRIM_MAX - (low >> 3)) << 3 | (low & 7u);  // key_low() of this is `low`
}

// Edge values at pixel (cx0, cy0) of the triangle's clipped bbox, the edge steps and the depth plane.
// A triangle under 64 px on a side (the common case) takes 32-bit arithmetic: |a|, |b| < 2^14 and every
// pixel centre of its bbox lies within 2^14 of each vertex, so a (Xc - Xi) + b (Yc - Yi) - bias fits int32
// and its floor division by 256 is the 64-bit form's A cx0 + B cy0 + D exactly (no clamp can trigger);
// the area is the same exact integer, so the depth plane gets the same floats. Returns false when the
// 64-bit form rejects the triangle.
__device__ __forceinline__ bool edge_start(const TriRec& r, int32_t cx0, int32_t cy0, int32_t A[3], int32_t B[3],
                                          int32_t F[3], float& dzdX, float& dzdY) {
    const int32_t xmin = min(r.X[0], min(r.X[1], r.X[2])), xmax = max(r.X[0], max(r.X[1], r.X[2]));
    const int32_t ymin = min(r.Y[0], min(r.Y[1], r.Y[2])), ymax = max(r.Y[0], max(r.Y[1], r.Y[2]));
    if (xmax - xmin < 16384 && ymax - ymin < 16384) {
        const int32_t Xc = 256 * cx0 + 128, Yc = 256 * cy0 + 128;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int i = k, j = (k + 1) % 3;
            const int32_t a = r.Y[i] - r.Y[j];
            const int32_t bb = r.X[j] - r.X[i];
            const bool tl = (a > 0) || (a == 0 && bb > 0);
            A[k] = a;
            B[k] = bb;
            F[k] = (__mul24(a, Xc - r.X[i]) + __mul24(bb, Yc - r.Y[i]) - (tl ? 0 : 1)) >> 8;
        }
        const int32_t X1 = r.X[1] - r.X[0], Y1 = r.Y[1] - r.Y[0], X2 = r.X[2] - r.X[0], Y2 = r.Y[2] - r.Y[0];
        const float fS = (float)(__mul24(X1, Y2) - __mul24(Y1, X2));
        const float fX1 = (float)X1, fY1 = (float)Y1, fX2 = (float)X2, fY2 = (float)Y2;
        const float dz1 = r.z[1] - r.z[0], dz2 = r.z[2] - r.z[0];
        const RcpRef rS = rcp_ref(fS);
        dzdX = div_rn(dz1 * fY2 - dz2 * fY1, rS);
        dzdY = div_rn(dz2 * fX1 - dz1 * fX2, rS);
        return true;
    }
    EdgeSetup e;
    edge_setup(r, e);
    bool rej = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        A[k] = e.A[k];
        B[k] = e.B[k];
        F[k] = clamp_edge((int64_t)e.A[k] * cx0 + (int64_t)e.B[k] * cy0 + e.D[k], rej);
    }
    dzdX = e.dzdX;
    dzdY = e.dzdY;
    return !rej;
}

// Rows cy0 + sub, cy0 + sub + step, ... of the bbox (sub < step: `step` lanes share a triangle). The
// row starts are stepped exactly (integer edge values; float offsets in multiples of 256), so any
// split gives the same keys as one lane walking every row.
template <int BL>
__device__ __forceinline__ void raster_serial(const TriRec& r, int32_t cx0, int32_t cx1, int32_t cy0, int32_t cy1,
                                              int32_t ox, int32_t oy, uint64_t* keys, int32_t sub = 0,
                                              int32_t step = 1) {
    struct {
        int32_t A[3], B[3];
        float dzdX, dzdY;
    } e;
    int32_t F[3];
    if (!edge_start(r, cx0, cy0, e.A, e.B, F, e.dzdX, e.dzdY)) return;
    const bool far_clip = (r.z[0] > 1.0f) || (r.z[1] > 1.0f) || (r.z[2] > 1.0f);
    const uint32_t low = key_low(r.prim_sub);
    // frag_depth's pixel offsets stepped incrementally: |256 p + 128 - X0| < 2^24, so the float steps
    // of 256 are exact and equal its int -> float conversions; same (z0 + dzdX dx) + dzdY dy order
    const float fdx0 = (float)(256 * cx0 + 128 - r.X[0]);
    float fdy = (float)(256 * (cy0 + sub) + 128 - r.Y[0]);
    uint32_t row = (uint32_t)(((cy0 + sub - oy) << BL) + (cx0 - ox));
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] += e.B[k] * sub;
    for (int32_t py = cy0 + sub; py <= cy1; py += step) {
        const float t2 = e.dzdY * fdy;
        int32_t f0 = F[0], f1 = F[1], f2 = F[2];
        float fdx = fdx0;
        const uint32_t rend = row + (uint32_t)(cx1 - cx0);
        for (uint32_t a = row; a <= rend; ++a) {
            if ((f0 | f1 | f2) >= 0) {
                uint64_t key;
                if (depth_key((r.z[0] + e.dzdX * fdx) + t2, far_clip, low, key)) atomicMin(&keys[a], key);
            }
            f0 += e.A[0]; f1 += e.A[1]; f2 += e.A[2];
            fdx += 256.0f;
        }
        F[0] += e.B[0] * step; F[1] += e.B[1] * step; F[2] += e.B[2] * step;
        fdy += 256.0f * (float)step;
        row += (uint32_t)step << BL;
    }
}

// Span walk (the per-lane path of 32x32 bins, triangles under 64 px on a side): each row's covered pixels
// are the integer x with f_k(x) = F_k + A_k (x - cx0) >= 0 for k = 0..2, an interval [L, R] found from the
// three crossings v_k = -F_k / A_k instead of testing every bbox pixel (the bbox of a C3 triangle is ~3x
// its area). Exact: with |A_k| < 2^14, |F_k| < 2^22 (exact in float, and stepped by B_k exactly) and v_rcp's 1-ulp
// reciprocal, t = fma(-F, 1/A, -/+delta) lies within 2^-16 of v -/+ delta for |v| <= 64, and a
// non-integer v is at least 1/|A| > 2^-14 from every integer, so with delta = 2^-15 ceil(t) = ceil(v) on
// the left (A > 0) and floor(t) = floor(v) on the right (A < 0), integer v included; crossings further
// than 64 px lie outside the 32-px bin either way. A horizontal edge (A = 0) empties the row when F < 0
// (scale 2^100 on the left side). Then the same keys as raster_serial over [L, R] only.
template <int BL>
__device__ __forceinline__ void raster_span(const TriRec& r, int32_t cx0, int32_t cx1, int32_t cy0, int32_t cy1,
                                            int32_t ox, int32_t oy, uint64_t* keys, int32_t sub = 0,
                                            int32_t step = 1) {
    const int32_t xmin = min(r.X[0], min(r.X[1], r.X[2])), xmax = max(r.X[0], max(r.X[1], r.X[2]));
    const int32_t ymin = min(r.Y[0], min(r.Y[1], r.Y[2])), ymax = max(r.Y[0], max(r.Y[1], r.Y[2]));
    if (!(xmax - xmin < 16384 && ymax - ymin < 16384)) {
        raster_serial<BL>(r, cx0, cx1, cy0, cy1, ox, oy, keys, sub, step);
        return;
    }
    int32_t A[3], B[3], F[3];
    float dzdX, dzdY;
    edge_start(r, cx0, cy0, A, B, F, dzdX, dzdY);  // the 32-bit form: never rejects
    constexpr float kDelta = 0x1p-15f;
    float nrl[3], dl[3], nrr[3], dr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float rc = -__builtin_amdgcn_rcpf((float)A[k]);
        nrl[k] = A[k] > 0 ? rc : (A[k] == 0 ? -0x1p100f : 0.0f);
        dl[k] = A[k] >= 0 ? -kDelta : -INFINITY;
        nrr[k] = A[k] < 0 ? rc : 0.0f;
        dr[k] = A[k] < 0 ? kDelta : INFINITY;
    }
    const bool far_clip = (r.z[0] > 1.0f) || (r.z[1] > 1.0f) || (r.z[2] > 1.0f);
    const uint32_t low = key_low(r.prim_sub);
    const float wmax = (float)(cx1 - cx0);
    const int32_t fx0 = 256 * cx0 + 128 - r.X[0];
    float fdy = (float)(256 * (cy0 + sub) + 128 - r.Y[0]);
    uint32_t row = (uint32_t)(((cy0 + sub - oy) << BL) + (cx0 - ox));
    // the edge values stay exact integers below 2^22 over the bbox: stepped in float without rounding
    float Ff[3], Bs[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        Ff[k] = (float)(F[k] + B[k] * sub);
        Bs[k] = (float)(B[k] * step);
    }
    for (int32_t py = cy0 + sub; py <= cy1; py += step) {
        const float f0 = Ff[0], f1 = Ff[1], f2 = Ff[2];
        const float tl = fmaxf(fmaxf(__builtin_fmaf(f0, nrl[0], dl[0]), __builtin_fmaf(f1, nrl[1], dl[1])),
                               __builtin_fmaf(f2, nrl[2], dl[2]));
        const float tr = fminf(fminf(__builtin_fmaf(f0, nrr[0], dr[0]), __builtin_fmaf(f1, nrr[1], dr[1])),
                               __builtin_fmaf(f2, nrr[2], dr[2]));
        const float Lf = fmaxf(ceilf(tl), 0.0f), Rf = fminf(floorf(tr), wmax);
        if (Lf <= Rf) {  // both in [0, wmax] here: the conversions are exact
            const int32_t L = (int32_t)Lf, R = (int32_t)Rf;
            const float t2 = dzdY * fdy;
            float fdx = (float)(fx0 + 256 * L);
            const uint32_t rend = row + (uint32_t)R;
            if (!far_clip) {  // (nearly every triangle: no per-pixel far-plane test)
                for (uint32_t a = row + (uint32_t)L; a <= rend; ++a) {
                    uint64_t key;
                    depth_key((r.z[0] + dzdX * fdx) + t2, false, low, key);
                    atomicMin(&keys[a], key);
                    fdx += 256.0f;
                }
            } else {
                for (uint32_t a = row + (uint32_t)L; a <= rend; ++a) {
                    uint64_t key;
                    if (depth_key((r.z[0] + dzdX * fdx) + t2, true, low, key)) atomicMin(&keys[a], key);
                    fdx += 256.0f;
                }
            }
        }
        Ff[0] += Bs[0]; Ff[1] += Bs[1]; Ff[2] += Bs[2];
        fdy += 256.0f * (float)step;
        row += (uint32_t)step << BL;
    }
}

// ------------------------------------------------------------------------------------------
// tile_raster_shade: Default.frag
// ------------------------------------------------------------------------------------------
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 muls(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f3 norm3(f3 v) { return muls(v, 1.0f / sqrtf(dot3(v, v))); }

// fast-path primitives (hardware v_rcp / v_rsq / v_exp / v_log, explicit FMA)
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fdot(f3 a, f3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
__device__ __forceinline__ f3 fnorm(f3 v) { return muls(v, frsq(fdot(v, v))); }
__device__ __forceinline__ float fpow(float x, float y) {  // x >= 0
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}
__device__ __forceinline__ float sat(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

__device__ __forceinline__ uint32_t wrap_repeat(float f, uint32_t n) {  // REPEAT addressing of floor(f)
    const int32_t i = (int32_t)fminf(fmaxf(f, -1.0e9f), 1.0e9f);
    if ((n & (n - 1)) == 0) return (uint32_t)i & (n - 1);  // power-of-two size: the mask is the modulo
    int32_t r = i % (int32_t)n;                             // (two's complement: negative i wraps too)
    if (r < 0) r += (int32_t)n;
    return (uint32_t)r;
}

// TRI_TEXEL_PAIRS / TRI_MAP_PAIRS: the bilinear footprint of a texture / the shadow map as two 8-B row loads
// instead of four 4-B gathers (C5's fragment stage is bound by the texture units' data return, which costs per
// load instruction)
#ifndef TRI_TEXEL_PAIRS
#define TRI_TEXEL_PAIRS 1
#endif
#ifndef TRI_MAP_PAIRS
#define TRI_MAP_PAIRS 1
#endif
// Two adjacent 4-B texels as one 8-B load (4-B aligned: a dwordx2 load needs no more)
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ u32x2a ld_pair(TRI_G const uint32_t* p) { return *reinterpret_cast<TRI_G const u32x2a*>(p); }
// texture(): R8G8B8A8_SRGB decode before LINEAR filtering, REPEAT, level 0 (Renderer.cpp:3592-3607)
__device__ __forceinline__ float4 sample_tex(const TriTexDesc& t, float u0, float v0, const float* lut) {
    if (t.w == 1 && t.h == 1)  // 1x1 (the default white slot): all four taps are texel (0,0)
        return make_float4(t.solid[0], t.solid[1], t.solid[2], t.solid[3]);
    const float u = u0 * (float)t.w - 0.5f;
    const float v = v0 * (float)t.h - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const float a = u - fu, bb = v - fv;
    const uint32_t x0 = wrap_repeat(fu, t.w), y0 = wrap_repeat(fv, t.h);
    const uint32_t x1 = (x0 + 1 == t.w) ? 0u : x0 + 1, y1 = (y0 + 1 == t.h) ? 0u : y0 + 1;
    TRI_G const uint32_t* tx = (TRI_G const uint32_t*)t.texels;  // device texture memory (global loads)
    uint32_t p00, p10, p01, p11;
    if (TRI_TEXEL_PAIRS && x1 == x0 + 1) {  // the two taps of a row are adjacent: one 8-B load per row
        const u32x2a r0 = ld_pair(tx + y0 * t.w + x0), r1 = ld_pair(tx + y1 * t.w + x0);
        p00 = r0.x; p10 = r0.y; p01 = r1.x; p11 = r1.y;
    } else {  // REPEAT wrapped x1 to column 0
        p00 = tx[y0 * t.w + x0]; p10 = tx[y0 * t.w + x1];
        p01 = tx[y1 * t.w + x0]; p11 = tx[y1 * t.w + x1];
    }
    float4 r;
    float* rp = &r.x;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        auto ch = [&](uint32_t px) -> float {
            const uint32_t by = (px >> (8 * c)) & 0xFFu;
            return lut[c == 3 ? 256 + by : by];
        };
        const float t00 = ch(p00), t10 = ch(p10), t01 = ch(p01), t11 = ch(p11);
        const float l0 = t00 + a * (t10 - t00);
        const float l1 = t01 + a * (t11 - t01);
        rp[c] = l0 + bb * (l1 - l0);
    }
    return r;
}

__device__ __forceinline__ uint32_t unorm8(float c) {
    const float cc = fminf(fmaxf(c, 0.0f), 1.0f);
    return (uint32_t)(int)(cc * 255.0f + 0.5f);
}

// Fast build's tone curve output (Default.frag:185-189 then the UNORM8 store): the channel comes back
// already scaled by 255 — 255 t^(1/2.2) as one exp2 with log2(255) folded into its argument (t = c / (c + 1)
// lies in [0, 1), so no clamp is needed), within a small fraction of an LSB of the IEEE value before rounding.
__device__ __forceinline__ float tone_out(float t) {
    constexpr float g = 1.0f / 2.2f;
    return __builtin_amdgcn_exp2f(__builtin_fmaf(g, __builtin_amdgcn_logf(t), 7.99435343685886f));
}
// The fast build's BGRA8 word from tone_out's channels (in [0, 255]) and the alpha byte. TRI_PK_U8:
// v_cvt_pk_u8_f32 rounds each channel to nearest (ties to even: it differs from floor(v + 0.5) only on an
// exact .5, inside the 1-LSB bar) and inserts it into its byte — one instruction per channel instead of a
// round, a conversion and a shift/or.
#ifndef TRI_PK_U8
#define TRI_PK_U8 1
#endif
__device__ __forceinline__ uint32_t fast_bgra(float r, float g, float b, uint32_t a8) {
    if (TRI_PK_U8)
        return __builtin_amdgcn_cvt_pk_u8_f32(r, 2u, __builtin_amdgcn_cvt_pk_u8_f32(g, 1u, __builtin_amdgcn_cvt_pk_u8_f32(b, 0u, a8 << 24)));
    auto u8 = [](float v) { return (uint32_t)(int)(v + 0.5f); };
    return u8(b) | (u8(g) << 8) | (u8(r) << 16) | (a8 << 24);
}

struct __attribute__((aligned(16))) V4 {
    float x, y, z, w;
};

struct Frag {  // flat scalars: nested f3 members are ABI-coerced and defeat SROA in the pair path
    float wx, wy, wz;  // world position
    float nx, ny, nz;  // interpolated normal
    float cx, cy, cz;  // vertex colour
    float u, v;
    float sx, sy, sz, sw;  // sampled texel (linear rgb, alpha)
    float tx, ty, tz, tw;  // draw tint
    float vis;             // shadow pre-pass: fraction of the sun's light reaching the fragment (1 without it)
};
__device__ __forceinline__ f3 fworld(const Frag& f) { return mk(f.wx, f.wy, f.wz); }
__device__ __forceinline__ f3 fnrm(const Frag& f) { return mk(f.nx, f.ny, f.nz); }
__device__ __forceinline__ f3 fvcol(const Frag& f) { return mk(f.cx, f.cy, f.cz); }
__device__ __forceinline__ f3 ftex(const Frag& f) { return mk(f.sx, f.sy, f.sz); }
__device__ __forceinline__ f3 ftint(const Frag& f) { return mk(f.tx, f.ty, f.tz); }

// ---- EXACT build: Default.frag with IEEE div/sqrt/powf in the oracle's operation order ----------
__device__ __forceinline__ float schlick_ggx(float NdotV, float roughness) {
    const float r = roughness + 1.0f;
    const float k = (r * r) / 8.0f;
    const float denom = NdotV * (1.0f - k) + k;
    return NdotV / fmaxf(denom, 1e-4f);
}

__device__ __forceinline__ f3 eval_pbr_exact(f3 L, f3 rad, f3 N, f3 V, f3 albedo, float metallic, float roughness,
                                             f3 F0) {
    const f3 H = norm3(add(V, L));
    const float a = roughness * roughness;
    const float a2 = a * a;
    const float NdotH = fmaxf(dot3(N, H), 0.0f);
    const float NdotH2 = NdotH * NdotH;
    const float dd = (NdotH2 * (a2 - 1.0f) + 1.0f);
    const float NDF = a2 / ((kPi * dd) * dd);
    const float NdotV = fmaxf(dot3(N, V), 0.0f);
    const float NdotL = fmaxf(dot3(N, L), 0.0f);
    const float G = schlick_ggx(NdotL, roughness) * schlick_ggx(NdotV, roughness);
    const float p = powf(sat(1.0f - fmaxf(dot3(H, V), 0.0f)), 5.0f);
    const f3 F = mk(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
    const f3 num = muls(F, NDF * G);
    const float den = fmaxf((4.0f * NdotV) * NdotL, 1e-4f);
    const f3 spec = mk(num.x / den, num.y / den, num.z / den);
    const f3 kD = muls(mk(1.0f - F.x, 1.0f - F.y, 1.0f - F.z), 1.0f - metallic);
    const f3 diff = mk((kD.x * albedo.x) / kPi, (kD.y * albedo.y) / kPi, (kD.z * albedo.z) / kPi);
    return muls(mul(add(diff, spec), rad), NdotL);
}

__device__ __forceinline__ float4 fs_exact(const TriFrameParams& fp, const Frag& f) {
    const tri_global_ubo& g = fp.ubo;
    const tri_material_record& mat = fp.mat0;
    const f3 N = norm3(norm3(fnrm(f)));
    const f3 V = norm3(sub3(mk(g.camera_position[0], g.camera_position[1], g.camera_position[2]), fworld(f)));
    const f3 albedo = mul(mul(mul(ftex(f), mk(mat.base_color_factor[0], mat.base_color_factor[1],
                                                               mat.base_color_factor[2])),
                              ftint(f)),
                          fvcol(f));
    const float metallic = sat(mat.material_factors[0]);
    const float roughness = fminf(fmaxf(mat.material_factors[1], 0.045f), 1.0f);
    const float amb_s = sat(mat.material_factors[2]);
    const float om = 0.04f * (1.0f - metallic);
    const f3 F0 = mk(om + albedo.x * metallic, om + albedo.y * metallic, om + albedo.z * metallic);
    f3 direct = mk(0.f, 0.f, 0.f);
    if (g.light_counts[0] > 0u) {
        const f3 L = norm3(mk(-g.directional_light_direction[0], -g.directional_light_direction[1],
                              -g.directional_light_direction[2]));
        const f3 rad = muls(muls(mk(g.directional_light_color[0], g.directional_light_color[1], g.directional_light_color[2]),
                                 g.directional_light_color[3]),
                            f.vis);
        direct = add(direct, eval_pbr_exact(L, rad, N, V, albedo, metallic, roughness, F0));
    }
    const uint32_t np = min(g.light_counts[1], 8u);
    for (uint32_t i = 0; i < np; ++i) {
        const tri_point_light& pl = g.point_lights[i];
        const f3 to = sub3(mk(pl.position_range[0], pl.position_range[1], pl.position_range[2]), fworld(f));
        const float dist = sqrtf(dot3(to, to));
        if (dist <= 1e-4f) continue;
        const f3 L = mk(to.x / dist, to.y / dist, to.z / dist);
        const float radius = fmaxf(pl.position_range[3], 1e-4f);
        const float nd = sat(dist / radius);
        float att = 1.0f - nd;
        att = att * att;
        const f3 rad = muls(muls(mk(pl.color_intensity[0], pl.color_intensity[1], pl.color_intensity[2]),
                                 pl.color_intensity[3]),
                            att);
        direct = add(direct, eval_pbr_exact(L, rad, N, V, albedo, metallic, roughness, F0));
    }
    const f3 amb = muls(mul(muls(mk(g.ambient_color_intensity[0], g.ambient_color_intensity[1],
                                    g.ambient_color_intensity[2]),
                                 g.ambient_color_intensity[3]),
                            albedo),
                        amb_s);
    f3 col = add(amb, direct);
    col = mk(col.x / (col.x + 1.0f), col.y / (col.y + 1.0f), col.z / (col.z + 1.0f));
    const float gamma = 1.0f / 2.2f;
    col = mk(powf(col.x, gamma), powf(col.y, gamma), powf(col.z, gamma));
    const float alpha = (mat.base_color_factor[3] * f.tw) * f.sw;
    return make_float4(col.x, col.y, col.z, alpha);
}

// ---- fast build: same algebra, frame constants hoisted, hardware transcendental approximations ---
// Per light: one v_rsq (half vector) and ONE v_rcp for NDF * G_L / (4 NdotV NdotL) together. For unit
// V and L, |V + L|^2 = 2 + 2 L.V, N.H = (N.V + N.L) / |V + L| and H.V = (1 + L.V) / |V + L|.
// G_V NdotL / max(4 NdotV NdotL, 1e-4) (the NDF's a2 / pi and G_L's 1 / (1 - k) folded in), the part of the
// specular weight before the per-light denominator dd^2 gden. For N.L > 0,
// NdotL / max(4 NdotV NdotL, 1e-4) = min(1 / (4 NdotV), 1e4 NdotL), so with spA = gVa / (4 NdotV) (formed
// without NdotV: a2 / (4 pi (1 - k) gden_V), finite at NdotV = 0) and spB = 1e4 gVa it is min(spA, spB NdotL):
// two operations per light instead of four, and one product fewer inside the reciprocal. TRI_SPEC_IMIN: both
// operands are non-negative and not NaN (spA > 0; spB >= 0 and N.L > 0 here), so their minimum is the integer
// minimum of their bits — v_min_i32, which needs no canonicalising v_max of spA in every light as the
// IEEE-mode v_min_f32 does.
#ifndef TRI_SPEC_IMIN
#define TRI_SPEC_IMIN 1
#endif
__device__ __forceinline__ float spec_num(float spA, float spB, float NdotL) {
    if (TRI_SPEC_IMIN) return __int_as_float(min(__float_as_int(spA), __float_as_int(spB * NdotL)));
    return fminf(spA, spB * NdotL);
}
// Point-light attenuation (1 - min(d / r, 1))^2's base, max(1 - d / r, 0) as one fma
__device__ __forceinline__ float att_base(float d, float ir) { return fmaxf(__builtin_fmaf(-d, ir, 1.0f), 0.0f); }

struct PbrPix {
    f3 N, V, F0, omF0, diffK;
    float NdotVr;   // unclamped N.V
    float spA, spB; // spec_num's per-pixel factors
};

// One light with unclamped N.L and L.V given (the caller forms them without normalising L first).
__device__ __forceinline__ void eval_pbr_fast(const TriShadeConst& sc, const PbrPix& px, float NdotLr, float LdotV,
                                              f3 rad, float scale, f3& c) {
#pragma clang fp contract(fast)  // fast build only: FMA contraction is inside the 1-LSB budget
    // N.L <= 0 makes the light's weight 0 and every term finite: c + X * 0 == c exactly, so a wave
    // whose lanes all face away skips the rest (Default.frag evaluates it to the same zero)
    if (!(NdotLr > 0.0f)) return;
    const float ih = frsq(fmaxf(__builtin_fmaf(2.0f, LdotV, 2.0f), 1e-30f));
    const float NdotH = fmaxf((px.NdotVr + NdotLr) * ih, 0.0f);
    const float NdotL = NdotLr;  // > 0 here: max(N.L, 0) is the identity
    const float dd = __builtin_fmaf(NdotH * NdotH, sc.a2m1, 1.0f);
    // Default.frag's max(., 1e-4) on G_L's denominator is the identity here: N.L > 0 and k = (r + 1)^2 / 8
    // >= 0.136 for roughness >= 0.045, so N.L (1 - k) + k >= k
    const float gden = NdotL + sc.kgo;  // G_L's denominator divided through by 1 - k (sc.a2pio carries 1 / (1 - k))
    // NDF * G_L * G_V / den with NDF = a2 / (pi dd^2), G_L = NdotL / gden
    const float sp = spec_num(px.spA, px.spB, NdotL) * frcp((dd * dd) * gden);
    // 1 - max(H.V, 0), clamped to [0, 1]: one clamped subtract
    const float q = sat(1.0f - __builtin_fmaf(LdotV, ih, ih));
    const float q2 = q * q;
    const float p5 = q2 * q2 * q;
    const float w = NdotL * scale;
    // (kD albedo / pi + F s) = diffK + F (s - diffK), F = F0 + (1 - F0) p5
    c.x = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(px.omF0.x, p5, px.F0.x), sp - px.diffK.x, px.diffK.x), rad.x * w, c.x);
    c.y = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(px.omF0.y, p5, px.F0.y), sp - px.diffK.y, px.diffK.y), rad.y * w, c.y);
    c.z = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(px.omF0.z, p5, px.F0.z), sp - px.diffK.z, px.diffK.z), rad.z * w, c.z);
}

// ONE: the texel, base colour and tint are uniform and their product is a kernel argument (sc.sbt)
// Packed colour pairs: kept for the shadow instantiation (C5 k_raster 197.4 -> 195.8 us); k_raster_plain is
// faster with scalar channels (C3 103.9 vs 105.7 us).
#ifndef TRI_PK_SHADE
#ifdef TRI_RASTER_PLAIN_TU
#define TRI_PK_SHADE 0
#else
#define TRI_PK_SHADE 1
#endif
#endif
#if TRI_PK_SHADE
// Colour channels x, y as one packed-FP32 pair (v_pk_fma_f32 / v_pk_mul_f32: two IEEE operations per
// instruction, the same bits as the scalar form) and z on its own; written out by hand, not left to the SLP
// vectoriser, so that only these values occupy register pairs (raster_plain.hip is built without SLP).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v splat(float x) { return f2v{x, x}; }
struct PbrPixP {
    f3 N, V;
    f2v F0xy, omF0xy, diffKxy;
    float F0z, omF0z, diffKz;
    float NdotVr;
    float spA, spB;
};
__device__ __forceinline__ void eval_pbr_fast_p(const TriShadeConst& sc, const PbrPixP& px, float NdotLr, float LdotV,
                                                f2v radxy, float radz, float scale, f2v& cxy, float& cz) {
#pragma clang fp contract(fast)
    if (!(NdotLr > 0.0f)) return;  // (see eval_pbr_fast)
    const float ih = frsq(fmaxf(__builtin_fmaf(2.0f, LdotV, 2.0f), 1e-30f));
    const float NdotH = fmaxf((px.NdotVr + NdotLr) * ih, 0.0f);
    const float NdotL = NdotLr;
    const float dd = __builtin_fmaf(NdotH * NdotH, sc.a2m1, 1.0f);
    // Default.frag's max(., 1e-4) on G_L's denominator is the identity here: N.L > 0 and k = (r + 1)^2 / 8
    // >= 0.136 for roughness >= 0.045, so N.L (1 - k) + k >= k
    const float gden = NdotL + sc.kgo;
    const float sp = spec_num(px.spA, px.spB, NdotL) * frcp((dd * dd) * gden);
    const float q = sat(1.0f - __builtin_fmaf(LdotV, ih, ih));
    const float q2 = q * q;
    const float p5 = q2 * q2 * q;
    const float w = NdotL * scale;
    cxy = pk_fma(pk_fma(pk_fma(px.omF0xy, splat(p5), px.F0xy), splat(sp) - px.diffKxy, px.diffKxy), radxy * splat(w), cxy);
    cz = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(px.omF0z, p5, px.F0z), sp - px.diffKz, px.diffKz), radz * w, cz);
}
#endif

// TRI_ONE_FOLD: single-draw solid frames shade from the vertex colour with host-folded factors (TriShadeConst::
// sbtm / sbtkd / sbtamb), never forming the albedo (-6 VALU per pixel)
#ifndef TRI_ONE_FOLD
#define TRI_ONE_FOLD 1
#endif
template <bool ONE = false>
__device__ __forceinline__ float4 fs_fast(const TriShadeConst& sc, const Frag& f) {
#pragma clang fp contract(fast)
#if TRI_PK_SHADE
    PbrPixP px;
    px.N = fnorm(fnrm(f));
    px.V = fnorm(sub3(mk(sc.cam[0], sc.cam[1], sc.cam[2]), fworld(f)));
    f2v albxy;
    float albz;
    if (ONE) {
        albxy = f2v{sc.sbt[0], sc.sbt[1]} * f2v{f.cx, f.cy};
        albz = sc.sbt[2] * f.cz;
    } else {
        albxy = ((f2v{f.sx, f.sy} * f2v{sc.base[0], sc.base[1]}) * f2v{f.tx, f.ty}) * f2v{f.cx, f.cy};
        albz = ((f.sz * sc.base[2]) * f.tz) * f.cz;
    }
    const float m = sc.metallic;
    const float om = sc.om;
    px.F0xy = pk_fma(albxy, splat(m), splat(om));
    px.F0z = __builtin_fmaf(albz, m, om);
    px.omF0xy = splat(1.0f) - px.F0xy;
    px.omF0z = 1.0f - px.F0z;
    const float kd = sc.kd;
    px.diffKxy = albxy * splat(kd);
    px.diffKz = albz * kd;
    px.NdotVr = fdot(px.N, px.V);
    const float NdotV = fmaxf(px.NdotVr, 0.0f);
    const float rgV = frcp(fmaxf(__builtin_fmaf(NdotV, sc.omkg, sc.kg), 1e-4f));
    px.spA = sc.spAk * rgV;                   // 0.25 a2 / pi / (1 - k) / max(G_V's denominator, 1e-4)
    px.spB = sc.spBk * (NdotV * rgV);         // 1e4 a2 / pi * G_V / (1 - k)
    f2v cxy = (f2v{sc.amb[0], sc.amb[1]} * albxy) * splat(sc.amb_strength);
    float cz = (sc.amb[2] * albz) * sc.amb_strength;
    if (kAblate & 64) return make_float4(cxy.x, cxy.y, cz, 1.0f);  // diagnostics: 64 = no lights
    if (sc.has_sun && f.vis > 0.0f) {  // vis = 0 (fully shadowed): the sun adds exactly nothing
        const f3 L = mk(sc.sun_l[0], sc.sun_l[1], sc.sun_l[2]);
        eval_pbr_fast_p(sc, px, fdot(px.N, L), fdot(L, px.V), f2v{sc.sun_rad[0], sc.sun_rad[1]}, sc.sun_rad[2], f.vis,
                        cxy, cz);
    }
    const f3 wp = fworld(f);
    for (uint32_t i = 0; i < sc.npt; ++i) {
        const f3 to = sub3(mk(sc.pl[i].pos[0], sc.pl[i].pos[1], sc.pl[i].pos[2]), wp);
        const float d2 = fdot(to, to);
        const float inv = frsq(d2);
        const float att0 = att_base(d2 * inv, sc.pl[i].pos[3]);
        if (!(d2 > 1e-8f && att0 > 0.0f)) continue;  // dist <= 1e-4, or beyond the range (see below)
        eval_pbr_fast_p(sc, px, fdot(px.N, to) * inv, fdot(to, px.V) * inv, f2v{sc.pl[i].rad[0], sc.pl[i].rad[1]},
                        sc.pl[i].rad[2], att0 * att0, cxy, cz);
    }
    const f2v c1 = cxy + splat(1.0f);
    const f2v txy = cxy * f2v{frcp(c1.x), frcp(c1.y)};
    const float tz = cz * frcp(cz + 1.0f);
    return make_float4(tone_out(txy.x), tone_out(txy.y), tone_out(tz), ONE ? sc.sbt[3] : (sc.base[3] * f.tw) * f.sw);
#else
    PbrPix px;
    px.N = fnorm(fnrm(f));
    px.V = fnorm(sub3(mk(sc.cam[0], sc.cam[1], sc.cam[2]), fworld(f)));
    const float m = sc.metallic;
    const float om = sc.om;  // 0.04 (1 - metallic), folded on the host with the other frame constants
    f3 c;
    if (ONE && TRI_ONE_FOLD) {  // albedo = sbt * colour: every term from the colour and a folded factor (TriShadeConst::sbtm)
        const f3 col = fvcol(f);
        px.F0 = mk(__builtin_fmaf(col.x, sc.sbtm[0], om), __builtin_fmaf(col.y, sc.sbtm[1], om),
                   __builtin_fmaf(col.z, sc.sbtm[2], om));
        px.diffK = mul(col, mk(sc.sbtkd[0], sc.sbtkd[1], sc.sbtkd[2]));
        c = mul(col, mk(sc.sbtamb[0], sc.sbtamb[1], sc.sbtamb[2]));
    } else {
        const f3 albedo = ONE ? mul(mk(sc.sbt[0], sc.sbt[1], sc.sbt[2]), fvcol(f))
                              : mul(mul(mul(ftex(f), mk(sc.base[0], sc.base[1], sc.base[2])), ftint(f)), fvcol(f));
        px.F0 = mk(__builtin_fmaf(albedo.x, m, om), __builtin_fmaf(albedo.y, m, om), __builtin_fmaf(albedo.z, m, om));
        px.diffK = muls(albedo, sc.kd);
        c = mk(sc.amb[0] * albedo.x * sc.amb_strength, sc.amb[1] * albedo.y * sc.amb_strength,
               sc.amb[2] * albedo.z * sc.amb_strength);
    }
    px.omF0 = mk(1.0f - px.F0.x, 1.0f - px.F0.y, 1.0f - px.F0.z);
    px.NdotVr = fdot(px.N, px.V);
    const float NdotV = fmaxf(px.NdotVr, 0.0f);
    const float rgV = frcp(fmaxf(__builtin_fmaf(NdotV, sc.omkg, sc.kg), 1e-4f));
    px.spA = sc.spAk * rgV;                   // 0.25 a2 / pi / (1 - k) / max(G_V's denominator, 1e-4)
    px.spB = sc.spBk * (NdotV * rgV);         // 1e4 a2 / pi * G_V / (1 - k)
    if (kAblate & 64) return make_float4(c.x, c.y, c.z, 1.0f);  // diagnostics: 64 = no lights
    if (sc.has_sun && f.vis > 0.0f) {  // vis = 0 (fully shadowed): the sun adds exactly nothing
        const f3 L = mk(sc.sun_l[0], sc.sun_l[1], sc.sun_l[2]);
        eval_pbr_fast(sc, px, fdot(px.N, L), fdot(L, px.V), mk(sc.sun_rad[0], sc.sun_rad[1], sc.sun_rad[2]), f.vis, c);
    }
    const f3 wp = fworld(f);
    for (uint32_t i = 0; i < sc.npt; ++i) {
        float lp[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) { lp[k] = sc.pl[i].pos[k]; lp[4 + k] = sc.pl[i].rad[k]; }
        const f3 to = sub3(mk(lp[0], lp[1], lp[2]), wp);
        const float d2 = fdot(to, to);
        const float inv = frsq(d2);
        const float att0 = att_base(d2 * inv, lp[3]);
        // dist <= 1e-4 (Default.frag skips it; d2 = 0 gives att0 = 0 here too), or beyond the light's
        // range: (1 - d/r)^2 = 0 adds exactly nothing. One exact skip instead of two.
        if (!(d2 > 1e-8f && att0 > 0.0f)) continue;
        // L = to / |to| is never formed: N.L and L.V are the dot products with `to`, scaled once
        eval_pbr_fast(sc, px, fdot(px.N, to) * inv, fdot(to, px.V) * inv, mk(lp[4], lp[5], lp[6]), att0 * att0, c);
    }
    const f3 t = mk(c.x * frcp(c.x + 1.0f), c.y * frcp(c.y + 1.0f), c.z * frcp(c.z + 1.0f));
    return make_float4(tone_out(t.x), tone_out(t.y), tone_out(t.z), ONE ? sc.sbt[3] : (sc.base[3] * f.tw) * f.sw);
#endif
}

__device__ __forceinline__ float interp_exact(float w0, float w1, float w2, float x0, float x1, float x2) {
    return (w0 * x0 + w1 * x1) + w2 * x2;  // the oracle's order, no contraction
}
__device__ __forceinline__ float interp_fast(float w0, float w1, float w2, float x0, float x1, float x2) {
    return __builtin_fmaf(w2, x2, __builtin_fmaf(w1, x1, w0 * x0));
}

// Fast build's perspective-correct weights from the pixel-centre offsets (dx, dy) to vertex 0: the three
// edge functions at the pixel, e0 = S + (y1 - y2) dx + (x2 - x1) dy, e1 = y2 dx - x2 dy, e2 = x1 dy - y1 dx
// (S the exact doubled area, so e0 + e1 + e2 = S), weighted by 1/w: q_k = e_k iw_k, w_k = q_k / (q0 + q1 + q2).
// This is the barycentric form scaled by S iw0, which cancels in the normalisation, so the only reciprocal is
// that of the sum (no 1/S, no 1/iw0). e0 is formed about vertex 1, e0 = (x2 - x1)(dy - y1) - (y2 - y1)(dx - x1)
// (the same function: its constant term is S), so no area product is needed. Every offset is an exact
// integer below 2^24 inside the guard band, converted once. Relative to the triangle's own vertices, not to a
// bin: every bin, band and code path gives a pixel the same bits.
__device__ __forceinline__ void fast_weights(const TriRec& r, int32_t px, int32_t py, float& w0, float& w1, float& w2) {
    const int32_t x1 = r.X[1] - r.X[0], y1 = r.Y[1] - r.Y[0], x2 = r.X[2] - r.X[0], y2 = r.Y[2] - r.Y[0];
    const float fx1 = (float)x1, fy1 = (float)y1, fx2 = (float)x2, fy2 = (float)y2;
    const int32_t idx = 256 * px + 128 - r.X[0], idy = 256 * py + 128 - r.Y[0];
    const float dx = (float)idx, dy = (float)idy;
    const float e1 = __builtin_fmaf(-fx2, dy, fy2 * dx);
    const float e2 = __builtin_fmaf(fx1, dy, -fy1 * dx);
    // e0 = S - e1 - e2 with the area in float (a weight then carries an absolute error of a few 2^-24, far
    // inside the colour bar; depth never uses these weights)
    const float e0 = (__builtin_fmaf(fx1, fy2, -fy1 * fx2) - e1) - e2;
    const float q0 = e0 * r.iw[0], q1 = e1 * r.iw[1], q2 = e2 * r.iw[2];
    const float iq = frcp((q0 + q1) + q2);
    w0 = q0 * iq; w1 = q1 * iq; w2 = q2 * iq;
}

// fast_weights of the unclipped triangle rec_from_snaps(a0, a1, a2) would build (v1 <-> v2 swapped), straight
// from the TRI_SNAP_F floats: the vertex differences and the pixel-centre offsets are exact in float either way,
// so the weights are the same bits without the integer sign extensions and conversions.
__device__ __forceinline__ void fast_weights_snaps(const TriSnap& a0, const TriSnap& a1, const TriSnap& a2, int32_t px,
                                                   int32_t py, float& w0, float& w1, float& w2) {
    const float X0 = snap_Xf(a0), Y0 = snap_Yf(a0);
    const float fx1 = snap_Xf(a2) - X0, fy1 = snap_Yf(a2) - Y0, fx2 = snap_Xf(a1) - X0, fy2 = snap_Yf(a1) - Y0;
    const float dx = (float)(256 * px + 128) - X0, dy = (float)(256 * py + 128) - Y0;
    const float e1 = __builtin_fmaf(-fx2, dy, fy2 * dx);
    const float e2 = __builtin_fmaf(fx1, dy, -fy1 * dx);
    const float e0 = (__builtin_fmaf(fx1, fy2, -fy1 * fx2) - e1) - e2;
    const float q0 = e0 * a0.iw, q1 = e1 * a2.iw, q2 = e2 * a1.iw;
    const float iq = frcp((q0 + q1) + q2);
    w0 = q0 * iq; w1 = q1 * iq; w2 = q2 * iq;
}

// Perspective-correct barycentric weights of pixel (px, py) in the oracle's order: exact int64 edge
// functions at the pixel centre, IEEE divides (the EXACT build's interpolation; the shadow lookup uses
// them in both builds so its compare sees the oracle's light-space depth bit for bit).
__device__ __forceinline__ void exact_weights(const TriRec& r, int32_t px, int32_t py, float& w0, float& w1, float& w2) {
    // The edge functions and the area are exact integers converted to float once (round to nearest):
    // a triangle under 125 px on a side (the common case) has every product below 2^30, so 32-bit
    // arithmetic gives the same integers, and so the same floats, as the 64-bit form.
    float fe[3], fS;
    const int32_t xmin = min(r.X[0], min(r.X[1], r.X[2])), xmax = max(r.X[0], max(r.X[1], r.X[2]));
    const int32_t ymin = min(r.Y[0], min(r.Y[1], r.Y[2])), ymax = max(r.Y[0], max(r.Y[1], r.Y[2]));
    if (xmax - xmin < 32000 && ymax - ymin < 32000) {  // |a|, |b|, |pixel - vertex| < 2^15 for a covered pixel
        const int32_t Xp = 256 * px + 128, Yp = 256 * py + 128;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int i = k, j = (k + 1) % 3;
            fe[k] = (float)((r.Y[i] - r.Y[j]) * (Xp - r.X[i]) + (r.X[j] - r.X[i]) * (Yp - r.Y[i]));
        }
        fS = (float)((r.X[1] - r.X[0]) * (r.Y[2] - r.Y[0]) - (r.Y[1] - r.Y[0]) * (r.X[2] - r.X[0]));
    } else {
        const int64_t Xp = 256 * (int64_t)px + 128, Yp = 256 * (int64_t)py + 128;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int i = k, j = (k + 1) % 3;
            const int64_t a = (int64_t)r.Y[i] - r.Y[j];
            const int64_t bb = (int64_t)r.X[j] - r.X[i];
            const int64_t c = -(a * r.X[i] + bb * r.Y[i]);
            fe[k] = (float)(a * Xp + bb * Yp + c);
        }
        fS = (float)((int64_t)(r.X[1] - r.X[0]) * (int64_t)(r.Y[2] - r.Y[0]) -
                     (int64_t)(r.Y[1] - r.Y[0]) * (int64_t)(r.X[2] - r.X[0]));
    }
    const RcpRef rS = rcp_ref(fS);
    const float l0 = div_rn(fe[1], rS), l1 = div_rn(fe[2], rS), l2 = div_rn(fe[0], rS);
    const float q0 = l0 * r.iw[0], q1 = l1 * r.iw[1], q2 = l2 * r.iw[2];
    const float qs = (q0 + q1) + q2;
    const RcpRef rq = rcp_ref(qs);
    w0 = div_rn(q0, rq); w1 = div_rn(q1, rq); w2 = div_rn(q2, rq);
}

// Shadow lookup (oracle shadow_visibility): the fraction of the 2x2 bilinear depth compare
// (zref - bias <= map) that passes at light-NDC point (lx, ly, lz); 1 outside the map. IEEE mul/add in
// the oracle's order (this file is compiled without contraction).
__device__ __forceinline__ float shadow_vis(const TriFrameParams& fp, const uint32_t* smap, float lx, float ly, float lz) {
    const float u = lx * 0.5f + 0.5f, v = ly * 0.5f + 0.5f;
    if (!(u >= 0.0f && u <= 1.0f && v >= 0.0f && v <= 1.0f)) return 1.0f;
    const int32_t n = (int32_t)fp.s_size;
    const float fx = u * (float)n - 0.5f, fy = v * (float)n - 0.5f;
    const float x0 = floorf(fx), y0 = floorf(fy);
    const float a = fx - x0, bb = fy - y0;
    const int32_t i0 = (int32_t)x0, j0 = (int32_t)y0;
    const float zref = lz - fp.s_bias;
    const int32_t ia = min(max(i0, 0), n - 1), ib = min(max(i0 + 1, 0), n - 1);
    const int32_t ja = min(max(j0, 0), n - 1), jb = min(max(j0 + 1, 0), n - 1);
    float m00, m10, m01, m11;
    TRI_G const uint32_t* sm = (TRI_G const uint32_t*)smap;
    if (TRI_MAP_PAIRS && ib == ia + 1) {  // adjacent columns: one 8-B load per row (as sample_tex)
        const u32x2a r0 = ld_pair(sm + (size_t)ja * n + ia), r1 = ld_pair(sm + (size_t)jb * n + ia);
        m00 = __uint_as_float(r0.x); m10 = __uint_as_float(r0.y);
        m01 = __uint_as_float(r1.x); m11 = __uint_as_float(r1.y);
    } else {  // a clamped column at the map's edge
        m00 = __uint_as_float(sm[(size_t)ja * n + ia]); m10 = __uint_as_float(sm[(size_t)ja * n + ib]);
        m01 = __uint_as_float(sm[(size_t)jb * n + ia]); m11 = __uint_as_float(sm[(size_t)jb * n + ib]);
    }
    const float c00 = zref <= m00 ? 1.0f : 0.0f;
    const float c10 = zref <= m10 ? 1.0f : 0.0f;
    const float c01 = zref <= m01 ? 1.0f : 0.0f;
    const float c11 = zref <= m11 ? 1.0f : 0.0f;
    const float l0 = c00 + a * (c10 - c00), l1 = c01 + a * (c11 - c01);
    return l0 + bb * (l1 - l0);
}

// The varyings of the triangle's three vertex slots: 16-B gathers, issued before the weights are
// computed (their addresses need only the slots, the weights need the snapped vertices too). With
// TRI_COLOUR_LATE the three colour gathers are issued once the weights are done and the
// snapped vertices' registers are free: the peak register count falls enough for 7 waves/SIMD.
// Both translation units (round 4: the shadow instantiation too, 92 -> 86 VGPRs, which with 6 waves/SIMD spills
// 6 instead of 20: C5 k_raster 166.5 -> 158.7 us).
#ifndef TRI_COLOUR_LATE
#define TRI_COLOUR_LATE 1
#endif
// TRI_COLOUR_EARLY_ONE: the single-draw solid instantiation (C3's) issues its colour gathers with the other
// varyings after all: within its 56-VGPR cap the scheduler keeps them without a spill, and their latency no longer
// sits between the weights and the shading (C3 10.89k -> 11.03k frames/s, same box; every other instantiation
// spills with them early, so keeps them late)
#ifndef TRI_COLOUR_EARLY_ONE
#define TRI_COLOUR_EARLY_ONE 1
#endif
struct Taps {
    V4 a0, a1, a2, b0, b1, b2, c0, c1, c2;
};
// SRC: an unclipped primitive's vertex (fb.src), else a clipped polygon's (fb.vary); the same buffer unless ONE.
template <bool ONE = false, bool SRC = false>
__device__ __forceinline__ V4 ld_vary(const FetchBufs& fb, uint32_t slot, uint32_t j) {
    if (ONE && TRI_VARY36) {  // 36-B prefixes: 12-B pieces, no texture coordinate (the stride is the buffer's)
        const u32x3v q = rec96<36>(SRC ? fb.src : fb.vary, slot, j * 12u);
        return V4{__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]), 0.0f};
    }
    // plain-float views (HIP vector unions defeat SROA); fb.src is fb.vary unless obj48 (the input records)
    const uint4 q = rec128<48>(SRC ? fb.src : fb.vary, slot, j * 16u);
    return V4{__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w)};
}
template <bool ONE = false, bool SRC = false, bool EARLY = !TRI_COLOUR_LATE>
__device__ __forceinline__ Taps load_taps(const FetchBufs& fb, uint32_t v0, uint32_t v1, uint32_t v2, bool colour = true) {
    Taps t;
    t.a0 = ld_vary<ONE, SRC>(fb, v0, 0); t.a1 = ld_vary<ONE, SRC>(fb, v0, 1);
    t.b0 = ld_vary<ONE, SRC>(fb, v1, 0); t.b1 = ld_vary<ONE, SRC>(fb, v1, 1);
    t.c0 = ld_vary<ONE, SRC>(fb, v2, 0); t.c1 = ld_vary<ONE, SRC>(fb, v2, 1);
    if (EARLY && colour) {
        t.a2 = ld_vary<ONE, SRC>(fb, v0, 2); t.b2 = ld_vary<ONE, SRC>(fb, v1, 2); t.c2 = ld_vary<ONE, SRC>(fb, v2, 2);
    }
    return t;
}

// The draw's 48-B shade record (tint, texture descriptor).
struct ShadeRec {
    uint4 st, sd, ss;
};
// TRI_SHADE_SCALAR: when every lane of the wave shades the same draw (the common case: a bin is mostly one
// mesh), the record comes through three scalar buffer loads instead of three wave-wide gathers (the texture
// units' data return is what C5's fragment stage waits on).
#ifndef TRI_SHADE_SCALAR
#define TRI_SHADE_SCALAR 1
#endif
__device__ u32x4v tri_s_buffer_load_v4(u32x4v rsrc, int offset, int aux) __asm("llvm.amdgcn.s.buffer.load.v4i32");
__device__ __forceinline__ ShadeRec load_shade(const FetchBufs& fb, uint32_t d) {
    if (TRI_SHADE_SCALAR) {
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
        if (__ballot(d != d0) == 0ull) {  // wave-uniform draw
            const uint64_t base = (uint64_t)fb.shade_base;  // a raw descriptor: base, 0 stride, size, flags
            const u32x4v r = u32x4v{(uint32_t)base, (uint32_t)(base >> 32) & 0xFFFFu, fb.shade_bytes, 0x00020000u};
            const int off = (int)(d0 * (uint32_t)sizeof(TriDrawShade));
            const u32x4v a = tri_s_buffer_load_v4(r, off, 0), b = tri_s_buffer_load_v4(r, off + 16, 0),
                         c = tri_s_buffer_load_v4(r, off + 32, 0);
            return ShadeRec{make_uint4(a[0], a[1], a[2], a[3]), make_uint4(b[0], b[1], b[2], b[3]),
                            make_uint4(c[0], c[1], c[2], c[3])};
        }
    }
    return ShadeRec{rec128<48>(fb.shade, d, 0u), rec128<48>(fb.shade, d, 16u), rec128<48>(fb.shade, d, 32u)};
}


// The varyings at weights (w0, w1, w2), the draw d's texture sample and tint: Frag fields 0..18 through
// `put`.
// XF48: the instantiation may apply obj48's per-draw model and normal matrices (not the shadow instantiation: the
// host keeps frames with the pre-pass and a non-identity obj48 draw on world-space varyings, so that kernel carries
// none of this code's registers)
template <bool EXACT, bool ONE, bool XF48, typename Put>
__device__ __forceinline__ void fetch_attrs(const TriFrameParams& fp, const TriDeviceBuffers& b, const FetchBufs& fb,
                                            const Taps& t, uint32_t d, float w0, float w1, float w2, const float* lut,
                                            Put&& put) {
    auto ip = [&](float x0, float x1, float x2) {
        return EXACT ? interp_exact(w0, w1, w2, x0, x1, x2) : interp_fast(w0, w1, w2, x0, x1, x2);
    };
    const V4 &a0 = t.a0, &a1 = t.a1, &a2 = t.a2, &b0 = t.b0, &b1 = t.b1, &b2 = t.b2, &c0 = t.c0, &c1 = t.c1, &c2 = t.c2;
    // field-wise stores (a struct-valued f3 store is ABI-coerced to <2 x float> + float, which
    // keeps the pixel-pair path's fragments from being promoted to registers)
    auto row = [](float c0v, float c1v, float c2v, float x, float y, float z, float w) {
        return __builtin_fmaf(c0v, x, __builtin_fmaf(c1v, y, __builtin_fmaf(c2v, z, w)));
    };
    if (ONE && obj_mode(fp) && fp.obj_xform) {  // object-space position and normal: the model / normal matrices
        const float px = ip(a0.x, b0.x, c0.x), py = ip(a0.y, b0.y, c0.y), pz = ip(a0.z, b0.z, c0.z);
        const float nx = ip(a1.x, b1.x, c1.x), ny = ip(a1.y, b1.y, c1.y), nz = ip(a1.z, b1.z, c1.z);
        const float* m = fp.draw0.model;  // column-major, affine (vary_obj)
        const float* n = fp.draw0.nm;     // NM[c*3+r]
        put(0, row(m[0], m[4], m[8], px, py, pz, m[12]));
        put(1, row(m[1], m[5], m[9], px, py, pz, m[13]));
        put(2, row(m[2], m[6], m[10], px, py, pz, m[14]));
        put(3, row(n[0], n[3], n[6], nx, ny, nz, 0.0f));
        put(4, row(n[1], n[4], n[7], nx, ny, nz, 0.0f));
        put(5, row(n[2], n[5], n[8], nx, ny, nz, 0.0f));
    } else if (!ONE && XF48 && obj48_mode(fp) && fp.obj48_xform) {
        // obj48: the fragment's own draw's matrices, one draw of the wave at a time (a waterfall: usually one
        // pass), read with scalar loads, so they live in SGPRs
        const float px = ip(a0.x, b0.x, c0.x), py = ip(a0.y, b0.y, c0.y), pz = ip(a0.z, b0.z, c0.z);
        const float nx = ip(a1.x, b1.x, c1.x), ny = ip(a1.y, b1.y, c1.y), nz = ip(a1.z, b1.z, c1.z);
        float o[6];
        for (;;) {
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
            if (d == d0) {
                TRI_G const TriDrawDev& dr = b.draws[d0];
                TRI_G const float* m = dr.model;
                TRI_G const float* n = dr.nm;
                o[0] = row(m[0], m[4], m[8], px, py, pz, m[12]);
                o[1] = row(m[1], m[5], m[9], px, py, pz, m[13]);
                o[2] = row(m[2], m[6], m[10], px, py, pz, m[14]);
                o[3] = row(n[0], n[3], n[6], nx, ny, nz, 0.0f);
                o[4] = row(n[1], n[4], n[7], nx, ny, nz, 0.0f);
                o[5] = row(n[2], n[5], n[8], nx, ny, nz, 0.0f);
                break;
            }
        }
        for (int i = 0; i < 6; ++i) put(i, o[i]);
    } else {
        put(0, ip(a0.x, b0.x, c0.x)); put(1, ip(a0.y, b0.y, c0.y)); put(2, ip(a0.z, b0.z, c0.z));
        put(3, ip(a1.x, b1.x, c1.x)); put(4, ip(a1.y, b1.y, c1.y)); put(5, ip(a1.z, b1.z, c1.z));
    }
    if (ONE && obj_mode(fp) && fp.obj_ucol) {  // one colour for every vertex (its interpolation is the colour)
        put(6, fp.ucol[0]); put(7, fp.ucol[1]); put(8, fp.ucol[2]);
    } else {
        put(6, ip(a2.x, b2.x, c2.x)); put(7, ip(a2.y, b2.y, c2.y)); put(8, ip(a2.z, b2.z, c2.z));
    }
    const float u = ip(a0.w, b0.w, c0.w), v = ip(a1.w, b1.w, c1.w);
    put(9, u); put(10, v);
    if (ONE || fp.shade_solid) {  // uniform: one draw with a 1x1 slot, its texel and tint are kernel arguments
        for (int i = 0; i < 4; ++i) put(11 + i, fp.sc.solid[i]);
        for (int i = 0; i < 4; ++i) put(15 + i, fp.sc.tint[i]);
        return;
    }
    const ShadeRec sh = load_shade(fb, d);
    const uint4 &st = sh.st, &sd = sh.sd, &ss = sh.ss;
    TriTexDesc td;
    td.texels = reinterpret_cast<const uint32_t*>(((uint64_t)sd.y << 32) | sd.x);
    td.w = sd.z; td.h = sd.w;
    td.solid[0] = __uint_as_float(ss.x); td.solid[1] = __uint_as_float(ss.y);
    td.solid[2] = __uint_as_float(ss.z); td.solid[3] = __uint_as_float(ss.w);
    const float4 tx = (kAblate & 128) ? make_float4(u, v, u, 1.0f) : sample_tex(td, u, v, lut);  // 128: no texture
    const float4 tint = make_float4(__uint_as_float(st.x), __uint_as_float(st.y), __uint_as_float(st.z), __uint_as_float(st.w));
    put(11, tx.x); put(12, tx.y); put(13, tx.z); put(14, tx.w);
    put(15, tint.x); put(16, tint.y); put(17, tint.z); put(18, tint.w);
}

// Interpolate the visible triangle's varyings at pixel (px, py) (perspective-correct).
// Writes the fragment through `put(field_index, value)` (fields in Frag order), so one body serves
// the single-pixel Frag and the lane-pair FragP without an intermediate in scratch memory.
// Rejected (round 4): the sun visibility of every visible pixel in a pass of its own before shading, so that
// the shading loop would not hold the light-space gathers and the map taps in its registers: C5 k_raster
// 188.6 -> 206.4 us (the pass fetches each fragment's index and snapped vertices a second time).
// The fast build's shadow instantiation shades with the exact weights its lookup needs (TRI_SHADOW_SHARED_WEIGHTS:
// one weight computation per fragment instead of two; C5 +1 % over both). Rejected (round 4): the lookup from
// the fast weights, recomputed with the exact ones only where a depth compare or the map border is within a few
// ulps: the fallback's registers cost 5 spilled VGPRs and C5 -3 %.
#ifndef TRI_SHADOW_SHARED_WEIGHTS
#define TRI_SHADOW_SHARED_WEIGHTS 1
#endif

// CLIPM: 0 = the key may name a clipped sub-triangle (tested per pixel), 1 = it never does (the shading loop
// defers clipped pixels, TRI_CLIP_DEFER), 2 = it always does (the deferred pass).
template <bool EXACT, bool SHADOW, bool ONE, int CLIPM = 0, typename Put>
__device__ __forceinline__ void fetch_fragment_to(const TriFrameParams& fp, const TriDeviceBuffers& b, uint64_t key,
                                                  int32_t px, int32_t py, const float* lut, Put&& put,
                                                  const uint32_t* qtab = nullptr) {
    constexpr bool kInlineVis = SHADOW;
    const uint32_t low = (uint32_t)key;
    // qtab (TRI_QTAB bins, uniform): the key names the primitive above its queue position (qenc)
    const uint32_t prim = qtab ? kQPrimMax - (low >> 11) : TRI_PRIM_MAX - (low >> 3);
    const uint32_t sub = CLIPM == 1 ? 0u : (qtab ? (low >> 8) & 7u : low & 7u);  // >= 1: sub-triangle of a clipped primitive
    const FetchBufs fb = fetch_bufs<ONE>(fp, b);
    constexpr bool kEarly = !TRI_COLOUR_LATE || (TRI_COLOUR_EARLY_ONE && ONE && !EXACT && !SHADOW);
    // (issued early, the colour gathers are unconditional: on a frame with one vertex colour (obj_ucol) they read the
    // records' colours beside their positions, unused; a uniform branch around them cost the instantiation 4 spills)
    const bool vcol = kEarly || !(ONE && TRI_VARY_OBJ && obj_mode(fp) && fp.obj_ucol);
    uint32_t sl[3] = {0, 0, 0}, d = 0;
    TriSnap a0{}, a1{}, a2{};
    uint32_t v0 = 0, v1 = 0, v2 = 0, dl = 0;
    Taps taps;
    if (CLIPM != 2) {
        if (TRI_QTAB && qtab) {  // the coverage pass's table: three LDS words (four with the draw), no index gather
            const uint32_t q = low & 0xFFu;
            sl[0] = qtab[q]; sl[1] = qtab[kQtab + q]; sl[2] = qtab[2 * kQtab + q];
            if (!ONE) d = qtab[3 * kQtab + q];
        } else {
            prim_slots<ONE, kIdxOk<SHADOW>>(fp, b, prim, sl, d);
        }
        // Every gather that needs only the slots is issued before the first wait: the snapped vertices and
        // the varyings are one round trip after the index fetch (the snaps are loaded for a clipped primitive
        // too, unused: its sub-triangle's record names its slots).
        a0 = ld_snap_xyw(fb, sl[0]); a1 = ld_snap_xyw(fb, sl[1]); a2 = ld_snap_xyw(fb, sl[2]);
        v0 = sl[0]; v1 = sl[2]; v2 = sl[1];  // set-up orientation (rec_from_snaps swaps v1 and v2)
        // obj48: the geometry's input records at slot + vdelta[draw]
        if (!ONE) dl = obj_delta(fp, d);  // (0 unless obj48: the host zeroes vdelta)
        // the varyings are gathered before the (rare) clipped branch: its record loads are waited for inside
        // it, and a wait at the join would otherwise hold the snaps and varyings in two round trips
        taps = load_taps<ONE, true, kEarly>(fb, v0 + dl, v1 + dl, v2 + dl, vcol);
    } else if (!ONE) {
        prim_slots<ONE, kIdxOk<SHADOW>>(fp, b, prim, sl, d);  // the draw (its shade record); the slots come from the record
    }
    TriRec rc;
    if (CLIPM == 2 || (CLIPM == 0 && sub)) {  // a clipped primitive's sub-triangle: its own slots and varyings
        rc = load_rec(b.recs, b.clip_slot[prim] + sub - 1u);
        v0 = rc.v[0]; v1 = rc.v[1]; v2 = rc.v[2];
        taps = load_taps<ONE, false, kEarly>(fb, v0, v1, v2, vcol);
    }
    const bool from_rec = CLIPM == 2 || (CLIPM == 0 && sub);
    // the three vertices' light-space positions (rejected in round 4: recomputing them from the varyings' world
    // positions, k_vertex's own operations and so the same bits, instead of three 16-B gathers: 63 VALU per pixel
    // for 3 gathers, C5 k_raster +3.5 us)
    uint4 L0, L1, L2;
    if constexpr (kInlineVis) {
        const RecBuf lr = rec_buf(b.lpos, 16u, (uint64_t)fp.nslots + fp.ovf_vert_cap);
        L0 = rec128<16>(lr, v0, 0u); L1 = rec128<16>(lr, v1, 0u); L2 = rec128<16>(lr, v2, 0u);
    }
    const TriRec r = from_rec ? rc : rec_from_snaps(prim, sl, a0, a1, a2);
    // obj48: past the light-space gathers (slot-indexed) an unclipped primitive's vertices are only needed as
    // input-record indices (one register each instead of the slot and the offset)
    if (!ONE && !from_rec) { v0 += dl; v1 += dl; v2 += dl; }
    float w0, w1, w2;
    // exact int64 edge functions, IEEE divides (oracle order). The shadow lookup needs these weights in both
    // builds (TRI_SHADOW_SHARED_WEIGHTS: the fast build shades with them too instead of forming its own)
    if (EXACT || (kInlineVis && TRI_SHADOW_SHARED_WEIGHTS && !(kAblate & 2048))) {
        exact_weights(r, px, py, w0, w1, w2);
    } else if (TRI_SNAP_F && CLIPM == 1) {  // never clipped here: the floats of the snaps directly
        fast_weights_snaps(a0, a1, a2, px, py, w0, w1, w2);
    } else {
        fast_weights(r, px, py, w0, w1, w2);
    }
    if (kAblate & 1024) {  // diagnostics: 1024 = no colour gathers (3 of the fragment's 13 loads; same VALU)
        taps.a2 = V4{w0, w1, w2, 0.0f}; taps.b2 = taps.a2; taps.c2 = taps.a2;
    } else if (ONE && TRI_VARY_OBJ && obj_mode(fp) && fp.obj_ucol) {
        // one colour for every vertex: fetch_attrs takes it from the frame arguments
    } else if (!kEarly) {
        if (!from_rec) {  // an unclipped primitive's vertices: fb.src (fb.vary unless ONE or obj48; with CLIPM 0 a
                          // per-lane choice: both masked)
            taps.a2 = ld_vary<ONE, true>(fb, v0, 2); taps.b2 = ld_vary<ONE, true>(fb, v1, 2);
            taps.c2 = ld_vary<ONE, true>(fb, v2, 2);
        } else {
            taps.a2 = ld_vary<ONE>(fb, v0, 2); taps.b2 = ld_vary<ONE>(fb, v1, 2); taps.c2 = ld_vary<ONE>(fb, v2, 2);
        }
    }

    float vis = 1.0f;
    if constexpr (kInlineVis && !(kAblate & 2048)) {  // light-space position at the pixel with the oracle's weights,
                                                       // then the compare (diagnostics: 2048 = no lookup)
        float e0 = w0, e1 = w1, e2 = w2;
        if (!EXACT && !TRI_SHADOW_SHARED_WEIGHTS && !(kAblate & 512))  // 512: fast weights (diagnostics)
            exact_weights(r, px, py, e0, e1, e2);
        auto ix = [&](uint32_t a, uint32_t bq, uint32_t c) {
            return interp_exact(e0, e1, e2, __uint_as_float(a), __uint_as_float(bq), __uint_as_float(c));
        };
        vis = shadow_vis(fp, b.shadow_map, ix(L0.x, L1.x, L2.x), ix(L0.y, L1.y, L2.y), ix(L0.z, L1.z, L2.z));
    }
    put(19, vis);
    fetch_attrs<EXACT, ONE, !SHADOW>(fp, b, fb, taps, d, w0, w1, w2, lut, put);
}

template <bool EXACT, bool SHADOW, bool ONE, int CLIPM = 0>
__device__ __forceinline__ void fetch_fragment(const TriFrameParams& fp, const TriDeviceBuffers& b, uint64_t key,
                                               int32_t px, int32_t py, const float* lut, Frag& f,
                                               const uint32_t* qtab = nullptr) {
    fetch_fragment_to<EXACT, SHADOW, ONE, CLIPM>(fp, b, key, px, py, lut, [&](int i, float x) { (&f.wx)[i] = x; }, qtab);
}

// ------------------------------------------------------------------------------------------
// skybox pass (Skybox.cpp:13-79, Skybox.vert:30-41, Skybox.frag:28-35, cull FRONT / depth LEQUAL
// without writes, recorded before the meshes, Renderer.cpp:5076-5082). Same arithmetic as the
// oracle's sky_pixel(): a background pixel's interpolated direction is the view-space point where
// its ray leaves the 20-unit cube; Vulkan cube sampling with seamless LINEAR filtering.
// ------------------------------------------------------------------------------------------
template <bool FAST = false>
__device__ __forceinline__ int cube_face(f3 d, float& s, float& t) {
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
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
    if (FAST) {
        const float h = 0.5f * frcp(ma);
        s = sc * h + 0.5f;
        t = tc * h + 0.5f;
    } else {
        s = 0.5f * (sc / ma) + 0.5f;
        t = 0.5f * (tc / ma) + 0.5f;
    }
    return face;
}

__device__ __forceinline__ f3 face_dir(int face, float sc, float tc) {
    switch (face) {
        case 0: return mk(1.0f, -tc, -sc);
        case 1: return mk(-1.0f, -tc, sc);
        case 2: return mk(sc, 1.0f, tc);
        case 3: return mk(sc, -1.0f, -tc);
        case 4: return mk(sc, -tc, 1.0f);
        default: return mk(-sc, -tc, -1.0f);
    }
}

struct SkyTex {
    TRI_G const uint32_t* t;
    int32_t n;
    const float* lut;
    __device__ __forceinline__ f3 decode(uint32_t p) const {
        return mk(lut[p & 0xFFu], lut[(p >> 8) & 0xFFu], lut[(p >> 16) & 0xFFu]);
    }
    __device__ __forceinline__ f3 texel(int face, int32_t i, int32_t j) const {
        return decode(t[((uint32_t)face * (uint32_t)n + (uint32_t)j) * (uint32_t)n + (uint32_t)i]);
    }
    __device__ __forceinline__ f3 across(int face, int32_t i, int32_t j) const {
        const float sc = 2.0f * (((float)i + 0.5f) / (float)n) - 1.0f;
        const float tc = 2.0f * (((float)j + 0.5f) / (float)n) - 1.0f;
        float s, tt;
        const int f2 = cube_face(face_dir(face, sc, tc), s, tt);
        const int32_t i2 = min(max((int32_t)floorf(s * (float)n), 0), n - 1);
        const int32_t j2 = min(max((int32_t)floorf(tt * (float)n), 0), n - 1);
        return texel(f2, i2, j2);
    }
    __device__ __forceinline__ f3 fetch(int face, int32_t i, int32_t j) const {
        const bool in_i = i >= 0 && i < n, in_j = j >= 0 && j < n;
        if (in_i && in_j) return texel(face, i, j);
        if (in_i || in_j) return across(face, i, j);
        const int32_t ci = min(max(i, 0), n - 1), cj = min(max(j, 0), n - 1);
        const f3 a = texel(face, ci, cj), b = across(face, i, cj), c = across(face, ci, j);
        return mk(((a.x + b.x) + c.x) / 3.0f, ((a.y + b.y) + c.y) / 3.0f, ((a.z + b.z) + c.z) / 3.0f);
    }
    template <bool FAST = false>
    __device__ __forceinline__ f3 sample(f3 d) const {
        float s, tt;
        const int face = cube_face<FAST>(d, s, tt);
        const float u = s * (float)n - 0.5f, v = tt * (float)n - 0.5f;
        const float fu = floorf(u), fv = floorf(v);
        const float a = u - fu, bb = v - fv;
        const int32_t i0 = (int32_t)fu, j0 = (int32_t)fv;
        f3 t00, t10, t01, t11;
        if (TRI_TEXEL_PAIRS && i0 >= 0 && i0 + 1 < n && j0 >= 0 && j0 + 1 < n) {  // inside the face: 8-B row loads
            TRI_G const uint32_t* r = t + ((uint32_t)face * (uint32_t)n + (uint32_t)j0) * (uint32_t)n + (uint32_t)i0;
            const u32x2a r0 = ld_pair(r), r1 = ld_pair(r + n);
            t00 = decode(r0.x); t10 = decode(r0.y); t01 = decode(r1.x); t11 = decode(r1.y);
        } else {  // a tap across an edge or corner of the face (seamless filtering)
            t00 = fetch(face, i0, j0); t10 = fetch(face, i0 + 1, j0);
            t01 = fetch(face, i0, j0 + 1); t11 = fetch(face, i0 + 1, j0 + 1);
        }
        auto lp = [](float x, float y, float w) { return x + w * (y - x); };
        return mk(lp(lp(t00.x, t10.x, a), lp(t01.x, t11.x, a), bb), lp(lp(t00.y, t10.y, a), lp(t01.y, t11.y, a), bb),
                  lp(lp(t00.z, t10.z, a), lp(t01.z, t11.z, a), bb));
    }
};

// BGRA8 sky colour of pixel (px, py), or the clear colour where the skybox does not cover it.
// Inlined into its own pass of k_raster (a call here costs the whole kernel a scratch stack and the
// callee-saved register set: measured 5x slower at C3).
__device__ __forceinline__ uint32_t sky_bgra(const TriFrameParams& fp, const TriDeviceBuffers& b, int32_t px, int32_t py,
                                          const float* lut) {
    const float xn = (float)(2 * px + 1) / (float)fp.W - 1.0f;
    const float yn = (float)(2 * py + 1) / (float)fp.H - 1.0f;
    const float* m = fp.sky_ip;
    auto unproject = [&](float zn) {
        const float x = ((m[0] * xn + m[4] * yn) + m[8] * zn) + m[12];
        const float y = ((m[1] * xn + m[5] * yn) + m[9] * zn) + m[13];
        const float z = ((m[2] * xn + m[6] * yn) + m[10] * zn) + m[14];
        const float w = ((m[3] * xn + m[7] * yn) + m[11] * zn) + m[15];
        return mk(x / w, y / w, z / w);
    };
    const f3 o = unproject(0.0f), o1 = unproject(1.0f);
    const f3 r = sub3(o1, o);
    const float* R = fp.sky_R;
    const float oa[3] = {(R[0] * o.x + R[1] * o.y) + R[2] * o.z, (R[3] * o.x + R[4] * o.y) + R[5] * o.z,
                         (R[6] * o.x + R[7] * o.y) + R[8] * o.z};
    const float ra[3] = {(R[0] * r.x + R[1] * r.y) + R[2] * r.z, (R[3] * r.x + R[4] * r.y) + R[5] * r.z,
                         (R[6] * r.x + R[7] * r.y) + R[8] * r.z};
    const float half = 20.0f;
    float t_in = -INFINITY, t_out = INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (ra[a] != 0.0f) {
            const float t0 = (-half - oa[a]) / ra[a], t1 = (half - oa[a]) / ra[a];
            t_in = fmaxf(t_in, fminf(t0, t1));
            t_out = fminf(t_out, fmaxf(t0, t1));
        } else if (oa[a] < -half || oa[a] > half) {
            return fp.clear_bgra;
        }
    }
    if (!(t_out >= t_in)) return fp.clear_bgra;
    const f3 h = mk(o.x + r.x * t_out, o.y + r.y * t_out, o.z + r.z * t_out);
    const float w = ((fp.sky_pw[0] * h.x + fp.sky_pw[1] * h.y) + fp.sky_pw[2] * h.z) + fp.sky_pw[3];
    if (!(w > 0.0f)) return fp.clear_bgra;
    const SkyTex sky{b.sky, (int32_t)fp.sky_size, lut};
    const f3 c = sky.sample(norm3(h));
    return unorm8(c.z) | (unorm8(c.y) << 8) | (unorm8(c.x) << 16) | (255u << 24);
}

// TRI_SKY_PERSP (fast build): the ray of a pixel starts at the eye, the centre of the skybox cube,
// so it always leaves the cube and its exit point has the direction of the far-plane point; cube
// sampling only uses direction ratios, so no normalisation and no cube intersection is needed.
__device__ __forceinline__ uint32_t sky_bgra_persp(const TriFrameParams& fp, const TriDeviceBuffers& b, int32_t px,
                                                   int32_t py, const float* lut) {
    const float xn = (float)(2 * px + 1) / (float)fp.W - 1.0f;
    const float yn = (float)(2 * py + 1) / (float)fp.H - 1.0f;
    const float* m = fp.sky_far;
    f3 d = mk(m[0] * xn + m[1] * yn + m[2], m[4] * xn + m[5] * yn + m[6], m[8] * xn + m[9] * yn + m[10]);
    if (m[12] * xn + m[13] * yn + m[14] < 0.0f) d = mk(-d.x, -d.y, -d.z);  // homogeneous w < 0
    const SkyTex sky{b.sky, (int32_t)fp.sky_size, lut};
    const f3 c = sky.sample<true>(d);
    return unorm8(c.z) | (unorm8(c.y) << 8) | (unorm8(c.x) << 16) | (255u << 24);
}

#ifndef TRI_RASTER_WAVES
#define TRI_RASTER_WAVES 6  // k_raster occupancy target at 32x32 bins (waves per SIMD)
#endif
#ifndef TRI_RASTER_WAVES_PLAIN
#define TRI_RASTER_WAVES_PLAIN 7  // k_raster_plain (raster_plain.hip, no SLP): 69 VGPRs, no spill
#endif
#ifndef TRI_RASTER_WAVES_SHADOW
#define TRI_RASTER_WAVES_SHADOW 6  // the fast build's shadow instantiation (80 VGPRs, 6 spilled: C5 raster 158.7 us
                                   // against 166.5 at 5 waves; the exact build keeps 5)
#endif

// bbox∩bin pixels above which a triangle is rasterized by the whole workgroup (cooperatively):
// 32x32 bins 96 (64: C3 raster 119 -> 143 us; 160: unchanged), 16x16 bins 160 (96 -> 160: C2 raster
// 41.8 -> 35.7 us, C2 28.4k -> 33.3k fps)
#ifndef TRI_BIG_AREA
#define TRI_BIG_AREA 96
#endif
#ifndef TRI_BIG_AREA16
#define TRI_BIG_AREA16 160
#endif
template <int BL>
constexpr int big_area() { return BL == 4 ? TRI_BIG_AREA16 : TRI_BIG_AREA; }
constexpr int kBigQueue = 1024;

// Bijective XCD-aware block -> bin remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): workgroups b, b+8, b+16 ... share an XCD's L2, so give them consecutive bins — each
// XCD then rasterizes one contiguous band of the screen and re-reads neighbours' records from L2.
__device__ __forceinline__ int xcd_bin(int b, int nb) {
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Balanced coverage (16x16 bins, i.e. sparse frames; dense 32x32 bands keep the per-lane walk, where
// C3's ~4-px rows made the per-job overhead cost more than the divergence it removed: 127 -> 136 us,
// while C2 went 16.8k -> 19.0k fps): a pass takes up to kCovPass queue entries; each entry's edge/depth constants at its
// clipped bbox corner go to LDS, and its bbox rows become jobs spread evenly over the workgroup, so a
// wave no longer issues its longest triangle's whole bbox walk while most lanes idle. A row job steps
// exactly like raster_serial (integer edge functions, float depth offsets in steps of 256: exact), so
// the keys are bit-identical.
// 32x32 bins: one lane per triangle (two lanes per triangle paid with the per-pixel bbox walk in round 2; with
// the span walk one lane per triangle is faster: C3 k_raster 95.3 -> 94.0 us, four lanes 94.5)
// lanes per triangle in the shadow pre-pass's per-lane walk (two paid with the per-texel walk; with the span
// walk one: C5 k_shadow_raster 44.5 -> 43.9 us)
#ifndef TRI_SHADOW_SHARE
#define TRI_SHADOW_SHARE 1
#endif
// Raised wave priority (s_setprio 1) from a 32x32 bin's start to the end of its coverage: the latency-bound
// init and coverage phases issue ahead of other workgroups' shading waves (C3 k_raster 101.7 -> 99.6 us,
// round 3 A/B; at 16x16 bins it was slower, so BL == 5 only). Scheduling only: output unchanged.
#ifndef TRI_RASTER_PRIO  // the rest of the bin (shading, stores) at this priority: above a concurrent frame's front end
#define TRI_RASTER_PRIO 0
#endif
#ifndef TRI_COV_PRIO
#define TRI_COV_PRIO 1
#endif
#ifndef TRI_COV_BALANCED
#define TRI_COV_BALANCED 1
#endif
// 32x32 bins: the per-lane walk visits each row's covered span only (raster_span)
#ifndef TRI_SPAN_WALK
#define TRI_SPAN_WALK 1
#endif
constexpr int kCovPass = 160;   // entries per pass (LDS: 64 B each)
constexpr int kCovJobs = 1024;  // row jobs per pass (u16: entry << 6 | row); rows beyond stay with their lane
struct __attribute__((aligned(16))) CovEntry {
    int32_t A[3], B[3], F[3];
    float dzdX, dzdY, z0, fdx0, fdy0;
    uint32_t low;
    uint32_t pk;  // row0 (12 bits) | width - 1 (6 bits) << 12 | far_clip << 18
};
static_assert(sizeof(CovEntry) == 64, "CovEntry: 64 bytes");

template <int BL>
__device__ __forceinline__ void cov_row(const CovEntry& c, uint32_t r, uint64_t* keys) {
    int32_t f0 = c.F[0] + c.B[0] * (int32_t)r, f1 = c.F[1] + c.B[1] * (int32_t)r, f2 = c.F[2] + c.B[2] * (int32_t)r;
    const float t2 = c.dzdY * (c.fdy0 + 256.0f * (float)r);
    const bool far_clip = (c.pk >> 18) & 1u;
    const uint32_t row = (c.pk & 0xFFFu) + (r << BL);
    const uint32_t rend = row + ((c.pk >> 12) & 0x3Fu);
    float fdx = c.fdx0;
    for (uint32_t a = row; a <= rend; ++a) {
        if ((f0 | f1 | f2) >= 0) {
            uint64_t key;
            if (depth_key((c.z0 + c.dzdX * fdx) + t2, far_clip, c.low, key)) atomicMin(&keys[a], key);
        }
        f0 += c.A[0]; f1 += c.A[1]; f2 += c.A[2];
        fdx += 256.0f;
    }
}

// texture(AiBlendTexture, gl_FragCoord.xy * AiBlendConfig.yz) (Default.frag:186-188): R8G8B8A8_UNORM (the UNORM
// decode b / 255, no sRGB), LINEAR, CLAMP_TO_EDGE, level 0 (the sampler of EnsureAiTextureResources,
// Renderer.cpp:1462-1470). Same float operations as the oracle's ai_sample.
__device__ __forceinline__ float4 sample_ai(const TriFrameParams& fp, const TriDeviceBuffers& b, int32_t px, int32_t py) {
    const float u = ((float)px + 0.5f) * fp.ai_sx, v = ((float)py + 0.5f) * fp.ai_sy;
    const float x = u * (float)fp.ai_tw - 0.5f, y = v * (float)fp.ai_th - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float a = x - fx, bb = y - fy;
    const int32_t i0 = (int32_t)fminf(fmaxf(fx, -1.0f), 1.0e9f), j0 = (int32_t)fminf(fmaxf(fy, -1.0f), 1.0e9f);
    const int32_t tw = (int32_t)fp.ai_tw, th = (int32_t)fp.ai_th;
    const int32_t xa = min(max(i0, 0), tw - 1), xb = min(max(i0 + 1, 0), tw - 1);
    const int32_t ya = min(max(j0, 0), th - 1), yb = min(max(j0 + 1, 0), th - 1);
    TRI_G const uint32_t* t = b.ai_frame;
    const uint32_t p00 = t[(size_t)ya * tw + xa], p10 = t[(size_t)ya * tw + xb];
    const uint32_t p01 = t[(size_t)yb * tw + xa], p11 = t[(size_t)yb * tw + xb];
    float r[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        auto ch = [&](uint32_t q) { return (float)((q >> (8 * c)) & 0xFFu) / 255.0f; };
        const float t00 = ch(p00), t10 = ch(p10), t01 = ch(p01), t11 = ch(p11);
        const float l0 = t00 + a * (t10 - t00), l1 = t01 + a * (t11 - t01);
        r[c] = l0 + bb * (l1 - l0);
    }
    return make_float4(r[0], r[1], r[2], r[3]);
}
// mix(x, y, a) = x * (1 - a) + y * a (GLSL)
__device__ __forceinline__ float mix_ai(float x, float y, float w) { return x * (1.0f - w) + y * w; }

// Default.frag for one fragment at pixel (px, py), stored as B8G8R8A8_UNORM. AI: the instantiation for frames with
// the AI frame blend (k_raster_ai; the other kernels carry none of its registers)
template <bool EXACT, bool ONE, bool AI>
__device__ __forceinline__ uint32_t shade_bgra(const TriFrameParams& fp, const TriDeviceBuffers& b, const Frag& f,
                                               int32_t px, int32_t py) {
    if (EXACT) {
        float4 c = fs_exact(fp, f);
        if (AI && fp.ai_on) {  // (an AI frame-generation model is loaded) the blend with the AI frame's sample
            const float4 ai = sample_ai(fp, b, px, py);
            const float w = fp.ai_wgt;
            c = make_float4(mix_ai(c.x, ai.x, w), mix_ai(c.y, ai.y, w), mix_ai(c.z, ai.z, w), mix_ai(c.w, ai.w, w));
        }
        return unorm8(c.z) | (unorm8(c.y) << 8) | (unorm8(c.x) << 16) | (unorm8(c.w) << 24);
    }
    float4 c = fs_fast<ONE>(fp.sc, f);
    if (AI && fp.ai_on) {  // the fast build's channels are already scaled by 255 (tone_out): mix there
        const float4 ai = sample_ai(fp, b, px, py);
        const float w = fp.ai_wgt;
        const float alpha = ONE ? fp.sc.sbt[3] : c.w;
        return fast_bgra(mix_ai(c.x, 255.0f * ai.x, w), mix_ai(c.y, 255.0f * ai.y, w), mix_ai(c.z, 255.0f * ai.z, w),
                         unorm8(mix_ai(alpha, ai.w, w)));
    }
    return fast_bgra(c.x, c.y, c.z, ONE ? fp.sc.a8 : unorm8(c.w));  // ONE: the uniform alpha byte, host-folded
}

#ifndef TRI_CLIP_DEFER
#define TRI_CLIP_DEFER 1
#endif

// One bin: coverage into the LDS key tile, then shading and stores. Reached by the whole workgroup.
template <bool EXACT, int BL, bool SHADOW, bool ONE = false, bool AI = false>
__device__ __forceinline__ void raster_bin(const TriFrameParams& fp, const TriDeviceBuffers& b, const int bin) {
    constexpr int BIN = 1 << BL;
    __shared__ uint64_t keys[BIN * BIN];
    constexpr bool kBalanced = TRI_COV_BALANCED && BL == 4;
    constexpr bool kQt = TRI_QTAB && BL == 5 && (ONE || (SHADOW && TRI_QTAB_SHADOW));
    constexpr uint32_t kQw = ONE ? 3u : 4u;  // table words per entry: the slots (and the draw)
    // (the queue-position table's 3 KB come from the large-triangle queue, so that 8 workgroups still fit the LDS;
    // 192 entries rather than 384: a bin with more large triangles walks the rest per lane, C3 +0.3 %, same box)
#ifndef TRI_QTAB_BIGN
#define TRI_QTAB_BIGN 192
#endif
    constexpr int kBigN = kBalanced ? kBigQueue / 2 : ((kQt && ONE) ? TRI_QTAB_BIGN : kBigQueue);
    __shared__ uint32_t bigq[kBigN];  // queue entries of the large triangles
    __shared__ float lut[512];
    constexpr int kJobWords = (kBalanced && kCovJobs > BIN * BIN ? kCovJobs : BIN * BIN);
    __shared__ uint16_t skyq[kJobWords];  // the coverage pass's row jobs, then the skybox queue
    __shared__ CovEntry cov[kBalanced ? kCovPass : 1];
    __shared__ uint32_t wsum[TRI_BLOCK / 64];
    __shared__ uint32_t nbig, nsky;
    __shared__ uint32_t qtab[kQt ? kQw * kQtab : 1];  // TRI_QTAB: per queue position, the entry's vertex slots
    __shared__ uint16_t bigqp[kQt ? kBigN : 1];      // ... and the large triangles' queue positions
    const int tid = threadIdx.x;
    TRI_STAMP(0);
    if constexpr (TRI_COV_PRIO && BL == 5) __builtin_amdgcn_s_setprio(1 + TRI_RASTER_PRIO);  // (TRI_COV_PRIO above)
    const int bx = bin % fp.nbx, by = bin / fp.nbx;
    const int32_t ox = bx * BIN, oy = fp.y0 + by * BIN;
    const int32_t bw = min(BIN, fp.W - ox), bh = min(BIN, fp.y1 - oy);
    // Every lane loads the bin's entry count with a vector (buffer) load issued before the key-tile clear:
    // the barrier below fences LDS only, so the load stays in flight across it instead of being waited for
    // in front of it (a scalar or a lane-0 load would sit on the barrier's critical path).
    const uint32_t cnt_v = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(b.bin_count, 4ull * fp.nbins), (uint32_t)bin * 4u, 0, 0);
#ifndef TRI_QUEUE_PREFETCH
#define TRI_QUEUE_PREFETCH 1  // round-3 A/B: C3 k_raster 98.9 -> 98.0 us, C5 195.6 -> 193.3 us
#endif
    // the lane's first queue entry of the per-lane walk, in flight likewise (entries past the count are loaded
    // and ignored: the queue holds bin_cap >= 256 slots)
    uint32_t pre1 = 0;
    if constexpr (TRI_QUEUE_PREFETCH && !(TRI_COV_BALANCED && BL == 4)) {
        const Rsrc qr = make_rsrc(b.bin_list + (size_t)bin * fp.bin_cap, 4ull * fp.bin_cap);
        pre1 = __builtin_amdgcn_raw_buffer_load_b32(qr, (uint32_t)tid * 4u, 0, 0);
    }
    for (int i = tid; i < BIN * BIN; i += TRI_BLOCK) keys[i] = kBgKey;
    if (fp.need_lut)
        for (int i = tid; i < 512; i += TRI_BLOCK) lut[i] = b.srgb_lut[i];
    if (tid == 0) {
        nbig = 0;
        nsky = 0;
    }
    lds_barrier();
    TRI_STAMP(1);
    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readfirstlane((int)cnt_v);
    const uint32_t* queue = b.bin_list + (size_t)bin * fp.bin_cap;
    uint32_t s0 = 0, s1 = min(cnt, fp.bin_cap);
    // TRI_QTAB: this bin's keys carry queue positions (uniform: small bins of frames within kQPrimMax primitives)
    const bool qmode = kQt && cnt <= kQtab && fp.nprims <= kQPrimMax;
    if (kAblate & 2) {  // diagnostics: no coverage; every pixel shades the bin's first triangle
        if (s1 > s0) {
            const TriRec r = load_entry<ONE, kIdxOk<SHADOW>>(fp, b, queue[0]);
            const uint64_t key = (0x3F000000ull << 32) | key_low(r.prim_sub);
            for (int i = tid; i < BIN * BIN; i += TRI_BLOCK) keys[i] = key;
        }
        s1 = s0;
    }
  if constexpr (kBalanced) {
    uint16_t* jobs = skyq;
    const uint32_t lane = lanes_below(~0ull);
    for (uint32_t base = s0; base < s1; base += kCovPass) {  // uniform trip count
        const uint32_t i = base + tid;
        uint32_t nrows = 0;
        TriRec r;
        int32_t cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
        if (tid < kCovPass && i < s1) {
            const uint32_t ri = queue[i];
            r = load_entry<ONE, kIdxOk<SHADOW>>(fp, b, ri);
            rec_bbox(r, ox, oy, bw, bh, cx0, cx1, cy0, cy1);
            if (cx0 <= cx1 && cy0 <= cy1) {
                bool big = false;
                if ((cx1 - cx0 + 1) * (cy1 - cy0 + 1) > big_area<BL>()) {
                    const uint32_t q = atomicAdd(&nbig, 1u);
                    if (q < (uint32_t)kBigN) { bigq[q] = ri; big = true; }
                }
                if (!big) {
                    EdgeSetup e;
                    edge_setup(r, e);
                    bool rej = false;
                    CovEntry c;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        c.F[k] = clamp_edge((int64_t)e.A[k] * cx0 + (int64_t)e.B[k] * cy0 + e.D[k], rej);
                        c.A[k] = e.A[k];
                        c.B[k] = e.B[k];
                    }
                    if (!rej) {
                        c.dzdX = e.dzdX; c.dzdY = e.dzdY; c.z0 = r.z[0];
                        c.fdx0 = (float)(256 * cx0 + 128 - r.X[0]);
                        c.fdy0 = (float)(256 * cy0 + 128 - r.Y[0]);
                        c.low = key_low(r.prim_sub);
                        const bool far_clip = (r.z[0] > 1.0f) || (r.z[1] > 1.0f) || (r.z[2] > 1.0f);
                        c.pk = (uint32_t)(((cy0 - oy) << BL) + (cx0 - ox)) | ((uint32_t)(cx1 - cx0) << 12) |
                               (far_clip ? 1u << 18 : 0u);
                        cov[tid] = c;
                        nrows = (uint32_t)(cy1 - cy0 + 1);
                    }
                }
            }
        }
        // exclusive prefix sum of the row counts over the workgroup
        const uint32_t incl = wave_incl_sum(nrows);
        if (lane == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        uint32_t start = incl - nrows, total = 0;
#pragma unroll
        for (int w = 0; w < TRI_BLOCK / 64; ++w) {
            const uint32_t ws = wsum[w];
            if (w < (tid >> 6)) start += ws;
            total += ws;
        }
        for (uint32_t k = 0; k < nrows && start + k < (uint32_t)kCovJobs; ++k)
            jobs[start + k] = (uint16_t)((tid << 6) | k);
        __syncthreads();
        const uint32_t njobs = min(total, (uint32_t)kCovJobs);
        for (uint32_t j = tid; j < njobs; j += TRI_BLOCK) {
            const uint32_t jb = jobs[j];
            cov_row<BL>(cov[jb >> 6], jb & 63u, keys);
        }
        for (uint32_t k = (start < (uint32_t)kCovJobs ? (uint32_t)kCovJobs - start : 0u); k < nrows; ++k)
            cov_row<BL>(cov[tid], k, keys);  // rows past the job table: the owner walks them
        __syncthreads();  // cov / jobs / wsum are reused by the next pass
    }
  } else {
    auto cover = [&](uint32_t i, int32_t sub, int32_t step, bool first) {
        const uint32_t ri = (TRI_QUEUE_PREFETCH && first) ? pre1 : queue[i];
        uint32_t dq;
        TriRec r = load_entry_d<ONE, kIdxOk<SHADOW>>(fp, b, ri, dq);
        if (kQt && qmode) {  // the entry's slots (set-up orientation undone) at its queue position; the key's payload
            if (!(ri & TRI_ENTRY_CLIPPED)) {
                qtab[i] = r.v[0]; qtab[kQtab + i] = r.v[2]; qtab[2 * kQtab + i] = r.v[1];
                if (!ONE) qtab[3 * kQtab + i] = dq;
            }
            r.prim_sub = qenc(r.prim_sub, i);
        }
        int32_t cx0, cx1, cy0, cy1;
        rec_bbox(r, ox, oy, bw, bh, cx0, cx1, cy0, cy1);
        if (cx0 > cx1 || cy0 > cy1) return;
        if ((cx1 - cx0 + 1) * (cy1 - cy0 + 1) > big_area<BL>()) {
            if (sub != 0) return;  // the first lane of the group hands it over
            const uint32_t q = atomicAdd(&nbig, 1u);
            if (q < (uint32_t)kBigN) {
                bigq[q] = ri;
                if (kQt) bigqp[q] = (uint16_t)i;
                return;
            }
            raster_serial<BL>(r, cx0, cx1, cy0, cy1, ox, oy, keys);  // queue full: this lane walks it all
            return;
        }
#if TRI_SPAN_WALK
        raster_span<BL>(r, cx0, cx1, cy0, cy1, ox, oy, keys, sub, step);
#else
        raster_serial<BL>(r, cx0, cx1, cy0, cy1, ox, oy, keys, sub, step);
#endif
    };
    // (Pairing only as many entries as there are spare lanes when the bin holds 129..256 entries, so that
    // every lane works, measured slower: 105.5 -> 109.8 us at C3. The duplicated fetch and set-up of a
    // pair costs issue slots the CU's other workgroups would use; a wave with no entry costs none.)
    for (uint32_t i = s0 + tid; i < s1; i += TRI_BLOCK) cover(i, 0, 1, i < (uint32_t)TRI_BLOCK);
    __syncthreads();
  }
    TRI_STAMP(2);
    const uint32_t nb = min(nbig, (uint32_t)kBigN);
    for (uint32_t q = 0; q < nb; ++q) {  // large triangles: all lanes share the pixels
        TriRec r = load_entry<ONE, kIdxOk<SHADOW>>(fp, b, bigq[q]);
        if (kQt && qmode) r.prim_sub = qenc(r.prim_sub, bigqp[q]);
        int32_t cx0, cx1, cy0, cy1;
        rec_bbox(r, ox, oy, bw, bh, cx0, cx1, cy0, cy1);
        EdgeSetup e;
        edge_setup(r, e);
        bool rej = false;
        int32_t F[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) F[k] = clamp_edge((int64_t)e.A[k] * cx0 + (int64_t)e.B[k] * cy0 + e.D[k], rej);
        if (rej) continue;  // uniform across the workgroup
        const bool far_clip = (r.z[0] > 1.0f) || (r.z[1] > 1.0f) || (r.z[2] > 1.0f);
        const uint32_t low = key_low(r.prim_sub);
        const int32_t rw = cx1 - cx0 + 1, rh = cy1 - cy0 + 1;
        for (int j = tid; j < rw * rh; j += TRI_BLOCK) {
            const int32_t dy = j / rw, dx = j - dy * rw;
            const int32_t f0 = F[0] + e.A[0] * dx + e.B[0] * dy;
            const int32_t f1 = F[1] + e.A[1] * dx + e.B[1] * dy;
            const int32_t f2 = F[2] + e.A[2] * dx + e.B[2] * dy;
            if ((f0 | f1 | f2) >= 0) {
                const int32_t px = cx0 + dx, py = cy0 + dy;
                uint64_t key;
                if (depth_key(frag_depth(r, e, px, py), far_clip, low, key))
                    atomicMin(&keys[((py - oy) << BL) + (px - ox)], key);
            }
        }
    }
    __syncthreads();
    TRI_STAMP(3);
    // queue consumed (every wave's count load has completed: each waited for it, and the barrier's fence
    // covers this workgroup's global accesses): ready for the next frame
    if (tid == 0) {
#ifndef TRI_DIAG_FRONT  // diagnostics (tri_render): later frames re-raster the first frame's queues
        b.bin_count[bin] = 0;
#endif
        if (cnt > fp.bin_cap) note_bin_overflow(b, cnt);
    }
    if constexpr (TRI_COV_PRIO && BL == 5) __builtin_amdgcn_s_setprio(TRI_RASTER_PRIO);
    // shade + store: each wave covers whole BIN-pixel row pieces -> coalesced colour/depth stores.
    // Background pixels go to an LDS queue for the skybox pass below (lane-dense, and its registers
    // are not live during shading).
    const int lx = tid & (BIN - 1);
    const bool sky_on = fp.sky_size != 0;
    const bool sky_const = sky_on && !EXACT && fp.sky_mode == TRI_SKY_UNIFORM;
    const bool sky_queue = sky_on && !sky_const;
    // the background colour stays a scalar to its store (its VGPR copy, hoisted out of the loop, was the shadow
    // instantiation's one spilled register)
    const uint32_t bg_sgpr = sky_const ? fp.sky_bgra : fp.clear_bgra;
    auto bg_bgra = [&]() {
        uint32_t v = bg_sgpr;
        asm volatile("" : "+s"(v));
        return v;
    };
    // Clipped sub-triangles' pixels (rare: near-plane and guard-band crossings) are shaded after the loop, from
    // a per-wave LDS queue (a wave shades exactly BIN * BIN / 4 pixels, so its slice never overflows): the
    // loop then carries no clipped branch and no register merge at its join.
    constexpr bool kDefer = TRI_CLIP_DEFER && BL <= 5;
    constexpr int kWaveQ = BIN * BIN / (TRI_BLOCK / 64);
    __shared__ uint16_t clipq[kDefer ? BIN * BIN : 1];
    uint32_t nclip = 0;  // this wave's deferred pixels (wave-uniform)
    // (TRI_QTAB: the loop compiled twice, for bins with and without the queue-position keys, so that neither
    // carries the other's registers)
    auto shade_loop = [&](auto QT) {
        constexpr bool kq = decltype(QT)::value;
        for (int ly = tid >> BL; ly < bh; ly += TRI_BLOCK / BIN) {
            const bool in = lx < bw;
            const uint64_t key = in ? keys[(ly << BL) + lx] : 0ull;
            const bool bg = in && key == kBgKey;
            if constexpr (kDefer) {
                const bool clipped = in && !bg && (((uint32_t)key >> (kq ? 8 : 0)) & 7u) != 0u;
                const uint64_t m = __ballot(clipped);
                if (m) {  // uniform
                    if (clipped) clipq[(tid >> 6) * kWaveQ + nclip + lanes_below(m)] = (uint16_t)((ly << BL) + lx);
                    nclip += (uint32_t)__builtin_popcountll(m);
                }
                if (clipped) continue;
            }
            if (sky_queue) {  // wave-aggregated append (uniform control flow here)
                const uint64_t m = __ballot(bg);
                if (m) {
                    const uint32_t lane = lanes_below(~0ull);
                    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
                    uint32_t base = 0;
                    if (lane == leader) base = atomicAdd(&nsky, (uint32_t)__builtin_popcountll(m));
                    base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);  // leader: uniform
                    if (bg) skyq[base + lanes_below(m)] = (uint16_t)((ly << BL) + lx);
                }
            }
    #ifdef TRI_PRIM_GROUPS
            {
                const bool shade = in && !bg;
                uint64_t m = __ballot(shade);
                const uint32_t pid = shade ? ((uint32_t)key >> 3) : 0u;
                const uint32_t active = (uint32_t)__builtin_popcountll(m);
                uint32_t groups = 0;
                while (m) {
                    const uint32_t lp = (uint32_t)__shfl((int)pid, (int)__builtin_ctzll(m));
                    m &= ~__ballot(shade && pid == lp);
                    ++groups;
                }
                if ((uint32_t)(tid & 63) == (uint32_t)__builtin_ctzll(__ballot(true)) && active) {
                    atomicAdd(&g_tri_groups[0], 1ull);
                    atomicAdd(&g_tri_groups[1], (unsigned long long)groups);
                    atomicAdd(&g_tri_groups[2], (unsigned long long)active);
                }
            }
    #endif
            if (!in) continue;
            int32_t px = ox + lx;
            const int32_t py = oy + ly;
            // (the shadow instantiation: px re-formed each pixel, so that 256 px + 128, loop-invariant, is not hoisted
            // into a register held across the loop, the one its table-reading variant had to spill)
            if constexpr (SHADOW) asm volatile("" : "+v"(px));
            uint32_t out;
            float z;
            if (bg) {
                const size_t o = (size_t)(py - fp.y0) * fp.W + px;
                if (!sky_queue) b.color[o] = bg_bgra();
                if (fp.write_depth) b.depth[o] = 1.0f;
                continue;
            } else if (kAblate & 1) {  // diagnostics: coverage only
                z = __uint_as_float((uint32_t)(key >> 32));
                out = (uint32_t)key;
            } else {
                z = __uint_as_float((uint32_t)(key >> 32));
                Frag f;
                if (kAblate & 256) {  // diagnostics: 256 = no varyings fetch (a fragment made from the key)
                    const float k0 = __uint_as_float(((uint32_t)key & 0x7FFFFFu) | 0x3F000000u);
                    for (int q = 0; q < 20; ++q) (&f.wx)[q] = k0 + 0.01f * q;
                } else {
                    fetch_fragment<EXACT, SHADOW, ONE, kDefer ? 1 : 0>(fp, b, key, px, py, lut, f, kq ? qtab : nullptr);
                }
                out = shade_bgra<EXACT, ONE, AI>(fp, b, f, px, py);
            }
            const size_t o = (size_t)(py - fp.y0) * fp.W + px;
            b.color[o] = out;
            if (fp.write_depth) b.depth[o] = z;
        }
    };
    if (kQt && qmode) shade_loop(std::true_type{});
    else shade_loop(std::false_type{});
    if constexpr (kDefer) {  // this wave's clipped pixels (its own LDS slice: no workgroup barrier)
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = (uint32_t)(tid & 63); i < nclip; i += 64) {
            const uint32_t li = clipq[(tid >> 6) * kWaveQ + i];
            const int32_t qx = (int32_t)(li & (BIN - 1)), qy = (int32_t)(li >> BL);
            const uint64_t key = keys[li];
            const int32_t px = ox + qx, py = oy + qy;
            Frag f;
            fetch_fragment<EXACT, SHADOW, ONE, 2>(fp, b, key, px, py, lut, f, (kQt && qmode) ? qtab : nullptr);
            const size_t o = (size_t)(py - fp.y0) * fp.W + px;
            b.color[o] = shade_bgra<EXACT, ONE, AI>(fp, b, f, px, py);
            if (fp.write_depth) b.depth[o] = __uint_as_float((uint32_t)(key >> 32));
        }
    }
#ifdef TRI_PHASE_TIMING
    __syncthreads();
    TRI_STAMP(4);
    if (!sky_queue) { TRI_STAMP(5); return; }
#endif
    if (!sky_queue) return;
    __syncthreads();
    const uint32_t ns = nsky;
    if (fp.sky_lut && !fp.need_lut && ns > 0) {  // uniform: only bins showing sky stage the LUT
        for (int i = tid; i < 512; i += TRI_BLOCK) lut[i] = b.srgb_lut[i];
        __syncthreads();
    }
    const bool persp = !EXACT && fp.sky_mode == TRI_SKY_PERSP;
    for (uint32_t i = tid; i < ns; i += TRI_BLOCK) {  // skybox pass over the queued background pixels
        const uint32_t li = skyq[i];
        const int32_t px = ox + (int32_t)(li & (BIN - 1)), py = oy + (int32_t)(li >> BL);
        b.color[(size_t)(py - fp.y0) * fp.W + px] =
            persp ? sky_bgra_persp(fp, b, px, py, lut) : sky_bgra(fp, b, px, py, lut);
    }
#ifdef TRI_PHASE_TIMING
    __syncthreads();
    TRI_STAMP(5);
#endif
}

// 6 waves/SIMD at 32x32 bins: the fast build fits 80 VGPRs without spilling (the exact build spills
// a little); 64x64 bins are LDS-limited to 3. One workgroup per bin: a persistent grid (one resident
// round of workgroups, each walking bins blockIdx + k * gridDim on its XCD) measured 121.5 -> 154 us at C3
// (13 VGPRs spilled by values hoisted out of the bin loop, and a static bin order that balances worse
// than the dispatcher's).
template <bool EXACT, int BL, bool SHADOW>
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu(BL <= 5 ? (SHADOW ? (EXACT ? 5 : TRI_RASTER_WAVES_SHADOW) : TRI_RASTER_WAVES) : 3))) void k_raster(TRI_KARGS) {
    TRI_BIND_ARGS;
    if constexpr (SHADOW)  // the map bins' counts for the next frame (k_shadow_raster's parts only read them)
        for (uint32_t i = blockIdx.x * TRI_BLOCK + threadIdx.x; i < fp.s_nbins; i += gridDim.x * TRI_BLOCK)
            b.sbin_count[i] = 0u;
    raster_bin<EXACT, BL, SHADOW>(fp, b, xcd_bin(blockIdx.x, fp.nbins));
}
// Frames without the shadow pre-pass: this instantiation lives in its own translation unit
// (raster_plain.hip), compiled without SLP vectorisation: packed-FP32 pairs need their uniform operands
// copied into VGPR pairs, and without them the fast build fits 7 waves/SIMD with no spill (C3 k_raster
// 117 -> 112 us). Frames with the pre-pass keep k_raster<.., true> (5 waves, SLP: faster there).
template <bool EXACT, int BL, bool ONE>
// The fast single-draw solid instantiation (C3's) at 8 waves/SIMD: with its parameters read through the frame's
// argument pointer the compiler fills a 7-wave budget (71 VGPRs) where 8 waves fit in 58 with a few SGPRs
// spilled to VGPR lanes.
#ifndef TRI_RASTER_WAVES_PLAIN_ONE
#define TRI_RASTER_WAVES_PLAIN_ONE 8
#endif
// TRI_RASTER_ONE_VGPRS: cap the fast single-draw instantiation's VGPRs below the 64 that 8 waves/SIMD allow, so that a
// concurrent frame's front-end wave (k_setup within 64, TRI_SETUP_WAVES_ONE) fits the register file beside 8 raster
// waves instead of displacing one. On gfx950's unified register file the attribute's value is doubled: 28 caps at 56
// VGPRs; 0 = no cap.
#ifndef TRI_RASTER_ONE_VGPRS
#define TRI_RASTER_ONE_VGPRS 28
#endif
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu(BL <= 5 ? ((ONE && !EXACT) ? TRI_RASTER_WAVES_PLAIN_ONE : TRI_RASTER_WAVES_PLAIN) : 3))) void k_raster_plain(TRI_KARGS) {
    TRI_BIND_ARGS;
    raster_bin<EXACT, BL, false, ONE>(fp, b, xcd_bin(blockIdx.x, fp.nbins));
}
#if TRI_RASTER_ONE_VGPRS && defined(TRI_RASTER_PLAIN_TU)  // C3's instantiation as an explicit specialization: the cap
                                                        // takes no template-dependent value (raster_plain.hip's)
template <>
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu(8))) __attribute__((amdgpu_num_vgpr(TRI_RASTER_ONE_VGPRS))) void k_raster_plain<false, 5, true>(TRI_KARGS) {
    TRI_BIND_ARGS;
    raster_bin<false, 5, false, true>(fp, b, xcd_bin(blockIdx.x, fp.nbins));
}
#endif
// Frames with Default.frag's AI frame blend (AiBlendConfig.w > 0, an uploaded AI frame; never with the shadow
// pre-pass, which the reference does not have): the general instantiation plus the blend
template <bool EXACT, int BL>
__global__ __launch_bounds__(TRI_BLOCK) __attribute__((amdgpu_waves_per_eu(BL <= 5 ? TRI_RASTER_WAVES_PLAIN : 3))) void k_raster_ai(TRI_KARGS) {
    TRI_BIND_ARGS;
    raster_bin<EXACT, BL, false, false, true>(fp, b, xcd_bin(blockIdx.x, fp.nbins));
}

// ------------------------------------------------------------------------------------------
// shadow pre-pass raster (oracle shadow_raster_triangle): one workgroup per 32x32 bin of the s_size^2
// map, the bin's depth tile in LDS (min over covering fragments of the [0, 1]-clamped plane depth, as
// uint32 bits: order-free), then one coalesced store of the tile. The triangle of a queue entry is
// rebuilt from its three map snaps (prim_slots -> lsnap), oriented like the set-up (v1 <-> v2 swapped when
// S < 0, kept when S > 0: no culling).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ TriRec load_shadow_entry(const TriFrameParams& fp, const TriDeviceBuffers& b, uint32_t e) {
    const Rsrc snr = make_rsrc(b.lsnap, 16ull * fp.nslots);
    uint32_t sl[3], d;
    prim_slots<false, kIdxOk<true>>(fp, b, e, sl, d);
    const uint4 q0 = ld128(snr, sl[0] * 16u), q1 = ld128(snr, sl[1] * 16u), q2 = ld128(snr, sl[2] * 16u);
    const int32_t X0 = ((int32_t)q0.x << 8) >> 8, X1 = ((int32_t)q1.x << 8) >> 8, X2 = ((int32_t)q2.x << 8) >> 8;
    const int32_t Y0 = (int32_t)q0.y, Y1 = (int32_t)q1.y, Y2 = (int32_t)q2.y;
    const int64_t S = (int64_t)(X1 - X0) * (int64_t)(Y2 - Y0) - (int64_t)(Y1 - Y0) * (int64_t)(X2 - X0);
    const bool sw = S < 0;
    TriRec r;
    r.X[0] = X0; r.Y[0] = Y0; r.z[0] = __uint_as_float(q0.w);
    r.X[1] = sw ? X2 : X1; r.Y[1] = sw ? Y2 : Y1; r.z[1] = __uint_as_float(sw ? q2.w : q1.w);
    r.X[2] = sw ? X1 : X2; r.Y[2] = sw ? Y1 : Y2; r.z[2] = __uint_as_float(sw ? q1.w : q2.w);
    r.iw[0] = r.iw[1] = r.iw[2] = 1.0f;
    r.prim_sub = e << 3;
    r.v[0] = r.v[1] = r.v[2] = 0;
    return r;
}

// Depth clamp to [0, 1] on the float bits (finite depth: the plane of snapped vertices with S != 0):
// negative (sign set, -0 included) -> +0, above 1 -> 1.
__device__ __forceinline__ uint32_t clamp_depth_bits(float z) {
    return (uint32_t)min(max(__float_as_int(z), 0), 0x3F800000);
}

// Slope-scaled depth bias of a caster (depthBiasSlopeFactor): slope * its largest depth change per texel.
__device__ __forceinline__ float slope_offset(const TriFrameParams& fp, const EdgeSetup& e) {
    return fp.s_slope * (fmaxf(fabsf(e.dzdX), fabsf(e.dzdY)) * 256.0f);
}

__device__ __forceinline__ void shadow_serial(const TriFrameParams& fp, const TriRec& r, int32_t cx0, int32_t cx1,
                                              int32_t cy0, int32_t cy1, int32_t ox, int32_t oy, uint32_t* dep,
                                              int32_t sub, int32_t step) {
    EdgeSetup e;
    edge_setup(r, e);
    const float off = slope_offset(fp, e);
    bool rej = false;
    int32_t F[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] = clamp_edge((int64_t)e.A[k] * cx0 + (int64_t)e.B[k] * cy0 + e.D[k], rej);
    if (rej) return;
    const float fdx0 = (float)(256 * cx0 + 128 - r.X[0]);
    float fdy = (float)(256 * (cy0 + sub) + 128 - r.Y[0]);
    uint32_t row = (uint32_t)(((cy0 + sub - oy) << 5) + (cx0 - ox));
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] += e.B[k] * sub;
    for (int32_t py = cy0 + sub; py <= cy1; py += step) {
        const float t2 = e.dzdY * fdy;
        int32_t f0 = F[0], f1 = F[1], f2 = F[2];
        float fdx = fdx0;
        const uint32_t rend = row + (uint32_t)(cx1 - cx0);
        for (uint32_t a = row; a <= rend; ++a) {
            if ((f0 | f1 | f2) >= 0) atomicMin(&dep[a], clamp_depth_bits(((r.z[0] + e.dzdX * fdx) + t2) + off));
            f0 += e.A[0]; f1 += e.A[1]; f2 += e.A[2];
            fdx += 256.0f;
        }
        F[0] += e.B[0] * step; F[1] += e.B[1] * step; F[2] += e.B[2] * step;
        fdy += 256.0f * (float)step;
        row += (uint32_t)step << 5;
    }
}

// The span walk of raster_span for the map (triangles under 64 px on a side; the rest keep shadow_serial):
// each map row's covered texels from the three edge crossings, exact by the same argument, the same depth
// (plane + slope bias, clamped) as shadow_serial.
__device__ __forceinline__ void shadow_span(const TriFrameParams& fp, const TriRec& r, int32_t cx0, int32_t cx1,
                                            int32_t cy0, int32_t cy1, int32_t ox, int32_t oy, uint32_t* dep,
                                            int32_t sub, int32_t step) {
    const int32_t xmin = min(r.X[0], min(r.X[1], r.X[2])), xmax = max(r.X[0], max(r.X[1], r.X[2]));
    const int32_t ymin = min(r.Y[0], min(r.Y[1], r.Y[2])), ymax = max(r.Y[0], max(r.Y[1], r.Y[2]));
    if (!(xmax - xmin < 16384 && ymax - ymin < 16384)) {
        shadow_serial(fp, r, cx0, cx1, cy0, cy1, ox, oy, dep, sub, step);
        return;
    }
    int32_t A[3], B[3], F[3];
    EdgeSetup e;
    edge_start(r, cx0, cy0, A, B, F, e.dzdX, e.dzdY);  // the 32-bit form (same integers and depth plane)
    const float off = slope_offset(fp, e);
    constexpr float kDelta = 0x1p-15f;
    float nrl[3], dl[3], nrr[3], dr[3], Ff[3], Bs[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float rc = -__builtin_amdgcn_rcpf((float)A[k]);
        nrl[k] = A[k] > 0 ? rc : (A[k] == 0 ? -0x1p100f : 0.0f);
        dl[k] = A[k] >= 0 ? -kDelta : -INFINITY;
        nrr[k] = A[k] < 0 ? rc : 0.0f;
        dr[k] = A[k] < 0 ? kDelta : INFINITY;
        Ff[k] = (float)(F[k] + B[k] * sub);
        Bs[k] = (float)(B[k] * step);
    }
    const float wmax = (float)(cx1 - cx0);
    const int32_t fx0 = 256 * cx0 + 128 - r.X[0];
    float fdy = (float)(256 * (cy0 + sub) + 128 - r.Y[0]);
    uint32_t row = (uint32_t)(((cy0 + sub - oy) << 5) + (cx0 - ox));
    for (int32_t py = cy0 + sub; py <= cy1; py += step) {
        const float tl = fmaxf(fmaxf(__builtin_fmaf(Ff[0], nrl[0], dl[0]), __builtin_fmaf(Ff[1], nrl[1], dl[1])),
                               __builtin_fmaf(Ff[2], nrl[2], dl[2]));
        const float tr = fminf(fminf(__builtin_fmaf(Ff[0], nrr[0], dr[0]), __builtin_fmaf(Ff[1], nrr[1], dr[1])),
                               __builtin_fmaf(Ff[2], nrr[2], dr[2]));
        const float Lf = fmaxf(ceilf(tl), 0.0f), Rf = fminf(floorf(tr), wmax);
        if (Lf <= Rf) {
            const int32_t L = (int32_t)Lf, R = (int32_t)Rf;
            const float t2 = e.dzdY * fdy;
            float fdx = (float)(fx0 + 256 * L);
            const uint32_t rend = row + (uint32_t)R;
            for (uint32_t a = row + (uint32_t)L; a <= rend; ++a) {
                atomicMin(&dep[a], clamp_depth_bits(((r.z[0] + e.dzdX * fdx) + t2) + off));
                fdx += 256.0f;
            }
        }
        Ff[0] += Bs[0]; Ff[1] += Bs[1]; Ff[2] += Bs[2];
        fdy += 256.0f * (float)step;
        row += (uint32_t)step << 5;
    }
}

// The map's bins are very uneven (C5: 1294 of 4096 hold casters, 773 on average, 4042 at most — the light sees
// the grid at a grazing angle), and one workgroup per bin made the heaviest bins the whole kernel. Each bin now
// has TRI_SHADOW_PARTS workgroups: part p takes the bin's entries in blocks of 256, every TRI_SHADOW_PARTS-th block,
// into its own LDS tile. A bin with one block keeps one workgroup and stores its tile; with more, every part
// atomicMin's the texels it covered into the map, which k_setup<true> cleared to 1.0 (k_raster zeroes the bins'
// counts for the next frame: the parts of a bin cannot tell which of them reads its count last).
#ifndef TRI_SHADOW_PARTS
#define TRI_SHADOW_PARTS 4
#endif
#if TRI_MAIN_TU
__global__ __launch_bounds__(TRI_BLOCK) void k_shadow_raster(TRI_KARGS) {
    TRI_BIND_ARGS;
    constexpr int BIN = 32;
    constexpr uint32_t kParts = TRI_SHADOW_PARTS;
    __shared__ uint32_t dep[BIN * BIN];
    __shared__ uint32_t bigq[kBigQueue];
    __shared__ uint32_t nbig, nentries;
    const int tid = threadIdx.x;
    // parts of one bin lie s_nbins workgroups apart: the same XCD (s_nbins is a multiple of 8) and its L2
    const uint32_t part = blockIdx.x / fp.s_nbins;
    const int bin = xcd_bin((int)(blockIdx.x - part * fp.s_nbins), (int)fp.s_nbins);
    const int32_t S = (int32_t)fp.s_size;
    const int32_t ox = (bin % (int)fp.s_nbx) * BIN, oy = (bin / (int)fp.s_nbx) * BIN;
    const int32_t bw = min(BIN, S - ox), bh = min(BIN, S - oy);
    if (tid == 0) {
        nbig = 0;
        const uint32_t cnt = b.sbin_count[bin];
        if (cnt > fp.s_bin_cap && part == 0) note_shadow_bin_overflow(b, cnt);
        nentries = min(cnt, fp.s_bin_cap);
    }
    __syncthreads();
    const uint32_t n = nentries;
    // nothing for this part (the map is already 1.0 there: k_setup<true> cleared it — unless the frame had no
    // primitives, no k_setup, and part 0 writes the empty tile itself)
    const bool store_empty = part == 0 && fp.nchunks == 0;
    if (n <= part * (uint32_t)TRI_BLOCK && !store_empty) return;
    for (int i = tid; i < BIN * BIN; i += TRI_BLOCK) dep[i] = 0x3F800000u;  // clear 1.0
    __syncthreads();
    const uint32_t* queue = b.sbin_list + (size_t)bin * fp.s_bin_cap;
    const int share = n <= (uint32_t)(TRI_BLOCK / TRI_SHADOW_SHARE) ? TRI_SHADOW_SHARE : 1;
    const int sub = tid % share;
    const uint32_t step = share > 1 ? (uint32_t)(TRI_BLOCK / share) : (uint32_t)TRI_BLOCK * kParts;
    for (uint32_t i = tid / share + part * (uint32_t)TRI_BLOCK; i < n; i += step) {
        const uint32_t ri = queue[i];
        const TriRec r = load_shadow_entry(fp, b, ri);
        int32_t cx0, cx1, cy0, cy1;
        rec_bbox(r, ox, oy, bw, bh, cx0, cx1, cy0, cy1);
        if (cx0 > cx1 || cy0 > cy1) continue;
        if ((cx1 - cx0 + 1) * (cy1 - cy0 + 1) > big_area<5>()) {
            if (sub != 0) continue;
            const uint32_t q = atomicAdd(&nbig, 1u);
            if (q < kBigQueue) { bigq[q] = ri; continue; }
            shadow_serial(fp, r, cx0, cx1, cy0, cy1, ox, oy, dep, 0, 1);
            continue;
        }
#if TRI_SPAN_WALK
        shadow_span(fp, r, cx0, cx1, cy0, cy1, ox, oy, dep, sub, share);
#else
        shadow_serial(fp, r, cx0, cx1, cy0, cy1, ox, oy, dep, sub, share);
#endif
    }
    __syncthreads();
    const uint32_t nb = min(nbig, (uint32_t)kBigQueue);
    for (uint32_t q = 0; q < nb; ++q) {  // large triangles: all lanes share the texels
        const TriRec r = load_shadow_entry(fp, b, bigq[q]);
        int32_t cx0, cx1, cy0, cy1;
        rec_bbox(r, ox, oy, bw, bh, cx0, cx1, cy0, cy1);
        EdgeSetup e;
        edge_setup(r, e);
        bool rej = false;
        int32_t F[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) F[k] = clamp_edge((int64_t)e.A[k] * cx0 + (int64_t)e.B[k] * cy0 + e.D[k], rej);
        if (rej) continue;  // uniform across the workgroup
        const float off = slope_offset(fp, e);
        const int32_t rw = cx1 - cx0 + 1, rh = cy1 - cy0 + 1;
        for (int j = tid; j < rw * rh; j += TRI_BLOCK) {
            const int32_t dy = j / rw, dx = j - dy * rw;
            if ((F[0] + e.A[0] * dx + e.B[0] * dy | F[1] + e.A[1] * dx + e.B[1] * dy | F[2] + e.A[2] * dx + e.B[2] * dy) >= 0) {
                const int32_t px = cx0 + dx, py = cy0 + dy;
                atomicMin(&dep[((py - oy) << 5) + (px - ox)], clamp_depth_bits(frag_depth(r, e, px, py) + off));
            }
        }
    }
    __syncthreads();
    const bool alone = n <= (uint32_t)TRI_BLOCK || kParts == 1 || store_empty;  // one part: its tile is the bin's
    for (int i = tid; i < BIN * BIN; i += TRI_BLOCK) {
        const int32_t ly = i >> 5, lx = i & 31;
        if (lx < bw && ly < bh) {
            const size_t o = (size_t)(oy + ly) * S + ox + lx;
            if (alone) b.shadow_map[o] = dep[i];
            else if (dep[i] != 0x3F800000u) atomicMin(&b.shadow_map[o], dep[i]);  // depth bits order as integers
        }
    }
}
#endif

// ------------------------------------------------------------------------------------------
// presentation blit (Renderer.cpp:5346-5361, vkCmdBlitImage with VK_FILTER_LINEAR): one lane per
// destination texel; the source coordinate of its centre is (x + 0.5) * (W / dw), filtered
// bilinearly over clamp-to-edge taps on UNORM values (b / 255), rounded to UNORM8. Same float
// operation order as the oracle's blit_linear (bit-exact). Rows are coalesced per wave. The 256-entry
// UNORM table is staged in LDS: read from global memory it was 16 wave-level gathers per texel on the texture
// path, which held a 4K blit at ≈ 70 µs beside the next frame's raster (tri_launch_blit copies an equal-size
// blit instead: its weights are 0 and every channel rounds back to its byte).
// ------------------------------------------------------------------------------------------
#if TRI_MAIN_TU
__global__ __launch_bounds__(TRI_BLOCK) void k_blit(const uint32_t* __restrict__ src, int32_t w, int32_t h,
                                                    uint32_t* __restrict__ dst, int32_t dw, int32_t dh, float sx,
                                                    float sy, const float* __restrict__ lut) {
    __shared__ float tab[256];
    for (int i = (int)threadIdx.x; i < 256; i += TRI_BLOCK) tab[i] = lut[i];
    __syncthreads();
    const int32_t x = (int32_t)(blockIdx.x * 64 + (threadIdx.x & 63));
    const int32_t y = (int32_t)(blockIdx.y * (TRI_BLOCK / 64) + (threadIdx.x >> 6));
    if (x >= dw || y >= dh) return;
    const float u = ((float)x + 0.5f) * sx - 0.5f;
    const float v = ((float)y + 0.5f) * sy - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const float a = u - fu, bb = v - fv;
    const int32_t i0 = (int32_t)fu, j0 = (int32_t)fv;
    const int32_t xa = min(max(i0, 0), w - 1), xb = min(max(i0 + 1, 0), w - 1);
    const int32_t ya = min(max(j0, 0), h - 1), yb = min(max(j0 + 1, 0), h - 1);
    const uint32_t p00 = src[(size_t)ya * w + xa], p10 = src[(size_t)ya * w + xb];
    const uint32_t p01 = src[(size_t)yb * w + xa], p11 = src[(size_t)yb * w + xb];
    uint32_t out = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float t00 = tab[(p00 >> (8 * c)) & 0xFFu], t10 = tab[(p10 >> (8 * c)) & 0xFFu];
        const float t01 = tab[(p01 >> (8 * c)) & 0xFFu], t11 = tab[(p11 >> (8 * c)) & 0xFFu];
        const float l0 = t00 + a * (t10 - t00);
        const float l1 = t01 + a * (t11 - t01);
        out |= unorm8(l0 + bb * (l1 - l0)) << (8 * c);
    }
    dst[(size_t)y * dw + x] = out;
}
#endif

}  // namespace

#ifdef TRI_VERTEX_TU
const void* tri_vertex_stage_kernel(TriFrontKernel k) {
    auto f = [](auto kernel) { return reinterpret_cast<const void*>(kernel); };
    return k == kFrontVertex ? f(k_vertex) : k == kFrontBand ? f(k_vertex_band) : f(k_reset);
}
#endif

#ifdef TRI_RASTER_PLAIN_TU
const void* tri_raster_plain_kernel(const TriFrameParams& fp) {
    // ONE: a single draw over a 1x1 texture slot (the common untextured mesh), the specialised instantiation
    const bool one = fp.one_draw && fp.shade_solid;
    const int bl = fp.bin_log2 == 5 ? 5 : fp.bin_log2 == 4 ? 4 : 6;
    const int sel = (fp.exact_shading ? 1 : 0) | (one ? 2 : 0);
    auto f = [](auto kernel) { return reinterpret_cast<const void*>(kernel); };
    if (fp.ai_on) {  // (the host keeps such frames off the ONE instantiation's 36-B varyings)
        if (bl == 5) return fp.exact_shading ? f(k_raster_ai<true, 5>) : f(k_raster_ai<false, 5>);
        if (bl == 4) return fp.exact_shading ? f(k_raster_ai<true, 4>) : f(k_raster_ai<false, 4>);
        return fp.exact_shading ? f(k_raster_ai<true, 6>) : f(k_raster_ai<false, 6>);
    }
    if (bl == 5) {
        if (sel == 0) return f(k_raster_plain<false, 5, false>); if (sel == 1) return f(k_raster_plain<true, 5, false>);
        if (sel == 2) return f(k_raster_plain<false, 5, true>); return f(k_raster_plain<true, 5, true>);
    }
    if (bl == 4) {
        if (sel == 0) return f(k_raster_plain<false, 4, false>); if (sel == 1) return f(k_raster_plain<true, 4, false>);
        if (sel == 2) return f(k_raster_plain<false, 4, true>); return f(k_raster_plain<true, 4, true>);
    }
    if (sel == 0) return f(k_raster_plain<false, 6, false>); if (sel == 1) return f(k_raster_plain<true, 6, false>);
    if (sel == 2) return f(k_raster_plain<false, 6, true>); return f(k_raster_plain<true, 6, true>);
}
#ifdef TRI_PRIM_GROUPS
extern "C" int tri_debug_prim_groups(unsigned long long* out3, int reset) {  // k_raster_plain's counts
    if (reset) {
        const unsigned long long z[3] = {0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_tri_groups), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(out3, HIP_SYMBOL(g_tri_groups), 3 * sizeof(unsigned long long), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
#ifdef TRI_PHASE_TIMING
extern "C" int tri_debug_phase_times(unsigned long long* out, int nslots) {  // k_raster_plain's stamps
    const size_t n = (size_t)(nslots < kPhaseSlots ? nslots : kPhaseSlots) * 6 * sizeof(unsigned long long);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tri_phase), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
#endif  // TRI_RASTER_PLAIN_TU

#if TRI_MAIN_TU
hipError_t tri_kernels_init() { return hipSuccess; }

template <bool EXACT, int BL>
static const void* raster_kernel(const TriFrameParams& fp) {
    if (fp.shadow_on) return reinterpret_cast<const void*>(k_raster<EXACT, BL, true>);
    return tri_raster_plain_kernel(fp);  // raster_plain.hip
}

void tri_plan_frame(const TriFrameParams& fp, TriFramePlan& plan) {
    plan.n = 0;
    auto add = [&](const void* f, dim3 g, dim3 t, int stage) { plan.k[plan.n++] = TriKernelLaunch{f, g, t, stage}; };
    auto F = [](auto kernel) { return reinterpret_cast<const void*>(kernel); };
    const dim3 t(TRI_BLOCK);
    if (fp.nslots > 0 && fp.cull_vertex && fp.one_draw)
        // one workgroup per four vertex blocks (TRI_VBLOCK == TRI_BLOCK slots each)
        add(tri_vertex_stage_kernel(kFrontBand), dim3((fp.nslots + 4u * TRI_VBLOCK - 1) / (4u * TRI_VBLOCK)), t, kStageVertex);
    else if (fp.nslots > 0)
        // with cluster culling every (draw, cluster) flag needs a lane, even when a mesh has fewer vertices
        add(tri_vertex_stage_kernel(kFrontVertex), dim3(((fp.cull_on && fp.ncl_total > fp.nslots ? fp.ncl_total : fp.nslots) + TRI_BLOCK - 1) / TRI_BLOCK),
            t, kStageVertex);
    else
        add(tri_vertex_stage_kernel(kFrontReset), dim3(1), dim3(TRI_BLOCK), kStageVertex);
    if (fp.nchunks > 0) {  // with the pre-pass, one set-up pass bins each primitive for the frame and the map
        const dim3 g(fp.setup_multi ? (fp.nchunks + 3u) / 4u : fp.nchunks);
        const void* k = fp.shadow_on ? (fp.one_draw ? F(k_setup<true, true>) : F(k_setup<true, false>))
                                     : (fp.one_draw ? F(k_setup<false, true>) : F(k_setup<false, false>));
        add(k, g, t, kStageSetup);
    }
    if (fp.shadow_on)  // the map's depth raster, before the frame's raster samples it
        add(F(k_shadow_raster), dim3(fp.s_nbins * TRI_SHADOW_PARTS), t, kStageShadow);
    const void* r;
    if (fp.bin_log2 == 5) r = fp.exact_shading ? raster_kernel<true, 5>(fp) : raster_kernel<false, 5>(fp);
    else if (fp.bin_log2 == 4) r = fp.exact_shading ? raster_kernel<true, 4>(fp) : raster_kernel<false, 4>(fp);
    else r = fp.exact_shading ? raster_kernel<true, 6>(fp) : raster_kernel<false, 6>(fp);
    add(r, dim3(fp.nbins), t, kStageRaster);
}

#ifdef TRI_DIAG_FRONT
// Diagnostics build: what the front end costs a frame beside its raster (tri_render): 1 = after a context's first
// frame only k_raster runs (over that frame's queues, which it keeps), 2 = the same with two empty launches in place
// of k_vertex and k_setup (the launches and their stream order, without their work), 3 = k_vertex and k_raster
__global__ void k_diag_empty(const TriLaunchArgs*) {}
void tri_diag_front_plan(TriFramePlan& plan) {
    TriFramePlan q;
    q.n = 0;
    for (uint32_t i = 0; i < plan.n; ++i) {
        if (plan.k[i].stage == kStageRaster || (TRI_DIAG_FRONT == 3 && plan.k[i].stage == kStageVertex)) q.k[q.n++] = plan.k[i];
        else if (TRI_DIAG_FRONT == 2) q.k[q.n++] = TriKernelLaunch{reinterpret_cast<const void*>(k_diag_empty), dim3(1), dim3(64), kStageSetup};
    }
    plan = q;
}
#endif

hipError_t tri_run_plan(const TriFramePlan& plan, const TriLaunchArgs& args, TriLaunchArgs* d_args,
                        hipStream_t stream, hipEvent_t* ev) {
    hipError_t e = hipSuccess;
    bool setup_stamped = false;
    if (ev && (plan.n == 0 || plan.k[0].stage != kStageVertex)) (void)hipEventRecord(ev[kStageVertex], stream);
    for (uint32_t i = 0; i < plan.n; ++i) {
        const TriKernelLaunch& k = plan.k[i];
        if (ev) {
            // stamps in the order the stages run; a frame without set-up still stamps it (zero length)
            if ((k.stage == kStageRaster || k.stage == kStageShadow) && !setup_stamped) {
                (void)hipEventRecord(ev[kStageSetup], stream);
                setup_stamped = true;
            }
            if (k.stage == kStageSetup) setup_stamped = true;
            (void)hipEventRecord(ev[k.stage], stream);
        }
        void* first[] = {const_cast<TriLaunchArgs*>(&args), &d_args};
        void* later[] = {&d_args};
        // the frame's first kernel (k_vertex's stage) takes the arguments by value and publishes them
        e = hipLaunchKernel(k.func, k.grid, k.block, k.stage == kStageVertex ? first : later, 0, stream);
        if (e != hipSuccess) return e;
    }
    if (ev) (void)hipEventRecord(ev[kStageCount], stream);
    return hipGetLastError();
}

hipError_t tri_launch_blit(const uint32_t* src, int32_t w, int32_t h, uint32_t* dst, int32_t dw, int32_t dh,
                           const float* unorm_lut, hipStream_t stream) {
    if (w == dw && h == dh)  // u = x, v = y: both weights 0, and unorm8(b / 255) == b for every byte
        return hipMemcpyAsync(dst, src, (size_t)w * h * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream);
    const float sx = (float)w / (float)dw, sy = (float)h / (float)dh;
    const dim3 g((uint32_t)((dw + 63) / 64), (uint32_t)((dh + TRI_BLOCK / 64 - 1) / (TRI_BLOCK / 64)));
    hipLaunchKernelGGL(k_blit, g, dim3(TRI_BLOCK), 0, stream, src, w, h, dst, dw, dh, sx, sy, unorm_lut);
    return hipGetLastError();
}

#ifdef TRI_PHASE_TIMING
extern "C" int tri_debug_setup_times(unsigned long long* out, int nslots) {
    const size_t n = (size_t)(nslots < kPhaseSlots ? nslots : kPhaseSlots) * 4 * sizeof(unsigned long long);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tri_setup_phase), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
#endif
