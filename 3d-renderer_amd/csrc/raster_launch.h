// raster_launch.h — host-side launchers for the gfx950 kernels (implemented in raster_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include "raster_common.h"

// k_setup occupancy target (waves per SIMD); with 4 waves per workgroup, also its workgroups per CU
// TRI_IDX_ROUTE: frames of a few draws over concatenated meshes reach a primitive's vertex slots through the index
// buffer (TriFrameParams::idx_route) instead of a per-primitive prim_vs record; 0 keeps the records
#ifndef TRI_IDX_ROUTE
#define TRI_IDX_ROUTE 1
#endif
// TRI_IDX_ROUTE_SHADOW: the route on frames with the shadow pre-pass too (its fragments read their slots and draw from
// the queue-position table, so only the coverage pass, the map raster and the table's fallback search the draws)
#ifndef TRI_IDX_ROUTE_SHADOW
#define TRI_IDX_ROUTE_SHADOW 0
#endif
#ifndef TRI_SETUP_WAVES
#define TRI_SETUP_WAVES 6
#endif
#ifndef TRI_SETUP_WGS_PER_CU
#define TRI_SETUP_WGS_PER_CU TRI_SETUP_WAVES
#endif
// k_setup workgroups per CU for frames without the shadow pre-pass. With frames in flight, one frame's set-up runs
// beside another frame's k_raster, and every resident set-up workgroup holds wave slots and LDS that the raster's
// bins cannot use while it waits on its fetch -> atomic -> store chain. Fewer, longer workgroups (more primitives
// per lane) make the set-up slower alone (C3 27.9 -> 37 us) but the frame rate higher (C3 10.39-10.43k -> 10.55k,
// C3 under a TRS draw +1 %, C2 unchanged: its set-up is one primitive per lane either way). The shadow set-up bins
// every primitive twice and keeps the resident round (C5 4.90k -> 4.75k with 2). Round 6: with the single-draw set-up
// within 64 VGPRs and the raster's C3 instantiation within 56 (raster_kernels.hip: TRI_SETUP_WAVES_ONE,
// TRI_RASTER_ONE_VGPRS) a set-up wave displaces at most one raster wave, and 3 per CU beat 2 (same-box A/B).
// k_setup's chunk target for bands (cluster culling): most chunks are culled and exit at once
#ifndef TRI_SETUP_BAND_CHUNKS
#define TRI_SETUP_BAND_CHUNKS 4096
#endif
#ifndef TRI_SETUP_WGS_PER_CU_OVERLAP
#define TRI_SETUP_WGS_PER_CU_OVERLAP 3
#endif

// Device pointers in the global address space (device compilation only; the host sees plain pointers of the same
// size). The later kernels of a frame read these pointers from the device copy of their arguments, not from
// kernel-argument memory, so without the qualifier the compiler cannot tell them from LDS pointers: every access
// became a flat instruction, which counts against the LDS wait counter too (a wait for an LDS result then also
// waits for every outstanding memory load).
// (Only in the kernels' translation units, TRI_KERNEL_TU: host code elsewhere fills the struct with plain pointers,
// and the device pass of a host-only file still type-checks those assignments.)
#if defined(__HIP_DEVICE_COMPILE__) && defined(TRI_KERNEL_TU)
#define TRI_G __attribute__((address_space(1)))
#else
#define TRI_G
#endif

// TRI_UCOL: vary_obj frames over a geometry whose vertices share one colour take it from the frame arguments
// (TriFrameParams::obj_ucol)
#ifndef TRI_UCOL
#define TRI_UCOL 1
#endif
// TRI_OBJ48: object-space varyings outside the ONE instantiation (TriFrameParams::obj48); 0 keeps world-space varyings
#ifndef TRI_OBJ48
#define TRI_OBJ48 1
#endif

struct TriDeviceBuffers {
    TRI_G const TriVsIn* vin;
    TRI_G const float* vpos;           // 12 B per vertex: the positions alone (k_vertex's only input with vary_obj)
    TRI_G const float* vattr;          // 36 B per vertex {pos, normal, colour}: the fragment stage's records with vary_obj
    TRI_G const TriVsSkin* vskin;      // may be null when no draw skins
    TRI_G const float* bones;
    uint64_t vertex_count;
    TRI_G const uint32_t* indices;
    TRI_G const TriDrawDev* draws;
    TRI_G const TriDrawShade* draw_shade;
    TRI_G const uint32_t* draw_vbase;  // ndraws+1
    TRI_G const uint32_t* draw_pbase;  // ndraws+1
    TRI_G const uint32_t* sky;         // 6 * sky_size^2 RGBA8 sRGB texels (+X,-X,+Y,-Y,+Z,-Z)
    TRI_G const float* srgb_lut;       // 256 sRGB -> linear (host, double) + 256 alpha b/255
    TRI_G float4* clip;                // nslots (read only when a primitive is clipped)
    TRI_G TriSnap* snap;               // nslots (TRI_SNAP_F: {X, Y as exact floats, 1/w, z})
    TRI_G uint8_t* oc;                 // nslots outcodes (TRI_SNAP_F; otherwise they ride in snap's X word)
    TRI_G float4* vary;                // 3 * (nslots + ovf_vert_cap)
    TRI_G TriRec* recs;                // ovf_rec_cap clipped sub-triangles
    TRI_G uint32_t* clip_slot;         // nprims: first sub-triangle record of a clipped primitive
    TRI_G uint4* prim_vs;              // nprims: {vertex slot 0, 1, 2, draw | TRI_PRIM_CLIPPED} of every
                                 // primitive k_setup passed on (visible or clipped)
    TRI_G uint32_t* bin_count;         // nbins entry counters (zero between frames: k_raster re-zeroes)
    TRI_G uint32_t* bin_list;          // nbins * bin_cap record ids (fixed-capacity queue per bin)
    TRI_G TriCounters* counters;
    TRI_G uint2* setup_stats;          // nchunks {triangles set up, bin entries} per k_setup workgroup
    TRI_G uint32_t* color;             // band rows * W
    TRI_G float* depth;                // band rows * W (may be null)
    // cluster culling (only when TriFrameParams::cull_on)
    TRI_G const TriCluster* clusters;  // all meshes' clusters
    TRI_G const TriCluster* vbox;      // per mesh vertex block: the union box of the clusters referencing it
    TRI_G const uint32_t* draw_cbase;  // ndraws+1: first (draw, cluster) pair of each draw
    TRI_G uint32_t* cvis;              // ncl_total visibility flags, written by k_vertex each frame
    // shadow-map pre-pass (only when TriFrameParams::shadow_on)
    TRI_G float4* lpos;                // nslots + ovf_vert_cap: light-NDC position per vertex slot (xyz, 0)
    TRI_G TriSnap* lsnap;              // nslots: the light-NDC position snapped to the map ({X | outcode << 24, Y, 1, z})
    TRI_G uint32_t* sbin_count;        // s_nbins shadow-map bin counters (zeroed by k_shadow_raster)
    TRI_G uint32_t* sbin_list;         // s_nbins * s_bin_cap primitive ids
    TRI_G uint32_t* shadow_map;        // s_size * s_size float32 depth bits
    TRI_G const uint32_t* ai_frame;    // the AI blend's RGBA8 UNORM frame (only when TriFrameParams::ai_on)
};

// One frame's arguments (DESIGN.md §2 "launch cost"). The frame's first kernel (k_vertex, k_vertex_band or
// k_reset) takes them by value — kernel-argument memory, which its many short waves read fastest — and its
// workgroup 0 publishes them to a device copy that every later kernel of the frame reads through a 16-B
// pointer argument (k_setup, k_shadow_raster, k_raster: one kernarg block of 1.8 KB per frame instead of one
// per launch). Stream order makes the copy complete before k_setup starts and keeps the next frame's copy
// behind this frame's raster.
struct TriLaunchArgs {
    TriFrameParams fp;
    TriDeviceBuffers b;
};
static_assert(sizeof(TriLaunchArgs) % 16 == 0, "TriLaunchArgs moves in 16-B pieces");

// The kernels of one frame in launch order (which instantiation, grid, block) — computed on the host from the
// frame's parameters; the same plan is launched directly or as a cached HIP graph.
struct TriKernelLaunch {
    const void* func;  // the first launch takes (TriLaunchArgs by value, TriLaunchArgs* copy); the others the copy
    dim3 grid, block;
    int stage;  // TriStage stamped before this launch when timing (-1: none)
};
struct TriFramePlan {
    uint32_t n = 0;
    TriKernelLaunch k[4];
};
void tri_plan_frame(const TriFrameParams& fp, TriFramePlan& plan);
#ifdef TRI_DIAG_FRONT
void tri_diag_front_plan(TriFramePlan& plan);  // diagnostics build only (raster_kernels.hip)
#endif
// k_raster_plain's instantiation for a frame without the shadow pre-pass (raster_plain.hip)
const void* tri_raster_plain_kernel(const TriFrameParams& fp);
// The frame's first kernel (vertex_stage.hip): k_vertex, k_vertex_band (row bands with cluster culling) or k_reset
// (a frame without vertex work)
enum TriFrontKernel { kFrontVertex = 0, kFrontBand, kFrontReset };
const void* tri_vertex_stage_kernel(TriFrontKernel k);

// Event stamps of one frame, in launch order: vertex, setup (+ clip, + the shadow map binning), shadow-map
// raster (only with the pre-pass), raster, end.
enum TriStage { kStageVertex = 0, kStageShadow, kStageSetup, kStageRaster, kStageCount };

hipError_t tri_kernels_init();

// One frame = 3 dependent launches on `stream` (k_vertex, k_setup with in-wave clipping, k_raster), 4 with the
// shadow pre-pass (k_shadow_raster after k_setup<shadow>); `events` (may be null) gets kStageCount + 1 stamps
// (the kStageShadow stamp only when the pre-pass runs).
hipError_t tri_run_plan(const TriFramePlan& plan, const TriLaunchArgs& args, TriLaunchArgs* d_args,
                        hipStream_t stream, hipEvent_t* events);

// Presentation blit (tri_blit_linear): src W x H B8G8R8A8 -> dst dw x dh, linear, clamp-to-edge.
hipError_t tri_launch_blit(const uint32_t* src, int32_t w, int32_t h, uint32_t* dst, int32_t dw, int32_t dh,
                           const float* unorm_lut, hipStream_t stream);

// The band codec (band_codec.hip): B8G8R8A8 <-> 3-byte BGR with a known alpha. The sender's status reaches the
// display with the band (tri_xfer): pack_bgr24 also ORs its alpha flag into `trailer` (a word after the packed pixels,
// zero at allocation, sticky like the flags), which unpack_bgr24 ORs into the display's `flags`; a dbp slot carries
// its own alpha mark (header word 1) and overflow (its payload count), which unpack ORs into `flags` (both nullable).
hipError_t tri_launch_pack_bgr24(const uint32_t* src, uint8_t* dst, uint64_t n, uint32_t alpha, uint32_t* flag,
                                 hipStream_t stream, uint32_t* trailer = nullptr);
hipError_t tri_launch_unpack_bgr24(const uint8_t* src, uint32_t* dst, uint64_t n, uint32_t alpha, hipStream_t stream,
                                   const uint32_t* trailer = nullptr, uint32_t* flags = nullptr);
hipError_t tri_launch_dbp_pack(const uint32_t* src, uint64_t n, uint32_t alpha, uint8_t* dst, uint32_t slot_bytes,
                               uint32_t* flags, hipStream_t stream);
hipError_t tri_launch_dbp_unpack(const uint8_t* src, uint64_t n, uint32_t alpha, uint32_t slot_bytes, uint32_t* dst,
                                 hipStream_t stream);
uint64_t tri_dbp_stream_bytes(uint64_t pixels, uint32_t slot_bytes);
hipError_t tri_launch_dbp_unpack_bands(const uint8_t* const* src, uint32_t* const* dst, const uint64_t* n, uint32_t count,
                                       uint32_t alpha, uint32_t slot_bytes, hipStream_t stream, uint32_t* flags = nullptr);

// Internal accessors for the group layer (tri_group.hip): a context's stream and device.
hipStream_t tri_internal_stream(tri_ctx* ctx);
int tri_internal_device(tri_ctx* ctx);
// Record an error message for tri_last_error (returns `code`).
int tri_internal_fail(int code, const char* msg);
// The device a geometry object lives on; the UNORM8 decode table (b / 255) on a context's device.
int tri_internal_geometry_device(const tri_geometry* geometry);
const float* tri_internal_unorm_lut(tri_ctx* ctx);
