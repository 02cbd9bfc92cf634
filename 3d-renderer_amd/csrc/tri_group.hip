// tri_group.hip — one frame over N band contexts (include/tri_raster.h "multi-device frames").
//
// Sort-first screen partition: band r renders rows [r*H/N, (r+1)*H/N) on its device with
// the whole scene (every band context culls clusters to its rows). The B8G8R8A8 frame is assembled on
// the display band's device: bands on that device render straight into it (tri_bind_output at their row
// offset, no copy), bands on other devices render into a band buffer that one RCCL group of ncclSend /
// ncclRecv moves over xGMI — each remote band crosses one link once, all links at the same time (a
// gather, not an all-gather: (N-1)/N of a frame lands on one GPU instead of on every GPU).
//
// Geometry: ONE tri_geometry per distinct device, bound by every band context on it (N bands on one
// device hold one copy, as the editor's viewports share one vertex/index buffer, Renderer.cpp:1965-2116),
// or the caller's own per-device geometry objects (tri_group_bind_geometry).
//
// Frames in flight: the assembled frame and every remote band buffer are double-buffered. Frame k renders
// into frame[k & 1]; a remote band's buffer k & 1 is reused by frame k + 2 only after frame k's assembly
// read it (a device-side wait on that assembly's event); an in-place band of frame k + 2 waits for the
// consumer's fence on frame k (tri_group_present), so a presenter still reading frame k is never
// overwritten while frame k + 1 renders into the other buffer.
//
// Streams: each band renders on its context's stream; per distinct device the group owns an assembly
// stream that waits (events) for that device's bands and carries the device's RCCL calls, so every
// communicator sees one stream.
#include "raster_launch.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <vector>

struct tri_group {
    uint32_t W = 0, H = 0, n = 0, display = 0;
    uint32_t gflags = 0;               // TRI_GROUP_*
    std::vector<int32_t> dev;        // per band
    std::vector<uint32_t> y0, y1;    // per band rows
    std::vector<tri_ctx*> ctx;       // per band
    std::vector<int32_t> udev;       // distinct devices
    std::vector<int> urank;          // band -> index of its device in udev (its RCCL rank)
    std::vector<tri_geometry*> geom; // per distinct device: the group's own geometry
    std::vector<ncclComm_t> comm;    // per distinct device (only when there are several)
    std::vector<hipStream_t> astream;  // per distinct device: assembly stream
    std::vector<hipEvent_t> band_done;   // per band: its render of the current frame finished
    std::vector<hipEvent_t> asm_done[2]; // per buffer parity, per distinct device: that frame's assembly finished
    std::vector<uint32_t*> band_buf[2];  // per buffer parity, per band on a non-display device: its colour band
    std::vector<uint8_t*> band_pack[2];  // ... the band packed (band_codec.hip: 3-byte or dbp), on the band's device
    std::vector<uint8_t*> rx[2];         // ... its packed bytes received on the display device
    // per remote band, on its device: [0] the packer's sticky flags (1 alpha differs, 2 a dbp slot overflowed;
    // 0 = lossless), [1] the largest dbp slot its frames needed since the last tri_group_synchronize
    std::vector<uint32_t*> flag;
    uint32_t slot = TRI_DBP_MAX_SLOT;    // the dbp slot size the next frame uses (refitted at synchronize)
    uint32_t fmt_last = TRI_GROUP_FMT_BGRA32, slot_last = 0;  // the most recent frame's transfer
    uint64_t inbound_last = 0;
    uint32_t* frame[2] = {nullptr, nullptr};  // W*H on the display device
    hipEvent_t present_done[2] = {nullptr, nullptr};  // consumer fence per buffer (tri_group_present)
    bool present_armed[2] = {false, false};
    hipEvent_t blit_done[2] = {nullptr, nullptr};  // per buffer: the group's blit of it (tri_group_blit_linear)
    bool blit_armed[2] = {false, false};
    bool asm_recorded[2] = {false, false};  // asm_done[p] holds a recorded assembly
    uint64_t frames = 0;                    // frames enqueued
    uint32_t* present = nullptr;            // tri_group_blit_linear's owned target (display device)
    size_t cap_present = 0;
    uint32_t present_w = 0, present_h = 0;
};

namespace {

// A band that travels to the display device (another device, or every band with TRI_GROUP_STAGE_BANDS).
bool travels(const tri_group* g, uint32_t r) {
    return r != g->display && (g->dev[r] != g->dev[g->display] || (g->gflags & TRI_GROUP_STAGE_BANDS));
}

int hip_fail(hipError_t e, const char* what) {
    const std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return tri_internal_fail(e == hipErrorOutOfMemory ? TRI_E_OOM : TRI_E_HIP, m.c_str());
}

int nccl_fail(ncclResult_t r, const char* what) {
    const std::string m = std::string(what) + ": " + ncclGetErrorString(r);
    return tri_internal_fail(TRI_E_HIP, m.c_str());
}

#define GH(expr)                                            \
    do {                                                    \
        const hipError_t _e = (expr);                       \
        if (_e != hipSuccess) return hip_fail(_e, #expr);   \
    } while (0)
#define GN(expr)                                            \
    do {                                                    \
        const ncclResult_t _r = (expr);                     \
        if (_r != ncclSuccess) return nccl_fail(_r, #expr); \
    } while (0)

template <typename F>
int each(tri_group* g, F&& f) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group: null group");
    for (tri_ctx* c : g->ctx) {
        const int rc = f(c);
        if (rc) return rc;
    }
    return TRI_OK;
}

// Bytes a packed band of px pixels may take: the 3-byte format, or the delta bit-plane format at its largest slot.
size_t packed_capacity(size_t px) {
    return std::max(px * 3, (size_t)tri_dbp_stream_bytes(px, TRI_DBP_MAX_SLOT));
}

// The transfer format of a frame whose alpha tri_frame_alpha returned (-1: not proven uniform).
uint32_t frame_format(const tri_group* g, int32_t alpha) {
    if ((g->gflags & TRI_GROUP_NO_PACK) || alpha < 0) return TRI_GROUP_FMT_BGRA32;
    return (g->gflags & TRI_GROUP_PACK_BGR24) ? TRI_GROUP_FMT_BGR24 : TRI_GROUP_FMT_DBP;
}

// Buffer parity of the most recent frame (the one tri_group_frame / readback / present refer to).
uint32_t last_parity(const tri_group* g) { return g->frames ? (uint32_t)((g->frames - 1) & 1u) : 0u; }

}  // namespace

extern "C" {

int tri_group_destroy(tri_group* g) {
    if (!g) return TRI_OK;
    for (size_t u = 0; u < g->astream.size(); ++u) {
        (void)hipSetDevice(g->udev[u]);
        if (g->astream[u]) (void)hipStreamSynchronize(g->astream[u]);
    }
    for (tri_ctx* c : g->ctx) tri_destroy(c);  // before the geometry they bind
    for (tri_geometry* geo : g->geom) tri_geometry_destroy(geo);
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    for (int p = 0; p < 2; ++p)
        for (uint32_t r = 0; r < g->band_buf[p].size(); ++r) {
            (void)hipSetDevice(g->dev[r]);
            if (g->band_buf[p][r]) (void)hipFree(g->band_buf[p][r]);
            if (r < g->band_pack[p].size() && g->band_pack[p][r]) (void)hipFree(g->band_pack[p][r]);
            if (p == 0 && r < g->flag.size() && g->flag[r]) (void)hipFree(g->flag[r]);
            if (!g->dev.empty() && r < g->rx[p].size() && g->rx[p][r]) {
                (void)hipSetDevice(g->dev[g->display]);
                (void)hipFree(g->rx[p][r]);
            }
        }
    for (uint32_t r = 0; r < g->band_done.size(); ++r)
        if (g->band_done[r]) {
            (void)hipSetDevice(g->dev[r]);
            (void)hipEventDestroy(g->band_done[r]);
        }
    for (size_t u = 0; u < g->udev.size(); ++u) {
        (void)hipSetDevice(g->udev[u]);
        for (int p = 0; p < 2; ++p)
            if (u < g->asm_done[p].size() && g->asm_done[p][u]) (void)hipEventDestroy(g->asm_done[p][u]);
        if (u < g->astream.size() && g->astream[u]) (void)hipStreamDestroy(g->astream[u]);
    }
    if (!g->dev.empty()) {
        (void)hipSetDevice(g->dev[g->display]);
        for (int p = 0; p < 2; ++p) {
            if (g->frame[p]) (void)hipFree(g->frame[p]);
            if (g->present_done[p]) (void)hipEventDestroy(g->present_done[p]);
            if (g->blit_done[p]) (void)hipEventDestroy(g->blit_done[p]);
        }
        if (g->present) (void)hipFree(g->present);
    }
    delete g;
    return TRI_OK;
}

int tri_group_create(const tri_group_config* cfg, tri_group** out) {
    if (!cfg || !out) return tri_internal_fail(TRI_E_INVALID, "tri_group_create: null argument");
    *out = nullptr;
    if (cfg->device_count == 0 || cfg->display >= cfg->device_count || cfg->height < cfg->device_count)
        return tri_internal_fail(TRI_E_INVALID, "tri_group_create: need 1 <= display < device_count <= height");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return tri_internal_fail(TRI_E_HIP, "tri_group_create: no HIP device available");
    tri_group* g = new tri_group();
    g->W = cfg->width;
    g->H = cfg->height;
    g->n = cfg->device_count;
    g->display = cfg->display;
    g->gflags = cfg->group_flags;
    auto bail = [&](int rc) { tri_group_destroy(g); return rc; };
    for (uint32_t r = 0; r < g->n; ++r) {
        const int32_t d = cfg->devices ? cfg->devices[r] : (int32_t)r;
        if (d < 0 || d >= ndev) return bail(tri_internal_fail(TRI_E_INVALID, "tri_group_create: device ordinal out of range"));
        g->dev.push_back(d);
        g->y0.push_back((uint32_t)((uint64_t)r * g->H / g->n));
        g->y1.push_back((uint32_t)((uint64_t)(r + 1) * g->H / g->n));
        if (std::find(g->udev.begin(), g->udev.end(), d) == g->udev.end()) g->udev.push_back(d);
    }
    for (uint32_t r = 0; r < g->n; ++r)
        g->urank.push_back((int)(std::find(g->udev.begin(), g->udev.end(), g->dev[r]) - g->udev.begin()));
    g->geom.assign(g->udev.size(), nullptr);
    for (size_t u = 0; u < g->udev.size(); ++u) {
        const int rc = tri_geometry_create(g->udev[u], &g->geom[u]);
        if (rc) return bail(rc);
    }
    const int32_t ddev = g->dev[g->display];
    for (uint32_t r = 0; r < g->n; ++r) {
        tri_config c{g->W, g->H, g->y0[r], g->y1[r], g->dev[r], cfg->flags};
        tri_ctx* ctx = nullptr;
        int rc = tri_create(&c, &ctx);
        if (rc) return bail(rc);
        g->ctx.push_back(ctx);
        if ((rc = tri_bind_geometry(ctx, g->geom[g->urank[r]]))) return bail(rc);
    }
    if (hipSetDevice(ddev) != hipSuccess)
        return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: hipSetDevice failed"));
    for (int p = 0; p < 2; ++p) {
        if (hipMalloc(&g->frame[p], (size_t)g->W * g->H * 4) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_OOM, "tri_group_create: frame allocation failed"));
        if (hipEventCreateWithFlags(&g->present_done[p], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->blit_done[p], hipEventDisableTiming) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: event creation failed"));
        g->band_buf[p].assign(g->n, nullptr);
        g->band_pack[p].assign(g->n, nullptr);
        g->rx[p].assign(g->n, nullptr);
    }
    g->flag.assign(g->n, nullptr);
    g->band_done.assign(g->n, nullptr);
    for (uint32_t r = 0; r < g->n; ++r) {
        if (hipSetDevice(g->dev[r]) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: hipSetDevice failed"));
        if (travels(g, r)) {
            const size_t px = (size_t)(g->y1[r] - g->y0[r]) * g->W;
            for (int p = 0; p < 2; ++p)
                if (hipMalloc(&g->band_buf[p][r], px * 4) != hipSuccess ||
                    (!(g->gflags & TRI_GROUP_NO_PACK) && hipMalloc(&g->band_pack[p][r], packed_capacity(px)) != hipSuccess))
                    return bail(tri_internal_fail(TRI_E_OOM, "tri_group_create: band buffer allocation failed"));
            if (!(g->gflags & TRI_GROUP_NO_PACK)) {
                // zeroed on the band context's own stream: its packer runs on that stream, so the clear is ordered
                // before every pack (a null-stream memset is not ordered with a non-blocking stream)
                if (hipMalloc(&g->flag[r], 8) != hipSuccess ||
                    hipMemsetAsync(g->flag[r], 0, 8, tri_internal_stream(g->ctx[r])) != hipSuccess)
                    return bail(tri_internal_fail(TRI_E_OOM, "tri_group_create: flag allocation failed"));
                if (hipSetDevice(ddev) != hipSuccess)
                    return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: hipSetDevice failed"));
                for (int p = 0; p < 2; ++p)
                    if (hipMalloc(&g->rx[p][r], packed_capacity(px)) != hipSuccess)
                        return bail(tri_internal_fail(TRI_E_OOM, "tri_group_create: receive buffer allocation failed"));
                if (hipSetDevice(g->dev[r]) != hipSuccess)
                    return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: hipSetDevice failed"));
            }
        }
        if (hipEventCreateWithFlags(&g->band_done[r], hipEventDisableTiming) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: event creation failed"));
    }
    g->astream.assign(g->udev.size(), nullptr);
    for (int p = 0; p < 2; ++p) g->asm_done[p].assign(g->udev.size(), nullptr);
    for (size_t u = 0; u < g->udev.size(); ++u) {
        if (hipSetDevice(g->udev[u]) != hipSuccess ||
            hipStreamCreateWithFlags(&g->astream[u], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&g->asm_done[0][u], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->asm_done[1][u], hipEventDisableTiming) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: assembly stream creation failed"));
    }
    for (int32_t d : g->udev)  // every device's allocations and clears complete before the group is handed out
        if (hipSetDevice(d) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: device synchronisation failed"));
    if (g->udev.size() > 1) {  // one RCCL communicator per distinct device, in this process
        g->comm.assign(g->udev.size(), nullptr);
        const ncclResult_t r = ncclCommInitAll(g->comm.data(), (int)g->udev.size(), g->udev.data());
        if (r != ncclSuccess) {
            g->comm.clear();
            return bail(nccl_fail(r, "tri_group_create: ncclCommInitAll"));
        }
    }
    *out = g;
    return TRI_OK;
}

int tri_group_context(tri_group* g, uint32_t band, tri_ctx** out) {
    if (!g || !out || band >= g->n) return tri_internal_fail(TRI_E_INVALID, "tri_group_context: bad argument");
    *out = g->ctx[band];
    return TRI_OK;
}

int tri_group_upload_geometry(tri_group* g, const tri_vertex* v, uint64_t nv, const uint32_t* idx, uint64_t ni,
                              const tri_mesh_range* m, uint32_t nm) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_upload_geometry: null group");
    int rc = tri_group_bind_geometry(g, 0, nullptr);  // back to the group's own per-device copies
    if (rc) return rc;
    for (tri_geometry* geo : g->geom)  // one upload per distinct device
        if ((rc = tri_geometry_upload(geo, v, nv, idx, ni, m, nm))) return rc;
    return TRI_OK;
}

int tri_group_bind_geometry(tri_group* g, uint32_t count, tri_geometry* const* geometries) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_bind_geometry: null group");
    if (count && !geometries) return tri_internal_fail(TRI_E_INVALID, "tri_group_bind_geometry: null geometry list");
    for (uint32_t r = 0; r < g->n; ++r) {
        tri_geometry* use = g->geom[g->urank[r]];
        if (count) {
            use = nullptr;
            for (uint32_t i = 0; i < count && !use; ++i)
                if (geometries[i] && tri_internal_geometry_device(geometries[i]) == g->dev[r]) use = geometries[i];
            if (!use) return tri_internal_fail(TRI_E_INVALID, "tri_group_bind_geometry: no geometry on a band's device");
        }
        const int rc = tri_bind_geometry(g->ctx[r], use);
        if (rc) return rc;
    }
    return TRI_OK;
}

int tri_group_upload_materials(tri_group* g, const tri_material_record* r, uint32_t n) {
    return each(g, [&](tri_ctx* c) { return tri_upload_materials(c, r, n); });
}
int tri_group_upload_texture(tri_group* g, uint32_t slot, const uint8_t* rgba, uint32_t w, uint32_t h) {
    return each(g, [&](tri_ctx* c) { return tri_upload_texture(c, slot, rgba, w, h); });
}
int tri_group_upload_bone_palette(tri_group* g, const float* m, uint32_t n) {
    return each(g, [&](tri_ctx* c) { return tri_upload_bone_palette(c, m, n); });
}
int tri_group_upload_ai_frame(tri_group* g, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    return each(g, [&](tri_ctx* c) { return tri_upload_ai_frame(c, rgba8, w, h); });
}
int tri_group_upload_skybox(tri_group* g, const uint8_t* faces, uint32_t size) {
    return each(g, [&](tri_ctx* c) { return tri_upload_skybox(c, faces, size); });
}
int tri_group_set_shadow(tri_group* g, const tri_shadow_config* s) {
    return each(g, [&](tri_ctx* c) { return tri_set_shadow(c, s); });
}
int tri_group_set_frame(tri_group* g, const tri_global_ubo* ubo, const float clear[4]) {
    return each(g, [&](tri_ctx* c) { return tri_set_frame(c, ubo, clear); });
}
int tri_group_set_draws(tri_group* g, const tri_draw* d, uint32_t n) {
    return each(g, [&](tri_ctx* c) { return tri_set_draws(c, d, n); });
}

int tri_group_render(tri_group* g) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_render: null group");
    const int32_t ddev = g->dev[g->display];
    const uint32_t p = (uint32_t)(g->frames & 1u);
    // a packed transfer when every pixel's alpha is provably one value (every band context holds the same
    // frame state: tri_group_set_* broadcasts it)
    int32_t alpha = -1;
    if (!(g->gflags & TRI_GROUP_NO_PACK)) {
        const int rc = tri_frame_alpha(g->ctx[g->display], &alpha);
        if (rc) return rc;
    }
    const uint32_t fmt = frame_format(g, alpha);
    const bool pack = fmt != TRI_GROUP_FMT_BGRA32, dbp = fmt == TRI_GROUP_FMT_DBP;
    const uint32_t slot = g->slot;  // this frame's dbp slot size (both ends of every band use it)
    auto pixels = [&](uint32_t r) { return (uint64_t)(g->y1[r] - g->y0[r]) * g->W; };
    for (uint32_t r = 0; r < g->n; ++r) {
        GH(hipSetDevice(g->dev[r]));
        hipStream_t s = tri_internal_stream(g->ctx[r]);
        uint32_t* out_ptr;
        if (!travels(g, r)) {
            out_ptr = g->frame[p] + (size_t)g->y0[r] * g->W;  // in place
            // the consumer of frame k - 2 (same buffer) has released it, and the group's blit has read it
            if (g->present_armed[p]) GH(hipStreamWaitEvent(s, g->present_done[p], 0));
            if (g->blit_armed[p]) GH(hipStreamWaitEvent(s, g->blit_done[p], 0));
        } else {
            out_ptr = g->band_buf[p][r];
            // frame k - 2's assembly read this buffer (and its packed copy)
            if (g->asm_recorded[p]) GH(hipStreamWaitEvent(s, g->asm_done[p][g->urank[r]], 0));
        }
        int rc = tri_bind_output(g->ctx[r], out_ptr, nullptr);  // depth stays in the band context
        if (rc) return rc;
        if ((rc = tri_render(g->ctx[r]))) return rc;
        if (pack && travels(g, r)) {  // behind the band's raster on its stream
            if (dbp)
                GH(tri_launch_dbp_pack(g->band_buf[p][r], pixels(r), (uint32_t)alpha, g->band_pack[p][r], slot, g->flag[r], s));
            else
                GH(tri_launch_pack_bgr24(g->band_buf[p][r], g->band_pack[p][r], pixels(r), (uint32_t)alpha, g->flag[r], s));
        }
        GH(hipEventRecord(g->band_done[r], s));
    }
    const int disp = g->urank[g->display];
    for (size_t u = 0; u < g->udev.size(); ++u) {  // each device's assembly stream waits for its bands
        GH(hipSetDevice(g->udev[u]));
        for (uint32_t r = 0; r < g->n; ++r)
            if (g->urank[r] == (int)u) GH(hipStreamWaitEvent(g->astream[u], g->band_done[r], 0));
        // the receives into frame[p] wait for the consumer's fence on frame k - 2 as well (the blit of frame
        // k - 2 ran on this same stream, so it is ordered already)
        if ((int)u == disp && g->present_armed[p]) GH(hipStreamWaitEvent(g->astream[u], g->present_done[p], 0));
    }
    // where band r's bytes land on the display device: straight into the frame, or its receive buffer
    auto landing = [&](uint32_t r) -> void* {
        return pack ? static_cast<void*>(g->rx[p][r]) : static_cast<void*>(g->frame[p] + (size_t)g->y0[r] * g->W);
    };
    auto source = [&](uint32_t r) -> const void* {
        return pack ? static_cast<const void*>(g->band_pack[p][r]) : static_cast<const void*>(g->band_buf[p][r]);
    };
    auto bytes = [&](uint32_t r) -> size_t {
        return dbp ? (size_t)tri_dbp_stream_bytes(pixels(r), slot) : (size_t)pixels(r) * (pack ? 3u : 4u);
    };
    if (!g->comm.empty()) {
        GN(ncclGroupStart());
        for (uint32_t r = 0; r < g->n; ++r) {
            if (g->dev[r] == ddev) continue;
            GN(ncclSend(source(r), bytes(r), ncclUint8, disp, g->comm[g->urank[r]], g->astream[g->urank[r]]));
            GN(ncclRecv(landing(r), bytes(r), ncclUint8, g->urank[r], g->comm[disp], g->astream[disp]));
        }
        GN(ncclGroupEnd());
    }
    GH(hipSetDevice(ddev));
    for (uint32_t r = 0; r < g->n; ++r)  // staged bands on the display device itself: a device-local copy
        if (travels(g, r) && g->dev[r] == ddev)
            GH(hipMemcpyAsync(landing(r), source(r), bytes(r), hipMemcpyDeviceToDevice, g->astream[disp]));
    if (pack) {  // restore the 4-byte pixels with the proven alpha, behind the receives
        std::vector<const uint8_t*> from;
        std::vector<uint32_t*> to;
        std::vector<uint64_t> npx;
        for (uint32_t r = 0; r < g->n; ++r)
            if (travels(g, r)) {
                from.push_back(g->rx[p][r]);
                to.push_back(g->frame[p] + (size_t)g->y0[r] * g->W);
                npx.push_back(pixels(r));
                if (!dbp) GH(tri_launch_unpack_bgr24(from.back(), to.back(), npx.back(), (uint32_t)alpha, g->astream[disp]));
            }
        for (size_t k = 0; dbp && k < from.size(); k += TRI_DBP_MAX_BANDS)  // every remote band in one launch
            GH(tri_launch_dbp_unpack_bands(from.data() + k, to.data() + k, npx.data() + k,
                                           (uint32_t)std::min<size_t>(TRI_DBP_MAX_BANDS, from.size() - k),
                                           (uint32_t)alpha, slot, g->astream[disp]));
    }
    for (size_t u = 0; u < g->udev.size(); ++u) {
        GH(hipSetDevice(g->udev[u]));
        GH(hipEventRecord(g->asm_done[p][u], g->astream[u]));
    }
    g->asm_recorded[p] = true;
    g->present_armed[p] = false;  // waited for; the consumer re-arms it for this frame
    g->blit_armed[p] = false;
    g->fmt_last = fmt;
    g->slot_last = dbp ? slot : 0u;
    g->inbound_last = 0;
    for (uint32_t r = 0; r < g->n; ++r)
        if (g->dev[r] != ddev) g->inbound_last += bytes(r);
    ++g->frames;
    return TRI_OK;
}

int tri_group_present(tri_group* g, void* hip_stream) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_present: null group");
    if (!g->frames) return tri_internal_fail(TRI_E_STATE, "tri_group_present: no frame rendered");
    const uint32_t p = last_parity(g);
    GH(hipSetDevice(g->dev[g->display]));
    // host release: stamp it behind the frame's own assembly, so the fence can never precede the frame
    hipStream_t s = hip_stream ? static_cast<hipStream_t>(hip_stream) : g->astream[g->urank[g->display]];
    GH(hipEventRecord(g->present_done[p], s));
    g->present_armed[p] = true;
    return TRI_OK;
}

int tri_group_synchronize(tri_group* g) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_synchronize: null group");
    int status = TRI_OK;
    for (tri_ctx* c : g->ctx) {  // every band (an overflow in any band re-renders the frame)
        const int rc = tri_synchronize(c);
        if (rc && status == TRI_OK) status = rc;
    }
    for (size_t u = 0; u < g->udev.size(); ++u) {
        GH(hipSetDevice(g->udev[u]));
        GH(hipStreamSynchronize(g->astream[u]));
    }
    // every packed band kept the proven alpha and fitted its dbp slots; the dbp slot is refitted to the largest
    // slot the frames since the previous synchronize needed (+ 1/16)
    uint32_t need = 0;
    bool alpha_bad = false, overflow = false;
    for (uint32_t r = 0; r < g->n; ++r) {
        if (!g->flag[r]) continue;
        uint32_t f[2] = {0, 0};
        GH(hipSetDevice(g->dev[r]));
        GH(hipMemcpy(f, g->flag[r], 8, hipMemcpyDeviceToHost));
        if (f[0] || f[1])
            // reported once: cleared on the band's stream (idle here), so a later lossless frame synchronises clean.
            // Frames handed out (tri_group_frame / get_output / blit) without a synchronize are not checked.
            GH(hipMemsetAsync(g->flag[r], 0, 8, tri_internal_stream(g->ctx[r])));
        alpha_bad |= (f[0] & 1u) != 0;
        overflow |= (f[0] & 2u) != 0;
        need = std::max(need, f[1]);
    }
    if (need) {
        const uint32_t fit = (need + need / 16u + 15u) / 16u * 16u;
        g->slot = std::min<uint32_t>(TRI_DBP_MAX_SLOT, std::max<uint32_t>(TRI_DBP_MIN_SLOT, fit));
    }
    if (status == TRI_OK && alpha_bad)
        status = tri_internal_fail(TRI_E_STATE, "tri_group: a band's alpha was not the proven value (lossy packed transfer)");
    if (status == TRI_OK && overflow)
        status = tri_internal_fail(TRI_E_OVERFLOW, "tri_group: a band outgrew its dbp slots (slot refitted: render the frame again)");
    return status;
}

int tri_group_transfer_info(tri_group* g, uint32_t* bytes_per_pixel, uint64_t* inbound_bytes) {
    if (!g || !bytes_per_pixel || !inbound_bytes) return tri_internal_fail(TRI_E_INVALID, "tri_group_transfer_info: null argument");
    uint64_t px = 0, bytes = 0;  // every band that travelled (staged bands too), for the bytes per pixel
    for (uint32_t r = 0; r < g->n; ++r)
        if (travels(g, r)) {
            const uint64_t n = (uint64_t)(g->y1[r] - g->y0[r]) * g->W;
            px += n;
            bytes += g->fmt_last == TRI_GROUP_FMT_DBP ? tri_dbp_stream_bytes(n, g->slot_last)
                                                       : n * (g->fmt_last == TRI_GROUP_FMT_BGR24 ? 3u : 4u);
        }
    *bytes_per_pixel = g->fmt_last == TRI_GROUP_FMT_DBP ? (uint32_t)((bytes + px - 1) / std::max<uint64_t>(px, 1))
                                                        : (g->fmt_last == TRI_GROUP_FMT_BGR24 ? 3u : 4u);
    *inbound_bytes = g->inbound_last;
    return TRI_OK;
}

int tri_group_transfer_format(tri_group* g, uint32_t* format, uint32_t* slot_bytes) {
    if (!g || !format || !slot_bytes) return tri_internal_fail(TRI_E_INVALID, "tri_group_transfer_format: null argument");
    if (g->frames) {
        *format = g->fmt_last;
        *slot_bytes = g->slot_last;
    } else {  // what the next frame would use with a proven alpha
        *format = frame_format(g, 0);
        *slot_bytes = *format == TRI_GROUP_FMT_DBP ? g->slot : 0u;
    }
    return TRI_OK;
}

int tri_group_readback(tri_group* g, uint8_t* bgra, uint32_t* depth) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_readback: null group");
    int rc = tri_group_synchronize(g);
    if (rc) return rc;
    if (bgra) {
        GH(hipSetDevice(g->dev[g->display]));
        GH(hipMemcpy(bgra, g->frame[last_parity(g)], (size_t)g->W * g->H * 4, hipMemcpyDeviceToHost));
    }
    if (depth)
        for (uint32_t r = 0; r < g->n; ++r)
            if ((rc = tri_readback(g->ctx[r], nullptr, depth + (size_t)g->y0[r] * g->W))) return rc;
    return TRI_OK;
}

int tri_group_frame(tri_group* g, void** ptr, int32_t* device) {
    if (!g || !ptr || !device) return tri_internal_fail(TRI_E_INVALID, "tri_group_frame: null argument");
    *ptr = g->frame[last_parity(g)];
    *device = g->dev[g->display];
    return TRI_OK;
}

int tri_group_get_output(tri_group* g, tri_image* out) {
    if (!g || !out) return tri_internal_fail(TRI_E_INVALID, "tri_group_get_output: null argument");
    out->device_ptr = g->frame[last_parity(g)];
    out->width = g->W;
    out->height = g->H;
    out->pitch_bytes = g->W * 4u;
    out->format = TRI_FORMAT_B8G8R8A8_UNORM;
    out->device = g->dev[g->display];
    out->reserved = 0;
    return TRI_OK;
}

int tri_group_blit_linear(tri_group* g, void* dst, uint32_t width, uint32_t height) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_blit_linear: null group");
    if (width == 0 || height == 0 || width > TRI_MAX_DIM || height > TRI_MAX_DIM)
        return tri_internal_fail(TRI_E_INVALID, "tri_group_blit_linear: destination size out of range");
    if (!g->frames) return tri_internal_fail(TRI_E_STATE, "tri_group_blit_linear: no frame rendered");
    const int32_t ddev = g->dev[g->display];
    GH(hipSetDevice(ddev));
    hipStream_t s = g->astream[g->urank[g->display]];  // behind the frame's assembly
    uint32_t* out = static_cast<uint32_t*>(dst);
    if (!out) {
        const size_t need = (size_t)width * height;
        if (need > g->cap_present) {
            GH(hipStreamSynchronize(s));
            if (g->present) GH(hipFree(g->present));
            g->present = nullptr;
            g->cap_present = 0;
            GH(hipMalloc(&g->present, need * 4));
            g->cap_present = need;
        }
        out = g->present;
        g->present_w = width;
        g->present_h = height;
    } else {
        g->present_w = g->present_h = 0;  // the owned target no longer holds the latest blit: read_present fails
    }
    const uint32_t p = last_parity(g);
    GH(tri_launch_blit(g->frame[p], (int32_t)g->W, (int32_t)g->H, out, (int32_t)width, (int32_t)height,
                       tri_internal_unorm_lut(g->ctx[g->display]), s));
    // the blit reads frame[p] on the assembly stream: frame k + 2's in-place bands (context streams) wait for it
    GH(hipEventRecord(g->blit_done[p], s));
    g->blit_armed[p] = true;
    return TRI_OK;
}

int tri_group_read_present(tri_group* g, uint8_t* bgra) {
    if (!g || !bgra) return tri_internal_fail(TRI_E_INVALID, "tri_group_read_present: null argument");
    if (!g->present || !g->present_w) return tri_internal_fail(TRI_E_STATE, "tri_group_read_present: nothing was blitted");
    GH(hipSetDevice(g->dev[g->display]));
    GH(hipStreamSynchronize(g->astream[g->urank[g->display]]));
    GH(hipMemcpy(bgra, g->present, (size_t)g->present_w * g->present_h * 4, hipMemcpyDeviceToHost));
    return TRI_OK;
}

}  // extern "C"
