// tri_group.hip — one frame over N band contexts (include/tri_raster.h "multi-device frames").
//
// Sort-first screen partition: band r renders rows [r*H/N, (r+1)*H/N) on its device with
// the whole scene (every band context culls clusters to its rows). The B8G8R8A8 frame is assembled on
// the display band's device: bands on that device render straight into it (tri_bind_output at their row
// offset, no copy), bands on other devices render into a band buffer that one RCCL group of ncclSend /
// ncclRecv moves over xGMI — each remote band crosses one link once, all links at the same time (a
// gather, not an all-gather: (N-1)/N of a frame lands on one GPU instead of on every GPU).
//
// Streams: each band renders on its context's stream; per distinct device the group owns an assembly
// stream that waits (events) for that device's bands and carries the device's RCCL calls, so every
// communicator sees one stream. A band's next frame waits for the assembly that read its buffer.
#include "raster_launch.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <vector>

struct tri_group {
    uint32_t W = 0, H = 0, n = 0, display = 0;
    std::vector<int32_t> dev;        // per band
    std::vector<uint32_t> y0, y1;    // per band rows
    std::vector<tri_ctx*> ctx;       // per band
    std::vector<int32_t> udev;       // distinct devices
    std::vector<int> urank;          // band -> index of its device in udev (its RCCL rank)
    std::vector<ncclComm_t> comm;    // per distinct device (only when there are several)
    std::vector<hipStream_t> astream;  // per distinct device: assembly stream
    std::vector<hipEvent_t> band_done;   // per band: its render finished
    std::vector<hipEvent_t> asm_done;    // per distinct device: its part of the assembly finished
    std::vector<uint32_t*> band_buf;     // per band on a non-display device: its colour band
    uint32_t* frame = nullptr;           // W*H on the display device
    bool assembled_once = false;
};

namespace {

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

}  // namespace

extern "C" {

int tri_group_destroy(tri_group* g) {
    if (!g) return TRI_OK;
    for (size_t u = 0; u < g->astream.size(); ++u) {
        (void)hipSetDevice(g->udev[u]);
        if (g->astream[u]) (void)hipStreamSynchronize(g->astream[u]);
    }
    for (tri_ctx* c : g->ctx) tri_destroy(c);
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    for (uint32_t r = 0; r < g->band_buf.size(); ++r)
        if (g->band_buf[r]) {
            (void)hipSetDevice(g->dev[r]);
            (void)hipFree(g->band_buf[r]);
        }
    for (uint32_t r = 0; r < g->band_done.size(); ++r)
        if (g->band_done[r]) {
            (void)hipSetDevice(g->dev[r]);
            (void)hipEventDestroy(g->band_done[r]);
        }
    for (size_t u = 0; u < g->udev.size(); ++u) {
        (void)hipSetDevice(g->udev[u]);
        if (u < g->asm_done.size() && g->asm_done[u]) (void)hipEventDestroy(g->asm_done[u]);
        if (u < g->astream.size() && g->astream[u]) (void)hipStreamDestroy(g->astream[u]);
    }
    if (g->frame) {
        (void)hipSetDevice(g->dev[g->display]);
        (void)hipFree(g->frame);
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
    const int32_t ddev = g->dev[g->display];
    for (uint32_t r = 0; r < g->n; ++r) {
        tri_config c{g->W, g->H, g->y0[r], g->y1[r], g->dev[r], cfg->flags};
        tri_ctx* ctx = nullptr;
        const int rc = tri_create(&c, &ctx);
        if (rc) return bail(rc);
        g->ctx.push_back(ctx);
    }
    if (hipSetDevice(ddev) != hipSuccess || hipMalloc(&g->frame, (size_t)g->W * g->H * 4) != hipSuccess)
        return bail(tri_internal_fail(TRI_E_OOM, "tri_group_create: frame allocation failed"));
    g->band_buf.assign(g->n, nullptr);
    g->band_done.assign(g->n, nullptr);
    for (uint32_t r = 0; r < g->n; ++r) {
        uint32_t* out_ptr;
        if (g->dev[r] == ddev) {
            out_ptr = g->frame + (size_t)g->y0[r] * g->W;  // renders in place
        } else {
            if (hipSetDevice(g->dev[r]) != hipSuccess ||
                hipMalloc(&g->band_buf[r], (size_t)(g->y1[r] - g->y0[r]) * g->W * 4) != hipSuccess)
                return bail(tri_internal_fail(TRI_E_OOM, "tri_group_create: band buffer allocation failed"));
            out_ptr = g->band_buf[r];
        }
        int rc = tri_bind_output(g->ctx[r], out_ptr, nullptr);  // depth stays in the band context
        if (rc) return bail(rc);
        if (hipSetDevice(g->dev[r]) != hipSuccess ||
            hipEventCreateWithFlags(&g->band_done[r], hipEventDisableTiming) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: event creation failed"));
    }
    g->astream.assign(g->udev.size(), nullptr);
    g->asm_done.assign(g->udev.size(), nullptr);
    for (size_t u = 0; u < g->udev.size(); ++u) {
        if (hipSetDevice(g->udev[u]) != hipSuccess ||
            hipStreamCreateWithFlags(&g->astream[u], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&g->asm_done[u], hipEventDisableTiming) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_group_create: assembly stream creation failed"));
    }
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
    return each(g, [&](tri_ctx* c) { return tri_upload_geometry(c, v, nv, idx, ni, m, nm); });
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
    for (uint32_t r = 0; r < g->n; ++r) {
        GH(hipSetDevice(g->dev[r]));
        hipStream_t s = tri_internal_stream(g->ctx[r]);
        // the previous frame's assembly read this band's buffer: the band waits for it (device-side)
        if (g->assembled_once && g->dev[r] != ddev) GH(hipStreamWaitEvent(s, g->asm_done[g->urank[r]], 0));
        const int rc = tri_render(g->ctx[r]);
        if (rc) return rc;
        GH(hipEventRecord(g->band_done[r], s));
    }
    for (size_t u = 0; u < g->udev.size(); ++u) {  // each device's assembly stream waits for its bands
        GH(hipSetDevice(g->udev[u]));
        for (uint32_t r = 0; r < g->n; ++r)
            if (g->urank[r] == (int)u) GH(hipStreamWaitEvent(g->astream[u], g->band_done[r], 0));
    }
    if (!g->comm.empty()) {
        const int disp = g->urank[g->display];
        GN(ncclGroupStart());
        for (uint32_t r = 0; r < g->n; ++r) {
            if (g->dev[r] == ddev) continue;
            const size_t bytes = (size_t)(g->y1[r] - g->y0[r]) * g->W * 4;
            GN(ncclSend(g->band_buf[r], bytes, ncclUint8, disp, g->comm[g->urank[r]], g->astream[g->urank[r]]));
            GN(ncclRecv(g->frame + (size_t)g->y0[r] * g->W, bytes, ncclUint8, g->urank[r], g->comm[disp], g->astream[disp]));
        }
        GN(ncclGroupEnd());
    }
    for (size_t u = 0; u < g->udev.size(); ++u) {
        GH(hipSetDevice(g->udev[u]));
        GH(hipEventRecord(g->asm_done[u], g->astream[u]));
    }
    g->assembled_once = true;
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
    return status;
}

int tri_group_readback(tri_group* g, uint8_t* bgra, uint32_t* depth) {
    if (!g) return tri_internal_fail(TRI_E_INVALID, "tri_group_readback: null group");
    int rc = tri_group_synchronize(g);
    if (rc) return rc;
    if (bgra) {
        GH(hipSetDevice(g->dev[g->display]));
        GH(hipMemcpy(bgra, g->frame, (size_t)g->W * g->H * 4, hipMemcpyDeviceToHost));
    }
    if (depth)
        for (uint32_t r = 0; r < g->n; ++r)
            if ((rc = tri_readback(g->ctx[r], nullptr, depth + (size_t)g->y0[r] * g->W))) return rc;
    return TRI_OK;
}

int tri_group_frame(tri_group* g, void** ptr, int32_t* device) {
    if (!g || !ptr || !device) return tri_internal_fail(TRI_E_INVALID, "tri_group_frame: null argument");
    *ptr = g->frame;
    *device = g->dev[g->display];
    return TRI_OK;
}

}  // extern "C"
