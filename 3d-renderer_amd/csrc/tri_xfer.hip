// tri_xfer.hip — one rank's band exchange for a process-per-GPU caller (bench.py at N > 1).
//
// The torch.distributed route costs the host ≈ 20 µs per point-to-point operation (torch's P2POp / batch_isend_irecv
// bookkeeping, measured on an MI355X with tools/p2p_host_cost.py: one send/receive pair 42 µs per frame, seven 218
// µs), so a display rank that receives seven bands per frame would be host-bound far below one GPU's frame rate. This
// file drives the same exchange natively, one call per frame: render the rank's band (tri_bind_output +
// tri_set_frame + tri_set_draws + tri_render on the context's stream), then on that same stream pack and send it (a
// sender) or receive every remote band and decode it into the frame (the display rank):
//
//   context stream of slot s:  [render frame k] ─ pack ─ ncclSend (comm s)                       (sender)
//                              [render own band] ─ ncclRecv × (N-1) (comm s) ─ decode bands       (display)
//
// Each slot (one per frame in flight) has its own RCCL communicator (tri_xfer_comm, bootstrapped from a unique id
// the caller broadcasts once), so every communicator's operations stay on one stream and frame k + nbuf, which
// reuses the slot's buffers on the same stream, is ordered behind frame k's transfer with no event: HIP event
// record/wait calls cost the host ≈ 2 µs each (tools/xfer_host_cost.py: a fenced version of this call took 26.8 µs
// against 16 µs for the render alone). If a slot changes streams (a different context), it is fenced with events.
// Band formats are tri_group's (TRI_GROUP_FMT_*): the delta bit-plane stream with the slot size every rank agreed,
// 3-byte pixels, or 4. A packed band carries its sender's status (an alpha that broke the proof, a dbp slot that
// overflowed), which the display's decode ORs into its own flags, so tri_xfer_synchronize on the display rank reports a
// lossy frame as well as the sender's does.
//
// Fail-safe waits: tri_xfer_synchronize polls every slot's stream against a deadline (tri_xfer_set_timeout) and each
// communicator's asynchronous error; on expiry or error it aborts the communicators (ncclCommAbort, which releases
// kernels stuck in a transfer) and returns TRI_E_TIMEOUT, so a caller process exits instead of hanging its job.
//
// Loopback transport (tri_xfer_loopback, tests only): N exchanges of one process on one device stand in for N ranks,
// because RCCL refuses two ranks on one GPU. A loopback communicator replaces ncclSend/ncclRecv and nothing else: the
// sender records an event behind its pack and posts {buffer, bytes, event}; the display's receive waits for that event
// and copies the bytes into the same receive buffer ncclRecv would fill, then records a "consumed" event that the
// sender's next frame on the slot waits for (ncclSend's rendezvous: a sender's stream does not run past a send until it
// is received). Everything else — the pack, the receive buffers, the batched decode and an assemble-only display's
// own streams — is the code the N-GPU run executes. The caller drives the ranks frame by frame, senders before the
// display (a receive whose send was not posted yet is TRI_E_STATE).
#include "raster_launch.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <thread>
#include <vector>

static_assert(sizeof(ncclUniqueId) == TRI_XFER_ID_BYTES, "tri_xfer: RCCL unique id size");

namespace {
struct LbMsg {  // one posted loopback send
    const void* src = nullptr;
    uint64_t bytes = 0;
    hipEvent_t ready = nullptr, consumed = nullptr;
    bool received = false;
    ~LbMsg() {
        if (ready) (void)hipEventDestroy(ready);
        if (consumed) (void)hipEventDestroy(consumed);
    }
};
}  // namespace

struct tri_xfer_loopback {
    uint32_t world = 0;
    std::vector<uint32_t> made;  // communicators created per rank: the k-th of every rank forms channel k
    // channel -> sender rank -> posted sends in order
    std::vector<std::vector<std::deque<std::shared_ptr<LbMsg>>>> chan;
};

struct tri_xfer_comm {
    ncclComm_t comm = nullptr;
    int32_t device = 0;
    uint32_t world = 0, rank = 0;
    tri_xfer_loopback* lb = nullptr;  // loopback transport (tests): the hub and this communicator's channel
    uint32_t channel = 0;
    bool aborted = false;
    // a communicator shared by several slots (fewer communicators than frames in flight): its operations are fenced
    // across streams (the stream of its last operation, and an event recorded after it)
    hipStream_t last = nullptr;
    hipEvent_t after = nullptr;
};

struct tri_xfer {
    std::vector<tri_xfer_comm*> xc;          // slot s uses xc[s % xc.size()]
    int32_t device = 0;
    uint32_t world = 1, rank = 0;
    uint32_t W = 0, display = 0, fmt = TRI_GROUP_FMT_BGRA32, slot_bytes = 0, alpha = 0, nbuf = 0;
    std::vector<uint32_t> y;                 // world + 1 row boundaries
    std::vector<hipStream_t> own;            // per slot: exchange-only frames of a slot that never rendered (an
                                             // assemble-only display's frames: slots overlap like render streams)
    std::vector<uint32_t*> pixels;           // per slot: this rank's band (sender) or the frame (display)
    std::vector<uint8_t*> stage;             // per slot: the sender's packed band
    std::vector<std::vector<uint8_t*>> rx;   // per slot, per rank: the display's received packed bands
    std::vector<hipStream_t> stream;         // per slot: the stream its last frame ran on
    std::vector<hipEvent_t> freed;           // per slot: fences a change of stream
    uint32_t* flags = nullptr;               // [sticky flags, largest dbp slot]: this rank's packs, or on the display
                                             // its decodes of the senders' status
    std::vector<std::shared_ptr<LbMsg>> lb_sent;  // loopback: per slot, the last send its next frame waits for
    uint32_t timeout_ms = 60000;             // tri_xfer_synchronize's deadline (0: none)
};

namespace {

int xfail(hipError_t e, const char* what) {
    const std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return tri_internal_fail(e == hipErrorOutOfMemory ? TRI_E_OOM : TRI_E_HIP, m.c_str());
}
int nfail(ncclResult_t r, const char* what) {
    const std::string m = std::string(what) + ": " + ncclGetErrorString(r);
    return tri_internal_fail(TRI_E_HIP, m.c_str());
}
#define XH(expr)                                          \
    do {                                                  \
        const hipError_t _e = (expr);                     \
        if (_e != hipSuccess) return xfail(_e, #expr);    \
    } while (0)
#define XN(expr)                                          \
    do {                                                  \
        const ncclResult_t _r = (expr);                   \
        if (_r != ncclSuccess) return nfail(_r, #expr);   \
    } while (0)

uint64_t band_pixels(const tri_xfer* x, uint32_t r) { return (uint64_t)(x->y[r + 1] - x->y[r]) * x->W; }

uint64_t band_bytes(const tri_xfer* x, uint32_t r) {
    const uint64_t px = band_pixels(x, r);
    if (x->fmt == TRI_GROUP_FMT_DBP) return tri_dbp_stream_bytes(px, x->slot_bytes);
    // 3-byte bands end in a 16-B aligned status word (the sender's sticky alpha flag), so the display sees it
    if (x->fmt == TRI_GROUP_FMT_BGR24) return (px * 3u + 15u) / 16u * 16u + 16u;
    return px * 4u;
}
uint64_t bgr24_trailer(uint64_t px) { return (px * 3u + 15u) / 16u * 16u; }

int lb_send(tri_xfer_comm* c, const void* src, uint64_t bytes, uint32_t peer, hipStream_t s, std::shared_ptr<LbMsg>& out) {
    (void)peer;  // (the display; one receiver per channel)
    auto m = std::make_shared<LbMsg>();
    m->src = src;
    m->bytes = bytes;
    XH(hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
    XH(hipEventCreateWithFlags(&m->consumed, hipEventDisableTiming));
    XH(hipEventRecord(m->ready, s));
    c->lb->chan[c->channel][c->rank].push_back(m);
    out = m;
    return TRI_OK;
}

int lb_recv(tri_xfer_comm* c, void* to, uint64_t bytes, uint32_t peer, hipStream_t s) {
    auto& q = c->lb->chan[c->channel][peer];
    if (q.empty()) return tri_internal_fail(TRI_E_STATE, "tri_xfer loopback: a sender has not posted this frame's band");
    std::shared_ptr<LbMsg> m = q.front();
    q.pop_front();
    if (m->bytes != bytes) return tri_internal_fail(TRI_E_STATE, "tri_xfer loopback: send and receive sizes differ");
    XH(hipStreamWaitEvent(s, m->ready, 0));
    XH(hipMemcpyAsync(to, m->src, bytes, hipMemcpyDeviceToDevice, s));
    XH(hipEventRecord(m->consumed, s));
    m->received = true;
    return TRI_OK;
}

void abort_comms(tri_xfer* x) {
    for (tri_xfer_comm* c : x->xc)
        if (c->comm && !c->aborted) {
            (void)ncclCommAbort(c->comm);  // releases kernels blocked in a transfer; frees the communicator
            c->comm = nullptr;
            c->aborted = true;
        }
}

}  // namespace

extern "C" {

int tri_xfer_unique_id(uint8_t* id) {
    if (!id) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_unique_id: null argument");
    ncclUniqueId u;
    XN(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return TRI_OK;
}

int tri_xfer_comm_create(const uint8_t* id, uint32_t world, uint32_t rank, int32_t device, tri_xfer_comm** out) {
    if (!id || !out || world == 0 || rank >= world) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_comm_create: bad argument");
    *out = nullptr;
    XH(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    tri_xfer_comm* xc = new tri_xfer_comm();
    xc->device = device;
    xc->world = world;
    xc->rank = rank;
    const ncclResult_t r = ncclCommInitRank(&xc->comm, (int)world, u, (int)rank);
    if (r != ncclSuccess) {
        delete xc;
        return nfail(r, "tri_xfer_comm_create: ncclCommInitRank");
    }
    *out = xc;
    return TRI_OK;
}

int tri_xfer_comm_destroy(tri_xfer_comm* xc) {
    if (!xc) return TRI_OK;
    (void)hipSetDevice(xc->device);
    if (xc->comm) (void)ncclCommDestroy(xc->comm);
    if (xc->after) (void)hipEventDestroy(xc->after);
    delete xc;
    return TRI_OK;
}

int tri_xfer_loopback_create(uint32_t world, tri_xfer_loopback** out) {
    if (!out || world == 0) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_loopback_create: bad argument");
    tri_xfer_loopback* lb = new tri_xfer_loopback();
    lb->world = world;
    lb->made.assign(world, 0u);
    *out = lb;
    return TRI_OK;
}

int tri_xfer_loopback_destroy(tri_xfer_loopback* lb) {
    delete lb;
    return TRI_OK;
}

int tri_xfer_comm_create_loopback(tri_xfer_loopback* lb, uint32_t rank, int32_t device, tri_xfer_comm** out) {
    if (!lb || !out || rank >= lb->world) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_comm_create_loopback: bad argument");
    *out = nullptr;
    XH(hipSetDevice(device));
    tri_xfer_comm* xc = new tri_xfer_comm();
    xc->device = device;
    xc->world = lb->world;
    xc->rank = rank;
    xc->lb = lb;
    xc->channel = lb->made[rank]++;
    if (lb->chan.size() <= xc->channel) lb->chan.resize(xc->channel + 1, std::vector<std::deque<std::shared_ptr<LbMsg>>>(lb->world));
    *out = xc;
    return TRI_OK;
}

int tri_xfer_destroy(tri_xfer* x) {
    if (!x) return TRI_OK;
    (void)hipSetDevice(x->device);
    for (hipStream_t st : x->stream)
        if (st) (void)hipStreamSynchronize(st);
    for (uint8_t* p : x->stage)
        if (p) (void)hipFree(p);
    for (auto& v : x->rx)
        for (uint8_t* p : v)
            if (p) (void)hipFree(p);
    for (hipEvent_t e : x->freed)
        if (e) (void)hipEventDestroy(e);
    if (x->flags) (void)hipFree(x->flags);
    for (hipStream_t st : x->own)
        if (st) (void)hipStreamDestroy(st);
    delete x;
    return TRI_OK;
}

int tri_xfer_create(tri_xfer_comm* const* comms, uint32_t ncomm, const tri_xfer_config* cfg, tri_xfer** out) {
    if (!comms || ncomm == 0 || !cfg || !out || !cfg->band_y)
        return tri_internal_fail(TRI_E_INVALID, "tri_xfer_create: null argument");
    *out = nullptr;
    for (uint32_t i = 0; i < ncomm; ++i)
        if (!comms[i] || comms[i]->world != comms[0]->world || comms[i]->rank != comms[0]->rank ||
            comms[i]->device != comms[0]->device || (comms[i]->lb == nullptr) != (comms[0]->lb == nullptr))
            return tri_internal_fail(TRI_E_INVALID, "tri_xfer_create: the communicators differ in world, rank, device or transport");
    const uint32_t N = comms[0]->world;
    if (cfg->display >= N || cfg->nbuf == 0 || cfg->width == 0 || cfg->alpha > 255u ||
        cfg->format > TRI_GROUP_FMT_DBP ||
        (cfg->format == TRI_GROUP_FMT_DBP && (cfg->slot_bytes < TRI_DBP_MIN_SLOT || cfg->slot_bytes % 16u)))
        return tri_internal_fail(TRI_E_INVALID, "tri_xfer_create: bad configuration");
    // every band has rows, except that the display's may be empty (it then only assembles the others)
    for (uint32_t r = 0; r < N; ++r)
        if (cfg->band_y[r + 1] < cfg->band_y[r] || (cfg->band_y[r + 1] == cfg->band_y[r] && (r != cfg->display || N == 1)))
            return tri_internal_fail(TRI_E_INVALID, "tri_xfer_create: every band but the display's needs at least one row");
    XH(hipSetDevice(comms[0]->device));
    tri_xfer* x = new tri_xfer();
    x->xc.assign(comms, comms + ncomm);
    x->device = comms[0]->device;
    x->world = N;
    x->rank = comms[0]->rank;
    x->W = cfg->width;
    x->display = cfg->display;
    x->fmt = cfg->format;
    x->slot_bytes = cfg->slot_bytes;
    x->alpha = cfg->alpha;
    x->nbuf = cfg->nbuf;
    x->y.assign(cfg->band_y, cfg->band_y + N + 1);
    auto bail = [&](int rc) { tri_xfer_destroy(x); return rc; };
    const bool packed = x->fmt != TRI_GROUP_FMT_BGRA32;
    x->pixels.assign(x->nbuf, nullptr);
    x->stage.assign(x->nbuf, nullptr);
    x->rx.assign(x->nbuf, std::vector<uint8_t*>(N, nullptr));
    x->stream.assign(x->nbuf, nullptr);
    x->freed.assign(x->nbuf, nullptr);
    x->own.assign(x->nbuf, nullptr);  // created on first use: a rank that renders every frame never needs them
    x->lb_sent.assign(x->nbuf, nullptr);
    for (uint32_t s = 0; s < x->nbuf; ++s) {
        if (hipEventCreateWithFlags(&x->freed[s], hipEventDisableTiming) != hipSuccess)
            return bail(tri_internal_fail(TRI_E_HIP, "tri_xfer_create: event creation failed"));
        if (!packed || N == 1) continue;
        if (x->rank != x->display) {
            if (hipMalloc(&x->stage[s], band_bytes(x, x->rank)) != hipSuccess)
                return bail(tri_internal_fail(TRI_E_OOM, "tri_xfer_create: staging allocation failed"));
        } else {
            for (uint32_t r = 0; r < N; ++r)
                if (r != x->display && hipMalloc(&x->rx[s][r], band_bytes(x, r)) != hipSuccess)
                    return bail(tri_internal_fail(TRI_E_OOM, "tri_xfer_create: receive allocation failed"));
        }
    }
    if (hipMalloc(&x->flags, 8) != hipSuccess || hipMemset(x->flags, 0, 8) != hipSuccess)
        return bail(tri_internal_fail(TRI_E_OOM, "tri_xfer_create: flag allocation failed"));
    if (packed && N > 1 && x->fmt == TRI_GROUP_FMT_BGR24 && x->rank != x->display)  // the status words start clear
        for (uint32_t s = 0; s < x->nbuf; ++s)
            if (hipMemset(x->stage[s] + bgr24_trailer(band_pixels(x, x->rank)), 0, 16) != hipSuccess)
                return bail(tri_internal_fail(TRI_E_HIP, "tri_xfer_create: status word initialisation failed"));
    // the null-stream memsets above are not ordered with the non-blocking streams that pack and decode: complete them
    if (hipDeviceSynchronize() != hipSuccess) return bail(tri_internal_fail(TRI_E_HIP, "tri_xfer_create: synchronisation failed"));
    *out = x;
    return TRI_OK;
}

int tri_xfer_bind_slot(tri_xfer* x, uint32_t slot, void* pixels) {
    if (!x || slot >= x->nbuf || !pixels || ((uintptr_t)pixels & 3u))
        return tri_internal_fail(TRI_E_INVALID, "tri_xfer_bind_slot: bad argument");
    x->pixels[slot] = static_cast<uint32_t*>(pixels);
    return TRI_OK;
}

int tri_xfer_frame(tri_xfer* x, uint32_t slot, tri_ctx* ctx, void* depth, const tri_global_ubo* ubo,
                   const float clear[4], const tri_draw* draws, uint32_t draw_count, uint32_t exchange) {
    if (!x || slot >= x->nbuf || !x->pixels[slot]) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_frame: bad slot");
    const uint32_t me = x->rank, N = x->world;
    if (ctx && band_pixels(x, me) == 0)
        return tri_internal_fail(TRI_E_INVALID, "tri_xfer_frame: an assemble-only display (empty band) renders nothing");
    const bool disp = me == x->display;
    XH(hipSetDevice(x->device));
    uint32_t* frame = x->pixels[slot];  // the band (sender) or the frame (display)
    // the slot's stream: its context's (render and transfer in one stream order), else the last one it ran on
    if (!ctx && !x->stream[slot] && !x->own[slot])  // an exchange-only slot that never rendered: a stream of its own
        XH(hipStreamCreateWithFlags(&x->own[slot], hipStreamNonBlocking));
    hipStream_t s = ctx ? tri_internal_stream(ctx) : (x->stream[slot] ? x->stream[slot] : x->own[slot]);
    if (x->stream[slot] && x->stream[slot] != s) {  // the slot moves to another stream: fence its last frame
        XH(hipEventRecord(x->freed[slot], x->stream[slot]));
        XH(hipStreamWaitEvent(s, x->freed[slot], 0));
    }
    x->stream[slot] = s;
    if (x->lb_sent[slot]) {  // loopback: the slot's previous send must be received before its buffers are reused
        if (!x->lb_sent[slot]->received)
            return tri_internal_fail(TRI_E_STATE, "tri_xfer loopback: the display has not received this slot's previous frame");
        XH(hipStreamWaitEvent(s, x->lb_sent[slot]->consumed, 0));
        x->lb_sent[slot].reset();
    }
    if (ctx) {
        uint32_t* out = disp ? frame + (size_t)x->y[me] * x->W : frame;
        int rc = tri_bind_output(ctx, out, depth);
        if (!rc && ubo) rc = tri_set_frame(ctx, ubo, clear);
        if (!rc && draws) rc = tri_set_draws(ctx, draws, draw_count);
        if (!rc) rc = tri_render(ctx);
        if (rc) return rc;
    }
    if (!exchange || N == 1) return TRI_OK;
    tri_xfer_comm* xc = x->xc[slot % x->xc.size()];
    if (xc->aborted) return tri_internal_fail(TRI_E_STATE, "tri_xfer_frame: the communicator was aborted (a timed-out wait)");
    // fewer communicators than slots: a communicator's operations on another stream are fenced behind its last ones
    const bool shared = x->xc.size() < x->nbuf;
    if (shared) {
        if (!xc->after) XH(hipEventCreateWithFlags(&xc->after, hipEventDisableTiming));
        if (xc->last && xc->last != s) XH(hipStreamWaitEvent(s, xc->after, 0));
    }
    ncclComm_t comm = xc->comm;
    if (!disp) {
        const void* src = frame;
        const uint64_t px = band_pixels(x, me);
        if (x->fmt == TRI_GROUP_FMT_DBP) {
            XH(tri_launch_dbp_pack(frame, px, x->alpha, x->stage[slot], x->slot_bytes, x->flags, s));
            src = x->stage[slot];
        } else if (x->fmt == TRI_GROUP_FMT_BGR24) {
            XH(tri_launch_pack_bgr24(frame, x->stage[slot], px, x->alpha, x->flags, s,
                                     reinterpret_cast<uint32_t*>(x->stage[slot] + bgr24_trailer(px))));
            src = x->stage[slot];
        }
        if (xc->lb) {
            const int rc = lb_send(xc, src, band_bytes(x, me), x->display, s, x->lb_sent[slot]);
            if (rc) return rc;
        } else {
            XN(ncclSend(src, band_bytes(x, me), ncclUint8, (int)x->display, comm, s));
        }
    } else {
        if (!xc->lb) XN(ncclGroupStart());
        for (uint32_t r = 0; r < N; ++r) {
            if (r == me) continue;
            void* to = x->fmt == TRI_GROUP_FMT_BGRA32 ? static_cast<void*>(frame + (size_t)x->y[r] * x->W)
                                                      : static_cast<void*>(x->rx[slot][r]);
            if (xc->lb) {
                const int rc = lb_recv(xc, to, band_bytes(x, r), r, s);
                if (rc) return rc;
            } else {
                XN(ncclRecv(to, band_bytes(x, r), ncclUint8, (int)r, comm, s));
            }
        }
        if (!xc->lb) XN(ncclGroupEnd());
        if (x->fmt == TRI_GROUP_FMT_DBP) {  // every remote band in one launch (up to TRI_DBP_MAX_BANDS)
            const uint8_t* from[TRI_DBP_MAX_BANDS];
            uint32_t* to[TRI_DBP_MAX_BANDS];
            uint64_t npx[TRI_DBP_MAX_BANDS];
            uint32_t k = 0;
            for (uint32_t r = 0; r < N; ++r) {
                if (r == me) continue;
                from[k] = x->rx[slot][r];
                to[k] = frame + (size_t)x->y[r] * x->W;
                npx[k] = band_pixels(x, r);
                if (++k == TRI_DBP_MAX_BANDS) {
                    XH(tri_launch_dbp_unpack_bands(from, to, npx, k, x->alpha, x->slot_bytes, s, x->flags));
                    k = 0;
                }
            }
            if (k) XH(tri_launch_dbp_unpack_bands(from, to, npx, k, x->alpha, x->slot_bytes, s, x->flags));
        } else if (x->fmt == TRI_GROUP_FMT_BGR24) {
            for (uint32_t r = 0; r < N; ++r)
                if (r != me) {
                    const uint64_t px = band_pixels(x, r);
                    XH(tri_launch_unpack_bgr24(x->rx[slot][r], frame + (size_t)x->y[r] * x->W, px, x->alpha, s,
                                               reinterpret_cast<const uint32_t*>(x->rx[slot][r] + bgr24_trailer(px)),
                                               x->flags));
                }
        }
    }
    if (shared) {
        XH(hipEventRecord(xc->after, s));
        xc->last = s;
    }
    return TRI_OK;
}

int tri_xfer_set_timeout(tri_xfer* x, uint32_t timeout_ms) {
    if (!x) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_set_timeout: null exchange");
    x->timeout_ms = timeout_ms;
    return TRI_OK;
}

int tri_xfer_wait(tri_xfer* x) {
    if (!x) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_wait: null exchange");
    XH(hipSetDevice(x->device));
    // every slot's stream, polled against the deadline together with the communicators' asynchronous errors: a
    // transfer whose peer never comes (a dead or diverged rank) must end the caller, not hang the whole job
    const auto t0 = std::chrono::steady_clock::now();
    for (hipStream_t st : x->stream) {
        if (!st) continue;
        for (;;) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) return xfail(e, "tri_xfer_wait: hipStreamQuery");
            for (tri_xfer_comm* c : x->xc) {
                ncclResult_t ae = ncclSuccess;
                if (c->comm && ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                    abort_comms(x);
                    return nfail(ae, "tri_xfer_wait: a communicator failed (aborted)");
                }
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (x->timeout_ms && ms > (double)x->timeout_ms) {
                abort_comms(x);
                return tri_internal_fail(TRI_E_TIMEOUT, "tri_xfer_wait: the exchange did not complete before the "
                                                        "deadline (communicators aborted)");
            }
            // (spinning for the first 2 ms: a timed region's closing wait must not add a sleep's granularity)
            if (ms < 2.0) std::this_thread::yield();
            else std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    return TRI_OK;
}

int tri_xfer_synchronize(tri_xfer* x) {
    const int rc = tri_xfer_wait(x);
    if (rc) return rc;
    uint32_t f[2] = {0, 0};
    XH(hipMemcpy(f, x->flags, 8, hipMemcpyDeviceToHost));
    if (f[0] & 1u) return tri_internal_fail(TRI_E_STATE, "tri_xfer: a band's alpha was not the proven value (lossy packed transfer)");
    if (f[0] & 2u) return tri_internal_fail(TRI_E_OVERFLOW, "tri_xfer: a band outgrew the agreed dbp slot size (lossy transfer)");
    return TRI_OK;
}

int tri_xfer_comm_count(tri_xfer* x, uint32_t* count) {
    if (!x || !count) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_comm_count: null argument");
    *count = (uint32_t)x->xc.size();
    return TRI_OK;
}

int tri_xfer_info(tri_xfer* x, uint64_t* sent_bytes, uint64_t* received_bytes, uint32_t* max_slot_bytes) {
    if (!x || !sent_bytes || !received_bytes) return tri_internal_fail(TRI_E_INVALID, "tri_xfer_info: null argument");
    const uint32_t N = x->world, me = x->rank;
    *sent_bytes = (N > 1 && me != x->display) ? band_bytes(x, me) : 0u;
    uint64_t in = 0;
    if (N > 1 && me == x->display)
        for (uint32_t r = 0; r < N; ++r)
            if (r != me) in += band_bytes(x, r);
    *received_bytes = in;
    if (max_slot_bytes) {
        const int rc = tri_xfer_synchronize(x);
        if (rc && rc != TRI_E_STATE && rc != TRI_E_OVERFLOW) return rc;
        uint32_t f[2] = {0, 0};
        XH(hipMemcpy(f, x->flags, 8, hipMemcpyDeviceToHost));
        *max_slot_bytes = f[1];
    }
    return TRI_OK;
}

}  // extern "C"
