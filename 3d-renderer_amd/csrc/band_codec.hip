// band_codec.hip — lossless 3-byte/pixel transfer format for the multi-GPU band assembly.
//
// The display GPU receives (N-1)/N of every frame over xGMI; at N = 8 that inbound traffic, not the
// raster, is expected to bound the whole-job frame rate. A band whose alpha bytes all equal
// one value (every frame of the reference's pipeline: opaque materials, tints and textures, Skybox.frag's
// alpha 1, an opaque clear colour — tri_alpha_uniform proves it from the context's state) travels as its
// B, G, R bytes only: 25 % fewer bytes per link, restored bit for bit on arrival with the known alpha.
//
//   k_pack_bgr24    4 pixels per lane: one 16-B load, one 12-B store (a wave writes 768 contiguous bytes);
//                   an alpha byte that differs from the promised one sets *flag (the sender's check that
//                   the transfer stayed lossless; tri_alpha_uniform makes it unreachable)
//   k_unpack_bgr24  4 pixels per lane: one 12-B load, one 16-B store
// Both are HBM-streaming kernels: 7 B moved per pixel (4 read + 3 written, or the reverse).
#include "raster_launch.h"

#include <hip/hip_runtime.h>

namespace {

constexpr uint32_t kCodecBlock = 256;

// VEC: the 4-byte side is 16-B aligned and the 3-byte side 4-B aligned (a band of a frame whose width is a
// multiple of 4); otherwise every pixel moves by itself (same bytes).
template <bool VEC>
__global__ __launch_bounds__(kCodecBlock) void k_pack_bgr24(const uint32_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                            uint64_t n, uint32_t alpha, uint32_t* __restrict__ flag) {
    const uint64_t q = (uint64_t)blockIdx.x * kCodecBlock + threadIdx.x;  // pixel quad
    const uint64_t p = q * 4;
    if (p >= n) return;
    bool bad = false;
    if (VEC && p + 4 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + p);
        bad = ((v.x >> 24) != alpha) | ((v.y >> 24) != alpha) | ((v.z >> 24) != alpha) | ((v.w >> 24) != alpha);
        // bytes b0 g0 r0 b1 | g1 r1 b2 g2 | r2 b3 g3 r3
        uint3 o;
        o.x = (v.x & 0x00FFFFFFu) | (v.y << 24);
        o.y = ((v.y >> 8) & 0x0000FFFFu) | (v.z << 16);
        o.z = ((v.z >> 16) & 0x000000FFu) | (v.w << 8);
        // 12-B aligned store: the quad's 3 dwords (dst is 4-B aligned and q * 12 is a multiple of 4)
        *reinterpret_cast<uint3*>(dst + q * 12) = o;
    } else {
        for (uint64_t i = p; i < n && i < p + 4; ++i) {  // unaligned bands, and a band's last 1-3 pixels
            const uint32_t v = src[i];
            bad |= (v >> 24) != alpha;
            dst[3 * i + 0] = (uint8_t)v;
            dst[3 * i + 1] = (uint8_t)(v >> 8);
            dst[3 * i + 2] = (uint8_t)(v >> 16);
        }
    }
    if (bad && flag) atomicOr(flag, 1u);
}

template <bool VEC>
__global__ __launch_bounds__(kCodecBlock) void k_unpack_bgr24(const uint8_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                              uint64_t n, uint32_t alpha) {
    const uint64_t q = (uint64_t)blockIdx.x * kCodecBlock + threadIdx.x;
    const uint64_t p = q * 4;
    if (p >= n) return;
    const uint32_t a = alpha << 24;
    if (VEC && p + 4 <= n) {
        const uint3 v = *reinterpret_cast<const uint3*>(src + q * 12);
        uint4 o;
        o.x = (v.x & 0x00FFFFFFu) | a;
        o.y = ((v.x >> 24) | (v.y << 8)) & 0x00FFFFFFu;
        o.y |= a;
        o.z = (((v.y >> 16) | (v.z << 16)) & 0x00FFFFFFu) | a;
        o.w = (v.z >> 8) | a;
        *reinterpret_cast<uint4*>(dst + p) = o;
    } else {
        for (uint64_t i = p; i < n && i < p + 4; ++i)
            dst[i] = (uint32_t)src[3 * i] | ((uint32_t)src[3 * i + 1] << 8) | ((uint32_t)src[3 * i + 2] << 16) | a;
    }
}

dim3 codec_grid(uint64_t n) { return dim3((uint32_t)((n + 4ull * kCodecBlock - 1) / (4ull * kCodecBlock))); }
bool vec_ok(const void* four, const void* three) { return ((uintptr_t)four & 15u) == 0 && ((uintptr_t)three & 3u) == 0; }

}  // namespace

hipError_t tri_launch_pack_bgr24(const uint32_t* src, uint8_t* dst, uint64_t n, uint32_t alpha, uint32_t* flag,
                                 hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (vec_ok(src, dst)) hipLaunchKernelGGL(k_pack_bgr24<true>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha, flag);
    else hipLaunchKernelGGL(k_pack_bgr24<false>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha, flag);
    return hipGetLastError();
}

hipError_t tri_launch_unpack_bgr24(const uint8_t* src, uint32_t* dst, uint64_t n, uint32_t alpha, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (vec_ok(dst, src)) hipLaunchKernelGGL(k_unpack_bgr24<true>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha);
    else hipLaunchKernelGGL(k_unpack_bgr24<false>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha);
    return hipGetLastError();
}

extern "C" {

int tri_pack_bgr24(const void* bgra, void* bgr, uint64_t pixels, uint32_t alpha, uint32_t* flag, void* stream) {
    if ((pixels && (!bgra || !bgr)) || alpha > 255u) return tri_internal_fail(TRI_E_INVALID, "tri_pack_bgr24: bad argument");
    if ((uintptr_t)bgra & 3u) return tri_internal_fail(TRI_E_INVALID, "tri_pack_bgr24: source must be 4-B aligned");
    const hipError_t e = tri_launch_pack_bgr24(static_cast<const uint32_t*>(bgra), static_cast<uint8_t*>(bgr), pixels,
                                               alpha, flag, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TRI_OK : tri_internal_fail(TRI_E_HIP, hipGetErrorString(e));
}

int tri_unpack_bgr24(const void* bgr, void* bgra, uint64_t pixels, uint32_t alpha, void* stream) {
    if ((pixels && (!bgra || !bgr)) || alpha > 255u) return tri_internal_fail(TRI_E_INVALID, "tri_unpack_bgr24: bad argument");
    if ((uintptr_t)bgra & 3u) return tri_internal_fail(TRI_E_INVALID, "tri_unpack_bgr24: destination must be 4-B aligned");
    const hipError_t e = tri_launch_unpack_bgr24(static_cast<const uint8_t*>(bgr), static_cast<uint32_t*>(bgra), pixels,
                                                 alpha, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TRI_OK : tri_internal_fail(TRI_E_HIP, hipGetErrorString(e));
}

}  // extern "C"
