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
                                                            uint64_t n, uint32_t alpha, uint32_t* __restrict__ flag,
                                                            uint32_t* __restrict__ trailer) {
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
    if (bad && trailer) atomicOr(trailer, 1u);  // the status that travels with the band (tri_xfer)
}

template <bool VEC>
__global__ __launch_bounds__(kCodecBlock) void k_unpack_bgr24(const uint8_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                              uint64_t n, uint32_t alpha, const uint32_t* __restrict__ trailer,
                                                              uint32_t* __restrict__ flags) {
    const uint64_t q = (uint64_t)blockIdx.x * kCodecBlock + threadIdx.x;
    const uint64_t p = q * 4;
    if (q == 0 && trailer && flags && (*trailer & 1u)) atomicOr(flags, 1u);  // the sender's alpha check failed
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

// ---- the delta bit-plane codec: a band as a 1-D pixel stream, 4096 pixels per fixed-size slot -------
// A slot is 4 segments of 1024 pixels, a segment 16 blocks of 64. Per block and channel (B, G, R) the pixel-to-pixel
// difference (mod 256; a segment's first pixel is stored whole in the slot header and coded as a zero difference) is
// zigzag-mapped, the block's bit width w (0..8) is the width of the largest value, and the block stores w bit planes,
// each a 64-bit ballot (bit i = pixel i). Shaded frames are smooth between neighbours (C3: 1.42 B/pixel on average,
// at most 1.59 in any slot; C5 with its textures 2.0 / 2.11), so a slot of S bytes carries 4096 pixels in far fewer
// than the 3-byte format's 12288. Slot layout (S bytes, a multiple of 16):
//   [0, 4)      the payload bytes P of the 64 blocks (the decoder's bound; P + 160 > S marks an overflowed slot)
//   [16, 160)   4 segment headers of 36 B: the first pixel (B, G, R, 0) and 16 block widths w_b | w_g << 4 | w_r << 8
//   [160, +P)   the blocks' planes in order, channel B's w_b planes, then G's, then R's
// One workgroup per slot. Both kernels are bound by instruction issue (the VALUs and the CU's one scalar unit), so
// every step is counted in instructions per 64-pixel block:
//   k_dbp_pack    1024 threads, wave w on blocks 4w..4w+3 (a one-band launch has about one slot per CU: sixteen
//                 waves keep it busy). The wave issues its 4 pixel loads at once; a pixel's predecessor comes from
//                 the lane before it (DPP wave_shr:1; lane 0 takes the previous block's last pixel, a readlane, or
//                 one scalar load at the wave's first block). The three channels' byte differences and zigzag maps
//                 are one 32-bit SWAR word and one DPP OR-scan gives the widths; the zigzag words stay in registers.
//                 After one barrier every wave's prefix sum over the 64 blocks' plane counts places its blocks; each
//                 plane that exists then costs a bit test, a ballot and two and-ors (plane j parked in lane j), and
//                 lanes < w store a channel's planes in place (8 B each).
//   k_dbp_unpack  256 threads, wave w on segment w (the carries never leave the wave; eight slots fit a CU at once).
//                 Every wave sums the 64 blocks' widths (lane = block, DPP scan) to find its blocks' planes and reads
//                 each channel's 8 candidate planes with one scalar buffer load (16 SGPRs, the next block's in flight
//                 while this one is summed; planes past the width are dropped, reads past the slot return 0). A plane
//                 then costs one VALU op: v_addc with the plane as its carry-in lane mask shifts the lane's bit into
//                 z (z = 2 z + bit, most significant plane first). The zigzag is inverted per byte (SWAR) and the
//                 differences summed with two DPP wave scans (B and R share one in 16-bit fields, G the other: only
//                 the sums mod 256 matter); the block's last pixel is the next block's carry (readlane). One launch
//                 decodes up to TRI_DBP_MAX_BANDS bands (the display GPU's remote bands), a workgroup per slot.
// Lossless whenever no slot overflows; an overflow (a slot whose pixels need more than S bytes) sets flags[0] bit 1
// and leaves the slot's pixels undecoded, so the caller grows S and sends the frame again (the bin-queue overflow
// protocol). A slot whose widths do not add up to its payload count is not decoded either (not this format).
constexpr uint32_t kDbpSlotPixels = 4096, kDbpHeader = 160, kDbpBlocks = 64, kDbpThreads = 256, kDbpSegBlocks = 16;
constexpr uint32_t kDbpMaxPayload = kDbpBlocks * 24u * 8u;  // 12288 B: 8 planes per channel in every block

// v[lane - k] within the lane's row of 16 (CTRL row_shr:k), or row_bcast:15 / :31 onto the rows in ROW_MASK; 0 elsewhere
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += dpp0<0x111>(v);
    v += dpp0<0x112>(v);
    v += dpp0<0x114>(v);
    v += dpp0<0x118>(v);
    v += dpp0<0x142, 0xa>(v);
    v += dpp0<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {  // the OR over the wave (uniform)
    v |= dpp0<0x111>(v);
    v |= dpp0<0x112>(v);
    v |= dpp0<0x114>(v);
    v |= dpp0<0x118>(v);
    v |= dpp0<0x142, 0xa>(v);
    v |= dpp0<0x143, 0xc>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// v of the lane before (DPP wave_shr:1); lane 0 gets `first`
__device__ __forceinline__ uint32_t lane_before(uint32_t v, uint32_t first) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xf, 0xf, false);
}
// B, G, R bytes of (v - p) mod 256, each zigzag-mapped (0, -1, 1, -2, ... -> 0, 1, 2, 3, ...); alpha byte 0
__device__ __forceinline__ uint32_t zigzag_diff3(uint32_t v, uint32_t p) {
    constexpr uint32_t H = 0x00808080u, L = 0x007F7F7Fu;
    const uint32_t d = (((v | H) - (p & L)) ^ ((v ^ ~p) & H)) & 0x00FFFFFFu;  // bytewise subtraction, no borrows
    const uint32_t neg = (d >> 7) & 0x00010101u;                                // each byte's sign
    return ((d << 1) & 0x00FEFEFEu) ^ (neg * 0xFFu);                            // (d << 1) ^ (d >> 7), per byte
}
__device__ __forceinline__ uint32_t width8(uint32_t x) { return x ? 32u - (uint32_t)__builtin_clz(x) : 0u; }
// planes J..wc-1 of channel C of the wave's zigzag words: plane j (a ballot, in SGPRs) parked in lane j of l (low
// word) and h (high word) by an and-or with the lane's mask lm[j] (all ones in lane j): one v_and_or per word,
// an ordinary per-lane operation (a v_writelane in inline asm would not survive the compiler's copies of the register
// under partial exec masks)
template <uint32_t C, uint32_t J>
__device__ __forceinline__ void park_planes(uint32_t zz, uint32_t wc, const uint32_t (&lm)[8], uint32_t& l, uint32_t& h) {
    if constexpr (J < 8) {
        if (J < wc) {
            const uint64_t pl = __ballot((zz >> (8 * C + J)) & 1u);
            // l and h start at 0 and every lane is written once: (lm & plane) | l, one v_and_or each (the compiler
            // splits it into an and and an or with an SGPR operand). The ballot's SGPRs were just written by a VALU
            // compare: two wait states before a VALU reads them (the compiler inserts them for its own code only)
            asm("s_nop 1\n\tv_and_or_b32 %0, %1, %2, %0" : "+v"(l) : "v"(lm[J]), "s"((uint32_t)pl));
            asm("v_and_or_b32 %0, %1, %2, %0" : "+v"(h) : "v"(lm[J]), "s"((uint32_t)(pl >> 32)));
            park_planes<C, J + 1>(zz, wc, lm, l, h);
        }
    }
}

constexpr uint32_t kDbpPackThreads = 1024, kDbpPackBlocks = kDbpBlocks / (kDbpPackThreads / 64);  // 4 per wave

__global__ __launch_bounds__(kDbpPackThreads) void k_dbp_pack(const uint32_t* __restrict__ src, uint64_t n,
                                                              uint32_t alpha, uint8_t* __restrict__ dst,
                                                              uint32_t slot_bytes, uint32_t* __restrict__ flags) {
    __shared__ uint32_t hdr[kDbpHeader / 4];
    __shared__ uint32_t cnt[kDbpBlocks];
    __shared__ uint32_t wave_bad[kDbpPackThreads / 64];  // a pixel's alpha differs (the slot's header word 1)
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t b0 = kDbpPackBlocks * w;  // this wave's first block in the slot
    const uint64_t px0 = (uint64_t)blockIdx.x * kDbpSlotPixels + 64u * b0;
    // pixels past the band repeat its last one (zero differences)
    uint32_t zz[kDbpPackBlocks], wq[kDbpPackBlocks];
    bool bad = false;
    {
        uint32_t v[kDbpPackBlocks];
#pragma unroll
        for (uint32_t k = 0; k < kDbpPackBlocks; ++k) {
            const uint64_t i = px0 + 64u * k + lane;
            v[k] = src[i < n ? i : n - 1];
        }
        // the pixel before this wave's first: a segment's first pixel is its own predecessor (a zero difference,
        // the pixel stored whole in the header); otherwise the previous wave's last pixel, one scalar load
        const bool seg_first = (b0 % kDbpSegBlocks) == 0;
        uint32_t carry = seg_first ? (uint32_t)__builtin_amdgcn_readlane((int)v[0], 0) : src[px0 - 1 < n ? px0 - 1 : n - 1];
        if (seg_first && lane == 0) hdr[4 + 9 * (b0 / kDbpSegBlocks)] = px0 < n ? carry & 0x00FFFFFFu : 0u;
#pragma unroll
        for (uint32_t k = 0; k < kDbpPackBlocks; ++k) {
            bad |= px0 + 64u * k + lane < n && (v[k] >> 24) != alpha;
            zz[k] = zigzag_diff3(v[k], lane_before(v[k], carry));
            carry = (uint32_t)__builtin_amdgcn_readlane((int)v[k], 63);
            const uint32_t any = wave_or(zz[k]);
            wq[k] = width8(any & 0xFFu) | (width8((any >> 8) & 0xFFu) << 4) | (width8((any >> 16) & 0xFFu) << 8);
            if (lane == 0) {
                const uint32_t b = b0 + k;
                reinterpret_cast<uint16_t*>(hdr + 4 + 9 * (b / kDbpSegBlocks) + 1)[b % kDbpSegBlocks] = (uint16_t)wq[k];
                cnt[b] = (wq[k] & 15u) + ((wq[k] >> 4) & 15u) + (wq[k] >> 8);
            }
        }
    }
    const bool wbad = __ballot(bad) != 0ull;
    if (wbad && lane == 0 && flags) atomicOr(flags, 1u);
    if (lane == 0) wave_bad[w] = wbad ? 1u : 0u;
    __syncthreads();
    // every wave places the slot's 64 blocks itself (lane = block): no second barrier
    const uint32_t c = cnt[lane];
    const uint32_t incl = wave_incl_sum(c);
    const uint32_t excl = incl - c;
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t bytes = kDbpHeader + 8u * total;
    uint8_t* slot = dst + (size_t)blockIdx.x * slot_bytes;
    if (threadIdx.x == 0 && flags) {
        atomicMax(flags + 1, bytes);
        if (bytes > slot_bytes) atomicOr(flags, 2u);
    }
    uint32_t slot_bad = 0u;  // (read by the two header threads only)
    if (threadIdx.x < 2) {
#pragma unroll
        for (uint32_t k = 0; k < kDbpPackThreads / 64; ++k) slot_bad |= wave_bad[k];
    }
    if (bytes > slot_bytes) {  // overflow: only the payload count and the alpha mark (the decoder leaves the slot alone)
        if (threadIdx.x < 2) reinterpret_cast<uint32_t*>(slot)[threadIdx.x] = threadIdx.x == 0 ? 8u * total : slot_bad;
        return;
    }
    if (threadIdx.x < kDbpHeader / 4)
        reinterpret_cast<uint32_t*>(slot)[threadIdx.x] =
            threadIdx.x == 0 ? 8u * total : threadIdx.x == 1 ? slot_bad : threadIdx.x < 4 ? 0u : hdr[threadIdx.x];
    // each block's planes, parked in lanes and stored straight to their place
    uint32_t lm[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        lm[j] = lane == j ? ~0u : 0u;
        asm volatile("" : "+v"(lm[j]));  // an opaque vector value: kept as a VGPR operand, not turned into lane masks
    }
    uint2* pay = reinterpret_cast<uint2*>(slot + kDbpHeader);
#pragma unroll
    for (uint32_t k = 0; k < kDbpPackBlocks; ++k) {
        const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)(b0 + k));
        const uint32_t w0 = wq[k] & 15u, w1 = (wq[k] >> 4) & 15u, w2 = wq[k] >> 8;
        uint32_t l0 = 0, h0 = 0, l1 = 0, h1 = 0, l2 = 0, h2 = 0;
        park_planes<0, 0>(zz[k], w0, lm, l0, h0);
        park_planes<1, 0>(zz[k], w1, lm, l1, h1);
        park_planes<2, 0>(zz[k], w2, lm, l2, h2);
        if (lane < w0) pay[o + lane] = make_uint2(l0, h0);
        if (lane < w1) pay[o + w0 + lane] = make_uint2(l1, h1);
        if (lane < w2) pay[o + w0 + w1 + lane] = make_uint2(l2, h2);
    }
}

struct DbpBands {  // the bands one k_dbp_unpack launch decodes (kernel argument)
    const uint8_t* src[TRI_DBP_MAX_BANDS];
    uint32_t* dst[TRI_DBP_MAX_BANDS];
    uint64_t n[TRI_DBP_MAX_BANDS];
    uint32_t first[TRI_DBP_MAX_BANDS + 1];  // first slot (workgroup) of each band; first[count] = the grid
    uint32_t count;
};

// DBP_ABLATE (diagnostic builds only, tools/codec_ablate.sh): 1 skips the plane decode, 2 the scans, 4 the stores
#ifndef DBP_ABLATE
#define DBP_ABLATE 0
#endif
typedef uint32_t dbp_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t dbp_u32x16 __attribute__((ext_vector_type(16)));
__device__ dbp_u32x16 dbp_s_load16(dbp_u32x4 rsrc, int offset, int aux) __asm("llvm.amdgcn.s.buffer.load.v16i32");
__device__ uint32_t dbp_s_load1(dbp_u32x4 rsrc, int offset, int aux) __asm("llvm.amdgcn.s.buffer.load.i32");

// z = 2 z + (bit `lane` of the 64-bit plane m): one v_addc with the plane as its carry-in lane mask
__device__ __forceinline__ uint32_t shift_in_plane(uint32_t z, uint64_t m) {
    uint64_t carry_out;  // unused (an SGPR pair of its own, so successive ops share no VCC)
    asm("v_addc_co_u32 %0, %1, %2, %2, %3" : "=v"(z), "=s"(carry_out) : "v"(z), "s"(m));
    return z;
}
// a channel's zigzag values from its wc (<= 8) planes p[0..7] (16 words from one scalar load), most significant plane
// first; the planes past wc belong to the next channel or block and are masked off afterwards (one VALU op instead of
// a scalar select per plane: the CU's one scalar unit, shared by its four SIMDs, is as scarce an issue port). A
// channel of at most 4 planes (most of them) takes 4 steps: one scalar branch saves 4 VALU ops.
__device__ __forceinline__ uint32_t planes_to_lanes(const dbp_u32x16& p, uint32_t wc) {
    uint32_t z = 0;
    if (wc > 4) {
#pragma unroll
        for (int j = 7; j >= 4; --j) z = shift_in_plane(z, ((uint64_t)p[2 * j + 1] << 32) | p[2 * j]);
    }
#pragma unroll
    for (int j = 3; j >= 0; --j) z = shift_in_plane(z, ((uint64_t)p[2 * j + 1] << 32) | p[2 * j]);
    return z & ((1u << wc) - 1u);
}

__global__ __launch_bounds__(kDbpThreads) void k_dbp_unpack(DbpBands bands, uint32_t alpha, uint32_t slot_bytes,
                                                             uint32_t* __restrict__ flags) {
    uint32_t band = 0;  // the band this slot belongs to (wave-uniform search over <= 16 entries)
    while (band + 1 < bands.count && blockIdx.x >= bands.first[band + 1]) ++band;
    const uint64_t n = bands.n[band];
    uint32_t* dst = bands.dst[band];
    const uint32_t sl = blockIdx.x - bands.first[band];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint8_t* slot = bands.src[band] + (size_t)sl * slot_bytes;
    // the slot as a raw buffer (scalar loads past its end return 0)
    const uint64_t base = (uint64_t)slot;
    const dbp_u32x4 r = dbp_u32x4{(uint32_t)base, (uint32_t)(base >> 32) & 0xFFFFu, slot_bytes, 0x00020000u};
    const uint32_t payload = dbp_s_load1(r, 0, 0);
    // the sender's status travels in the slot: its alpha mark (header word 1) and an overflow (the payload count), so
    // the display's own flags report a lossy frame (tri_xfer_synchronize on the display rank)
    if (flags && threadIdx.x == 0) {
        const uint32_t st = (dbp_s_load1(r, 4, 0) != 0u ? 1u : 0u) | (kDbpHeader + payload > slot_bytes ? 2u : 0u);
        if (st) atomicOr(flags, st);
    }
    // an overflowed slot (the sender flagged the frame), or more payload than the format has: left alone
    if (kDbpHeader + payload > slot_bytes || payload > kDbpMaxPayload) return;
    // lane l: block l's widths and plane count; the inclusive sum places every block's planes
    const uint32_t wl = reinterpret_cast<const uint16_t*>(slot + 16 + 36 * (lane >> 4) + 4)[lane & 15u];
    const uint32_t first = dbp_s_load1(r, 16 + 36 * (int)w, 0);
    const uint32_t cl = (wl & 15u) + ((wl >> 4) & 15u) + ((wl >> 8) & 15u);
    const uint32_t incl = wave_incl_sum(cl);
    if (8u * (uint32_t)__builtin_amdgcn_readlane((int)incl, 63) != payload) return;  // not a dbp slot (uniform)
    uint32_t c0 = first & 0x00FF00FFu, c1 = (first >> 8) & 0xFFu;  // the carries: B | R << 16, and G
    const uint32_t a = alpha << 24;
    const uint64_t seg0 = (uint64_t)sl * kDbpSlotPixels + (uint64_t)w * (kDbpSegBlocks * 64u);
    // the segment's pixels as a raw buffer: stores past the band's end are dropped by the bounds check (no compare,
    // no 64-bit address arithmetic per block)
    const uint64_t left = seg0 < n ? n - seg0 : 0;
    const __amdgpu_buffer_rsrc_t out = __builtin_amdgcn_make_buffer_rsrc(
        dst + (seg0 < n ? seg0 : 0), (short)0, (int)(uint32_t)(4u * (left < 1024u ? left : 1024u)), 0x00020000);
    // block k's planes: three scalar loads (one per channel), issued one block ahead of their use
    const uint32_t ol = incl - cl;  // lane l: block l's first plane
    uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)wl, (int)(kDbpSegBlocks * w));
    uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)ol, (int)(kDbpSegBlocks * w));
    dbp_u32x16 p0 = dbp_s_load16(r, (int)(kDbpHeader + 8u * o), 0);
    dbp_u32x16 p1 = dbp_s_load16(r, (int)(kDbpHeader + 8u * (o + (wb & 15u))), 0);
    dbp_u32x16 p2 = dbp_s_load16(r, (int)(kDbpHeader + 8u * (o + (wb & 15u) + ((wb >> 4) & 15u))), 0);
    for (uint32_t k = 0; k < kDbpSegBlocks; ++k) {
        const uint32_t zz = (DBP_ABLATE & 1) ? lane * (p0[0] + p1[0] + p2[0])
                                             : planes_to_lanes(p0, wb & 15u) | (planes_to_lanes(p1, (wb >> 4) & 15u) << 8) |
                                                   (planes_to_lanes(p2, (wb >> 8) & 15u) << 16);
        if (k + 1 < kDbpSegBlocks) {  // the next block's planes, in flight during this block's sums and stores
            const uint32_t nb = kDbpSegBlocks * w + k + 1;
            wb = (uint32_t)__builtin_amdgcn_readlane((int)wl, (int)nb);
            o = (uint32_t)__builtin_amdgcn_readlane((int)ol, (int)nb);
            p0 = dbp_s_load16(r, (int)(kDbpHeader + 8u * o), 0);
            p1 = dbp_s_load16(r, (int)(kDbpHeader + 8u * (o + (wb & 15u))), 0);
            p2 = dbp_s_load16(r, (int)(kDbpHeader + 8u * (o + (wb & 15u) + ((wb >> 4) & 15u))), 0);
        }
        // zigzag back to the differences (mod 256), per byte; then the running sums from the carry
        const uint32_t d = ((zz >> 1) & 0x007F7F7Fu) ^ ((zz & 0x00010101u) * 0xFFu);
        const uint32_t x0 = ((DBP_ABLATE & 2) ? (d & 0x00FF00FFu) : wave_incl_sum(d & 0x00FF00FFu)) + c0;
        const uint32_t x1 = ((DBP_ABLATE & 2) ? ((d >> 8) & 0xFFu) : wave_incl_sum((d >> 8) & 0xFFu)) + c1;
        if (!(DBP_ABLATE & 4) || x0 == 0x12345678u)
            __builtin_amdgcn_raw_buffer_store_b32(a | (x0 & 0x00FF00FFu) | ((x1 & 0xFFu) << 8), out, (int)(4u * lane),
                                                  (int)(256u * k), 0);
        c0 = (uint32_t)__builtin_amdgcn_readlane((int)x0, 63) & 0x00FF00FFu;
        c1 = (uint32_t)__builtin_amdgcn_readlane((int)x1, 63) & 0xFFu;
    }
}

dim3 codec_grid(uint64_t n) { return dim3((uint32_t)((n + 4ull * kCodecBlock - 1) / (4ull * kCodecBlock))); }
bool vec_ok(const void* four, const void* three) { return ((uintptr_t)four & 15u) == 0 && ((uintptr_t)three & 3u) == 0; }

}  // namespace

hipError_t tri_launch_pack_bgr24(const uint32_t* src, uint8_t* dst, uint64_t n, uint32_t alpha, uint32_t* flag,
                                 hipStream_t stream, uint32_t* trailer) {
    if (n == 0) return hipSuccess;
    if (vec_ok(src, dst))
        hipLaunchKernelGGL(k_pack_bgr24<true>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha, flag, trailer);
    else
        hipLaunchKernelGGL(k_pack_bgr24<false>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha, flag, trailer);
    return hipGetLastError();
}

hipError_t tri_launch_unpack_bgr24(const uint8_t* src, uint32_t* dst, uint64_t n, uint32_t alpha, hipStream_t stream,
                                   const uint32_t* trailer, uint32_t* flags) {
    if (n == 0) return hipSuccess;
    if (vec_ok(dst, src))
        hipLaunchKernelGGL(k_unpack_bgr24<true>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha, trailer, flags);
    else
        hipLaunchKernelGGL(k_unpack_bgr24<false>, codec_grid(n), dim3(kCodecBlock), 0, stream, src, dst, n, alpha, trailer, flags);
    return hipGetLastError();
}

uint64_t tri_dbp_stream_bytes(uint64_t pixels, uint32_t slot_bytes) {
    return (pixels + kDbpSlotPixels - 1) / kDbpSlotPixels * (uint64_t)slot_bytes;
}

hipError_t tri_launch_dbp_pack(const uint32_t* src, uint64_t n, uint32_t alpha, uint8_t* dst, uint32_t slot_bytes,
                               uint32_t* flags, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 g((uint32_t)((n + kDbpSlotPixels - 1) / kDbpSlotPixels));
    hipLaunchKernelGGL(k_dbp_pack, g, dim3(kDbpPackThreads), 0, stream, src, n, alpha, dst, slot_bytes, flags);
    return hipGetLastError();
}

hipError_t tri_launch_dbp_unpack_bands(const uint8_t* const* src, uint32_t* const* dst, const uint64_t* n, uint32_t count,
                                       uint32_t alpha, uint32_t slot_bytes, hipStream_t stream, uint32_t* flags) {
    DbpBands b{};
    uint32_t grid = 0;
    for (uint32_t k = 0; k < count; ++k) {
        b.src[b.count] = src[k];
        b.dst[b.count] = dst[k];
        b.n[b.count] = n[k];
        b.first[b.count] = grid;
        grid += (uint32_t)((n[k] + kDbpSlotPixels - 1) / kDbpSlotPixels);
        if (n[k]) ++b.count;  // empty bands take no slot
    }
    b.first[b.count] = grid;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_dbp_unpack, dim3(grid), dim3(kDbpThreads), 0, stream, b, alpha, slot_bytes, flags);
    return hipGetLastError();
}

hipError_t tri_launch_dbp_unpack(const uint8_t* src, uint64_t n, uint32_t alpha, uint32_t slot_bytes, uint32_t* dst,
                                 hipStream_t stream) {
    return tri_launch_dbp_unpack_bands(&src, &dst, &n, 1, alpha, slot_bytes, stream);
}

extern "C" {

int tri_dbp_pack(const void* bgra, uint64_t pixels, uint32_t alpha, void* stream_out, uint32_t slot_bytes, uint32_t* flags,
                 void* stream) {
    if ((pixels && (!bgra || !stream_out)) || alpha > 255u || slot_bytes < TRI_DBP_MIN_SLOT || slot_bytes % 16u)
        return tri_internal_fail(TRI_E_INVALID, "tri_dbp_pack: bad argument");
    if (((uintptr_t)bgra & 3u) || ((uintptr_t)stream_out & 15u))
        return tri_internal_fail(TRI_E_INVALID, "tri_dbp_pack: misaligned buffer");
    const hipError_t e = tri_launch_dbp_pack(static_cast<const uint32_t*>(bgra), pixels, alpha,
                                             static_cast<uint8_t*>(stream_out), slot_bytes, flags,
                                             static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TRI_OK : tri_internal_fail(TRI_E_HIP, hipGetErrorString(e));
}

int tri_dbp_unpack(const void* stream_in, uint64_t pixels, uint32_t alpha, uint32_t slot_bytes, void* bgra, void* stream) {
    if ((pixels && (!bgra || !stream_in)) || alpha > 255u || slot_bytes < TRI_DBP_MIN_SLOT || slot_bytes % 16u)
        return tri_internal_fail(TRI_E_INVALID, "tri_dbp_unpack: bad argument");
    if (((uintptr_t)bgra & 3u) || ((uintptr_t)stream_in & 15u))
        return tri_internal_fail(TRI_E_INVALID, "tri_dbp_unpack: misaligned buffer");
    const hipError_t e = tri_launch_dbp_unpack(static_cast<const uint8_t*>(stream_in), pixels, alpha, slot_bytes,
                                               static_cast<uint32_t*>(bgra), static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TRI_OK : tri_internal_fail(TRI_E_HIP, hipGetErrorString(e));
}

uint64_t tri_dbp_bytes(uint64_t pixels, uint32_t slot_bytes) { return tri_dbp_stream_bytes(pixels, slot_bytes); }

int tri_dbp_unpack_bands(const void* const* streams, void* const* bgra, const uint64_t* pixels, uint32_t count,
                         uint32_t alpha, uint32_t slot_bytes, void* stream) {
    if ((count && (!streams || !bgra || !pixels)) || count > TRI_DBP_MAX_BANDS || alpha > 255u ||
        slot_bytes < TRI_DBP_MIN_SLOT || slot_bytes % 16u)
        return tri_internal_fail(TRI_E_INVALID, "tri_dbp_unpack_bands: bad argument");
    const uint8_t* src[TRI_DBP_MAX_BANDS];
    uint32_t* dst[TRI_DBP_MAX_BANDS];
    for (uint32_t k = 0; k < count; ++k) {
        if (pixels[k] && (!streams[k] || !bgra[k]))
            return tri_internal_fail(TRI_E_INVALID, "tri_dbp_unpack_bands: null buffer");
        if (((uintptr_t)bgra[k] & 3u) || ((uintptr_t)streams[k] & 15u))
            return tri_internal_fail(TRI_E_INVALID, "tri_dbp_unpack_bands: misaligned buffer");
        src[k] = static_cast<const uint8_t*>(streams[k]);
        dst[k] = static_cast<uint32_t*>(bgra[k]);
    }
    const hipError_t e = tri_launch_dbp_unpack_bands(src, dst, pixels, count, alpha, slot_bytes,
                                                     static_cast<hipStream_t>(stream));
    return e == hipSuccess ? TRI_OK : tri_internal_fail(TRI_E_HIP, hipGetErrorString(e));
}

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
