// FETCH_SIZE calibration probe (MI355X_MICROARCH.md "HBM / rocprofv3").
//
// Each kernel reads a 1 GiB (or 768 MiB) buffer -- 3-4x the 256 MiB Infinity Cache -- in one access shape
// whose true line traffic is known from the shape alone, so the L2->fabric read counters (FETCH_SIZE and
// the sized TCC_EA0_RDREQ_{32B,64B,128B} requests) can be compared against known bytes:
//   k_cal_stream16 / k_cal_stream12  coalesced 16-B (b128) / 12-B (b96) per lane, every byte once:
//                                    truth = footprint.
//   k_cal_chunk16 / k_cal_chunk12    a wave reads one 1024-B / 768-B contiguous chunk, chunks in a
//                                    scrambled order (whole 128-B lines, lines never revisited): truth = footprint.
//   k_cal_line16 / k_cal_line12      one lane per distinct 128-B line, lines in scrambled order (k_raster's
//                                    gathers at their sparsest): truth = lines x request size, which the
//                                    sized counters decide (64 B or 128 B per line).
//   k_cal_dense16 / k_cal_dense12    packed 16-B / 12-B records, each read once in scrambled order (the
//                                    snap / varying gathers of k_raster over random triangle order):
//                                    footprint is the lower bound; the excess is re-fetch after eviction.
// Loads are raw buffer loads exactly as k_raster issues them (raster_kernels.hip ld128 / b96 snap reads).
// The kernels only read; one store happens only for an impossible checksum, so writes are ~0.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t scramble(uint32_t i, uint32_t mask) { return (i * 0x9E3779B1u) & mask; }
__device__ __forceinline__ uint32_t ld16(Rsrc r, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return v[0] ^ v[1] ^ v[2] ^ v[3];
}
__device__ __forceinline__ uint32_t ld12(Rsrc r, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0);
    return v[0] ^ v[1] ^ v[2];
}
__device__ __forceinline__ void sink(uint32_t acc, uint32_t* out) {
    if (acc == 0x9E3779B1u) out[0] = acc;  // never true for the zero-filled buffer: keeps the loads live
}

constexpr uint32_t kBytes = 1u << 30;          // 1 GiB buffer
constexpr uint32_t kRec16 = kBytes / 16;       // 2^26 records
constexpr uint32_t kRec12 = kRec16;            // 2^26 x 12 B = 768 MiB
constexpr uint32_t kLines = kBytes / 128;      // 2^23 lines
constexpr uint32_t kChunks16 = kBytes / 1024;  // 2^20 chunks of 1 KiB
constexpr uint32_t kChunks12 = 1u << 20;       // 2^20 chunks of 768 B = 768 MiB

__global__ __launch_bounds__(256) void k_cal_stream16(const uint8_t* buf, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    sink(ld16(rsrc(buf, kBytes), i * 16u), out);
}
__global__ __launch_bounds__(256) void k_cal_stream12(const uint8_t* buf, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    sink(ld12(rsrc(buf, kBytes), i * 12u), out);
}
__global__ __launch_bounds__(256) void k_cal_chunk16(const uint8_t* buf, uint32_t* out) {
    const uint32_t w = blockIdx.x * 4u + threadIdx.x / 64u, lane = threadIdx.x & 63u;
    sink(ld16(rsrc(buf, kBytes), scramble(w, kChunks16 - 1) * 1024u + lane * 16u), out);
}
__global__ __launch_bounds__(256) void k_cal_chunk12(const uint8_t* buf, uint32_t* out) {
    const uint32_t w = blockIdx.x * 4u + threadIdx.x / 64u, lane = threadIdx.x & 63u;
    sink(ld12(rsrc(buf, kBytes), scramble(w, kChunks12 - 1) * 768u + lane * 12u), out);
}
__global__ __launch_bounds__(256) void k_cal_line16(const uint8_t* buf, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    sink(ld16(rsrc(buf, kBytes), scramble(i, kLines - 1) * 128u), out);
}
__global__ __launch_bounds__(256) void k_cal_line12(const uint8_t* buf, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    sink(ld12(rsrc(buf, kBytes), scramble(i, kLines - 1) * 128u), out);
}
__global__ __launch_bounds__(256) void k_cal_dense16(const uint8_t* buf, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    sink(ld16(rsrc(buf, kBytes), scramble(i, kRec16 - 1) * 16u), out);
}
__global__ __launch_bounds__(256) void k_cal_dense12(const uint8_t* buf, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    sink(ld12(rsrc(buf, kBytes), scramble(i, kRec12 - 1) * 12u), out);
}

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef void (*Kern)(const uint8_t*, uint32_t*);
struct Case {
    const char* name;
    Kern k;
    uint32_t blocks;     // 256-lane workgroups
    double truth_bytes;  // known line bytes (0: decided by the sized counters / lower bound only)
    double footprint;
};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 0, kBytes));
    CHECK(hipMemset(out, 0, 64));
    const Case cases[] = {
        {"k_cal_stream16", k_cal_stream16, kRec16 / 256, (double)kBytes, (double)kBytes},
        {"k_cal_stream12", k_cal_stream12, kRec12 / 256, 12.0 * kRec12, 12.0 * kRec12},
        {"k_cal_chunk16", k_cal_chunk16, kChunks16 / 4, (double)kBytes, (double)kBytes},
        {"k_cal_chunk12", k_cal_chunk12, kChunks12 / 4, 768.0 * kChunks12, 768.0 * kChunks12},
        {"k_cal_line16", k_cal_line16, kLines / 256, 0.0, 128.0 * kLines},
        {"k_cal_line12", k_cal_line12, kLines / 256, 0.0, 128.0 * kLines},
        {"k_cal_dense16", k_cal_dense16, kRec16 / 256, 0.0, (double)kBytes},
        {"k_cal_dense12", k_cal_dense12, kRec12 / 256, 0.0, 12.0 * kRec12},
    };
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    printf("{\"cases\": [\n");
    for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
        const Case& k = cases[c];
        float best = 1e30f, sum = 0.f;
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(a, 0));
            hipLaunchKernelGGL(k.k, dim3(k.blocks), dim3(256), 0, 0, buf, out);
            CHECK(hipGetLastError());
            CHECK(hipEventRecord(b, 0));
            CHECK(hipEventSynchronize(b));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf(" {\"kernel\": \"%s\", \"lanes\": %u, \"truth_bytes\": %.0f, \"footprint\": %.0f, \"ms_min\": %.4f, "
               "\"ms_mean\": %.4f, \"footprint_gbs\": %.1f}%s\n",
               k.name, k.blocks * 256u, k.truth_bytes, k.footprint, best, sum / reps, k.footprint / (best * 1e6),
               c + 1 < sizeof(cases) / sizeof(cases[0]) ? "," : "");
    }
    printf("]}\n");
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
