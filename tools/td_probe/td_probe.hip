// TD / TA throughput probe: CU cycles per wave-level gather instruction for the access shapes of k_raster's
// fragment fetch, with the data resident in L1 / L2 (tools/td_probe.sh). Each wave issues
// batches of 8 independent raw buffer loads; every workgroup slot of the chip is filled (8 waves per SIMD).
//   full64    64 active lanes, 64 distinct 48-B records (b96 at the record start)
//   runs12    64 active lanes reading 12 distinct records (runs of 5-6 lanes, as pixels of one triangle)
//   first16   lanes 0..15 active (compacted), distinct records
//   every4    lanes 0, 4, 8, .. active (one per quad), distinct records
//   full64x4  64 active lanes, distinct records, b128
//   same1     64 active lanes, one record
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr int kIters = 256;

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(const uint8_t* buf, uint32_t nrec, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u, w = blockIdx.x * 4u + threadIdx.x / 64u;
    const Rsrc r = rsrc(buf, nrec * 48u);
    bool active = true;
    if (MODE == 2) active = lane < 16u;
    if (MODE == 3) active = (lane & 3u) == 0u;
    uint32_t rec = lane;
    if (MODE == 1) rec = lane * 12u / 64u;
    if (MODE == 5) rec = 0;
    uint32_t acc = 0;
    if (active) {
        for (int it = 0; it < kIters; ++it) {
            const uint32_t base = (w * 977u + (uint32_t)it * 131u) & (nrec - 1u);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t off = ((base + rec + (uint32_t)j * 64u) & (nrec - 1u)) * 48u;
                if (MODE == 4) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
                    acc += v[0] ^ v[1] ^ v[2] ^ v[3];
                } else {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0);
                    acc += v[0] ^ v[1] ^ v[2];
                }
            }
        }
    }
    if (acc == 0x9E3779B1u) out[0] = acc;
}

template <int MODE>
float run(const uint8_t* buf, uint32_t nrec, uint32_t* out, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) k_probe<MODE><<<grid, 256>>>(buf, nrec, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int rep = 0; rep < reps; ++rep) k_probe<MODE><<<grid, 256>>>(buf, nrec, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int grid = cus * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    uint8_t* buf;
    uint32_t* out;
    const uint32_t big = 1u << 22;  // 4 Mi records (192 MiB)
    hipMalloc(&buf, (size_t)big * 48);
    hipMemset(buf, 0, (size_t)big * 48);
    hipMalloc(&out, 64);
    const double instr_per_cu = (double)grid * 4 * kIters * 8 / cus;  // wave-level loads per CU
    const double ghz = 2.4;
    const char* names[] = {"full64", "runs12", "first16", "every4", "full64x4", "same1"};
    for (uint32_t nrec : {512u, 32768u, big}) {  // 24 KiB (L1), 1.5 MiB (L2), 192 MiB (MALL/HBM)
        float t[6];
        t[0] = run<0>(buf, nrec, out, grid);
        t[1] = run<1>(buf, nrec, out, grid);
        t[2] = run<2>(buf, nrec, out, grid);
        t[3] = run<3>(buf, nrec, out, grid);
        t[4] = run<4>(buf, nrec, out, grid);
        t[5] = run<5>(buf, nrec, out, grid);
        for (int m = 0; m < 6; ++m)
            printf("footprint %9u B  %-9s %8.3f ms  %6.1f CU cycles per wave load (at %.1f GHz)\n", nrec * 48, names[m], t[m],
                   t[m] * 1e-3 * ghz * 1e9 / instr_per_cu, ghz);
    }
    return 0;
}
