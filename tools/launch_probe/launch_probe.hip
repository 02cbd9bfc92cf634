// Host cost of enqueueing one frame's launches (VERDICT r3 "host cost per frame"): three empty
// kernels per "frame" with (a) a 1.7-KB by-value argument block (today's TriFrameParams + TriDeviceBuffers),
// (b) a 16-B argument (a pointer to device-resident parameters), (c) (b) preceded by a 1.7-KB pinned
// host-to-device copy of the parameters, (d) a HIP graph of the three kernels, (e) the graph with its three
// nodes' parameters updated before each launch. Host time per frame, median of bursts that never fill the queue.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Big { unsigned w[432]; };  // 1728 B
__global__ void k_big(Big p, unsigned* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && p.w[5] == 12345u) out[0] = p.w[7]; }
__global__ void k_small(const Big* p, unsigned* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && p->w[5] == 12345u) out[0] = p->w[7]; }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
using clk = std::chrono::steady_clock;

template <class F> double burst_us(hipStream_t s, F&& frame) {
    std::vector<double> v;
    for (int r = 0; r < 30; ++r) {
        (void)hipStreamSynchronize(s);
        auto t0 = clk::now();
        for (int i = 0; i < 16; ++i) frame();
        v.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count() / 16);
    }
    (void)hipStreamSynchronize(s);
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned* out; Big* dp; Big* hp;
    CK(hipMalloc(&out, 64)); CK(hipMalloc(&dp, sizeof(Big) * 8)); CK(hipHostMalloc(&hp, sizeof(Big) * 8));
    Big big{}; big.w[5] = 1;
    const dim3 g(2048), t(256);
    auto a = [&] { for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_big, g, t, 0, s, big, out); };
    auto b = [&] { for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_small, g, t, 0, s, dp, out); };
    int slot = 0;
    auto c = [&] {
        hp[slot] = big;
        (void)hipMemcpyAsync(dp + slot, hp + slot, sizeof(Big), hipMemcpyHostToDevice, s);
        for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_small, g, t, 0, s, dp + slot, out);
        slot = (slot + 1) & 7;
    };
    for (int w = 0; w < 3; ++w) { a(); b(); c(); }
    CK(hipStreamSynchronize(s));
    printf("a 3 launches, 1.7 KB args: %.2f us/frame\n", burst_us(s, a));
    printf("b 3 launches, 16 B args: %.2f us/frame\n", burst_us(s, b));
    printf("c pinned 1.7 KB copy + 3 launches, 16 B args: %.2f us/frame\n", burst_us(s, c));
    // graph
    hipGraph_t gr; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_big, g, t, 0, s, big, out);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    size_t nn = 0; CK(hipGraphGetNodes(gr, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn); CK(hipGraphGetNodes(gr, nodes.data(), &nn));
    auto d = [&] { (void)hipGraphLaunch(ge, s); };
    printf("d graph of 3 (1.7 KB args): %.2f us/frame\n", burst_us(s, d));
    std::vector<hipKernelNodeParams> kp(nn);
    for (size_t i = 0; i < nn; ++i) CK(hipGraphKernelNodeGetParams(nodes[i], &kp[i]));
    void* args[2] = {&big, &out};
    auto e = [&] {
        big.w[7]++;
        for (size_t i = 0; i < nn; ++i) { kp[i].kernelParams = args; (void)hipGraphExecKernelNodeSetParams(ge, nodes[i], &kp[i]); }
        (void)hipGraphLaunch(ge, s);
    };
    printf("e graph of 3, params updated: %.2f us/frame\n", burst_us(s, e));
    // f: a graph of a pinned-host -> device parameter copy + the 3 kernels reading the device copy (small args):
    // the host writes the slot, then one graph launch (no node updates)
    hipGraph_t gf; hipGraphExec_t gfe;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipMemcpyAsync(dp, hp, sizeof(Big), hipMemcpyHostToDevice, s));
    for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_small, g, t, 0, s, dp, out);
    CK(hipStreamEndCapture(s, &gf));
    CK(hipGraphInstantiate(&gfe, gf, nullptr, nullptr, 0));
    auto f = [&] { hp[0].w[7]++; (void)hipGraphLaunch(gfe, s); };
    printf("f graph: pinned param copy + 3 kernels: %.2f us/frame\n", burst_us(s, f));
    CK(hipStreamSynchronize(s));
    {
        auto t0 = clk::now();
        for (int i = 0; i < 2000; ++i) f();
        CK(hipStreamSynchronize(s));
        printf("f drained: %.2f us/frame\n", std::chrono::duration<double, std::micro>(clk::now() - t0).count() / 2000);
    }
    // g: the same graph without the copy node (device-resident parameters)
    hipGraph_t gg; hipGraphExec_t gge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_small, g, t, 0, s, dp, out);
    CK(hipStreamEndCapture(s, &gg));
    CK(hipGraphInstantiate(&gge, gg, nullptr, nullptr, 0));
    auto gl = [&] { (void)hipGraphLaunch(gge, s); };
    printf("g graph of 3 (16 B args): %.2f us/frame\n", burst_us(s, gl));
    // the GPU-side cost of the copy: frames back to back, drained
    for (auto* f : {"b", "c"}) {
        CK(hipStreamSynchronize(s));
        auto t0 = clk::now();
        for (int i = 0; i < 2000; ++i) { if (f[0] == 'b') b(); else c(); }
        CK(hipStreamSynchronize(s));
        printf("%s drained: %.2f us/frame\n", f, std::chrono::duration<double, std::micro>(clk::now() - t0).count() / 2000);
    }
    unsigned h = 0; CK(hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost));
    printf("ok %u\n", h);
    return 0;
}
