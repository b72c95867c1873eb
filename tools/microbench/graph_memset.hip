// Replays of captured graphs that hold memset nodes (the round-robin stall under torch's
// bundled HIP runtime): the graphs of round 4's round-robin iteration held two
// hipMemsetAsync nodes among their kernels, and under the ROCm 7.0 runtime torch bundles the
// host waited forever on the second replay of the first graph.  This program captures three
// graphs of kernel + memset + kernel + memset + kernel bodies (1, 2, 3 copies), each at its
// first use, replays them in turn R times (each replay followed by a 12-byte device-to-host
// copy and a stream sync, as launch_rr_iteration does), and checks the counters; with `kernels`
// the graphs hold no memset nodes (kernels clear the buffers instead).
// Run it against the runtime it was built with and against torch's (LD_LIBRARY_PATH).
// build: hipcc --offload-arch=gfx950 -O2 -o /tmp/graph_memset tools/microbench/graph_memset.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_add(unsigned* ctr, const unsigned* zero_a, const unsigned* zero_b, unsigned* out) {
    // counts the replays; records whether the cleared buffers were zero when it ran
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        ctr[0] += 1;
        out[0] = ctr[0];
        out[1] = zero_a ? zero_a[0] : 0u;
        out[2] = zero_b ? zero_b[0] : 0u;
    }
}
__global__ void k_dirty(unsigned* a, unsigned n) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = 0xFFFFFFFFu;
}
__global__ void k_clear(unsigned* a, unsigned n) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = 0u;
}

int main(int argc, char** argv) {
    const bool kernels_only = argc > 1 && strcmp(argv[1], "kernels") == 0;
    const int R = argc > 2 ? atoi(argv[2]) : 20;
    int rt = 0;
    CK(hipRuntimeGetVersion(&rt));
    printf("HIP runtime version %d, graph with %s\n", rt, kernels_only ? "kernel nodes only" : "memset nodes");
    const unsigned n = (argc > 3 ? (unsigned)atoi(argv[3]) : 4u) << 18;  // (argv[3]: MiB per cleared buffer)
    const int body = argc > 4 ? atoi(argv[4]) : 1;                          // (argv[4]: bodies per graph copy)
    unsigned *a, *b2, *ctr, *out, *h;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b2, n * 4));
    CK(hipMalloc(&ctr, 64));
    CK(hipMalloc(&out, 64));
    CK(hipHostMalloc((void**)&h, 64, 0));
    CK(hipMemset(ctr, 0, 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // G graphs of different lengths (as the loop's pre(P) / one-pass / post pieces), each captured
    // at its first use, after the others have been replayed -- the order in which the round
    // robin captured its graphs
    constexpr int G = 3;
    hipGraphExec_t ge[G] = {};
    int uses[G] = {};
    unsigned expect = 0;
    for (int r = 1; r <= R; ++r) {
        const int k = (r - 1) % G == 0 ? 0 : ((r - 1) % G == 1 ? 1 : 2);
        if (!ge[k]) {
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int rep = 0; rep < (k + 1) * body; ++rep) {  // (graph k: (k + 1) body copies)
                k_dirty<<<256, 256, 0, s>>>(a, n);
                k_dirty<<<256, 256, 0, s>>>(b2, n);
                if (kernels_only) k_clear<<<256, 256, 0, s>>>(a, n);
                else CK(hipMemsetAsync(a, 0, n * 4, s));
                k_add<<<1, 64, 0, s>>>(ctr, a, nullptr, out);
                if (kernels_only) k_clear<<<256, 256, 0, s>>>(b2, n);
                else CK(hipMemsetAsync(b2, 0, n * 4, s));
                k_add<<<1, 64, 0, s>>>(ctr, a, b2, out);
            }
            hipGraph_t g;
            CK(hipStreamEndCapture(s, &g));
            size_t nn = 0;
            CK(hipGraphGetNodes(g, nullptr, &nn));
            CK(hipGraphInstantiate(&ge[k], g, nullptr, nullptr, 0));
            CK(hipGraphUpload(ge[k], s));
            printf("graph %d captured at replay %d: %zu nodes\n", k, r, nn);
        }
        const auto t0 = std::chrono::steady_clock::now();
        CK(hipGraphLaunch(ge[k], s));
        CK(hipMemcpyAsync(h, out, 12, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        expect += 2u * (k + 1) * body;
        ++uses[k];
        const bool ok = h[0] == expect && h[1] == 0u && h[2] == 0u;
        printf("replay %d (graph %d, use %d): %.0f us, counter %u, cleared %u %u: %s\n", r, k, uses[k], us, h[0], h[1], h[2],
               ok ? "ok" : "WRONG");
        fflush(stdout);
        if (!ok) return 2;
    }
    printf("all %d replays completed\n", R);
    return 0;
}
