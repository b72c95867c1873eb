// Dependent-load latency on one MI355X (the repair rounds' critical path):
// one lane chases a random cycle through a buffer of S MiB, written by another kernel just
// before (as k_fp_turn / k_fp_bbuild leave the repair's inputs), and reports ns per hop;
// also the same after the buffer was read once by the chasing CU (L2-warm) and with 16 chases
// in flight per lane (the gather's memory-level parallelism).
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/chase tools/microbench/chase.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_fill(uint32_t* nxt, const uint32_t* perm, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        nxt[perm[i]] = perm[(i + 1) % n];
}

template <int W>
__global__ void k_chase(const uint32_t* nxt, uint32_t hops, uint32_t n, unsigned long long* out) {
    if (threadIdx.x != 0) return;
    uint32_t p[W];
#pragma unroll
    for (int w = 0; w < W; ++w) p[w] = (uint32_t)((w * 2654435761ull) % n);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t h = 0; h < hops; ++h) {
#pragma unroll
        for (int w = 0; w < W; ++w) p[w] = nxt[p[w]];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) acc += p[w];
    out[0] = t1 - t0;
    out[1] = acc;
}

int main(int argc, char** argv) {
    const uint32_t mib = argc > 1 ? atoi(argv[1]) : 32;
    const uint32_t n = mib * (1u << 18);  // 4-byte words
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    std::mt19937 rng(1);
    std::shuffle(perm.begin(), perm.end(), rng);
    uint32_t *d_nxt, *d_perm;
    unsigned long long* d_out;
    CK(hipMalloc(&d_nxt, 4ull * n));
    CK(hipMalloc(&d_perm, 4ull * n));
    CK(hipMalloc(&d_out, 16));
    CK(hipMemcpy(d_perm, perm.data(), 4ull * n, hipMemcpyHostToDevice));
    const uint32_t hops = 200;
    for (int rep = 0; rep < 3; ++rep) {
        unsigned long long h[2];
        k_fill<<<1024, 256>>>(d_nxt, d_perm, n);
        k_chase<1><<<1, 64>>>(d_nxt, hops, n, d_out);
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        const double cold = h[0] * 10.0 / hops;
        k_chase<1><<<1, 64>>>(d_nxt, hops, n, d_out);
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        const double again = h[0] * 10.0 / hops;
        k_fill<<<1024, 256>>>(d_nxt, d_perm, n);
        k_chase<16><<<1, 64>>>(d_nxt, hops, n, d_out);
        CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
        const double w16 = h[0] * 10.0 / hops;
        printf("%u MiB: ns per dependent hop: fresh %.0f, repeated %.0f; 16 chases in flight %.0f per step\n", mib, cold,
               again, w16);
    }
    return 0;
}
