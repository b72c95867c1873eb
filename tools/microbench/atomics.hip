// Microbenchmark (not product code): random-address atomicMin / load throughput on gfx950,
// sized like LFMIS round 0 at the 10M-clause config (2.7M updates into 2.5M variables).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k_min32(uint32_t* owner, const uint32_t* idx, uint32_t n, uint32_t key) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicMin(&owner[idx[i]], key + i);
}
__global__ void k_min64(unsigned long long* owner, const uint32_t* idx, uint32_t n, unsigned long long key) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicMin(&owner[idx[i]], key + i);
}
__global__ void k_load64(const unsigned long long* owner, const uint32_t* idx, uint32_t n, unsigned long long* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long v = 0;
    if (i < n) v = owner[idx[i]];
    if (v == 12345) out[0] = v;
}
__global__ void k_load32(const uint32_t* owner, const uint32_t* idx, uint32_t n, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v = 0;
    if (i < n) v = owner[idx[i]];
    if (v == 12345) out[0] = v;
}
__global__ void k_store32(uint32_t* owner, const uint32_t* idx, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) owner[idx[i]] = i;
}
__global__ void k_min32_ret(uint32_t* owner, const uint32_t* idx, uint32_t n, uint32_t key, uint32_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { uint32_t o = atomicMin(&owner[idx[i]], key + i); if (o == 7) out[0] = o; }
}

int main() {
    const uint32_t nv = 2500000, n = 2700000;
    std::vector<uint32_t> h(n);
    uint64_t s = 88172645463325252ull;
    for (auto& x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)(s % nv); }
    uint32_t *idx, *o32, *out32; unsigned long long *o64, *out64;
    hipMalloc(&idx, n * 4); hipMalloc(&o32, nv * 4); hipMalloc(&o64, nv * 8);
    hipMalloc(&out32, 64); hipMalloc(&out64, 64);
    hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(o32, 0xFF, nv * 4); hipMemset(o64, 0xFF, nv * 8);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    dim3 grid((n + 255) / 256);
    auto time = [&](const char* name, auto f) {
        for (int w = 0; w < 3; ++w) f();
        hipEventRecord(a);
        const int R = 20;
        for (int r = 0; r < R; ++r) f();
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-14s %8.1f us   %6.1f G ops/s\n", name, ms * 1000 / R, n / (ms / R * 1e-3) / 1e9);
    };
    uint32_t key = 1000000000u;
    time("atomicMin u32", [&] { k_min32<<<grid, 256>>>(o32, idx, n, key -= 3000000); });
    time("atomicMin u64", [&] { k_min64<<<grid, 256>>>(o64, idx, n, (unsigned long long)(key -= 3000000) << 20); });
    time("atomicMin ret", [&] { k_min32_ret<<<grid, 256>>>(o32, idx, n, key -= 3000000, out32); });
    time("load u32", [&] { k_load32<<<grid, 256>>>(o32, idx, n, out32); });
    time("load u64", [&] { k_load64<<<grid, 256>>>(o64, idx, n, out64); });
    time("store u32", [&] { k_store32<<<grid, 256>>>(o32, idx, n); });
    return 0;
}
