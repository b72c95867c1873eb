// Microbenchmark (not product code): the two primitives a dependency-driven LFMIS would rest on.
//  1. scattered 4-byte write-through (sc1) stores / relaxed agent loads, 2M of them over 128 MB,
//     against plain stores -- the per-message cost of pushing chain states to successors;
//  2. hop latency: a token passed L times between random workgroups (one per CU) that each poll
//     a mailbox region of P words with sc1 loads, the way a run workgroup would poll its pairs.
// Every spin is bounded by a device wall-clock timeout (s_memrealtime, 100 MHz).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

template <int MODE>  // 0 plain store, 1 sc1 (relaxed agent atomic) store, 2 relaxed agent load
__global__ void k_scatter(uint32_t* a, uint32_t mask, uint32_t per, uint32_t salt, uint32_t* sink) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t p = hsh(t * per + i + salt) & mask;
        if constexpr (MODE == 0) a[p] = t;
        else if constexpr (MODE == 1) __hip_atomic_store(a + p, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else acc += __hip_atomic_load(a + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (MODE == 2 && acc == 0x12345678u) sink[0] = acc;
}

// hop h lives at word pos[h] of workgroup wg[h]'s mailbox; its token value is tag + h.  A
// workgroup's threads each own P / blockDim words and poll the ones they still wait on.
template <int WPT>  // words per thread
__global__ void k_chain(uint32_t* mbox, const uint32_t* wg, const uint32_t* pos, uint32_t L, uint32_t tag,
                        unsigned long long* arrive, uint32_t* done, uint32_t* timeout, int sleep) {
    const uint32_t P = blockDim.x * WPT;
    uint32_t* my = mbox + (size_t)blockIdx.x * P;
    // which of my words carry a hop (host laid them out): hop index per word, ~0 = none
    uint32_t hop[WPT];
    uint32_t waiting = 0;
    for (int k = 0; k < WPT; ++k) {
        hop[k] = ~0u;
    }
    for (uint32_t h = 1; h < L; ++h)  // (L is small: a linear scan is fine for a microbenchmark)
        if (wg[h] == blockIdx.x && pos[h] / WPT == threadIdx.x) { hop[pos[h] % WPT] = h; waiting |= 1u << (pos[h] % WPT); }
    const unsigned long long t0 = now();
    if (blockIdx.x == wg[0] && threadIdx.x == 0) {  // start the chain
        arrive[0] = t0;
        const uint32_t n1 = 1;
        __hip_atomic_store(mbox + (size_t)wg[n1] * P + pos[n1], tag + n1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (;;) {
        // poll every word this thread owns (the worst case: a whole region per pass)
        uint32_t v[WPT];
#pragma unroll
        for (int k = 0; k < WPT; ++k) v[k] = __hip_atomic_load(my + threadIdx.x * WPT + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < WPT; ++k) {
            if (!((waiting >> k) & 1u) || v[k] != tag + hop[k]) continue;
            waiting &= ~(1u << k);
            const uint32_t h = hop[k];
            arrive[h] = now();
            if (h + 1 < L) __hip_atomic_store(mbox + (size_t)wg[h + 1] * P + pos[h + 1], tag + h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(done, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag) break;
        if (now() - t0 > 2000000ull) { atomicAdd(timeout, 1u); break; }  // 20 ms
        if (sleep) __builtin_amdgcn_s_sleep(1);
    }
}

int main() {
    int ncu = 256;
    {
        hipDeviceProp_t p;
        CK(hipGetDeviceProperties(&p, 0));
        ncu = p.multiProcessorCount;
        printf("device %s, %d CUs\n", p.gcnArchName, ncu);
    }
    const uint32_t words = 32u << 20;  // 128 MB
    uint32_t *a, *sink;
    CK(hipMalloc(&a, words * 4ull));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0, words * 4ull));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t per = 8, threads = 1024, blocks = ncu;
    const double nops = (double)per * threads * blocks;
    const char* names[3] = {"plain store", "sc1 store", "sc1 load"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            if (mode == 0) k_scatter<0><<<blocks, threads>>>(a, words - 1, per, rep * 977, sink);
            if (mode == 1) k_scatter<1><<<blocks, threads>>>(a, words - 1, per, rep * 977, sink);
            if (mode == 2) k_scatter<2><<<blocks, threads>>>(a, words - 1, per, rep * 977, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 2) printf("scatter %-12s %.0f ops in %.1f us = %.1f G ops/s\n", names[mode], nops, ms * 1e3, nops / (ms * 1e-3) / 1e9);
        }
    }
    // chains
    for (int cfg = 0; cfg < 6; ++cfg) {
        // (threads, words per thread): the 4096-word region by 256 x 16 and 1024 x 4 (residency
        // vs polling volume), then 1024 x 16 (four times the polling)
        const uint32_t th = cfg % 3 == 0 ? 256 : 1024;
        const uint32_t WPT = cfg % 3 == 1 ? 4 : 16;
        const int sleep = cfg / 3;
        const uint32_t L = 200, P = th * WPT;
        std::vector<uint32_t> wg(L), pos(L);
        uint64_t s = 0x9E3779B97F4A7C15ull + cfg;
        for (uint32_t h = 0; h < L; ++h) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            wg[h] = (uint32_t)(s % blocks);
            if (h && wg[h] == wg[h - 1]) wg[h] = (wg[h] + 1) % blocks;
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            pos[h] = (uint32_t)(s % P);
        }
        // distinct (wg, pos) per hop
        for (uint32_t h = 0; h < L; ++h) pos[h] = (pos[h] & ~255u) | (h & 255u);
        uint32_t *mb, *dwg, *dpos, *done, *tmo;
        unsigned long long* arr;
        CK(hipMalloc(&mb, (size_t)blocks * P * 4));
        CK(hipMalloc(&dwg, L * 4)); CK(hipMalloc(&dpos, L * 4)); CK(hipMalloc(&arr, L * 8));
        CK(hipMalloc(&done, 64)); CK(hipMalloc(&tmo, 64));
        CK(hipMemset(mb, 0, (size_t)blocks * P * 4)); CK(hipMemset(done, 0, 64)); CK(hipMemset(tmo, 0, 64));
        CK(hipMemcpy(dwg, wg.data(), L * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dpos, pos.data(), L * 4, hipMemcpyHostToDevice));
        for (int rep = 0; rep < 3; ++rep) {
            const uint32_t tag = 1000u * (rep + 1);
            CK(hipEventRecord(e0));
            if (WPT == 4) k_chain<4><<<blocks, th>>>(mb, dwg, dpos, L, tag, arr, done, tmo, sleep);
            else k_chain<16><<<blocks, th>>>(mb, dwg, dpos, L, tag, arr, done, tmo, sleep);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<unsigned long long> h(L);
            uint32_t to = 0;
            CK(hipMemcpy(h.data(), arr, L * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&to, tmo, 4, hipMemcpyDeviceToHost));
            std::vector<double> d;
            for (uint32_t i = 1; i < L; ++i) d.push_back((double)(h[i] - h[i - 1]) * 0.01);  // 100 MHz -> us
            std::sort(d.begin(), d.end());
            if (h[L - 1] < h[0] || to) { printf("chain threads %u words/thread %u sleep %d rep %d: kernel %.1f us, INCOMPLETE (%u timeouts)\n", th, WPT, sleep, rep, ms * 1e3, to); CK(hipMemset(tmo, 0, 64)); continue; }
            printf("chain threads %u words/thread %u sleep %d rep %d: kernel %.1f us, %u hops: total %.1f us, per hop median %.2f p90 %.2f max %.2f us, timeouts %u\n",
                   th, WPT, sleep, rep, ms * 1e3, L - 1, (double)(h[L - 1] - h[0]) * 0.01, d[d.size() / 2], d[d.size() * 9 / 10], d.back(), to);
        }
        hipFree(mb); hipFree(dwg); hipFree(dpos); hipFree(arr); hipFree(done); hipFree(tmo);
    }
    return 0;
}
