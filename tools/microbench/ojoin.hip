// Microbenchmark (not product code): round 0 of the LFMIS decided from static per-variable
// occurrence lists instead of claim pairs (the direction the round-3 review proposed).
//
// A violated clause c wins round 0 iff, in the occurrence list of each of its variables (clause
// ids ascending), no clause before c is violated.  Lists are stored back to back, each preceded
// by a sentinel word (~0u); opos[c * K + j] = the position of c's (first) occurrence in the list
// of its j-th variable.  A lane per violated clause scans backwards from opos until a sentinel
// (win) or a violated clause (lose), looking each one up in the violated bitmask (1.25 MB at
// M: L2-resident).  Times are hipEvent averages over back-to-back launches.
//   scan1  one dword per step
//   scan4  aligned uint4 loads of the preceding words, four bit lookups per load
//   scan16 four aligned uint4 loads per list and step, all 16 bit lookups issued unconditionally
//          (two dependent latencies per step; a step covers 13-16 preceding words)
// Config M: n = 2.5M, m = 10M, K = 3, ~7.5% violated.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int K = 3;

__device__ __forceinline__ bool vbit(const uint64_t* vm, uint32_t c) { return (vm[c >> 6] >> (c & 63)) & 1ull; }

__global__ __launch_bounds__(256) void k_scan1(const uint32_t* __restrict__ occ, const uint32_t* __restrict__ opos,
                                               const uint64_t* __restrict__ vm, const uint32_t* __restrict__ ent,
                                               uint32_t ne, uint8_t* __restrict__ lose) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ne) return;
    const uint32_t c = ent[i];
    bool lost = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        uint32_t p = opos[(uint64_t)c * K + j];
        for (;;) {
            const uint32_t x = occ[--p];
            if (x == ~0u) break;
            if (vbit(vm, x)) { lost = true; break; }
        }
    }
    lose[i] = lost;
}

__global__ __launch_bounds__(256) void k_scan4(const uint32_t* __restrict__ occ, const uint32_t* __restrict__ opos,
                                               const uint64_t* __restrict__ vm, const uint32_t* __restrict__ ent,
                                               uint32_t ne, uint8_t* __restrict__ lose) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ne) return;
    const uint32_t c = ent[i];
    uint32_t p[K];
#pragma unroll
    for (int j = 0; j < K; ++j) p[j] = opos[(uint64_t)c * K + j];
    bool lost = false;
    bool live[K];
#pragma unroll
    for (int j = 0; j < K; ++j) live[j] = true;
    // step: the aligned uint4 holding p - 1 (words below p only)
    for (int it = 0; it < 64; ++it) {
        uint4 w[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            w[j] = live[j] ? *reinterpret_cast<const uint4*>(occ + ((p[j] - 1) & ~3u)) : make_uint4(~0u, ~0u, ~0u, ~0u);
        bool any = false;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (!live[j]) continue;
            const uint32_t q = (p[j] - 1) & ~3u, n = p[j] - q;  // words q .. p-1 (1..4)
            const uint32_t x[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
            bool stop = false, v = false;
            for (int e = (int)n - 1; e >= 0; --e) {
                if (x[e] == ~0u) { stop = true; break; }
                if (vbit(vm, x[e])) { v = true; stop = true; break; }
            }
            lost |= v;
            live[j] = !stop && !v;
            p[j] = q;
            any |= live[j];
        }
        if (lost || !any) break;
    }
    lose[i] = lost;
}


__global__ __launch_bounds__(256) void k_scan16(const uint32_t* __restrict__ occ, const uint32_t* __restrict__ opos,
                                                const uint64_t* __restrict__ vm, const uint32_t* __restrict__ ent,
                                                uint32_t ne, uint8_t* __restrict__ lose) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ne) return;
    const uint32_t c = ent[i];
    uint32_t p[K];
#pragma unroll
    for (int j = 0; j < K; ++j) p[j] = opos[(uint64_t)c * K + j];
    bool lost = false, live[K];
#pragma unroll
    for (int j = 0; j < K; ++j) live[j] = true;
    for (int it = 0; it < 64; ++it) {
        uint32_t x[K][16];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t q = ((p[j] - 1) & ~3u) - 12;  // words q .. q + 15 (p - 1 in the top uint4)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t idx = q + 4u * u;  // (wraps below the first list: those words read as sentinels)
                const uint4 w = live[j] && idx < 0x80000000u ? *reinterpret_cast<const uint4*>(occ + idx)
                                                             : make_uint4(~0u, ~0u, ~0u, ~0u);
                x[j][4 * u] = w.x; x[j][4 * u + 1] = w.y; x[j][4 * u + 2] = w.z; x[j][4 * u + 3] = w.w;
            }
        }
        uint32_t vb[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            vb[j] = 0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t y = x[j][e];
                const uint64_t w = y != ~0u ? vm[y >> 6] : 0ull;
                vb[j] |= (uint32_t)((w >> (y & 63)) & 1ull) << e;
            }
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (!live[j]) continue;
            const uint32_t q = ((p[j] - 1) & ~3u) - 12, top = p[j] - 1 - q;  // word index of p - 1
            bool stop = false, v = false;
            for (int e = (int)top; e >= 0; --e) {
                if (x[j][e] == ~0u) { stop = true; break; }
                if ((vb[j] >> e) & 1u) { v = true; stop = true; break; }
            }
            lost |= v;
            live[j] = !stop;
            p[j] = q;
            any |= live[j];
        }
        if (lost || !any) break;
    }
    lose[i] = lost;
}

int main() {
    const uint32_t n = 2500000;
    const uint64_t m = 10000000;
    std::vector<uint32_t> lits(m * K);
    uint64_t s = 88172645463325252ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (uint64_t c = 0; c < m; ++c)
        for (int j = 0; j < K; ++j) lits[c * K + j] = (uint32_t)(rnd() % n);
    std::vector<uint32_t> deg(n, 0);
    for (uint64_t c = 0; c < m; ++c)
        for (int j = 0; j < K; ++j) {
            bool dup = false;
            for (int q = 0; q < j; ++q) dup |= lits[c * K + q] == lits[c * K + j];
            if (!dup) deg[lits[c * K + j]]++;
        }
    std::vector<uint64_t> off(n + 1, 0);
    for (uint32_t v = 0; v < n; ++v) off[v + 1] = off[v] + 1 + deg[v];
    const uint64_t L = off[n];
    std::vector<uint32_t> occ(L + 32, ~0u), opos(m * K), cur(n);
    for (uint32_t v = 0; v < n; ++v) cur[v] = (uint32_t)(off[v] + 1);
    for (uint64_t c = 0; c < m; ++c)
        for (int j = 0; j < K; ++j) {
            int first = j;
            for (int q = 0; q < j; ++q) if (lits[c * K + q] == lits[c * K + j]) { first = q; break; }
            if (first == j) {
                const uint32_t v = lits[c * K + j];
                opos[c * K + j] = cur[v];
                occ[cur[v]++] = (uint32_t)c;
            } else {
                opos[c * K + j] = opos[c * K + first];
            }
        }
    // violated: ~7.5% of clauses
    std::vector<uint64_t> vm((m + 63) / 64, 0);
    std::vector<uint32_t> ent;
    for (uint64_t c = 0; c < m; ++c)
        if (rnd() % 1000 < 75) { vm[c / 64] |= 1ull << (c % 64); ent.push_back((uint32_t)c); }
    const uint32_t ne = (uint32_t)ent.size();
    // CPU check of the win count
    uint64_t cpu_lose = 0;
    for (uint32_t i = 0; i < ne; ++i) {
        const uint32_t c = ent[i];
        bool lost = false;
        for (int j = 0; j < K; ++j) {
            uint32_t p = opos[(uint64_t)c * K + j];
            for (;;) {
                const uint32_t x = occ[--p];
                if (x == ~0u) break;
                if ((vm[x / 64] >> (x % 64)) & 1) { lost = true; break; }
            }
        }
        cpu_lose += lost;
    }
    printf("L %llu occurrences (+%u sentinels), %u violated, %llu lose (cpu)\n", (unsigned long long)(L - n), n, ne,
           (unsigned long long)cpu_lose);
    uint32_t *d_occ, *d_opos, *d_ent;
    uint64_t* d_vm;
    uint8_t* d_lose;
    CK(hipMalloc(&d_occ, occ.size() * 4));
    CK(hipMalloc(&d_opos, opos.size() * 4));
    CK(hipMalloc(&d_ent, ne * 4));
    CK(hipMalloc(&d_vm, vm.size() * 8));
    CK(hipMalloc(&d_lose, ne));
    CK(hipMemcpy(d_occ, occ.data(), occ.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_opos, opos.data(), opos.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ent, ent.data(), ne * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_vm, vm.data(), vm.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint8_t> lose(ne);
    for (int variant = 0; variant < 3; ++variant) {
        const int reps = 50;
        auto launch = [&]() {
            if (variant == 0) k_scan1<<<(ne + 255) / 256, 256>>>(d_occ, d_opos, d_vm, d_ent, ne, d_lose);
            else if (variant == 1) k_scan4<<<(ne + 255) / 256, 256>>>(d_occ, d_opos, d_vm, d_ent, ne, d_lose);
            else k_scan16<<<(ne + 255) / 256, 256>>>(d_occ, d_opos, d_vm, d_ent, ne, d_lose);
        };
        for (int r = 0; r < 5; ++r) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(lose.data(), d_lose, ne, hipMemcpyDeviceToHost));
        uint64_t gl = 0;
        for (uint32_t i = 0; i < ne; ++i) gl += lose[i];
        printf("%s: %.2f us per launch, lose %llu (%s)\n", variant == 0 ? "scan1" : variant == 1 ? "scan4" : "scan16", ms * 1000.0f / reps,
               (unsigned long long)gl, gl == cpu_lose ? "match" : "MISMATCH");
    }
    return 0;
}
