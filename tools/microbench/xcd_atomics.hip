// Microbenchmark (not product code): can LFMIS claims run as L2-local atomics?
// Random u64 atomicMin into a 2.5M-entry owner array, 2.7M updates (LFMIS round 0 at 10M
// clauses), as
//   A  agent-scope atomics from every workgroup (the current claim kernel's form);
//   B  workgroup-scope atomics, variables partitioned over the 8 XCDs by 128-B owner line,
//      each workgroup pulling chunks of its own XCD's list (XCC id read from HW_REG_XCC_ID);
//   C  as B with agent-scope atomics (separates the partitioning from the scope);
//   D  as B, but every workgroup reads ALL updates and keeps its XCD's (no pre-bucketing).
// Checks that B/C/D give A's final owner values.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}
__device__ __forceinline__ uint32_t part_of(uint32_t v) { return (v >> 4) & 7u; }

__global__ void k_agent(unsigned long long* owner, const uint32_t* idx, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicMin(&owner[idx[i]], ((unsigned long long)idx[i] << 20) ^ i);
}

template <int SCOPE>
__global__ void k_part(unsigned long long* owner, const uint32_t* lists, const uint32_t* list_off,
                       uint32_t* q, uint32_t chunk) {
    __shared__ uint32_t s_c;
    const uint32_t x = xcc_id();
    const uint32_t b = list_off[x], e = list_off[x + 1];
    for (;;) {
        if (threadIdx.x == 0) s_c = atomicAdd(&q[x], 1u);
        __syncthreads();
        const uint64_t c0 = b + (uint64_t)s_c * chunk;
        __syncthreads();
        if (c0 >= e) break;
        for (uint32_t t = threadIdx.x; t < chunk && c0 + t < e; t += blockDim.x) {
            const uint32_t w = lists[c0 + t];
            const uint32_t v = w;  // stored var
            const uint32_t i = lists[(list_off[8]) + c0 + t];
            __hip_atomic_fetch_min(&owner[v], ((unsigned long long)v << 20) ^ i, __ATOMIC_RELAXED, SCOPE);
        }
    }
}

__global__ void k_filter(unsigned long long* owner, const uint32_t* idx, uint32_t n) {
    const uint32_t x = xcc_id();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t v = idx[i];
        if (part_of(v) == x)
            __hip_atomic_fetch_min(&owner[v], ((unsigned long long)v << 20) ^ i, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

int main() {
    const uint32_t nv = 2500000, n = 2700000;
    std::vector<uint32_t> h(n);
    uint64_t s = 88172645463325252ull;
    for (auto& x : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x = (uint32_t)(s % nv); }
    // bucket by partition: lists = [vars of part 0..7][original index of each]
    std::vector<uint32_t> off(10, 0);
    for (uint32_t i = 0; i < n; ++i) off[((h[i] >> 4) & 7) + 1]++;
    for (int p = 0; p < 8; ++p) off[p + 1] += off[p];
    off[8] = n;  // second half offset
    std::vector<uint32_t> lists(2 * n), cur(off.begin(), off.begin() + 8);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t p = (h[i] >> 4) & 7, k = cur[p]++;
        lists[k] = h[i];
        lists[n + k] = i;
    }
    uint32_t *idx, *dl, *doff, *q;
    unsigned long long *o_ref, *o;
    hipMalloc(&idx, n * 4); hipMalloc(&dl, 2 * n * 4); hipMalloc(&doff, 10 * 4); hipMalloc(&q, 64);
    hipMalloc(&o_ref, nv * 8); hipMalloc(&o, nv * 8);
    hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dl, lists.data(), 2 * n * 4, hipMemcpyHostToDevice);
    hipMemcpy(doff, off.data(), 10 * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    std::vector<unsigned long long> r1(nv), r2(nv);
    auto run = [&](const char* name, unsigned long long* dst, auto f) {
        const int R = 20;
        float tot = 0;
        for (int r = 0; r < R + 3; ++r) {
            hipMemset(dst, 0xFF, nv * 8);
            hipMemset(q, 0, 64);
            hipEventRecord(a);
            f();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (r >= 3) tot += ms;
        }
        printf("%-34s %8.1f us  %6.1f G atomics/s\n", name, tot * 1000 / R, n / (tot / R * 1e-3) / 1e9);
    };
    run("A agent, all workgroups", o_ref, [&] { k_agent<<<(n + 255) / 256, 256>>>(o_ref, idx, n); });
    hipMemcpy(r1.data(), o_ref, nv * 8, hipMemcpyDeviceToHost);
    auto check = [&](const char* name) {
        hipMemcpy(r2.data(), o, nv * 8, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (uint32_t v = 0; v < nv; ++v) bad += r1[v] != r2[v];
        printf("   %s: %zu mismatches\n", name, bad);
    };
    for (uint32_t chunk : {1024u, 4096u}) {
        for (int grid : {256, 1024, 2048}) {
            char nm[64];
            snprintf(nm, sizeof nm, "B wg-scope part chunk %u grid %d", chunk, grid);
            run(nm, o, [&] { k_part<__HIP_MEMORY_SCOPE_WORKGROUP><<<grid, 256>>>(o, dl, doff, q, chunk); });
            check("B");
        }
    }
    run("C agent part chunk 1024 grid 1024", o, [&] { k_part<__HIP_MEMORY_SCOPE_AGENT><<<1024, 256>>>(o, dl, doff, q, 1024); });
    check("C");
    for (int grid : {1024, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "D wg-scope filter grid %d", grid);
        run(nm, o, [&] { k_filter<<<grid, 256>>>(o, idx, n); });
        check("D");
    }
    return 0;
}
