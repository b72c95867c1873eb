// Microbenchmark (not product code): streaming-read structure for the eval kernel's literal
// stream (config M: 10M clauses x 3 literals = 120 MB, 256-clause chunks of 3 KiB).
//   flat      grid-stride 16-B loads over many workgroups (the achievable reference)
//   chunk<U>  persistent grid (one workgroup per CU, 1024 threads), contiguous chunk range per
//             workgroup, a wave takes U chunks per step (3 x 16 B per lane per chunk) -- the
//             k_eval_hybrid skeleton
//   chunk256<U>  same with 256-thread workgroups, 4 per CU
// Every variant XOR-reduces what it reads and stores one word per wave.  Times are hipEvent
// averages of back-to-back launches, warm (MALL-resident) and after a 512 MB flush (cold).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t CHUNK_U4 = 192;  // 3 KiB per chunk = 192 uint4 (3 slots x 64 lanes)

__global__ __launch_bounds__(256) void k_flat(const uint4* __restrict__ p, uint64_t n4, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int U, int WG>
__global__ __launch_bounds__(WG) void k_chunk(const uint4* __restrict__ p, uint64_t nchunks, uint32_t* out) {
    constexpr uint32_t WAVES = WG / 64;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
    uint32_t acc = 0;
    for (uint64_t g0 = c0 + wave; g0 < c1; g0 += (uint64_t)U * WAVES) {
        uint4 x[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t g = g0 + (uint64_t)u * WAVES;
            if (g < c1) {
#pragma unroll
                for (int j = 0; j < 3; ++j) x[u][j] = p[g * CHUNK_U4 + j * 64 + lane];
            } else {
#pragma unroll
                for (int j = 0; j < 3; ++j) x[u][j] = make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 3; ++j) acc ^= x[u][j].x ^ x[u][j].y ^ x[u][j].z ^ x[u][j].w;
        const uint64_t bal = __ballot(acc & 1u);
        if (lane == 0 && bal == 0x1234567ull) out[1] = (uint32_t)bal;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_flush(uint4* p, uint64_t n4) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) p[i] = make_uint4(i, 0, 0, 0);
}

template <typename F>
int timeit(const char* name, F launch, uint4* fl, uint64_t fl4, double bytes) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    // warm: 20 back-to-back
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int i = 0; i < 20; ++i) launch(); CK(hipEventRecord(b));
    CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    const double warm = ms / 20;
    // cold: flush before each of 10 single launches
    double cold = 0;
    for (int i = 0; i < 10; ++i) {
        k_flush<<<4096, 256>>>(fl, fl4);
        CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        cold += ms / 10;
    }
    printf("%-22s warm %7.1f us %6.2f TB/s   cold %7.1f us %6.2f TB/s\n", name, warm * 1e3, bytes / warm / 1e9,
           cold * 1e3, bytes / cold / 1e9);
    return 0;
}

int main() {
    const uint64_t nchunks = 10000000ull / 256 + 1;  // config M
    const uint64_t n4 = nchunks * CHUNK_U4;
    const double bytes = (double)n4 * 16;
    uint4 *p, *fl;
    uint32_t* out;
    const uint64_t fl4 = (512ull << 20) / 16;
    CK(hipMalloc(&p, n4 * 16)); CK(hipMalloc(&fl, fl4 * 16)); CK(hipMalloc(&out, 64));
    CK(hipMemset(p, 1, n4 * 16));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs %d, %.1f MB\n", ncu, bytes / 1e6);
    timeit("flat 8192x256", [&] { k_flat<<<8192, 256>>>(p, n4, out); }, fl, fl4, bytes);
    timeit("flat 2048x256", [&] { k_flat<<<2048, 256>>>(p, n4, out); }, fl, fl4, bytes);
    timeit("chunk<1> 1024", [&] { k_chunk<1, 1024><<<ncu, 1024>>>(p, nchunks, out); }, fl, fl4, bytes);
    timeit("chunk<2> 1024", [&] { k_chunk<2, 1024><<<ncu, 1024>>>(p, nchunks, out); }, fl, fl4, bytes);
    timeit("chunk<4> 1024", [&] { k_chunk<4, 1024><<<ncu, 1024>>>(p, nchunks, out); }, fl, fl4, bytes);
    timeit("chunk<1> 256 x4/CU", [&] { k_chunk<1, 256><<<ncu * 4, 256>>>(p, nchunks, out); }, fl, fl4, bytes);
    timeit("chunk<2> 256 x4/CU", [&] { k_chunk<2, 256><<<ncu * 4, 256>>>(p, nchunks, out); }, fl, fl4, bytes);
    timeit("chunk<1> 256 x8/CU", [&] { k_chunk<1, 256><<<ncu * 8, 256>>>(p, nchunks, out); }, fl, fl4, bytes);
    timeit("chunk<1> 1024 x2/CU", [&] { k_chunk<1, 1024><<<ncu * 2, 1024>>>(p, nchunks, out); }, fl, fl4, bytes);
    return 0;
}
