// alll_kernels.hip -- CDNA4 (gfx950) kernels of the Moser-Tardos resample loop.
//
// One iteration of SATInstance<T>::parallel_solve (reference SATInstance.h:260-311) is
//   k_eval_*   clause evaluation (Clause.h:34-46) over the clause shard + violated-clause
//              compaction (SATInstance.h:264-280) via wave ballots: writes the violated
//              bitmask and per-tile lists of violated clause ids.
//   k_collect  (multi-GPU) rebuilds the per-tile lists of the other shards from the
//              all-gathered bitmask.
//   k_reduce   violated count + termination test (check_if_noUNSAT, SATInstance.h:326-338)
//              and the loop state update.
//   k_claim / k_join (x R)  round-synchronous exact lexicographically-first MIS of the
//              violated clauses in clause order (populate_mis_parallel with one set,
//              SATInstance.h:391-451; dependency = shared variable, :369-389).
//   k_tail     single-workgroup rounds until every violated clause is decided.
//   k_resample Philox4x32-10 per-variable resampling of every MIS clause
//              (resample_clauses, SATInstance.h:340-365).
// Integer / bit work only: no MFMA.  HBM-bound on the literal stream of k_eval.
#include <algorithm>

#include "alll_internal.h"

namespace alll {

#define ALLL_DISPATCH_K(KV, CALL)                      \
    switch (KV) {                                      \
        case 1: { constexpr int K = 1; CALL; } break;  \
        case 2: { constexpr int K = 2; CALL; } break;  \
        case 3: { constexpr int K = 3; CALL; } break;  \
        case 4: { constexpr int K = 4; CALL; } break;  \
        case 5: { constexpr int K = 5; CALL; } break;  \
        case 6: { constexpr int K = 6; CALL; } break;  \
        case 7: { constexpr int K = 7; CALL; } break;  \
        case 8: { constexpr int K = 8; CALL; } break;  \
        default: { constexpr int K = 0; CALL; } break; \
    }

// ------------------------------------------------------------------------------------
// Philox4x32-10, identical constants to oracle/alll_oracle.c (Random123 KAT-pinned).
__device__ __forceinline__ uint32_t philox_x(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                             uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c0;
}

// The AoS literal copy used by the LFMIS / resample kernels carries a "hot variable" flag in
// bit 31 (set by the host for the highest-degree variables of skewed instances).
constexpr uint32_t LIT_MASK = 0x7FFFFFFFu;
constexpr uint32_t LIT_HOT = 0x80000000u;
__device__ __forceinline__ uint32_t lvar(const ClauseView& cv, uint64_t j) {
    return (cv.lits[j] & LIT_MASK) >> 1;
}

__device__ __forceinline__ uint32_t abit(const uint32_t* __restrict__ A, uint32_t v) {
    return (A[v >> 5] >> (v & 31u)) & 1u;
}

// bits 0..15 of x -> bit positions 0,4,...,60 (4-way Morton spread)
__device__ __forceinline__ uint64_t spread4(uint64_t x) {
    x &= 0xFFFFull;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}

__device__ __forceinline__ bool eval_gate_closed(const DevState* st) {
    return st->done != 0 || st->n_iter >= st->limit_eval;
}

// Number of literals / variables of clause c.
template <int K>
__device__ __forceinline__ void clause_range(const ClauseView& cv, uint32_t c, uint64_t& b, uint64_t& e) {
    if constexpr (K > 0) { b = (uint64_t)c * K; e = b + K; }
    else { b = cv.offs[c]; e = cv.offs[c + 1]; }
}

// ------------------------------------------------------------------------------------
// Initial assignment: word w = Philox(seed, {w, 0, 0xFFFFFFFF, 0}).x (VariablesArray.h:23-34).
__global__ void k_init_assignment(uint32_t* A, uint32_t n_words, uint32_t n_vars, uint64_t seed) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_words) return;
    uint32_t x = philox_x(w, 0u, 0xFFFFFFFFu, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
    if (w == n_words - 1 && (n_vars & 31u)) x &= (1u << (n_vars & 31u)) - 1u;
    A[w] = x;
}

// Common epilogue of eval / collect: per-wave LDS lists -> contiguous tile list.
__device__ __forceinline__ void publish_tile(const LoopBuffers& b, uint32_t tile, uint32_t* s_idx,
                                             uint32_t* s_wcnt, uint32_t wcount, int lane, int wave) {
    if (lane == 0) s_wcnt[wave] = wcount;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t cw = s_wcnt[w];
        off += (w < wave) ? cw : 0u;
        tot += cw;
    }
    uint32_t* dst = b.stage + (uint64_t)tile * TILE + off;
    const uint32_t* src = s_idx + wave * (TILE / 4);
    for (uint32_t i = lane; i < wcount; i += 64) dst[i] = src[i];
    if (threadIdx.x == 0) {
        b.tile_cnt[tile] = tot;
        b.mis_cnt[tile] = 0;
    }
}

// ------------------------------------------------------------------------------------
// Clause evaluation, fixed width K, chunk-transposed literals: lane i of a wave evaluates
// clauses 4i..4i+3 of a 256-clause chunk with one 16-byte load per literal slot
// (1 KiB per wave-instruction).  4 chunks per wave, 16 per 256-thread workgroup (= TILE).
template <int K>
__global__ __launch_bounds__(EVAL_THREADS) void k_eval_fixed(ClauseView cv, LoopBuffers b,
                                                             uint32_t tile_begin, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    __shared__ uint32_t s_idx[TILE];
    __shared__ uint32_t s_wcnt[4];
    const uint32_t tile = tile_begin + blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = cv.m;
    const uint32_t* __restrict__ A = b.A;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t wcount = 0;
#pragma unroll 2
    for (int s = 0; s < 4; ++s) {
        const uint64_t g = (uint64_t)tile * (TILE / CHUNK) + wave * 4 + s;
        const uint64_t cb = g * CHUNK;
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        if (cb < m) {
            const uint4* src = reinterpret_cast<const uint4*>(cv.lits_t + cb * K) + lane;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint4 x = src[j * 64];
                s0 |= abit(A, x.x >> 1) ^ (x.x & 1u);
                s1 |= abit(A, x.y >> 1) ^ (x.y & 1u);
                s2 |= abit(A, x.z >> 1) ^ (x.z & 1u);
                s3 |= abit(A, x.w >> 1) ^ (x.w & 1u);
            }
        }
        const uint64_t c0 = cb + 4u * lane;
        const bool v0 = !s0 && c0 < m, v1 = !s1 && c0 + 1 < m;
        const bool v2 = !s2 && c0 + 2 < m, v3 = !s3 && c0 + 3 < m;
        const uint64_t b0 = __ballot(v0), b1 = __ballot(v1), b2 = __ballot(v2), b3 = __ballot(v3);
        if (lane < 4) {
            const int sh = 16 * lane;
            const uint64_t w = spread4(b0 >> sh) | (spread4(b1 >> sh) << 1) |
                               (spread4(b2 >> sh) << 2) | (spread4(b3 >> sh) << 3);
            b.vmask[g * 4 + lane] = w;
        }
        const uint32_t pre = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) +
                             __popcll(b3 & lt);
        uint32_t* dst = s_idx + wave * (TILE / 4) + wcount + pre;
        uint32_t q = 0;
        if (v0) dst[q++] = (uint32_t)c0;
        if (v1) dst[q++] = (uint32_t)(c0 + 1);
        if (v2) dst[q++] = (uint32_t)(c0 + 2);
        if (v3) dst[q++] = (uint32_t)(c0 + 3);
        wcount += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
    }
    publish_tile(b, tile, s_idx, s_wcnt, wcount, lane, wave);
}

// Clause evaluation, fixed width K, persistent hybrid (the loop's default for fixed k).
// One 1024-thread workgroup per CU owns a contiguous run of tiles.  The assignment words of
// the first min(n, LDS_VARS) variables are staged once in LDS by LDS-DMA; a literal whose
// variable lies there is looked up in LDS, the others in L2 (the whole bit-packed assignment
// stays L2-resident).  Lanes evaluate 4 clauses of a 256-clause chunk with one 16-byte load
// per literal slot from the chunk-transposed layout (as k_eval_fixed), so the literal stream
// is read once, perfectly coalesced.  Violated clauses go to the per-tile lists through
// per-tile LDS counters.
template <int K>
__global__ __launch_bounds__(HYB_THREADS) void k_eval_hybrid(ClauseView cv, LoopBuffers b,
                                                             uint32_t tile_begin, uint32_t tile_end,
                                                             int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_A[];
    __shared__ uint32_t s_tcnt[HYB_MAX_TILES];
    const uint32_t nblk = gridDim.x;
    const uint32_t ntiles = tile_end - tile_begin;
    const uint32_t t0 = tile_begin + (uint32_t)(((uint64_t)ntiles * blockIdx.x) / nblk);
    const uint32_t t1 = tile_begin + (uint32_t)(((uint64_t)ntiles * (blockIdx.x + 1)) / nblk);
    if (t0 >= t1) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t m = cv.m;
    const uint32_t lds_words = min(b.n_words, LDS_WORDS);
    const uint32_t lds_vars = lds_words * 32u;
    {
        // LDS-DMA fill (global_load_lds_dwordx4: no VGPR round trip; A padded to 4 words)
        const uint32_t n4 = (lds_words + 3) / 4;
        const uint4* src = reinterpret_cast<const uint4*>(b.A);
        const uint32_t wbase = __builtin_amdgcn_readfirstlane(wave * 64);
        for (uint32_t q0 = 0; q0 < n4; q0 += HYB_THREADS) {
            const uint32_t q = q0 + threadIdx.x;
            if (q < n4)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src + q),
                    (__attribute__((address_space(3))) void*)(reinterpret_cast<uint4*>(s_A) + q0 + wbase),
                    16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint32_t* __restrict__ A = b.A;
    for (uint32_t pt = t0; pt < t1; pt += HYB_MAX_TILES) {
        const uint32_t pe = min(t1, pt + HYB_MAX_TILES);
        if (threadIdx.x < HYB_MAX_TILES) s_tcnt[threadIdx.x] = 0;
        __syncthreads();  // also publishes the LDS fill
        const uint64_t gbeg = (uint64_t)pt * (TILE / CHUNK), gend = (uint64_t)pe * (TILE / CHUNK);
        for (uint64_t g = gbeg + wave; g < gend; g += HYB_THREADS / 64) {
            const uint64_t cb = g * CHUNK;
            uint32_t sat[4] = {0u, 0u, 0u, 0u};
            if (cb < m) {
                const uint4* src = reinterpret_cast<const uint4*>(cv.lits_t + cb * K) + lane;
                uint4 x[K];
#pragma unroll
                for (int j = 0; j < K; ++j) x[j] = src[j * 64];
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t v = xs[q] >> 1;
                        const uint32_t w = (v < lds_vars) ? s_A[v >> 5] : A[v >> 5];
                        sat[q] |= ((w >> (v & 31u)) & 1u) ^ (xs[q] & 1u);
                    }
                }
            }
            const uint64_t c0 = cb + 4u * lane;
            const bool v0 = !sat[0] && c0 < m, v1 = !sat[1] && c0 + 1 < m;
            const bool v2 = !sat[2] && c0 + 2 < m, v3 = !sat[3] && c0 + 3 < m;
            const uint64_t b0 = __ballot(v0), b1 = __ballot(v1), b2 = __ballot(v2), b3 = __ballot(v3);
            if (lane < 4) {
                const int sh = 16 * lane;
                const uint64_t w = spread4(b0 >> sh) | (spread4(b1 >> sh) << 1) |
                                   (spread4(b2 >> sh) << 2) | (spread4(b3 >> sh) << 3);
                b.vmask[g * 4 + lane] = w;
            }
            const uint32_t tot = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
            if (tot) {
                const uint32_t tile = (uint32_t)(g / (TILE / CHUNK));
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&s_tcnt[tile - pt], tot);
                base = __shfl(base, 0, 64);
                const uint32_t pre = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) +
                                     __popcll(b3 & lt);
                uint32_t* dst = b.stage + (uint64_t)tile * TILE + base + pre;
                uint32_t q = 0;
                if (v0) dst[q++] = (uint32_t)c0;
                if (v1) dst[q++] = (uint32_t)(c0 + 1);
                if (v2) dst[q++] = (uint32_t)(c0 + 2);
                if (v3) dst[q++] = (uint32_t)(c0 + 3);
            }
        }
        __syncthreads();
        if (threadIdx.x < pe - pt) {
            b.tile_cnt[pt + threadIdx.x] = s_tcnt[threadIdx.x];
            b.mis_cnt[pt + threadIdx.x] = 0;
        }
    }
}

// Clause evaluation, generic CSR (ragged widths): lane per clause, 64 consecutive
// clauses per wave step, 16 steps per wave.
__global__ __launch_bounds__(EVAL_THREADS) void k_eval_csr(ClauseView cv, LoopBuffers b,
                                                           uint32_t tile_begin, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    __shared__ uint32_t s_idx[TILE];
    __shared__ uint32_t s_wcnt[4];
    const uint32_t tile = tile_begin + blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = cv.m;
    const uint32_t* __restrict__ A = b.A;
    const uint32_t* __restrict__ offs = cv.offs;
    const uint32_t* __restrict__ lits = cv.lits;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t wcount = 0;
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
        const uint64_t c = (uint64_t)tile * TILE + wave * (TILE / 4) + s * 64 + lane;
        bool viol = false;
        if (c < m) {
            const uint32_t o0 = offs[c], o1 = offs[c + 1];
            uint32_t sat = 0;
            for (uint32_t j = o0; j < o1; ++j) {
                const uint32_t l = lits[j] & LIT_MASK;
                sat |= abit(A, l >> 1) ^ (l & 1u);
            }
            viol = !sat;
        }
        const uint64_t mask = __ballot(viol);
        if (lane == 0) b.vmask[c >> 6] = mask;
        if (viol) s_idx[wave * (TILE / 4) + wcount + __popcll(mask & lt)] = (uint32_t)c;
        wcount += __popcll(mask);
    }
    publish_tile(b, tile, s_idx, s_wcnt, wcount, lane, wave);
}

// Multi-GPU: tiles owned by other ranks get their violated lists from the all-gathered
// bitmask (same order and format as k_eval_*).
__global__ __launch_bounds__(EVAL_THREADS) void k_collect(ClauseView cv, LoopBuffers b,
                                                          uint32_t own_begin, uint32_t own_end) {
    if (eval_gate_closed(b.state)) return;
    const uint32_t tile = blockIdx.x;
    if (tile >= own_begin && tile < own_end) return;
    __shared__ uint32_t s_idx[TILE];
    __shared__ uint32_t s_wcnt[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t m = cv.m;
    uint32_t wcount = 0;
    for (int s = 0; s < 16; ++s) {
        const uint64_t c = (uint64_t)tile * TILE + wave * (TILE / 4) + s * 64 + lane;
        const uint64_t mask = b.vmask[c >> 6];  // uniform load
        const bool viol = ((mask >> lane) & 1ull) && c < m;
        if (viol) s_idx[wave * (TILE / 4) + wcount + __popcll(mask & lt)] = (uint32_t)c;
        wcount += __popcll(mask);
    }
    publish_tile(b, tile, s_idx, s_wcnt, wcount, lane, wave);
}

// ------------------------------------------------------------------------------------
// Single workgroup: violated count + loop state (mode 0) or standalone count (mode 1).
__global__ __launch_bounds__(1024) void k_reduce(LoopBuffers b, int mode) {
    DevState* st = b.state;
    if (mode == 0 && eval_gate_closed(st)) {
        if (threadIdx.x == 0) st->active = 0;
        return;
    }
    __shared__ unsigned long long s_sum;
    if (threadIdx.x == 0) s_sum = 0;
    __syncthreads();
    unsigned long long acc = 0;
    for (uint32_t t = threadIdx.x; t < b.n_tiles; t += blockDim.x) acc += b.tile_cnt[t];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_sum, acc);
    __syncthreads();
    if (threadIdx.x != 0) return;
    const unsigned long long u = s_sum;
    if (mode == 1) { st->count_out = u; return; }
    st->n_iter += 1;
    st->u_total = u;
    st->left_cnt = 0;
    st->tmis_cnt = 0;
    st->stamp = (uint32_t)st->n_iter ? (uint32_t)st->n_iter : 1u;
    st->round_base = st->round_next;
    if (u == 0) { st->done = 1; st->active = 0; }
    else if (st->n_iter >= st->limit_nores) { st->done = 2; st->active = 0; }
    else st->active = 1;
}

// ------------------------------------------------------------------------------------
// LFMIS round r, phase CLAIM: every undecided violated clause first drops out if a
// variable is covered by a clause that joined the MIS in an earlier round of this
// iteration (it depends on an MIS clause), otherwise it claims each of its variables with
// atomicMin(owner[v], key), key = (~epoch << 32) | clause: keys of later rounds/iterations
// are always smaller than stale ones, so owner[] is never reset.
template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_claim(ClauseView cv, LoopBuffers b, uint32_t r) {
    const DevState* st = b.state;
    if (!st->active) return;
    const uint32_t tile = blockIdx.x;
    const uint32_t cnt = b.tile_cnt[tile];
    if (cnt == 0) return;
    const uint32_t stamp = st->stamp;
    const unsigned long long keyhi = (unsigned long long)(~(st->round_base + r)) << 32;
    __shared__ uint32_t s_e[TILE];
    __shared__ uint32_t s_wp;
    // claims on hot variables are first reduced in an LDS hash table (one global atomic per
    // hot variable per block instead of one per clause: power-law hubs)
    __shared__ uint32_t s_hk[HOT_SLOTS];
    __shared__ unsigned long long s_hv[HOT_SLOTS];
    const bool hot = cv.n_hot != 0;
    uint32_t* list = b.stage + (uint64_t)tile * TILE;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) s_e[i] = list[i];
    if (hot)
        for (uint32_t i = threadIdx.x; i < HOT_SLOTS; i += blockDim.x) { s_hk[i] = 0xFFFFFFFFu; s_hv[i] = ~0ull; }
    if (threadIdx.x == 0) s_wp = 0;
    __syncthreads();
    const bool translate = (r == 0) && cv.perm != nullptr;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
        const uint32_t c = translate ? cv.perm[s_e[i]] : s_e[i];
        uint64_t lb, le;
        clause_range<K>(cv, c, lb, le);
        bool killed = false;
        if (r > 0)
            for (uint64_t j = lb; j < le; ++j) killed |= (b.cover[lvar(cv, j)] == stamp);
        if (!killed) {
            const unsigned long long key = keyhi | c;
            for (uint64_t j = lb; j < le; ++j) {
                const uint32_t raw = cv.lits[j];
                const uint32_t v = (raw & LIT_MASK) >> 1;
                if (raw & LIT_HOT) {
                    uint32_t h = (v * 2654435761u) & (HOT_SLOTS - 1);
                    for (;;) {
                        const uint32_t prev = atomicCAS(&s_hk[h], 0xFFFFFFFFu, v);
                        if (prev == 0xFFFFFFFFu || prev == v) break;
                        h = (h + 1) & (HOT_SLOTS - 1);
                    }
                    atomicMin(&s_hv[h], key);
                } else {
                    atomicMin(&b.owner[v], key);
                }
            }
            list[atomicAdd(&s_wp, 1u)] = c;
        }
    }
    __syncthreads();
    if (hot)
        for (uint32_t i = threadIdx.x; i < HOT_SLOTS; i += blockDim.x)
            if (s_hk[i] != 0xFFFFFFFFu) atomicMin(&b.owner[s_hk[i]], s_hv[i]);
    if (threadIdx.x == 0) b.tile_cnt[tile] = s_wp;
}

// Phase JOIN: a clause that owns all of its variables has no undecided lower-index
// neighbour, and every decided lower neighbour is out, so it is in the LFMIS: mark its
// variables covered and append it to the tile's MIS list.  In the last grid round the
// still-undecided clauses move to one compact list for the tail kernel.
template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_join(ClauseView cv, LoopBuffers b, uint32_t r, int last) {
    DevState* st = b.state;
    if (!st->active) return;
    const uint32_t tile = blockIdx.x;
    const uint32_t cnt = b.tile_cnt[tile];
    if (cnt == 0) return;
    const uint32_t stamp = st->stamp;
    const unsigned long long keyhi = (unsigned long long)(~(st->round_base + r)) << 32;
    __shared__ uint32_t s_e[TILE];
    __shared__ uint32_t s_keep[TILE];
    __shared__ uint32_t s_wp, s_mp, s_base;
    uint32_t* list = b.stage + (uint64_t)tile * TILE;
    uint32_t* mis = b.mis + (uint64_t)tile * TILE + b.mis_cnt[tile];
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) s_e[i] = list[i];
    if (threadIdx.x == 0) { s_wp = 0; s_mp = 0; }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
        const uint32_t c = s_e[i];
        uint64_t lb, le;
        clause_range<K>(cv, c, lb, le);
        const unsigned long long key = keyhi | c;
        bool own = true;
        for (uint64_t j = lb; j < le; ++j) own &= (b.owner[lvar(cv, j)] == key);
        if (own) {
            for (uint64_t j = lb; j < le; ++j) b.cover[lvar(cv, j)] = stamp;
            mis[atomicAdd(&s_mp, 1u)] = c;
        } else {
            s_keep[atomicAdd(&s_wp, 1u)] = c;
        }
    }
    __syncthreads();
    const uint32_t kept = s_wp;
    uint32_t* dst = list;
    if (last && kept) {
        if (threadIdx.x == 0) s_base = atomicAdd(&st->left_cnt, kept);
        __syncthreads();
        dst = b.left + s_base;
    }
    for (uint32_t i = threadIdx.x; i < kept; i += blockDim.x) dst[i] = s_keep[i];
    if (threadIdx.x == 0) {
        b.tile_cnt[tile] = last ? 0u : kept;
        b.mis_cnt[tile] += s_mp;
    }
}

// Tail: one workgroup finishes the LFMIS over the compact list handed over by the last grid
// round (rounds until no undecided clause is left).  Entries are processed in chunks of one
// per thread; survivors are compacted in place (a write position never passes the chunk being
// read).  owner / cover are accessed with agent-scope relaxed atomics so no stale L1 line is
// read across the barriers.
template <int K>
__global__ __launch_bounds__(TAIL_THREADS) void k_tail(ClauseView cv, LoopBuffers b, uint32_t first_round) {
    DevState* st = b.state;
    if (!st->active) return;
    const uint32_t stamp = st->stamp;
    __shared__ uint32_t s_wp, s_tm;
    uint32_t n = st->left_cnt;
    uint32_t epoch = st->round_base + first_round;
    uint32_t rounds = 0;
    if (threadIdx.x == 0) s_tm = 0;
    uint32_t* left = b.left;
    while (n > 0) {
        const unsigned long long keyhi = (unsigned long long)(~epoch) << 32;
        // CLAIM (with the kill test)
        if (threadIdx.x == 0) s_wp = 0;
        __syncthreads();
        for (uint32_t base = 0; base < n; base += blockDim.x) {
            const uint32_t i = base + threadIdx.x;
            const uint32_t c = (i < n) ? left[i] : 0u;
            __syncthreads();
            if (i < n) {
                uint64_t lb, le;
                clause_range<K>(cv, c, lb, le);
                bool killed = false;
                for (uint64_t j = lb; j < le; ++j)
                    killed |= (__hip_atomic_load(&b.cover[lvar(cv, j)], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) == stamp);
                if (!killed) {
                    const unsigned long long key = keyhi | c;
                    for (uint64_t j = lb; j < le; ++j) atomicMin(&b.owner[lvar(cv, j)], key);
                    left[atomicAdd(&s_wp, 1u)] = c;
                }
            }
        }
        __syncthreads();
        n = s_wp;
        __syncthreads();
        // JOIN
        if (threadIdx.x == 0) s_wp = 0;
        __syncthreads();
        for (uint32_t base = 0; base < n; base += blockDim.x) {
            const uint32_t i = base + threadIdx.x;
            const uint32_t c = (i < n) ? left[i] : 0u;
            __syncthreads();
            if (i < n) {
                uint64_t lb, le;
                clause_range<K>(cv, c, lb, le);
                const unsigned long long key = keyhi | c;
                bool own = true;
                for (uint64_t j = lb; j < le; ++j)
                    own &= (__hip_atomic_load(&b.owner[lvar(cv, j)], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) == key);
                if (own) {
                    for (uint64_t j = lb; j < le; ++j)
                        __hip_atomic_store(&b.cover[lvar(cv, j)], stamp, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    b.tmis[atomicAdd(&s_tm, 1u)] = c;
                } else {
                    left[atomicAdd(&s_wp, 1u)] = c;
                }
            }
        }
        __syncthreads();
        n = s_wp;
        ++rounds;
        ++epoch;
        if (rounds >= MAX_TAIL_ROUNDS && n > 0) {
            if (threadIdx.x == 0) { st->error = 1; st->done = 3; }
            break;
        }
        __syncthreads();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        st->round_next = epoch;
        st->tail_rounds = rounds;
        st->tmis_cnt = s_tm;
        const uint32_t total = first_round + rounds;
        if (total > st->max_rounds) st->max_rounds = total;
    }
}

// ------------------------------------------------------------------------------------
// Resample: every variable of every MIS clause gets Philox(seed, {v, it_lo, 0, it_hi}).x & 1
// with it = resample round (n_iter - 1).  A violated clause has every literal false, so the
// old value of v is l & 1 and only differing bits are flipped (atomicXor; MIS clauses are
// variable-disjoint).  A variable repeated inside one clause is applied once (its draws
// are equal anyway); n_resamples still counts every literal (SATInstance.h:363).
template <int K>
__device__ __forceinline__ uint64_t resample_clause(const ClauseView& cv, uint32_t* target, uint32_t c,
                                                    uint64_t it, uint32_t k0, uint32_t k1, bool apply) {
    uint64_t lb, le;
    clause_range<K>(cv, c, lb, le);
    if (apply) {
        for (uint64_t j = lb; j < le; ++j) {
            const uint32_t l = cv.lits[j] & LIT_MASK, v = l >> 1;
            bool dup = false;
            for (uint64_t q = lb; q < j; ++q) dup |= (lvar(cv, q) == v);
            if (dup) continue;
            const uint32_t nb = philox_x(v, (uint32_t)it, 0u, (uint32_t)(it >> 32), k0, k1) & 1u;
            if (nb != (l & 1u)) atomicXor(&target[v >> 5], 1u << (v & 31u));
        }
    }
    return le - lb;
}

template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_resample(ClauseView cv, LoopBuffers b,
                                                            uint32_t own_begin, uint32_t own_end,
                                                            int to_delta) {
    const DevState* st = b.state;
    if (!st->active) return;
    const uint32_t tile = blockIdx.x;
    const uint64_t it = st->n_iter - 1;
    const uint32_t k0 = (uint32_t)b.seed, k1 = (uint32_t)(b.seed >> 32);
    uint32_t* target = to_delta ? b.delta : b.A;
    if (tile == b.n_tiles) {
        // MIS clauses decided by the tail kernel (few): per-clause statistics to their tile
        const uint32_t cnt = st->tmis_cnt;
        for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
            const uint32_t c = b.tmis[i];
            const uint32_t t = c / TILE;
            const bool apply = !to_delta || (t >= own_begin && t < own_end);
            const uint64_t len = resample_clause<K>(cv, target, c, it, k0, k1, apply);
            atomicAdd(&b.tile_stats[2 * t], 1ull);
            atomicAdd(&b.tile_stats[2 * t + 1], (unsigned long long)len);
        }
        return;
    }
    const uint32_t cnt = b.mis_cnt[tile];
    if (cnt == 0) return;
    const bool apply = !to_delta || (tile >= own_begin && tile < own_end);
    __shared__ unsigned long long s_res;
    if (threadIdx.x == 0) s_res = 0;
    __syncthreads();
    const uint32_t* mis = b.mis + (uint64_t)tile * TILE;
    unsigned long long res = 0;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x)
        res += resample_clause<K>(cv, target, mis[i], it, k0, k1, apply);
    for (int o = 32; o > 0; o >>= 1) res += __shfl_down(res, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_res, res);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&b.tile_stats[2 * tile], (unsigned long long)cnt);
        atomicAdd(&b.tile_stats[2 * tile + 1], s_res);
    }
}

__global__ void k_apply_delta(LoopBuffers b) {
    if (!b.state->active) return;
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= b.n_words) return;
    const uint32_t d = b.delta[w];
    if (d) { b.A[w] ^= d; b.delta[w] = 0; }
}

// ------------------------------------------------------------------------------------
// Launchers.
hipError_t launch_init_assignment(const LoopBuffers& b, hipStream_t s) {
    if (b.n_words == 0) return hipSuccess;
    k_init_assignment<<<(b.n_words + 255) / 256, 256, 0, s>>>(b.A, b.n_words, b.n_vars, b.seed);
    return hipGetLastError();
}

hipError_t launch_eval(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                       uint32_t tile_end, bool gated, hipStream_t s) {
    if (tile_end <= tile_begin) return hipSuccess;
    const dim3 grid(tile_end - tile_begin);
    const int g = gated ? 1 : 0;
    switch (cv.k) {
        case 1: k_eval_fixed<1><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 2: k_eval_fixed<2><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 3: k_eval_fixed<3><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 4: k_eval_fixed<4><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 5: k_eval_fixed<5><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 6: k_eval_fixed<6><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 7: k_eval_fixed<7><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        case 8: k_eval_fixed<8><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
        default: k_eval_csr<<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g); break;
    }
    return hipGetLastError();
}

hipError_t launch_eval_hybrid(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                              uint32_t tile_end, bool gated, int n_blocks, hipStream_t s) {
    if (tile_end <= tile_begin) return hipSuccess;
    const uint32_t nt = tile_end - tile_begin;
    const dim3 grid(std::min<uint32_t>(nt, (uint32_t)std::max(1, n_blocks)));
    const size_t lds = (size_t)std::max<uint32_t>(4, (std::min(b.n_words, LDS_WORDS) + 3) / 4 * 4) * 4;
    const int g = gated ? 1 : 0;
    static bool attr_set[MAX_FIXED_K + 1] = {};
    if (cv.k >= 1 && cv.k <= (uint32_t)MAX_FIXED_K && !attr_set[cv.k]) {
        hipError_t e = hipSuccess;
        ALLL_DISPATCH_K(cv.k, (e = hipFuncSetAttribute((const void*)k_eval_hybrid<(K > 0 ? K : 1)>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)(LDS_WORDS * 4))));
        if (e != hipSuccess) return e;
        attr_set[cv.k] = true;
    }
    switch (cv.k) {
        case 1: k_eval_hybrid<1><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 2: k_eval_hybrid<2><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 3: k_eval_hybrid<3><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 4: k_eval_hybrid<4><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 5: k_eval_hybrid<5><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 6: k_eval_hybrid<6><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 7: k_eval_hybrid<7><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        case 8: k_eval_hybrid<8><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_collect(const ClauseView& cv, const LoopBuffers& b, uint32_t own_begin,
                          uint32_t own_end, hipStream_t s) {
    if (b.n_tiles == 0) return hipSuccess;
    k_collect<<<b.n_tiles, EVAL_THREADS, 0, s>>>(cv, b, own_begin, own_end);
    return hipGetLastError();
}

hipError_t launch_reduce(const LoopBuffers& b, int mode, hipStream_t s) {
    k_reduce<<<1, 1024, 0, s>>>(b, mode);
    return hipGetLastError();
}


hipError_t launch_round(const ClauseView& cv, const LoopBuffers& b, uint32_t r, bool last,
                        hipStream_t s) {
    if (b.n_tiles == 0) return hipSuccess;
    ALLL_DISPATCH_K(cv.k, (k_claim<K><<<b.n_tiles, ROUND_THREADS, 0, s>>>(cv, b, r)));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int l = last ? 1 : 0;
    ALLL_DISPATCH_K(cv.k, (k_join<K><<<b.n_tiles, ROUND_THREADS, 0, s>>>(cv, b, r, l)));
    return hipGetLastError();
}

hipError_t launch_tail(const ClauseView& cv, const LoopBuffers& b, uint32_t first_round, hipStream_t s) {
    ALLL_DISPATCH_K(cv.k, (k_tail<K><<<1, TAIL_THREADS, 0, s>>>(cv, b, first_round)));
    return hipGetLastError();
}

hipError_t launch_resample(const ClauseView& cv, const LoopBuffers& b, uint32_t own_begin,
                           uint32_t own_end, bool to_delta, hipStream_t s) {
    if (b.n_tiles == 0) return hipSuccess;
    const int td = to_delta ? 1 : 0;
    ALLL_DISPATCH_K(cv.k, (k_resample<K><<<b.n_tiles + 1, ROUND_THREADS, 0, s>>>(cv, b, own_begin, own_end, td)));
    return hipGetLastError();
}

hipError_t launch_apply_delta(const LoopBuffers& b, hipStream_t s) {
    if (b.n_words == 0) return hipSuccess;
    k_apply_delta<<<(b.n_words + 255) / 256, 256, 0, s>>>(b);
    return hipGetLastError();
}

}  // namespace alll
