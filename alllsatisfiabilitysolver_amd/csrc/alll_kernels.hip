// alll_kernels.hip -- CDNA4 (gfx950) kernels of the Moser-Tardos resample loop.
//
// One iteration of SATInstance<T>::parallel_solve (reference SATInstance.h:260-311) is
//   k_eval_*   clause evaluation (Clause.h:34-46) over the clause shard + violated-clause
//              compaction (SATInstance.h:264-280) via wave ballots: writes the violated
//              bitmask and per-tile lists of violated-clause entries {id, literals}.
//   k_collect  (multi-GPU) rebuilds the per-tile lists of the other shards from the
//              all-gathered bitmask.
//   k_reduce   violated count + termination test (check_if_noUNSAT, SATInstance.h:326-338)
//              and the loop state update.
//   round 0 (k_bscatter / k_bresolve / k_bjoin, or k_claim / k_join), rounds 1 .. G-1
//              (k_wclaim / k_wjoin), k_tail   round-synchronous exact lexicographically-first MIS of
//              the violated clauses in clause order (populate_mis_parallel with one set,
//              SATInstance.h:391-451; dependency = shared variable, :369-389).
//   k_resample_vars  Philox4x32-10 resampling of every variable of every MIS clause
//              (resample_clauses, SATInstance.h:340-365), one pass over the variables.
// Integer / bit work only: no MFMA.  HBM-bound on the literal stream of k_eval.
#include <algorithm>
#include <atomic>
#include <type_traits>

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

// Compiler fence after loads issued ahead of the branches that decide whether they are needed:
// the compiler may not sink a load past it, so the loads are in flight together (no wait).
__device__ __forceinline__ void spec_fence() { asm volatile("" ::: "memory"); }

// Wave-wide (64 lanes, all active) reductions and scans by DPP moves: a few cycles per step
// where a shuffle (ds_bpermute) costs an LDS round trip.  dpp<CTRL, ROWS>(v, old): v moved by the
// DPP control CTRL in the rows ROWS, old where a lane has no source (or its row is masked off).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xF, false);
}
// the minimum over the wave, in every lane
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, dpp<0xB1>(v, v));        // quad_perm [1,0,3,2]
    v = min(v, dpp<0x4E>(v, v));        // quad_perm [2,3,0,1]
    v = min(v, dpp<0x124>(v, v));       // row_ror:4
    v = min(v, dpp<0x128>(v, v));       // row_ror:8: every lane holds its row's minimum
    v = min(v, dpp<0x142, 0xA>(v, v));  // row_bcast:15 into rows 1, 3
    v = min(v, dpp<0x143, 0xC>(v, v));  // row_bcast:31 into rows 2, 3: lane 63 holds the minimum
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// inclusive prefix sum over the wave's lanes
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {
    v += dpp<0x111>(v, 0u);        // row_shr:1
    v += dpp<0x112>(v, 0u);        // row_shr:2
    v += dpp<0x114>(v, 0u);        // row_shr:4
    v += dpp<0x118>(v, 0u);        // row_shr:8: prefix within the row
    v += dpp<0x142, 0xA>(v, 0u);   // row_bcast:15: row 0's total into row 1, row 2's into row 3
    v += dpp<0x143, 0xC>(v, 0u);   // row_bcast:31: rows 0 + 1 into rows 2, 3
    return v;
}

__device__ __forceinline__ bool eval_gate_closed(const DevState* st) {
    return st->done != 0 || st->n_iter >= st->limit_eval;
}

// Streaming solve priorities (b.stream_batch > 0).  The reference's clause generator yields
// clause s_j = j*P mod m at step j (ClauseGenerator.h:47), so clause c comes at the steps
// j = pos(c) (mod m), pos(c) = c * P^-1 mod m in [1, m].  The iteration's window is steps
// (win_start, win_start + win_len]; the LFMIS key of c is its offset in the window + 1, or ~0
// when the window does not yield it.  Without streaming the key is the clause id.
__device__ __forceinline__ uint32_t prio(const LoopBuffers& b, const DevState* st, uint32_t c) {
    if (!b.stream_batch) return c;
    const uint64_t m = b.m;
    uint64_t pos = ((uint64_t)c * b.stream_pinv) % m;  // both factors < 2^32
    if (pos == 0) pos = m;
    const uint64_t off = (pos - 1 + m - st->win_start % m) % m;
    return off < st->win_len ? (uint32_t)(off + 1) : ~0u;
}
// Contribution of an MIS clause to the MIS-size statistic: 1, or in the streaming solve the
// number of batches after which it is counted (its batch and every later one, SATInstance.h:113)
__device__ __forceinline__ unsigned long long mis_weight(const LoopBuffers& b, const DevState* st, uint32_t key) {
    if (!b.stream_batch) return 1ull;
    const uint64_t nb = (st->win_len + b.stream_batch - 1) / b.stream_batch;
    return nb - (uint64_t)(key - 1) / b.stream_batch;
}

// In-loop timing stamps (ALLL_FLAG_KERNEL_TIMING): slot of iteration n_iter (see TIME_SLOTS).
__device__ __forceinline__ unsigned long long* time_slot(const LoopBuffers& b, uint64_t it) {
    return b.ktime + (it % TIME_SLOTS) * TIME_FIELDS;
}
__device__ __forceinline__ unsigned long long wall_now() {
    return (unsigned long long)__builtin_amdgcn_s_memrealtime();
}
// one stamp per workgroup (thread 0); only loop evaluations (gated) are timed
__device__ __forceinline__ void stamp_eval_begin(const LoopBuffers& b, int gated) {
    if (gated && b.ktime && threadIdx.x == 0) atomicMin(time_slot(b, b.state->n_iter), wall_now());
}
__device__ __forceinline__ void stamp_eval_end(const LoopBuffers& b, int gated) {
    if (gated && b.ktime && threadIdx.x == 0) atomicMax(time_slot(b, b.state->n_iter) + 1, wall_now());
}

// ------------------------------------------------------------------------------------
// Violated-clause entries.  Fixed width K: {clause id, K literals} (K+1 words, so a round
// kernel never re-reads the clause store); generic CSR (K = 0): {clause id}, literals from
// the CSR arrays.  Literals keep the hot-variable flag (bit 31).
template <int K>
struct Ent {
    static constexpr int S = K > 0 ? K + 1 : 1;
    uint32_t w[S];
};

template <int K>
__device__ __forceinline__ void load_ent(Ent<K>& e, const uint32_t* p) {
    if constexpr (K == 3) {
        const uint4 x = *reinterpret_cast<const uint4*>(p);
        e.w[0] = x.x; e.w[1] = x.y; e.w[2] = x.z; e.w[3] = x.w;
    } else {
#pragma unroll
        for (int i = 0; i < Ent<K>::S; ++i) e.w[i] = p[i];
    }
}

template <int K>
__device__ __forceinline__ void store_ent(uint32_t* p, const Ent<K>& e) {
    if constexpr (K == 3) {
        *reinterpret_cast<uint4*>(p) = make_uint4(e.w[0], e.w[1], e.w[2], e.w[3]);
    } else {
#pragma unroll
        for (int i = 0; i < Ent<K>::S; ++i) p[i] = e.w[i];
    }
}

// Literal range of the entry's clause: fixed K -> the entry itself; CSR -> offsets.
template <int K>
__device__ __forceinline__ uint32_t ent_len(const ClauseView& cv, const Ent<K>& e, uint64_t& lb) {
    if constexpr (K > 0) { lb = 0; return K; }
    else { lb = cv.offs[e.w[0]]; return cv.offs[e.w[0] + 1] - (uint32_t)lb; }
}

template <int K>
__device__ __forceinline__ uint32_t ent_lit(const ClauseView& cv, const Ent<K>& e, uint64_t lb, uint32_t j) {
    if constexpr (K > 0) return e.w[1 + j];
    else return cv.lits[lb + j];
}

__device__ __forceinline__ uint32_t lit_var(uint32_t raw) { return (raw & LIT_MASK) >> 1; }

// ------------------------------------------------------------------------------------
// Initial assignment: word w = Philox(seed, {w, 0, 0xFFFFFFFF, 0}).x (VariablesArray.h:23-34).
__global__ void k_init_assignment(uint32_t* A, uint32_t n_words, uint32_t n_vars, uint64_t seed) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_words) return;
    uint32_t x = philox_x(w, 0u, 0xFFFFFFFFu, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
    if (w == n_words - 1 && (n_vars & 31u)) x &= (1u << (n_vars & 31u)) - 1u;
    A[w] = x;
}

// Raw entry of the clause at evaluation position p with lits_t slots t[0..K-1], as the
// evaluation writes it (no per-clause unpacking in the streaming kernel): {p, slots with their
// packed id bits}.  The first LFMIS round-0 kernel (k_bscatter / CLAIM(0)) turns it into the
// entry every later kernel reads (ent_unpack): {clause id, literals without id bits}.
template <int K>
__device__ __forceinline__ void make_ent(Ent<K>& e, uint64_t p, const uint32_t* t) {
    e.w[0] = (uint32_t)p;
#pragma unroll
    for (int j = 0; j < K; ++j) e.w[1 + j] = t[j];
}

// Raw entry -> {clause id, literals}: the id from the slots' packed bits, or perm[position]
// when ids are not packed (cv.perm; a 4-byte gather).
template <int K>
__device__ __forceinline__ void ent_unpack(const ClauseView& cv, Ent<K>& e) {
    if (cv.id_bits) {
        const uint32_t fm = ((1u << cv.id_bits) - 1u) << cv.id_shift;
        uint32_t id = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            id |= ((e.w[1 + j] & fm) >> cv.id_shift) << (j * cv.id_bits);
            e.w[1 + j] &= ~fm;
        }
        e.w[0] = id;
    } else if (cv.perm) {
        e.w[0] = cv.perm[e.w[0]];
    }
}

// Writes the violated clauses of lane `lane` (four consecutive evaluation positions c0..c0+3,
// literals x[j] component q) as entries into tile `tile`'s list at base + rank.
template <int K>
__device__ __forceinline__ void emit4(const ClauseView& cv, uint32_t* list, uint32_t pos, uint64_t c0,
                                      const bool v[4], const uint4 (&x)[K]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!v[q]) continue;
        uint32_t t[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
            t[j] = xs[q];
        }
        Ent<K> e;
        make_ent<K>(e, c0 + q, t);
        store_ent<K>(list + (uint64_t)pos * Ent<K>::S, e);
        ++pos;
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Buffer resource over one tile's entry list (TILE entries; the range check drops the stores
// that emit4_bf sends out of range).
template <int K>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t list_rsrc(uint32_t* list_tile) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)list_tile);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)list_tile >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)hi << 32) | lo), (short)0, (int)(TILE * 4u * Ent<K>::S), 0x00020000);
}

// emit4 without branches: every lane stores its four entries, those of satisfied clauses to an
// out-of-range offset (no memory access), so the count of store instructions is fixed.
template <int K>
__device__ __forceinline__ void emit4_bf(__amdgpu_buffer_rsrc_t rs, uint32_t pos, uint64_t c0, const bool v[4],
                                         const uint4 (&x)[K]) {
    constexpr uint32_t S = Ent<K>::S;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t off = v[q] ? pos * (S * 4u) : 0x80000000u;
        pos += v[q] ? 1u : 0u;
        uint32_t w[S];
        w[0] = (uint32_t)(c0 + q);
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
            w[1 + j] = xs[q];
        }
        if constexpr (S == 4) {
            const u32x4 d = {w[0], w[1], w[2], w[3]};
            __builtin_amdgcn_raw_buffer_store_b128(d, rs, off, 0, 0);
        } else {
#pragma unroll
            for (uint32_t i = 0; i < S; ++i) __builtin_amdgcn_raw_buffer_store_b32(w[i], rs, off + 4u * i, 0, 0);
        }
    }
}

constexpr int BSC_THREADS = 1024;
constexpr uint32_t BKT_STAGE = 12288;  // pairs staged in LDS by k_bscatter (96 KiB)
// LDS of the bucket scatter of one run (the standalone kernel's arrays, or carved from the
// evaluation kernel's window once its tiles are done).
struct ScatterLds {
    uint32_t* hist;               // BKT_MAX bucket counters / cursors
    uint32_t* hk;                 // HOT_SLOTS hot-table keys
    unsigned long long* hv;       // HOT_SLOTS hot-table minima
    uint32_t* tc;                 // RUN_TILES_MAX tile counts
    uint32_t* pre;                // RUN_TILES_MAX + 1 prefix
    uint32_t* wsum;               // BSC_THREADS / 64
    unsigned long long* pairs;    // BKT_STAGE staged pairs
};
constexpr size_t SCATTER_LDS_BYTES = 8 * BKT_STAGE + 8 * HOT_SLOTS + 4 * BKT_MAX + 4 * HOT_SLOTS + 4 * RUN_TILES_MAX +
                                     4 * (RUN_TILES_MAX + 4) + 4 * (BSC_THREADS / 64);

__device__ __forceinline__ ScatterLds carve_scatter_lds(void* base) {
    char* p = static_cast<char*>(base);
    ScatterLds L;
    L.pairs = reinterpret_cast<unsigned long long*>(p); p += 8 * BKT_STAGE;
    L.hv = reinterpret_cast<unsigned long long*>(p); p += 8 * HOT_SLOTS;
    L.hist = reinterpret_cast<uint32_t*>(p); p += 4 * BKT_MAX;
    L.hk = reinterpret_cast<uint32_t*>(p); p += 4 * HOT_SLOTS;
    L.tc = reinterpret_cast<uint32_t*>(p); p += 4 * RUN_TILES_MAX;
    L.pre = reinterpret_cast<uint32_t*>(p); p += 4 * (RUN_TILES_MAX + 4);
    L.wsum = reinterpret_cast<uint32_t*>(p);
    return L;
}

template <int K>
__device__ void scatter_run(const ClauseView& cv, const LoopBuffers& b, uint32_t* list, uint32_t r, uint32_t epoch,
                            const ScatterLds& L);

// ------------------------------------------------------------------------------------
// Clause evaluation, fixed width K, chunk-transposed literals, one tile per 256-thread
// workgroup: lane i of a wave evaluates clauses 4i..4i+3 of a 256-clause chunk with one
// 16-byte load per literal slot (1 KiB per wave-instruction); every lookup of the
// assignment is an L2 gather.  (Alternative to k_eval_hybrid, ALLL_FLAG_NO_RANGED.)
template <int K>
__global__ __launch_bounds__(EVAL_THREADS) void k_eval_fixed(ClauseView cv, LoopBuffers b,
                                                             uint32_t tile_begin, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    stamp_eval_begin(b, gated);
    __shared__ uint32_t s_cnt;
    const uint32_t tile = tile_begin + blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = cv.m;
    const uint32_t* __restrict__ A = b.A;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t* list = b.stage[0] + (uint64_t)tile * TILE * Ent<K>::S;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    for (int s = 0; s < 4; ++s) {
        const uint64_t g = (uint64_t)tile * (TILE / CHUNK) + wave * 4 + s;
        const uint64_t cb = g * CHUNK;
        uint32_t sat[4] = {0u, 0u, 0u, 0u};
        uint4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = make_uint4(0u, 0u, 0u, 0u);
        if (cb < m) {
            const uint4* src = reinterpret_cast<const uint4*>(cv.lits_t + cb * K) + lane;
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = src[j * 64];
#pragma unroll
            for (int j = 0; j < K; ++j) {  // satisfied clauses skip their remaining lookups
                const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (j > 0 && sat[q]) continue;
                    const uint32_t l = xs[q] & cv.lit_mask;
                    sat[q] |= abit(A, l >> 1) ^ (l & 1u);
                }
            }
        }
        const uint64_t c0 = cb + 4u * lane;
        const bool v[4] = {!sat[0] && c0 < m, !sat[1] && c0 + 1 < m, !sat[2] && c0 + 2 < m,
                           !sat[3] && c0 + 3 < m};
        const uint64_t b0 = __ballot(v[0]), b1 = __ballot(v[1]), b2 = __ballot(v[2]), b3 = __ballot(v[3]);
        if (lane < 4) b.vmask[g * 4 + lane] = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
        const uint32_t tot = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
        if (tot) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&s_cnt, tot);
            base = __shfl(base, 0, 64);
            const uint32_t pre = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
            emit4<K>(cv, list, base + pre, c0, v, x);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        b.tile_cnt[tile] = s_cnt;
        b.mis_cnt[tile] = 0;
    }
    stamp_eval_end(b, gated);
}

// Clause evaluation, fixed width K, persistent hybrid (the loop's default for fixed k).
// One 1024-thread workgroup per CU owns a contiguous run of tiles.  The assignment words of
// a window of win_words * 32 consecutive variables (the block of the tile's smallest
// variables, b.win_base; refilled between tiles of different windows) are staged in LDS by
// LDS-DMA; a literal whose variable lies there is looked up in LDS, the others in L2 (the
// whole bit-packed assignment stays L2-resident).  Lanes evaluate 4 clauses of a 256-clause chunk with one 16-byte load
// per literal slot from the chunk-transposed layout (as k_eval_fixed), so the literal stream
// is read once, perfectly coalesced.  Violated clauses go to the per-tile lists through
// per-tile LDS counters.
// MODE: EV_LISTS the violated clauses go to the per-tile lists (k_eval_hybrid<K>); EV_SCATTER the
// evaluation workgroups also scatter LFMIS round 0's claims of their runs (one GPU, bucketed round
// 0: k_eval_scatter<K>, a kernel of its own so that profiles and the roofline keep the evaluation
// alone apart from the fused loop kernel); EV_FLAGS (the one-GPU round robin) each violated clause
// sets its byte of the clause-order flags rr_flag instead (k_eval_flags<K>: no lists, no k_rr_mark).
enum : int { EV_LISTS = 0, EV_SCATTER = 1, EV_FLAGS = 2 };
template <int K, int MODE>
__device__ __forceinline__ void eval_hybrid_body(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                                                 uint32_t tile_end, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_A[];
    __shared__ uint32_t s_tcnt[HYB_MAX_TILES];
    const uint32_t nblk = gridDim.x;
    const uint32_t ntiles = tile_end - tile_begin;
    const uint32_t t0 = tile_begin + (uint32_t)(((uint64_t)ntiles * blockIdx.x) / nblk);
    const uint32_t t1 = tile_begin + (uint32_t)(((uint64_t)ntiles * (blockIdx.x + 1)) / nblk);
    if (t0 >= t1) return;
    stamp_eval_begin(b, gated);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = cv.m;
    const uint32_t lds_words = min(b.n_words, b.win_words);
    // LDS-DMA fill of assignment words [wb, wb + lds_words) (global_load_lds_dwordx4: no VGPR
    // round trip; A padded to 4 words; wb + lds_words <= n_words)
    auto fill = [&](uint32_t wb) {
        const uint32_t n4 = (lds_words + 3) / 4;
        const uint4* src = reinterpret_cast<const uint4*>(b.A + wb);
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
    };
    // window of a tile (words; b.win_base: instances sorted by smallest-variable block, else 0)
    // (bit 31 of win_base[t]: the smallest variable of every clause of tile t lies in its
    // window, so slot K-1 is looked up in LDS only)
    auto window = [&](uint32_t t) -> uint32_t { return b.win_base ? b.win_base[t] & 0x7FFFFFFFu : 0u; };
    auto win_key = [&](uint32_t t) -> uint32_t { return b.win_base ? b.win_base[t] : 0u; };  // (with bit 31)
    // the whole assignment fits the LDS window: every lookup is an LDS read
    const bool all_lds = b.win_base == nullptr && b.n_words <= b.win_words;
    uint32_t wb = window(t0);
    // zero word for lanes that need no LDS word (past every word the fill writes)
    const uint32_t zslot = (lds_words + 3) / 4 * 4;
    if (threadIdx.x == 0) s_A[zslot] = 0u;
    fill(wb);
    const uint32_t a_lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)b.A);
    const uint32_t a_hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)b.A >> 32));
    const uint32_t wbits = __popc(cv.lit_mask) - 6u;  // word-index bits of a literal
    const auto rsV = __builtin_amdgcn_make_buffer_rsrc(
        (void*)b.vmask, (short)0, (int)__builtin_amdgcn_readfirstlane(b.n_tiles * (TILE_WORDS * 8u)), 0x00020000);
    // (EV_FLAGS: the clause-order flag bytes)
    const auto rsF = __builtin_amdgcn_make_buffer_rsrc(
        (void*)b.rr_flag, (short)0, (int)__builtin_amdgcn_readfirstlane(MODE == EV_FLAGS ? b.n_tiles * TILE : 0u), 0x00020000);
    // The four lookups of one literal slot (the lane's four clauses): the assignment word of
    // literal xs[q]'s variable, from LDS when the window holds it, else from L2.  Branch-free
    // per lane: a word a lane does not need from LDS (outside the window, or need[q] == false:
    // the clause is already satisfied) reads the zero word s_A[zslot], a word it does not need
    // from L2 gets an out-of-range buffer offset (the range check returns 0 without a memory
    // access), so w = gw | lw.  The four buffer loads are issued only when some lane of the
    // wave needs one (a wave-uniform branch: slot K-1 of a windowed tile and slot 0 of chunks
    // whose largest variables lie in the window need none).  AL: the whole assignment is in LDS.
    // MG: lanes that need no L2 word are masked off instead of sent out of range (instances
    // larger than the Infinity Cache, whose L2 lookups go to memory: C4 eval 456 -> 427 us; at
    // M, where they hit in L2, the out-of-range form is as fast or faster)
    // Offsets are bytes from the window's first word, for LDS and L2 alike (rsW is based at the
    // window): every variable of a clause is >= its smallest one, whose block starts at or
    // after its tile's window (§2 of DESIGN.md), so no offset is negative.
    const uint32_t lds_bytes = lds_words * 4u, zbyte = zslot * 4u;
    auto lookup4 = [&](auto al, auto mg, __amdgpu_buffer_rsrc_t rsW, uint32_t wb4n, const uint32_t (&xs)[4],
                       const bool (&need)[4], uint32_t (&gw)[4], uint32_t (&lw)[4]) {
        constexpr bool AL = decltype(al)::value;
        bool ng[4];
        uint32_t goff[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t db = __builtin_amdgcn_ubfe(xs[q], 6u, wbits) * 4u + wb4n;
            const bool inl = AL || db < lds_bytes;
            ng[q] = need[q] && !inl;
            goff[q] = ng[q] ? db : 0x80000000u;
            lw[q] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(s_A) + ((need[q] && inl) ? db : zbyte));
        }
        if constexpr (AL) {
#pragma unroll
            for (int q = 0; q < 4; ++q) gw[q] = 0u;
        } else if (__builtin_amdgcn_ballot_w64(ng[0] || ng[1] || ng[2] || ng[3])) {
            if constexpr (decltype(mg)::value) {
#pragma unroll
                for (int q = 0; q < 4; ++q) gw[q] = ng[q] ? __builtin_amdgcn_raw_buffer_load_b32(rsW, goff[q], 0, 0) : 0u;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) gw[q] = __builtin_amdgcn_raw_buffer_load_b32(rsW, goff[q], 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) gw[q] = 0u;
        }
    };
    // slot K-1 of a tile whose clauses all have their smallest variable in the window (bit 31 of
    // win_base): LDS reads only, no range test or L2 path
    auto lookup4_lds = [&](uint32_t wb4n, const uint32_t (&xs)[4], uint32_t (&lw)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            lw[q] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(s_A) +
                                                       __builtin_amdgcn_ubfe(xs[q], 6u, wbits) * 4u + wb4n);
    };
    // bit 0: the literal is true (its variable's bit of word w, xor the sign, bit 0 of xs; the
    // other bits are don't-care)
    auto lit_true = [](uint32_t w, uint32_t xs) -> uint32_t { return __builtin_amdgcn_ubfe(w, xs >> 1, 1u) ^ xs; };
    // The wave's chunks g = gbeg + wave, + 16, ... of one window segment, software-pipelined:
    // per chunk, the lookups of slots 0 (largest variable: coalesced gathers) and K-1 (smallest:
    // mostly in LDS) are issued together, then the literal loads of the wave's next chunk, and
    // only then are the lookups consumed; the middle slots follow, each only for the clauses
    // not yet satisfied.  So a wave waits for one literal load and one or two lookup round
    // trips per chunk, not for a chain of them.
    auto run_chunks_t = [&](auto al, auto nt, auto kl, uint64_t gbeg, uint64_t gend, uint32_t pt) {
        uint64_t g = gbeg + wave;
        if (g >= gend) return;
        // L2 lookups through a buffer descriptor over the assignment from the window on: its
        // range check returns 0 for the out-of-range offsets of lanes that need no L2 word
        const uint32_t wbu = __builtin_amdgcn_readfirstlane(wb);
        const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)a_hi << 32 | a_lo) + 4ull * wbu), (short)0,
                                                           (int)((b.n_words - wbu) * 4u), 0x00020000);
        const uint32_t wb4n = 0u - 4u * wbu;
        // NT: non-temporal literal loads (a stream larger than the Infinity Cache: it would
        // only evict the assignment words the L2 lookups need)
        auto load_chunk = [&](uint64_t gg, uint4 (&xx)[K]) {
            const uint4* src = reinterpret_cast<const uint4*>(cv.lits_t + gg * CHUNK * K) + lane;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                if constexpr (decltype(nt)::value) {
                    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + j * 64));
                    xx[j] = make_uint4(v.x, v.y, v.z, v.w);
                } else {
                    xx[j] = src[j * 64];
                }
            }
        };
        uint4 x[K], xn[K];
        load_chunk(g, x);
        for (;;) {
            // (the last chunk reloads itself instead of a next one: no branch around the loads)
            const uint64_t gn = g + HYB_THREADS / 64 < gend ? g + HYB_THREADS / 64 : g;
            const uint64_t cb = g * CHUNK;
            uint32_t sat[4];
            {
                const uint32_t xa[4] = {x[0].x, x[0].y, x[0].z, x[0].w};
                const uint32_t xb[4] = {x[K - 1].x, x[K - 1].y, x[K - 1].z, x[K - 1].w};
                uint32_t ga[4], la[4], gb[4], lb[4];
                const bool all4[4] = {true, true, true, true};
                lookup4(al, nt, rsW, wb4n, xa, all4, ga, la);
                if constexpr (K > 1) {
                    if constexpr (decltype(kl)::value) {
                        lookup4_lds(wb4n, xb, lb);
#pragma unroll
                        for (int q = 0; q < 4; ++q) gb[q] = 0u;
                    } else {
                        lookup4(al, nt, rsW, wb4n, xb, all4, gb, lb);
                    }
                }
                // (scheduling barriers keep the next chunk's loads between the lookups' issue
                // and their use)
                __builtin_amdgcn_sched_barrier(0);
                load_chunk(gn, xn);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    sat[q] = lit_true(ga[q] | la[q], xa[q]);
                    if constexpr (K > 1) sat[q] |= lit_true(gb[q] | lb[q], xb[q]);
                }
            }
#pragma unroll
            for (int j = 1; j < K - 1; ++j) {  // middle slots (by descending variable)
                const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
                uint32_t gw[4], lw[4];
                const bool need[4] = {!(sat[0] & 1u), !(sat[1] & 1u), !(sat[2] & 1u), !(sat[3] & 1u)};
                lookup4(al, nt, rsW, wb4n, xs, need, gw, lw);
#pragma unroll
                for (int q = 0; q < 4; ++q) sat[q] |= lit_true(gw[q] | lw[q], xs[q]);
            }
            const uint64_t c0 = cb + 4u * lane;
            // (wave-uniform: only the last chunk holds positions past m)
            const uint32_t lim = (uint32_t)min((uint64_t)CHUNK, m - cb);
            bool v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = !(sat[q] & 1u) && 4u * lane + q < lim;
            const uint64_t b0 = __ballot(v[0]), b1 = __ballot(v[1]), b2 = __ballot(v[2]), b3 = __ballot(v[3]);
            // Stores without branches, so that every chunk issues the same number of vector
            // memory instructions and the wait for the next chunk's literals (loaded before the
            // stores; the counter is in order) need not wait for the stores: lanes 0 and 1 write
            // the chunk's four bitmask words (32 aligned bytes), the other lanes and the
            // satisfied clauses store to an out-of-range offset (dropped by the range check).
            {
                const bool lo = lane == 0;
                const u32x4 vw = {(uint32_t)(lo ? b0 : b2), (uint32_t)((lo ? b0 : b2) >> 32),
                                  (uint32_t)(lo ? b1 : b3), (uint32_t)((lo ? b1 : b3) >> 32)};
                __builtin_amdgcn_raw_buffer_store_b128(vw, rsV, lane < 2 ? (uint32_t)g * 32u + lane * 16u : 0x80000000u, 0, 0);
            }
            const uint32_t tot = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
            // (wide clauses are rarely violated: their entries are stored only by chunks that
            // hold violated clauses, with the branching emit4)
            if constexpr (MODE == EV_FLAGS) {
                const uint32_t tile = (uint32_t)(g / (TILE / CHUNK));
                if (lane == 0 && tot) atomicAdd(&s_tcnt[tile - pt], tot);
                if (cv.id_bits) {
                    // Packed ids: four byte stores per chunk without branches (the satisfied
                    // clauses' to an out-of-range offset), so that, as for the bitmask above, the
                    // wait for the next chunk's literals need not wait for these scattered
                    // stores (with a branch per store the count varies: 51.8 -> 48.9 us at M,
                    // T = 16, profiles/r6_checks/rr/eval_flags_branchfree_ab.txt).
                    const uint32_t fm = ((1u << cv.id_bits) - 1u) << cv.id_shift;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t id = 0;
#pragma unroll
                        for (int j = 0; j < K; ++j) {
                            const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
                            id |= ((xs[q] & fm) >> cv.id_shift) << (j * cv.id_bits);
                        }
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)1u, rsF, v[q] ? id : 0x80000000u, 0, 0);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (!v[q]) continue;
                        Ent<K> e;
                        uint32_t t[K];
#pragma unroll
                        for (int j = 0; j < K; ++j) {
                            const uint32_t xs[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
                            t[j] = xs[q];
                        }
                        make_ent<K>(e, c0 + q, t);
                        ent_unpack<K>(cv, e);
                        b.rr_flag[e.w[0]] = 1u;
                    }
                }
            } else if (K <= 4 || tot) {
                const uint32_t tile = (uint32_t)(g / (TILE / CHUNK));
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&s_tcnt[tile - pt], tot);
                base = __builtin_amdgcn_readfirstlane(base);  // (every lane is active here)
                // rank of the lane's first violated clause: set bits of the four ballots below
                // the lane (mbcnt chain)
                uint32_t pre = 0;
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, pre));
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, pre));
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b2, pre));
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b3, pre));
                if constexpr (K <= 4) emit4_bf<K>(list_rsrc<K>(b.stage[0] + (uint64_t)tile * TILE * Ent<K>::S), base + pre, c0, v, x);
                else emit4<K>(cv, b.stage[0] + (uint64_t)tile * TILE * Ent<K>::S, base + pre, c0, v, x);
            }
            if (gn == g) break;
            g = gn;
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = xn[j];
        }
    };
    auto run_chunks = [&](uint64_t gbeg, uint64_t gend, uint32_t pt, bool kl) {
        if (all_lds) run_chunks_t(std::true_type{}, std::false_type{}, std::false_type{}, gbeg, gend, pt);
        else if (cv.lits_nt && kl) run_chunks_t(std::false_type{}, std::true_type{}, std::true_type{}, gbeg, gend, pt);
        else if (cv.lits_nt) run_chunks_t(std::false_type{}, std::true_type{}, std::false_type{}, gbeg, gend, pt);
        else if (kl) run_chunks_t(std::false_type{}, std::false_type{}, std::true_type{}, gbeg, gend, pt);
        else run_chunks_t(std::false_type{}, std::false_type{}, std::false_type{}, gbeg, gend, pt);
    };
    for (uint32_t pt = t0; pt < t1; pt += HYB_MAX_TILES) {
        const uint32_t pe = min(t1, pt + HYB_MAX_TILES);
        if (threadIdx.x < HYB_MAX_TILES) s_tcnt[threadIdx.x] = 0;
        __syncthreads();  // also publishes the LDS fill
      // segments of tiles with one window (and one bit 31: slot K-1 in LDS only); the LDS is
      // refilled between windows
      for (uint32_t sa = pt; sa < pe;) {
        const uint32_t wk = win_key(sa), ws = wk & 0x7FFFFFFFu;
        uint32_t se = sa + 1;
        while (se < pe && win_key(se) == wk) ++se;
        if (ws != wb) {
            __syncthreads();  // every wave is done with the old window
            fill(ws);
            __syncthreads();
            wb = ws;
        }
        // (chunks past m are skipped: their bitmask words stay 0 from the allocation)
        const uint64_t gbeg = (uint64_t)sa * (TILE / CHUNK);
        const uint64_t gend = min((uint64_t)se * (TILE / CHUNK), (m + CHUNK - 1) / CHUNK);
        sa = se;
        run_chunks(gbeg, gend, pt, (wk >> 31) != 0u);
      }
        __syncthreads();
        if (threadIdx.x < pe - pt) {
            b.tile_cnt[pt + threadIdx.x] = s_tcnt[threadIdx.x];
            b.mis_cnt[pt + threadIdx.x] = 0;
        }
    }
    stamp_eval_end(b, gated);
    if constexpr (MODE == EV_SCATTER) {
        // One GPU, bucketed LFMIS round 0: this workgroup's tiles form runs b.run_t0[r] ..
        // (rpw runs per workgroup), so the workgroup scatters their claims itself, from the
        // lists it has just written (L2-warm) and with the window's LDS, instead of a
        // separate k_bscatter launch; the reduce then runs in k_bresolve (pre-reduce epoch).
        __syncthreads();  // every wave is done with the window; the lists and counts are visible
        const ScatterLds L = carve_scatter_lds(s_A);
        const uint32_t rpw = b.n_runs / gridDim.x;
        for (uint32_t r = blockIdx.x * rpw; r < (blockIdx.x + 1) * rpw; ++r) {
            scatter_run<K>(cv, b, b.stage[0], r, b.state->round_next, L);
            __syncthreads();  // (the LDS is reused by the next run)
        }
    }
}

template <int K>
__global__ __launch_bounds__(HYB_THREADS) void k_eval_hybrid(ClauseView cv, LoopBuffers b, uint32_t tile_begin,
                                                             uint32_t tile_end, int gated) {
    eval_hybrid_body<K, EV_LISTS>(cv, b, tile_begin, tile_end, gated);
}

template <int K>
__global__ __launch_bounds__(HYB_THREADS) void k_eval_scatter(ClauseView cv, LoopBuffers b, uint32_t tile_begin,
                                                              uint32_t tile_end, int gated) {
    eval_hybrid_body<K, EV_SCATTER>(cv, b, tile_begin, tile_end, gated);
}

template <int K>
__global__ __launch_bounds__(HYB_THREADS) void k_eval_flags(ClauseView cv, LoopBuffers b, uint32_t tile_begin,
                                                            uint32_t tile_end, int gated) {
    eval_hybrid_body<K, EV_FLAGS>(cv, b, tile_begin, tile_end, gated);
}

// Clause evaluation, ragged widths (ClauseView::rg_off): the persistent LDS-window structure
// of k_eval_hybrid over the chunk-transposed ragged copy.  A chunk's width w (its widest
// clause; clauses are evaluated sorted by width, so chunks are nearly uniform) is wave-uniform;
// its slots are read RG_BATCH at a time (one 16-byte load per slot: 4 clauses per lane) and the
// chunk stops early once every one of its 256 clauses is satisfied.  Violated clauses go to the
// per-tile lists as evaluation positions (generic entries, one word); CLAIM(0) translates them
// through perm.  The bitmask has the four-ballots-per-chunk layout of the fixed-width kernels.
constexpr uint32_t RG_BATCH = 4;

__global__ __launch_bounds__(HYB_THREADS) void k_eval_ragged(ClauseView cv, LoopBuffers b, uint32_t tile_begin,
                                                             uint32_t tile_end, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_A[];
    __shared__ uint32_t s_tcnt[HYB_MAX_TILES];
    const uint32_t nblk = gridDim.x;
    const uint32_t ntiles = tile_end - tile_begin;
    const uint32_t t0 = tile_begin + (uint32_t)(((uint64_t)ntiles * blockIdx.x) / nblk);
    const uint32_t t1 = tile_begin + (uint32_t)(((uint64_t)ntiles * (blockIdx.x + 1)) / nblk);
    if (t0 >= t1) return;
    stamp_eval_begin(b, gated);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = cv.m;
    const uint32_t lds_words = min(b.n_words, b.win_words);
    auto fill = [&](uint32_t wb) {
        const uint32_t n4 = (lds_words + 3) / 4;
        const uint4* src = reinterpret_cast<const uint4*>(b.A + wb);
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
    };
    auto window = [&](uint32_t t) -> uint32_t { return b.win_base ? b.win_base[t] : 0u; };
    uint32_t wb = window(t0);
    const uint32_t zslot = (lds_words + 3) / 4 * 4;
    if (threadIdx.x == 0) s_A[zslot] = 0u;
    fill(wb);
    const uint32_t a_lo = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)b.A);
    const uint32_t a_hi = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)b.A >> 32));
    const uint32_t a_bytes = __builtin_amdgcn_readfirstlane(b.n_words * 4u);
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uintptr_t)a_hi << 32) | a_lo), (short)0, (int)a_bytes, 0x00020000);
    for (uint32_t pt = t0; pt < t1; pt += HYB_MAX_TILES) {
        const uint32_t pe = min(t1, pt + HYB_MAX_TILES);
        if (threadIdx.x < HYB_MAX_TILES) s_tcnt[threadIdx.x] = 0;
        __syncthreads();
      for (uint32_t sa = pt; sa < pe;) {
        const uint32_t ws = window(sa);
        uint32_t se = sa + 1;
        while (se < pe && window(se) == ws) ++se;
        if (ws != wb) {
            __syncthreads();
            fill(ws);
            __syncthreads();
            wb = ws;
        }
        const uint64_t gbeg = (uint64_t)sa * (TILE / CHUNK);
        const uint64_t gend = min((uint64_t)se * (TILE / CHUNK), (m + CHUNK - 1) / CHUNK);
        sa = se;
        for (uint64_t g = gbeg + wave; g < gend; g += HYB_THREADS / 64) {
            const uint64_t cb = g * CHUNK;
            const uint32_t o0 = __builtin_amdgcn_readfirstlane(cv.rg_off[g]);
            const uint32_t w = __builtin_amdgcn_readfirstlane(cv.rg_off[g + 1]) - o0;
            const uint4* src = reinterpret_cast<const uint4*>(cv.rg_lits + (uint64_t)o0 * CHUNK) + lane;
            uint32_t sat[4] = {0u, 0u, 0u, 0u};  // bit 0: clause satisfied (as k_eval_hybrid)
            for (uint32_t j0 = 0; j0 < w; j0 += RG_BATCH) {
                uint4 x[RG_BATCH];
#pragma unroll
                for (uint32_t u = 0; u < RG_BATCH; ++u)
                    x[u] = j0 + u < w ? src[(j0 + u) * 64] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (uint32_t u = 0; u < RG_BATCH; ++u) {
                    if (j0 + u >= w) break;  // (wave-uniform)
                    const uint32_t xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
                    uint32_t gw[4], lw[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t wi = __builtin_amdgcn_ubfe(xs[q], 6u, 25u);  // (bit 31: hot flag)
                        const uint32_t d = wi - wb;
                        const bool need = !(sat[q] & 1u);
                        const bool inl = d < lds_words;
                        gw[q] = __builtin_amdgcn_raw_buffer_load_b32(rsA, (need && !inl) ? wi * 4u : 0x80000000u, 0, 0);
                        lw[q] = s_A[(need && inl) ? d : zslot];
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        sat[q] |= __builtin_amdgcn_ubfe(gw[q] | lw[q], xs[q] >> 1, 1u) ^ xs[q];
                }
                if (!__any(!((sat[0] & sat[1] & sat[2] & sat[3]) & 1u))) break;  // chunk satisfied
            }
            const uint64_t c0 = cb + 4u * lane;
            const uint32_t lim = (uint32_t)min((uint64_t)CHUNK, m - cb);
            bool v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = !(sat[q] & 1u) && 4u * lane + q < lim;
            const uint64_t b0 = __ballot(v[0]), b1 = __ballot(v[1]), b2 = __ballot(v[2]), b3 = __ballot(v[3]);
            if (lane == 0) {
                uint4* vm = reinterpret_cast<uint4*>(b.vmask + g * 4);
                vm[0] = make_uint4((uint32_t)b0, (uint32_t)(b0 >> 32), (uint32_t)b1, (uint32_t)(b1 >> 32));
                vm[1] = make_uint4((uint32_t)b2, (uint32_t)(b2 >> 32), (uint32_t)b3, (uint32_t)(b3 >> 32));
            }
            const uint32_t tot = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
            if (tot) {
                const uint32_t tile = (uint32_t)(g / (TILE / CHUNK));
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&s_tcnt[tile - pt], tot);
                base = __builtin_amdgcn_readfirstlane(base);
                uint32_t pre = 0;
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, pre));
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, pre));
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b2, pre));
                pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b3, pre));
                uint32_t* list = b.stage[0] + (uint64_t)tile * TILE + base + pre;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (v[q]) *list++ = (uint32_t)(c0 + q);
            }
        }
      }
        __syncthreads();
        if (threadIdx.x < pe - pt) {
            b.tile_cnt[pt + threadIdx.x] = s_tcnt[threadIdx.x];
            b.mis_cnt[pt + threadIdx.x] = 0;
        }
    }
    stamp_eval_end(b, gated);
}

// Clause evaluation, generic CSR (ragged widths): lane per clause, 64 consecutive
// clauses per wave step, 16 steps per wave, one tile per workgroup.
__global__ __launch_bounds__(EVAL_THREADS) void k_eval_csr(ClauseView cv, LoopBuffers b,
                                                           uint32_t tile_begin, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    __shared__ uint32_t s_cnt;
    stamp_eval_begin(b, gated);
    const uint32_t tile = tile_begin + blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = cv.m;
    const uint32_t* __restrict__ A = b.A;
    const uint32_t* __restrict__ offs = cv.offs;
    const uint32_t* __restrict__ lits = cv.lits;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t* list = b.stage[0] + (uint64_t)tile * TILE;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    for (int s = 0; s < 16; ++s) {
        const uint64_t c = (uint64_t)tile * TILE + wave * (TILE / 4) + s * 64 + lane;
        bool viol = false;
        if (c < m) {
            const uint32_t o0 = offs[c], o1 = offs[c + 1];
            uint32_t sat = 0;
            for (uint32_t j = o0; j < o1 && !sat; ++j) {
                const uint32_t l = lits[j] & LIT_MASK;
                sat |= abit(A, l >> 1) ^ (l & 1u);
            }
            viol = !sat;
        }
        const uint64_t mask = __ballot(viol);
        if (lane == 0) b.vmask[c >> 6] = mask;
        if (mask) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&s_cnt, (uint32_t)__popcll(mask));
            base = __shfl(base, 0, 64);
            if (viol) list[base + __popcll(mask & lt)] = (uint32_t)c;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        b.tile_cnt[tile] = s_cnt;
        b.mis_cnt[tile] = 0;
    }
    stamp_eval_end(b, gated);
}

// Clause-sharded, evaluation order != clause order: the own shard's violated clauses set their
// bits of the clause-order mask (a wave per own tile, from the evaluation's raw entries), which
// is all-gathered instead of the evaluation-order bitmask.
template <int K>
__global__ __launch_bounds__(256) void k_cmark(ClauseView cv, LoopBuffers b, uint64_t base, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    constexpr int S = Ent<K>::S;
    const uint32_t tile = b.own_begin + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (tile >= b.own_end) return;
    const uint32_t cnt = b.tile_cnt[tile];
    const uint32_t* lin = b.stage[0] + (uint64_t)tile * TILE * S;
    for (uint32_t i = lane; i < cnt; i += 64) {
        Ent<K> e;
        load_ent<K>(e, lin + (uint64_t)i * S);
        if constexpr (K > 0) ent_unpack<K>(cv, e);
        else if (cv.perm) e.w[0] = cv.perm[e.w[0]];
        b.cflag[e.w[0] - base] = 1u;  // (a byte per clause: plain stores, packed by k_cpack)
    }
}

// The rank's clause flags → its words of the clause-order mask (every word written, so no
// clear), flags cleared once read; a thread per word of 64 clauses.
__global__ __launch_bounds__(256) void k_cpack(LoopBuffers b, uint64_t* words, uint32_t n_words, int gated) {
    if (gated && eval_gate_closed(b.state)) return;
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_words) return;
    uint4* f = reinterpret_cast<uint4*>(b.cflag + (uint64_t)w * 64);
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = f[k];
    unsigned long long bits = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t x[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                bits |= (unsigned long long)((x[j] >> (8 * e)) & 1u) << (16 * k + 4 * j + e);
    }
    words[w] = bits;
    if (bits)
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] = make_uint4(0u, 0u, 0u, 0u);
}

// Multi-GPU: tiles owned by other ranks get their violated lists from the all-gathered
// bitmask (evaluation positions; fixed K fetches the literals from the transposed store).
// Thread t takes 16 bits of word t / 4 of the tile: all bitmask loads are issued at once, a
// workgroup scan of the bit counts places every entry (ascending positions), and each thread's
// literal loads follow -- two dependent load rounds per tile instead of one per word.
template <int K>
__global__ __launch_bounds__(EVAL_THREADS) void k_collect(ClauseView cv, LoopBuffers b,
                                                          uint32_t own_begin, uint32_t own_end) {
    static_assert(EVAL_THREADS * 16 == TILE, "a thread per 16 positions of the tile");
    if (eval_gate_closed(b.state)) return;
    const uint32_t tile = blockIdx.x;
    if (tile >= own_begin && tile < own_end) return;
    __shared__ uint32_t s_wsum[EVAL_THREADS / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)tile * TILE_WORDS + (threadIdx.x >> 2);
    const uint32_t sl = (threadIdx.x & 3u) * 16u;
    // (bits past m are 0: the evaluation kernels never set them).  cmask: clause order (the
    // other ranks' shards are not laid out here: their literals come from the AoS copy)
    const bool co = b.cmask != nullptr;
    uint32_t bits = (uint32_t)((co ? b.cmask[w] : b.vmask[w]) >> sl) & 0xFFFFu;
    const uint32_t cnt = (uint32_t)__popc(bits);
    uint32_t incl = cnt;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t pos = incl - cnt, total = 0;
    for (int v = 0; v < EVAL_THREADS / 64; ++v) {
        if (v < wave) pos += s_wsum[v];
        total += s_wsum[v];
    }
    uint32_t* list = b.stage[0] + (uint64_t)tile * TILE * Ent<K>::S;
    while (bits) {
        const uint32_t i = sl + (uint32_t)__ffs(bits) - 1u;
        bits &= bits - 1u;
        // fixed K and ragged: word w of the bitmask holds positions (w / 4) * 256 + 4 * bit +
        // w % 4 (the kernels store their four ballots as they are); CSR: positions 64 * w + bit
        const uint64_t p = (!co && (K > 0 || cv.rg_off)) ? (w >> 2) * CHUNK + 4u * i + (w & 3u) : w * 64 + i;
        Ent<K> e;
        if constexpr (K > 0) {
            uint32_t t[K];
            if (co) {  // clause p: AoS literals with the clause id's pieces packed as the evaluation's
                const uint32_t idm = cv.id_bits ? (1u << cv.id_bits) - 1u : 0u;
#pragma unroll
                for (int j = 0; j < K; ++j)
                    t[j] = cv.lits[p * K + j] | (cv.id_bits ? (((uint32_t)(p >> (j * cv.id_bits)) & idm) << cv.id_shift) : 0u);
            } else {
                const uint32_t* tp = cv.lits_t + (p / CHUNK) * CHUNK * K + (p % CHUNK);
#pragma unroll
                for (int j = 0; j < K; ++j) t[j] = tp[j * CHUNK];
            }
            make_ent<K>(e, p, t);
        } else {
            e.w[0] = (uint32_t)p;
        }
        store_ent<K>(list + (uint64_t)pos * Ent<K>::S, e);
        ++pos;
    }
    if (threadIdx.x == 0) {
        b.tile_cnt[tile] = total;
        b.mis_cnt[tile] = 0;
    }
}

// ------------------------------------------------------------------------------------
// Violated count + loop state (mode 0) or standalone count (mode 1), by one 1024-thread
// workgroup: k_reduce, or the extra workgroup of k_bscatter (fused reduce).
__device__ void reduce_body(const LoopBuffers& b, int mode) {
    DevState* st = b.state;
    const unsigned long long reduce_t0 = wall_now();
    __shared__ unsigned long long s_sum;
    __shared__ uint32_t s_first;  // first tile with a violated clause (streaming window)
    if (threadIdx.x == 0) { s_sum = 0; s_first = ~0u; }
    __syncthreads();
    // 8-bit cover stamps cycle through 1 .. 255: when this iteration's stamp comes back to 1,
    // the marks of the last 255 iterations are cleared first (once per 255 iterations)
    if (mode == 0 && st->n_iter > 0 && st->n_iter % 255 == 0) {
        uint4* cv4 = reinterpret_cast<uint4*>(b.cover);  // n_words * 32 bytes
        for (uint32_t i = threadIdx.x; i < b.n_words * 2; i += blockDim.x) cv4[i] = make_uint4(0, 0, 0, 0);
    }
    unsigned long long acc = 0;
    uint32_t first = ~0u;
    // (mode 1, the standalone count: this rank's tiles, the only ones it evaluates)
    const uint32_t t_lo = mode == 1 ? b.own_begin : 0u, t_hi = mode == 1 ? b.own_end : b.n_tiles;
    for (uint32_t t = t_lo + threadIdx.x; t < t_hi; t += blockDim.x) {
        const uint32_t cnt = b.tile_cnt[t];
        acc += cnt;
        if (cnt && t < first) first = t;
    }
    if (b.stream_batch && first != ~0u) atomicMin(&s_first, first);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_sum, acc);
    __syncthreads();
    if (threadIdx.x != 0) return;
    const unsigned long long u = s_sum;
    if (mode == 1) {
        st->count_out = u;
        if (b.xcount) b.xcount[0] = (uint32_t)u;  // (summed over the ranks by the host)
        return;
    }
    if (b.ktime) {
        unsigned long long* ts = time_slot(b, st->n_iter);
        ts[2] = reduce_t0;
        unsigned long long* nx = time_slot(b, st->n_iter + 1);  // next iteration's slot
        nx[0] = ~0ull; nx[1] = 0; nx[2] = 0; nx[3] = 0;
    }
    st->n_iter += 1;
    st->u_total = u;
    st->left_cnt = 0;
    st->tmis_cnt = 0;
    st->stamp = (uint32_t)((st->n_iter - 1) % 255) + 1u;
    st->round_base = st->round_next;
    st->round_next = st->round_base + 1;  // the tail advances it past every epoch it used
    if (u == 0) { st->done = 1; st->active = 0; }
    else if (st->n_iter >= st->limit_nores) { st->done = 2; st->active = 0; }
    else st->active = 1;
    if (b.stream_batch && u) {
        // streaming window of this iteration: the first one takes all m steps; later ones
        // m - k0, k0 = first violated clause index + 1 (where the reference's end-of-iteration
        // check stopped), or m again when k0 == m (SATInstance.h:130-147, ClauseGenerator.h:73-90).
        // Streaming uses the clause-order (CSR) layout, so the bitmask is in clause order.
        if (st->n_iter == 1) {
            st->win_start = 0;
            st->win_len = b.m;
        } else {
            const uint32_t t = s_first;
            uint64_t first_c = (uint64_t)t * TILE;
            for (uint32_t w = 0; w < TILE_WORDS; ++w) {
                const uint64_t x = b.vmask[(uint64_t)t * TILE_WORDS + w];
                if (x) { first_c += 64u * w + (uint32_t)__builtin_ctzll(x); break; }
            }
            const uint64_t k0 = first_c + 1;
            st->win_start += st->win_len;
            st->win_len = (k0 == b.m) ? b.m : b.m - k0;
        }
    }
}

// Round robin (fixpoint passes): the iteration's start, run by the reduce's workgroup after the
// violated count (one launch less than a kernel of its own): entry count, set bounds, pass state.
// Owner keys and cover serials carry over from iteration to iteration (keys of later epochs are
// smaller, serials grow), so neither array needs clearing at every iteration; the restart rules
// below decide when they start over (k_fp_guess clears them then).
__device__ __forceinline__ uint32_t fp_ep_budget(const LoopBuffers& b);
__device__ __forceinline__ bool fp_ep_restart(const LoopBuffers& b, const RRFpCtl* ctl) {
    return ctl->ep_next >= fp_ep_budget(b) / 2;  // (every iteration gets at least half the epochs)
}
__device__ __forceinline__ bool fp_serial_restart(const LoopBuffers& b, const RRFpCtl* ctl) {
    return ctl->serial + b.fp_max + 2u > 255u;  // (8-bit cover serials, at most fp_max passes)
}
__device__ void fp_begin_body(const LoopBuffers& b) {
    RRFpCtl* ctl = b.fp_ctl;
    __shared__ uint32_t s_act, s_nu;
    if (threadIdx.x == 0) {
        s_act = b.state->active;  // (thread 0 wrote the state)
        s_nu = (uint32_t)b.state->u_total;
    }
    __syncthreads();
    if (!s_act) {
        if (threadIdx.x == 0) ctl->state = FP_OFF;
        return;
    }
    const uint32_t nu = s_nu, T = b.rr_T;
    // set starts (first entry with id >= the set's first clause): k_rr_entries writes those that
    // fall in a tile; the end and the starts past the last clause are nu
    for (uint32_t s = threadIdx.x; s <= T; s += blockDim.x)
        if (s == T || b.rr_sets[s] >= b.m) b.fp_sf[s] = nu;
    if (b.fp_log)  // (the per-pass counts; the timing rows only when they are written)
        for (uint32_t q = threadIdx.x; q < (b.ktime ? FP_LOG_WORDS : 4 * FP_LOG_PASSES); q += blockDim.x) b.fp_log[q] = 0;
    if (threadIdx.x == 0) {
        const bool ep0 = fp_ep_restart(b, ctl), ser0 = fp_serial_restart(b, ctl);
        ctl->restart = (ep0 ? 1u : 0u) | (ser0 ? 2u : 0u);
        ctl->state = FP_RUN;
        ctl->nu = nu;
        ctl->fp_iter = 0;
        ctl->changes = 0;
        ctl->ep_base = ep0 ? 0u : ctl->ep_next;
        ctl->ep_next = ctl->ep_base;
        if (ser0) ctl->serial = 0;
        ctl->tpre = 0;
        ctl->e0 = ~0u;
        ctl->nheavy = 0;
        ctl->inc = 0;  // (the first pass is a full one)
        ctl->pbsrc = 0;
        ctl->bail = 0;
        ctl->ran = 0;
        ctl->skip = 0;
        ctl->rep_rounds = 0;
        if (ctl->guess_den == 0) { ctl->guess_num = 1; ctl->guess_den = 2; }
    }
}

__global__ __launch_bounds__(1024) void k_reduce(LoopBuffers b, int mode) {
    if (mode == 0 && eval_gate_closed(b.state)) {
        if (threadIdx.x == 0) {
            b.state->active = 0;
            if (b.fp_ctl) b.fp_ctl->state = FP_OFF;
        }
        return;
    }
    reduce_body(b, mode);
    if (mode == 0 && b.fp_ctl) {
        __syncthreads();  // (thread 0 has written the loop state)
        fp_begin_body(b);
    }
}

// ------------------------------------------------------------------------------------
// LFMIS (exact lexicographically-first MIS of the violated clauses in clause order).
// Round r = CLAIM then JOIN, each its own kernel (the kernel boundary orders them):
//   CLAIM(r): an undecided clause touching a variable covered by a clause that already
//     joined in this iteration is out (it depends on an MIS clause); otherwise it claims each
//     of its variables with atomicMin(owner[v], key_r(c)), key_r(c) = (~(round_base+r) << 32)
//     | c, so keys of later rounds / iterations are always smaller than stale ones and
//     owner[] is never reset.
//   JOIN(r): a clause that holds every variable it claimed has no undecided lower-index
//     neighbour, and every decided lower neighbour is out, so it is in the LFMIS: its
//     variables are covered (cover[v] = stamp) and it leaves the list.
// Lists are double buffered: each kernel reads one buffer and compacts the survivors into
// the other.  Claims on hot variables (high-degree, flagged by the host) are reduced in an
// LDS hash table first: one global atomic per hot variable per workgroup (power-law hubs).
// Owner slot / bucket key of variable v (LoopBuffers::vmix_mul, identity unless skewed).
__device__ __forceinline__ uint32_t vmix(const LoopBuffers& b, uint32_t v) { return (v * b.vmix_mul) & b.vmix_mask; }
// inverse of vmix on [0, vmix_mask] (vmix_inv: the multiplier's inverse mod 2^k)
__device__ __forceinline__ uint32_t vunmix(const LoopBuffers& b, uint32_t x) { return (x * b.vmix_inv) & b.vmix_mask; }

struct HotTable {
    uint32_t* k;
    unsigned long long* v;
    __device__ void init() {
        for (uint32_t i = threadIdx.x; i < HOT_SLOTS; i += blockDim.x) { k[i] = 0xFFFFFFFFu; v[i] = ~0ull; }
    }
    __device__ void claim(uint32_t var, unsigned long long key) {
        uint32_t h = (var * 2654435761u) & (HOT_SLOTS - 1);
        for (;;) {
            const uint32_t prev = atomicCAS(&k[h], 0xFFFFFFFFu, var);
            if (prev == 0xFFFFFFFFu || prev == var) break;
            h = (h + 1) & (HOT_SLOTS - 1);
        }
        // workgroup scope: an LDS atomic (a different scope from the global claims keeps the
        // compiler from merging the two into one flat atomic through a selected pointer)
        __hip_atomic_fetch_min(&v[h], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // One claim per hot variable per workgroup.  The claim is tested against the owner key first
    // (agent-scope load): every workgroup of a round claims the top hubs, and memory-side
    // atomics on one address serialise (~11 ns each), so only keys below the current minimum
    // are sent.  A stale read is never below the true minimum (keys only decrease), so a
    // skipped claim could not have won.
    __device__ void flush(unsigned long long* owner, const LoopBuffers& b) {
        for (uint32_t i = threadIdx.x; i < HOT_SLOTS; i += blockDim.x) {
            if (k[i] == 0xFFFFFFFFu) continue;
            unsigned long long* o = &owner[vmix(b, k[i])];
            if (v[i] < __hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(o, v[i]);
        }
    }
};


template <int K>
__device__ __forceinline__ void claim_all(const ClauseView& cv, const LoopBuffers& b, const Ent<K>& e, uint64_t lb,
                                          uint32_t len, unsigned long long key, unsigned long long* owner,
                                          HotTable& ht, bool hot) {
    for (uint32_t j = 0; j < len; ++j) {
        const uint32_t raw = ent_lit<K>(cv, e, lb, j);
        if (hot && (raw & LIT_HOT)) ht.claim(lit_var(raw), key);
        else __hip_atomic_fetch_min(&owner[vmix(b, lit_var(raw))], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// CLAIM(0) (the atomic round 0): every violated clause of a tile claims its variables, in place
// (evaluation positions become clause ids here).  Rounds >= 1 run a wave per tile (k_wclaim).
template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_claim(ClauseView cv, LoopBuffers b, uint32_t* in) {
    const DevState* st = b.state;
    const uint32_t tile = blockIdx.x;
    constexpr int S = Ent<K>::S;
    uint32_t* lin = in + (uint64_t)tile * TILE * S;
    // loop state, count and the first entry of every thread (speculatively: TILE slots per
    // tile) in one round trip (k_wclaim)
    Ent<K> e0;
    load_ent<K>(e0, lin + (uint64_t)threadIdx.x * S);
    const uint32_t cnt = b.tile_cnt[tile];
    const uint32_t active = st->active, rbase = st->round_base;
    spec_fence();
    if (!active || cnt == 0) return;
    __shared__ uint32_t s_hk[HOT_SLOTS];
    __shared__ unsigned long long s_hv[HOT_SLOTS];
    HotTable ht{s_hk, s_hv};
    const bool hot = cv.n_hot != 0;
    if (hot) {
        ht.init();
        __syncthreads();
    }
    const unsigned long long keyhi = (unsigned long long)(~rbase) << 32;
    unsigned long long* owner = b.owner;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
        Ent<K> e;
        if (i == threadIdx.x) e = e0;
        else load_ent<K>(e, lin + (uint64_t)i * S);
        if (cv.id_bits || cv.perm) {  // raw entry from the evaluation
            ent_unpack<K>(cv, e);
            store_ent<K>(lin + (uint64_t)i * S, e);
        }
        uint64_t lb;
        const uint32_t len = ent_len<K>(cv, e, lb);
        const uint32_t key = prio(b, st, e.w[0]);
        if (key == ~0u) continue;  // streaming: not yielded this iteration (dropped by JOIN(0))
        claim_all<K>(cv, b, e, lb, len, keyhi | key, owner, ht, hot);
    }
    if (hot) {
        __syncthreads();
        ht.flush(owner, b);
    }
}

// Join one tile's undecided entries: own(e, i) says whether entry i holds every variable it
// claimed; such a clause is in the LFMIS (cover + MIS list + statistics), the others are
// compacted from `in` to `out` (in the last grid round: into the tail kernel's compact list).
template <int K, typename OwnFn>
__device__ __forceinline__ void join_tile(const ClauseView& cv, const LoopBuffers& b, uint32_t tile, uint32_t cnt,
                                          const uint32_t* in, uint32_t* out, int last,
                                          uint32_t stamp, uint32_t mis0, const Ent<K>& e0, OwnFn own) {
    DevState* st = b.state;
    constexpr int S = Ent<K>::S;
    __shared__ uint32_t s_keep, s_join, s_base;
    __shared__ unsigned long long s_lits, s_w;
    if (threadIdx.x == 0) { s_keep = 0; s_join = 0; s_lits = 0; s_w = 0; }
    __syncthreads();
    const uint32_t* lin = in + (uint64_t)tile * TILE * S;
    uint32_t* lout = out + (uint64_t)tile * TILE * S;
    uint32_t* mis = b.mis + (uint64_t)tile * TILE + mis0;
    unsigned long long my_lits = 0, my_w = 0;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
        Ent<K> e;
        if (i == threadIdx.x) e = e0;  // (loaded by the caller with the counts)
        else load_ent<K>(e, lin + (uint64_t)i * S);
        const uint32_t c = e.w[0];
        const uint32_t key = prio(b, st, c);
        if (key == ~0u) continue;  // streaming: not yielded this iteration, leaves the list
        uint64_t lb;
        const uint32_t len = ent_len<K>(cv, e, lb);
        if (own(e, i, lb, len)) {
            for (uint32_t j = 0; j < len; ++j) b.cover[lit_var(ent_lit<K>(cv, e, lb, j))] = (uint8_t)stamp;
            mis[atomicAdd(&s_join, 1u)] = c;
            my_lits += len;
            my_w += mis_weight(b, st, key);
        } else {
            store_ent<K>(lout + (uint64_t)atomicAdd(&s_keep, 1u) * S, e);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        my_lits += __shfl_down(my_lits, o, 64);
        my_w += __shfl_down(my_w, o, 64);
    }
    if ((threadIdx.x & 63) == 0 && my_w) {  // (an empty clause joins with no literals)
        atomicAdd(&s_lits, my_lits);
        atomicAdd(&s_w, my_w);
    }
    __syncthreads();
    const uint32_t kept = s_keep;
    if (last && kept) {
        if (threadIdx.x == 0) s_base = atomicAdd(&st->left_cnt, kept);
        __syncthreads();
        uint32_t* dst = b.left + (uint64_t)s_base * S;
        for (uint32_t i = threadIdx.x; i < kept * S; i += blockDim.x) dst[i] = lout[i];
    }
    if (threadIdx.x == 0) {
        b.tile_cnt[tile] = last ? 0u : kept;
        b.mis_cnt[tile] = mis0 + s_join;
        if (s_join) {
            atomicAdd(&b.tile_stats[2 * tile], s_w);  // = s_join unless streaming
            atomicAdd(&b.tile_stats[2 * tile + 1], s_lits);
        }
    }
    __syncthreads();  // the shared counters are reused by the next tile
}

// JOIN(r): a clause joins iff owner[v] holds its round-r key for every variable.
template <int K>
__global__ __launch_bounds__(JOIN_THREADS) void k_join(ClauseView cv, LoopBuffers b, uint32_t r,
                                                        const uint32_t* in, uint32_t* out,
                                                        int last) {
    const DevState* st = b.state;
    const uint32_t tile = blockIdx.x;
    // loop state, counts and the first entry of every thread in one round trip (k_wclaim)
    Ent<K> e0;
    load_ent<K>(e0, in + ((uint64_t)tile * TILE + threadIdx.x) * Ent<K>::S);
    const uint32_t cnt = b.tile_cnt[tile], mis0 = b.mis_cnt[tile];
    const uint32_t active = st->active, stamp = st->stamp, rbase = st->round_base;
    spec_fence();
    if (!active || cnt == 0) return;
    const unsigned long long keyhi = (unsigned long long)(~(rbase + r)) << 32;
    const unsigned long long* owner = b.owner;
    join_tile<K>(cv, b, tile, cnt, in, out, last, stamp, mis0, e0,
                 [&](const Ent<K>& e, uint32_t, uint64_t lb, uint32_t len) {
                     bool own = true;
                     const unsigned long long key = keyhi | prio(b, st, e.w[0]);
                     for (uint32_t j = 0; j < len; ++j) own &= owner[vmix(b, lit_var(ent_lit<K>(cv, e, lb, j)))] == key;
                     return own;
                 });
}

// Late rounds (r >= 2: ~60k undecided clauses of 1.25M at M, a few dozen per tile): the same
// CLAIM / JOIN over the same per-tile lists with a wave per tile instead of a workgroup per
// tile (a quarter of the workgroups to dispatch, no idle waves); positions in a tile's output
// and MIS lists come from the wave's ballots.  `last`: survivors go to the tail's list (one
// atomic per wave step that has survivors).
__device__ __forceinline__ uint32_t wave_tile() {
    return __builtin_amdgcn_readfirstlane(blockIdx.x * (ROUND_THREADS / 64) + (threadIdx.x >> 6));
}

template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_wclaim(ClauseView cv, LoopBuffers b, uint32_t r,
                                                          const uint32_t* in, uint32_t* out) {
    const DevState* st = b.state;
    constexpr int S = Ent<K>::S;
    const uint32_t tile = wave_tile();
    const int lane = threadIdx.x & 63;
    const bool tv = tile < b.n_tiles;
    const uint32_t* lin = in + (uint64_t)(tv ? tile : 0u) * TILE * S;
    // The loop state, the tile's count and the wave's first 64 entries are loaded together
    // (the entries speculatively: a tile's list always holds TILE slots), so the kernel pays one
    // memory round trip before its kill tests instead of three dependent ones.
    Ent<K> e0;
    load_ent<K>(e0, lin + (uint64_t)lane * S);
    const uint32_t cnt0 = b.tile_cnt[tv ? tile : 0u];
    const uint32_t active = st->active, stamp = st->stamp, rbase = st->round_base;
    spec_fence();
    if (!active) return;
    // hot-variable instances: the workgroup's claims on hot variables are reduced in an LDS
    // hash first and sent as one atomic per variable (a hub is claimed by hundreds of waves in
    // the early wave rounds; memory-side atomics on one address serialise), so every wave
    // reaches the workgroup barriers of the table
    const bool hot = cv.n_hot != 0;
    __shared__ uint32_t s_hk[HOT_SLOTS];
    __shared__ unsigned long long s_hv[HOT_SLOTS];
    HotTable ht{s_hk, s_hv};
    if (hot) {
        ht.init();
        __syncthreads();
    }
    const uint32_t cnt = tv ? __builtin_amdgcn_readfirstlane(cnt0) : 0u;
    if (cnt == 0 && !hot) return;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const unsigned long long keyhi = (unsigned long long)(~(rbase + r)) << 32;
    unsigned long long* owner = b.owner;
    uint32_t* lout = out + (uint64_t)tile * TILE * S;
    uint32_t kept = 0;
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
        const uint32_t i = i0 + lane;
        Ent<K> e;
        bool keep = false;
        if (i < cnt) {
            if (i0 == 0) e = e0;
            else load_ent<K>(e, lin + (uint64_t)i * S);
            uint64_t lb;
            const uint32_t len = ent_len<K>(cv, e, lb);
            const uint32_t key = prio(b, st, e.w[0]);
            if (key != ~0u) {
                bool killed = false;
                for (uint32_t j = 0; j < len; ++j) killed |= b.cover[lit_var(ent_lit<K>(cv, e, lb, j))] == stamp;
                if (!killed) {
                    for (uint32_t j = 0; j < len; ++j) {
                        const uint32_t raw = ent_lit<K>(cv, e, lb, j);
                        if (hot && (raw & LIT_HOT)) ht.claim(lit_var(raw), keyhi | key);
                        else __hip_atomic_fetch_min(&owner[vmix(b, lit_var(raw))], keyhi | key, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
                    }
                    keep = true;
                }
            }
        }
        const uint64_t km = __ballot(keep);
        if (keep) store_ent<K>(lout + (uint64_t)(kept + __popcll(km & lt)) * S, e);
        kept += (uint32_t)__popcll(km);
    }
    if (lane == 0 && cnt) b.tile_cnt[tile] = kept;
    if (hot) {
        __syncthreads();
        ht.flush(owner, b);
    }
}

template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_wjoin(ClauseView cv, LoopBuffers b, uint32_t r,
                                                         const uint32_t* in, uint32_t* out, int last) {
    DevState* st = b.state;
    constexpr int S = Ent<K>::S;
    const uint32_t tile = wave_tile();
    if (tile >= b.n_tiles) return;
    const int lane = threadIdx.x & 63;
    const uint32_t* lin = in + (uint64_t)tile * TILE * S;
    // loop state, counts and the first 64 entries (speculatively) in one round trip (k_wclaim)
    Ent<K> e0;
    load_ent<K>(e0, lin + (uint64_t)lane * S);
    const uint32_t cnt0 = b.tile_cnt[tile], mc0 = b.mis_cnt[tile];
    const uint32_t active = st->active, stamp = st->stamp, rbase = st->round_base;
    spec_fence();
    if (!active) return;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(cnt0);
    if (cnt == 0) return;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const unsigned long long keyhi = (unsigned long long)(~(rbase + r)) << 32;
    const unsigned long long* owner = b.owner;
    uint32_t* lout = out + (uint64_t)tile * TILE * S;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(mc0);
    uint32_t* mis = b.mis + (uint64_t)tile * TILE + m0;
    uint32_t kept = 0, joined = 0;
    unsigned long long lits = 0, w = 0;
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64) {
        const uint32_t i = i0 + lane;
        Ent<K> e;
        bool own = false, keep = false;
        if (i < cnt) {
            if (i0 == 0) e = e0;
            else load_ent<K>(e, lin + (uint64_t)i * S);
            uint64_t lb;
            const uint32_t len = ent_len<K>(cv, e, lb);
            const uint32_t kc = prio(b, st, e.w[0]);
            if (kc != ~0u) {  // (streaming: a clause not yielded this iteration leaves the list)
                own = true;
                for (uint32_t j = 0; j < len; ++j) own &= owner[vmix(b, lit_var(ent_lit<K>(cv, e, lb, j)))] == (keyhi | kc);
                keep = !own;
                if (own) {
                    for (uint32_t j = 0; j < len; ++j) b.cover[lit_var(ent_lit<K>(cv, e, lb, j))] = (uint8_t)stamp;
                    lits += len;
                    w += mis_weight(b, st, kc);
                }
            }
        }
        const uint64_t jm = __ballot(own), km = __ballot(keep);
        if (own) mis[joined + __popcll(jm & lt)] = e.w[0];
        if (last) {  // survivors straight into the tail's list
            uint32_t base = 0;
            if (km && lane == 0) base = atomicAdd(&st->left_cnt, (uint32_t)__popcll(km));
            base = __shfl(base, 0, 64);
            if (keep) store_ent<K>(b.left + (uint64_t)(base + __popcll(km & lt)) * S, e);
        } else if (keep) {
            store_ent<K>(lout + (uint64_t)(kept + __popcll(km & lt)) * S, e);
        }
        joined += (uint32_t)__popcll(jm);
        kept += (uint32_t)__popcll(km);
    }
    for (int o = 32; o > 0; o >>= 1) {
        lits += __shfl_down(lits, o, 64);
        w += __shfl_down(w, o, 64);
    }
    if (lane == 0) {
        b.tile_cnt[tile] = last ? 0u : kept;
        b.mis_cnt[tile] = m0 + joined;
        if (joined) {  // (the wave owns the tile: no other writer in this kernel)
            b.tile_stats[2 * tile] += w;
            b.tile_stats[2 * tile + 1] += lits;
        }
    }
}

// ------------------------------------------------------------------------------------
// Bucketed round 0 (fixed width K; same decisions as CLAIM(0) + JOIN(0)).  Round 0 claims
// ~k|U| random variables, which as global atomicMin runs at the chip's memory-side atomic
// rate; here the claims are grouped by variable bucket instead and each bucket's minima are
// taken in LDS:
//   k_bscatter (workgroup per run of run_tiles tiles): translates evaluation positions to
//     clause ids, histograms the run's claims by bucket, writes them as pairs grouped by
//     bucket into the run's area, and the per-bucket (start, count) into runtab[bucket][run].
//     Hot-variable claims are reduced in the LDS hash table and go to owner[] as before.
//   k_bresolve (workgroup per bucket): LDS minimum per variable over the bucket's pairs of
//     every run, then marks the pairs that are not the minimum (PAIR_LOSE).
//   k_bjoin (workgroup per run): a clause joins iff none of its pairs lost and it owns its hot
//     variables; joins and compaction as JOIN(0).
__device__ __forceinline__ unsigned long long make_pair(uint32_t c, uint32_t el, uint32_t vl) {
    return ((unsigned long long)c << 32) | ((unsigned long long)el << 15) | vl;
}

// Variable bucket of the bucketed round 0: v / bkt_width by multiply-high (the estimate is
// at most one low for v < 2^32, one correction step), and v's offset in the bucket.
__device__ __forceinline__ uint32_t bucket_of(const LoopBuffers& b, uint32_t v, uint32_t& off) {
    v = vmix(b, v);
    uint32_t q = __umulhi(v, b.bkt_magic);
    uint32_t r = v - q * b.bkt_width;
    if (r >= b.bkt_width) { ++q; r -= b.bkt_width; }
    off = r;
    return q;
}

// Run-local entry index f -> (tile of the run, index in that tile); pre = prefix of the
// run's tile counts (<= RUN_TILES_MAX + 1 entries, in LDS).
__device__ __forceinline__ uint32_t run_tile_of(const uint32_t* pre, uint32_t nt, uint32_t f) {
    uint32_t tt = 0;
    while (tt + 1 < nt && pre[tt + 1] <= f) ++tt;
    return tt;
}

// Loops below are unrolled by BKT_UNROLL independent items per thread so that their global
// loads are in flight together.  When a run's entries fit in one unrolled sweep of the
// workgroup (the common case: ~2.5k entries per run at 10M clauses), they stay in registers
// between the phases of a kernel instead of being re-read.
constexpr int BKT_UNROLL = 4;

// Tile counts of run r -> LDS prefix (nt + 1 entries); returns the run's entry count.
__device__ __forceinline__ uint32_t run_prefix(const LoopBuffers& b, uint32_t t0, uint32_t nt, uint32_t* s_tc,
                                               uint32_t* s_pre) {
    if (threadIdx.x < nt) s_tc[threadIdx.x] = b.tile_cnt[t0 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t tt = 0; tt < nt; ++tt) { s_pre[tt] = acc; acc += s_tc[tt]; }
        s_pre[nt] = acc;
    }
    __syncthreads();
    return s_pre[nt];
}

// Load the U entries f0 + u * blockDim.x of the run (ok[u] = exists; tt/idx = its tile / slot).
template <int K, int U>
__device__ __forceinline__ void load_run_entries(const uint32_t* list, uint32_t t0, uint32_t nt, const uint32_t* s_pre,
                                                 uint32_t E, uint32_t f0, Ent<K>* e, bool* ok, uint32_t* tt,
                                                 uint32_t* idx) {
    constexpr int S = Ent<K>::S;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t f = f0 + u * blockDim.x;
        ok[u] = f < E;
        if (ok[u]) {
            tt[u] = run_tile_of(s_pre, nt, f);
            idx[u] = f - s_pre[tt[u]];
            load_ent<K>(e[u], list + ((uint64_t)(t0 + tt[u]) * TILE + idx[u]) * S);
        }
    }
}

// Bucket scatter of run r (tiles run_t0[r] .. run_t0[r+1]) by the whole workgroup
// (BSC_THREADS threads): the pairs of its claims grouped by variable bucket into the run's
// pair area, the segment table column runtab[.][r], hot claims into owner[] under `epoch`.
// Every thread must call it (workgroup barriers inside).
template <int K>
__device__ void scatter_run(const ClauseView& cv, const LoopBuffers& b, uint32_t* list, uint32_t r, uint32_t epoch,
                            const ScatterLds& L) {
    constexpr int S = Ent<K>::S;
    constexpr int U = BKT_UNROLL;
    const uint32_t t0 = b.run_t0[r], nt = b.run_t0[r + 1] - t0;
    uint32_t* s_hist = L.hist;
    uint32_t* s_tc = L.tc;
    uint32_t* s_pre = L.pre;
    uint32_t* s_wsum = L.wsum;
    unsigned long long* s_pairs = L.pairs;
    HotTable ht{L.hk, L.hv};
    const bool hot = cv.n_hot != 0;
    if (hot) ht.init();
    const uint32_t nb = b.n_bkt;
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) s_hist[i] = 0;
    const uint32_t E = run_prefix(b, t0, nt, s_tc, s_pre);
    const bool single = E <= blockDim.x * U;
    const unsigned long long keyhi = (unsigned long long)(~epoch) << 32;
    Ent<K> e[U];
    bool ok[U];
    uint32_t tts[U], idx[U];
    // single sweep: the histogram's atomics return each claim's rank in its bucket, so pass 2
    // places the pair at bucket start + rank without a second (cursor) atomic
    uint32_t rk[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) ok[u] = false;  // threads past the last entry emit nothing
    // pass 1: bucket histogram (variables only: it runs while the clause-id loads are in
    // flight), clause ids (written back), hot claims
    for (uint32_t f0 = threadIdx.x; f0 < E; f0 += blockDim.x * U) {
        load_run_entries<K, U>(list, t0, nt, s_pre, E, f0, e, ok, tts, idx);
        // raw entries from the evaluation: packed ids are unpacked here (ALU); without packed
        // ids the perm loads are issued first and land while the histogram runs
        uint32_t id[U];
        if (cv.id_bits) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (ok[u]) ent_unpack<K>(cv, e[u]);
        } else if (cv.perm) {
#pragma unroll
            for (int u = 0; u < U; ++u) id[u] = ok[u] ? cv.perm[e[u].w[0]] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t raw = e[u].w[1 + j];
                uint32_t off;
                if (hot && (raw & LIT_HOT)) continue;
                if (single) rk[u][j] = atomicAdd(&s_hist[bucket_of(b, lit_var(raw), off)], 1u);
                else atomicAdd(&s_hist[bucket_of(b, lit_var(raw), off)], 1u);
            }
        }
        if (cv.id_bits) {  // the unpacked entries replace the raw ones (k_bjoin reads them)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (ok[u]) store_ent<K>(list + ((uint64_t)(t0 + tts[u]) * TILE + idx[u]) * S, e[u]);
        } else if (cv.perm) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ok[u]) continue;
                e[u].w[0] = id[u];
                list[((uint64_t)(t0 + tts[u]) * TILE + idx[u]) * S] = id[u];
            }
        }
        if (hot) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ok[u]) continue;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint32_t raw = e[u].w[1 + j];
                    if (raw & LIT_HOT) ht.claim(lit_var(raw), keyhi | e[u].w[0]);
                }
            }
        }
    }
    __syncthreads();
    if (hot) ht.flush(b.owner, b);
    // exclusive scan of the histogram: run-local start of every bucket
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t per = (nb + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = min(nb, threadIdx.x * per), b1 = min(nb, b0 + per);
    uint32_t sum = 0;
    for (uint32_t k = b0; k < b1; ++k) sum += s_hist[k];
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wave) wbase += s_wsum[w];
        total += s_wsum[w];
    }
    uint32_t run = wbase + incl - sum;
    for (uint32_t k = b0; k < b1; ++k) {
        const uint32_t c = s_hist[k];
        b.runtab[(uint64_t)k * b.n_runs + r] = run | ((unsigned long long)c << 32);
        s_hist[k] = run;
        run += c;
    }
    if (threadIdx.x == 0) b.run_pairs[r] = total;
    __syncthreads();
    // pass 2: pairs grouped by bucket, staged in LDS when they fit so that the run's area is
    // written with whole-line stores
    unsigned long long* gpr = b.pairs + (uint64_t)r * b.run_tiles * TILE * K;
    const bool staged = total <= BKT_STAGE;
    auto emit = [&]() {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const uint32_t el = tts[u] * TILE + idx[u];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t raw = e[u].w[1 + j];
                if (hot && (raw & LIT_HOT)) continue;
                const uint32_t v = lit_var(raw);
                uint32_t off;
                const uint32_t bk = bucket_of(b, v, off);
                const uint32_t pos = single ? s_hist[bk] + rk[u][j] : atomicAdd(&s_hist[bk], 1u);
                const unsigned long long x = make_pair(e[u].w[0], el, off);
                if (staged) s_pairs[pos] = x;
                else gpr[pos] = x;
            }
        }
    };
    if (single) {
        emit();  // this thread's entries are still in registers
    } else {
        for (uint32_t f0 = threadIdx.x; f0 < E; f0 += blockDim.x * U) {
            load_run_entries<K, U>(list, t0, nt, s_pre, E, f0, e, ok, tts, idx);
            emit();
        }
    }
    if (staged) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < total; i += blockDim.x) gpr[i] = s_pairs[i];
    }
}

template <int K>
// Standalone bucket scatter, workgroup per run.  pre_reduce: the loop's reduce has not run yet
// (one GPU: it runs in an extra workgroup of k_bresolve), so this iteration's owner epoch is
// state.round_next (the reduce makes it round_base), and the loop state is not read: an
// inactive iteration leaves pairs that k_bjoin never consumes.  Otherwise (multi-GPU, after
// k_reduce) the kernel is gated on state.active.
__global__ __launch_bounds__(BSC_THREADS) void k_bscatter(ClauseView cv, LoopBuffers b, uint32_t* list,
                                                          int pre_reduce) {
    const DevState* st = b.state;
    if (!pre_reduce && !st->active) return;
    __shared__ uint32_t s_hist[BKT_MAX];
    __shared__ uint32_t s_hk[HOT_SLOTS];
    __shared__ unsigned long long s_hv[HOT_SLOTS];
    __shared__ uint32_t s_tc[RUN_TILES_MAX], s_pre[RUN_TILES_MAX + 4];
    __shared__ uint32_t s_wsum[BSC_THREADS / 64];
    extern __shared__ unsigned long long s_pairs[];  // BKT_STAGE pairs
    const ScatterLds L{s_hist, s_hk, s_hv, s_tc, s_pre, s_wsum, s_pairs};
    scatter_run<K>(cv, b, list, blockIdx.x, pre_reduce ? st->round_next : st->round_base, L);
}

// Workgroup per bucket.  The run table column is processed in batches of BKT_RUN_BATCH runs:
// segment starts and a prefix of segment lengths in LDS make the batch's pairs one flat index
// space; a wave takes 64 consecutive items per step (coalesced loads: a segment is contiguous)
// and each lane finds its item's run by a fixed-depth branch-free binary search, U items
// interleaved (an LDS item -> segment table instead in the single-sweep case).  When the bucket's pairs fit one unrolled sweep of the workgroup (the
// common case), they stay in registers between the minimum and the marking pass; otherwise
// the marking pass re-reads them.  Every pair is written back, with PAIR_LOSE set when it is
// not its variable's minimum: a segment's pairs are contiguous, so these are whole-line stores.
constexpr int BRS_THREADS = 512;
// Items per thread and sweep: 20 (10240 pairs: ~8.9k per bucket at 10M clauses with one bucket
// per CU; 150 VGPRs, one workgroup per CU), or 16 (8192 pairs; two workgroups per CU) when
// there are more buckets than CUs.
constexpr int BRS_UNROLL_WIDE = 20, BRS_UNROLL_NARROW = 16, BRS_UNROLL_DEEP = 8;
constexpr int BRS_THREADS_DEEP = 1024;
constexpr uint32_t BRS_DEEP_LDS = 48u << 10;  // minima above this: the deep variant

struct ResolveLds {
    uint32_t* min;          // bkt_width
    uint32_t* start;        // batch: segment start in the run area
    uint32_t* pre;          // batch: exclusive prefix of segment lengths (pre[nr] = total)
    uint32_t* wsum;
};

// Batch setup: segments of runs [rb, rb+nr) of this bucket; returns the batch's pair count.
__device__ __forceinline__ uint32_t resolve_batch(const LoopBuffers& b, const ResolveLds& L, uint32_t rb, uint32_t nr) {
    const unsigned long long* tab = b.runtab + (uint64_t)blockIdx.x * b.n_runs;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t per = (nr + blockDim.x - 1) / blockDim.x;
    const uint32_t q0 = min(nr, threadIdx.x * per), q1 = min(nr, q0 + per);
    uint32_t sum = 0;
    for (uint32_t q = q0; q < q1; ++q) {
        const unsigned long long t = tab[rb + q];
        L.start[q] = (uint32_t)t;
        L.pre[q] = (uint32_t)(t >> 32);
        sum += (uint32_t)(t >> 32);
    }
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) L.wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum, total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wave) run += L.wsum[w];
        total += L.wsum[w];
    }
    for (uint32_t q = q0; q < q1; ++q) {
        const uint32_t c = L.pre[q];
        L.pre[q] = run;
        run += c;
    }
    if (threadIdx.x == 0) L.pre[nr] = total;
    __syncthreads();
    return total;
}

__device__ __forceinline__ unsigned long long resolve_mark(const ResolveLds& L, unsigned long long x) {
    return L.min[(uint32_t)x & 0x7FFFu] != (uint32_t)(x >> 32) ? (x | PAIR_LOSE) : x;
}

// Item -> segment table of one sweep: items [f0, f0 + cap) of the batch (nr <= BKT_RUN_BATCH
// segments, pre[nr] = the batch's pair count).  Every thread takes a contiguous range of items,
// finds the first one's segment by binary search and walks on, so the fill costs the same
// whatever the segment count (a thread per segment serialised on instances with few runs).
__device__ __forceinline__ void resolve_seg_table(const ResolveLds& L, uint32_t nr, uint32_t np, uint32_t f0,
                                                  uint32_t cap, uint16_t* s_seg) {
    const uint32_t f1 = min(np, f0 + cap);
    if (f1 <= f0) return;
    const uint32_t per = (f1 - f0 + blockDim.x - 1) / blockDim.x;
    uint32_t f = f0 + threadIdx.x * per;
    const uint32_t fe = min(f1, f + per);
    if (f >= fe) return;
    uint32_t q = 0;  // largest q < nr with pre[q] <= f
#pragma unroll
    for (int step = 9; step >= 0; --step) {
        const uint32_t mid = q + (1u << step);
        q = (mid < nr && L.pre[min(mid, nr)] <= f) ? mid : q;
    }
    for (; f < fe; ++f) {
        while (L.pre[q + 1] <= f) ++q;  // (skips empty segments; f < pre[nr])
        s_seg[f - f0] = (uint16_t)q;
    }
}

// T threads, U items per thread and sweep.  <20, 512>: one bucket per CU (minima <= 128 KB, ~9k
// pairs: one sweep); <16, 512>: more buckets than CUs with small minima (two workgroups per
// CU); <8, 1024>: more buckets than CUs with 128 KB minima (one workgroup per CU: 16 waves
// instead of 8 for the latency-bound sweeps).  Sweeps past the first use a per-sweep item ->
// segment table too (no binary search per item).
//
// fused_reduce (one GPU): the loop's reduce runs in workgroup 0 after its bucket, saving the
// k_reduce launch.  The bucket workgroups then read no loop
// state: when the iteration turns out inactive, their marks are never consumed (k_bjoin tests
// state.active, set by then), and a skipped evaluation leaves the previous pairs, which are
// resolved again to the same marks.
template <int U, int T>
__device__ void resolve_bucket(const LoopBuffers& b, uint32_t run_cap);

template <int U, int T>
__global__ __launch_bounds__(T, (U <= BRS_UNROLL_NARROW && T <= 512) ? 2 : 1) void k_bresolve(LoopBuffers b,
                                                                                              uint32_t run_cap,
                                                                                              int fused_reduce) {
    if (!fused_reduce && !b.state->active) return;
    resolve_bucket<U, T>(b, run_cap);
    if (fused_reduce && blockIdx.x == 0) {  // (no extra workgroup: every CU may hold a bucket)
        __syncthreads();
        if (eval_gate_closed(b.state)) {
            if (threadIdx.x == 0) b.state->active = 0;
        } else {
            reduce_body(b, 0);
        }
    }
}

template <int U, int T>
__device__ void resolve_bucket(const LoopBuffers& b, uint32_t run_cap) {
    extern __shared__ uint32_t s_min[];
    __shared__ uint32_t s_start[BKT_RUN_BATCH], s_pre[BKT_RUN_BATCH + 1];
    __shared__ uint32_t s_wsum[T / 64];
    __shared__ uint16_t s_seg[T * U];  // item -> segment of the current sweep
    const uint32_t bv = b.bkt_width;
    ResolveLds L{s_min, s_start, s_pre, s_wsum};
    for (uint32_t i = threadIdx.x; i < bv; i += blockDim.x) L.min[i] = ~0u;
    // items of a wave: f0 + 64 u, f0 = wave * 64 U + lane (+ stride per sweep)
    const uint32_t first = (threadIdx.x >> 6) * 64 * U + (threadIdx.x & 63);
    const uint32_t stride = T * U;
    uint32_t pos[U];  // pair positions (the pair area holds < 2^32 pairs, checked at create)
    unsigned long long x[U];
    if (b.n_runs <= BKT_RUN_BATCH) {
        const uint32_t np = resolve_batch(b, L, 0, b.n_runs);  // (its barriers also publish L.min)
        if (np <= stride) {
            if (np > 0) {
                // item -> segment table (one LDS read per item instead of a binary search)
                resolve_seg_table(L, b.n_runs, np, 0u, np, s_seg);
                __syncthreads();
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t f = min(first + 64 * u, np - 1);
                    const uint32_t q = s_seg[f];
                    pos[u] = q * run_cap + L.start[q] + (f - L.pre[q]);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = b.pairs[pos[u]];
#pragma unroll
                for (int u = 0; u < U; ++u)  // (clamped duplicates of the last pair would serialise)
                    if (first + 64 * u < np) atomicMin(&L.min[(uint32_t)x[u] & 0x7FFFu], (uint32_t)(x[u] >> 32));
            }
            __syncthreads();
            if (np > 0) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (first + 64 * u < np) b.pairs[pos[u]] = resolve_mark(L, x[u]);
            }
            return;
        }
    }
    __syncthreads();
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t rb = 0; rb < b.n_runs; rb += BKT_RUN_BATCH) {
            const uint32_t nr = min(BKT_RUN_BATCH, b.n_runs - rb);
            const uint32_t np = resolve_batch(b, L, rb, nr);
            for (uint32_t s0 = 0; s0 < np; s0 += stride) {
                resolve_seg_table(L, nr, np, s0, stride, s_seg);
                __syncthreads();
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t f = min(s0 + first + 64 * u, np - 1);
                    const uint32_t q = s_seg[f - s0];
                    pos[u] = (rb + q) * run_cap + L.start[q] + (f - L.pre[q]);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = b.pairs[pos[u]];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (s0 + first + 64 * u >= np) continue;
                    if (pass == 0) atomicMin(&L.min[(uint32_t)x[u] & 0x7FFFu], (uint32_t)(x[u] >> 32));
                    else b.pairs[pos[u]] = resolve_mark(L, x[u]);
                }
                __syncthreads();  // the table is rewritten by the next sweep
            }
            // (batch arrays are rewritten next; after pass 0: L.min is final -- the sweep's
            // last barrier orders it)
        }
    }
}

// Workgroup per run: lose marks -> LDS byte per entry; then every entry of the run's tiles in
// one flat loop: join (cover, MIS list of its tile) or survive (compacted into its tile's
// list in `out`, or the tail's compact list when `last`).
constexpr int BJN_THREADS = 1024;

template <int K>
__global__ __launch_bounds__(BJN_THREADS) void k_bjoin(ClauseView cv, LoopBuffers b, const uint32_t* in,
                                                       uint32_t* out, int last) {
    DevState* st = b.state;
    constexpr int S = Ent<K>::S;
    constexpr int U = K <= 4 ? 2 * BKT_UNROLL : BKT_UNROLL;
    const uint32_t r = blockIdx.x;
    // the loop state with the run's bounds and pair count (one round trip)
    const uint32_t t0 = b.run_t0[r], nt = b.run_t0[r + 1] - t0;
    const uint32_t np = b.run_pairs[r];
    const uint32_t active = st->active, stamp = st->stamp, rbase = st->round_base;
    spec_fence();
    if (!active) return;
    extern __shared__ uint32_t s_lost[];  // one byte per entry slot of the run's tiles
    __shared__ uint32_t s_tc[RUN_TILES_MAX], s_pre[RUN_TILES_MAX + 1], s_keep[RUN_TILES_MAX],
        s_join[RUN_TILES_MAX], s_mis0[RUN_TILES_MAX], s_base[RUN_TILES_MAX];
    __shared__ unsigned long long s_lits[RUN_TILES_MAX];
    for (uint32_t i = threadIdx.x; i < nt * TILE / 4; i += blockDim.x) s_lost[i] = 0;
    if (threadIdx.x < nt) {
        s_keep[threadIdx.x] = 0;
        s_join[threadIdx.x] = 0;
        s_lits[threadIdx.x] = 0;
        s_mis0[threadIdx.x] = b.mis_cnt[t0 + threadIdx.x];
    }
    const uint32_t E = run_prefix(b, t0, nt, s_tc, s_pre);
    const bool single = E <= blockDim.x * U;
    Ent<K> e[U];
    bool ok[U];
    uint32_t tts[U], idx[U];
    if (single) load_run_entries<K, U>(in, t0, nt, s_pre, E, threadIdx.x, e, ok, tts, idx);
    uint8_t* lost = reinterpret_cast<uint8_t*>(s_lost);
    const unsigned long long* pr = b.pairs + (uint64_t)r * b.run_tiles * TILE * K;
    constexpr int PU = 16;  // pairs per thread per sweep (~3 per clause: one sweep at 10M clauses)
    for (uint32_t i0 = threadIdx.x; i0 < np; i0 += blockDim.x * PU) {
        unsigned long long x[PU];
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            x[u] = i < np ? pr[i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < PU; ++u)
            if (x[u] & PAIR_LOSE) lost[(x[u] >> 15) & 0xFFFFu] = 1;
    }
    __syncthreads();
    const bool hot = cv.n_hot != 0;
    const unsigned long long keyhi = (unsigned long long)(~rbase) << 32;
    const unsigned long long* owner = b.owner;
    auto decide = [&]() {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const uint32_t tt = tts[u], tile = t0 + tt;
            bool own = !lost[tt * TILE + idx[u]];
            if (hot) {
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint32_t raw = e[u].w[1 + j];
                    if (raw & LIT_HOT) own &= owner[vmix(b, lit_var(raw))] == (keyhi | e[u].w[0]);
                }
            }
            if (own) {
#pragma unroll
                for (int j = 0; j < K; ++j) b.cover[lit_var(e[u].w[1 + j])] = (uint8_t)stamp;
                b.mis[(uint64_t)tile * TILE + s_mis0[tt] + atomicAdd(&s_join[tt], 1u)] = e[u].w[0];
                atomicAdd(&s_lits[tt], (unsigned long long)K);
            } else {
                store_ent<K>(out + ((uint64_t)tile * TILE + atomicAdd(&s_keep[tt], 1u)) * S, e[u]);
            }
        }
    };
    if (single) {
        decide();
    } else {
        for (uint32_t f0 = threadIdx.x; f0 < E; f0 += blockDim.x * U) {
            load_run_entries<K, U>(in, t0, nt, s_pre, E, f0, e, ok, tts, idx);
            decide();
        }
    }
    __syncthreads();
    if (threadIdx.x < nt) {
        const uint32_t tt = threadIdx.x, tile = t0 + tt, kept = s_keep[tt];
        if (last && kept) s_base[tt] = atomicAdd(&st->left_cnt, kept);
        b.tile_cnt[tile] = last ? 0u : kept;
        b.mis_cnt[tile] = s_mis0[tt] + s_join[tt];
        if (s_join[tt]) {
            atomicAdd(&b.tile_stats[2 * tile], (unsigned long long)s_join[tt]);
            atomicAdd(&b.tile_stats[2 * tile + 1], s_lits[tt]);
        }
    }
    if (last) {
        __syncthreads();
        for (uint32_t tt = 0; tt < nt; ++tt) {
            const uint32_t kept = s_keep[tt];
            if (!kept) continue;
            const uint32_t* src = out + (uint64_t)(t0 + tt) * TILE * S;
            uint32_t* dst = b.left + (uint64_t)s_base[tt] * S;
            for (uint32_t i = threadIdx.x; i < kept * S; i += blockDim.x) dst[i] = src[i];
        }
    }
}

// Tail: one workgroup finishes the LFMIS over the compact list handed over by the last grid
// round (CLAIM / barrier / JOIN passes until no undecided clause is left).  Entries are
// processed in chunks of one per thread; survivors are compacted in place (a write position
// never passes the chunk being read).  owner / cover are accessed with agent-scope relaxed
// atomics so no stale L1 line is read across the barriers.  (Round 6: the entries held in
// registers across the rounds, up to 12 per thread with their loads in flight together, was
// 6-7 us slower per iteration at M and C5 and no faster on longer lists, DESIGN.md §7.1: one
// CU's memory-level parallelism, not the chunk barriers, bounds a round of the tail.)
template <int K>
__global__ __launch_bounds__(TAIL_THREADS) void k_tail(ClauseView cv, LoopBuffers b, uint32_t first_round) {
    DevState* st = b.state;
    constexpr int S = Ent<K>::S;
    // the loop state and the first entry of every thread (speculatively: the list holds
    // n_tiles * TILE >= TAIL_THREADS entries) in one round trip
    Ent<K> e0;
    if (b.n_tiles) load_ent<K>(e0, b.left + (uint64_t)threadIdx.x * S);
    const uint32_t active = st->active, stamp = st->stamp, n0 = st->left_cnt, rbase = st->round_base;
    spec_fence();
    if (!active) return;
    __shared__ uint32_t s_wp, s_tm;
    uint32_t n = n0;
    uint32_t epoch = rbase + first_round;
    uint32_t rounds = 0;
    if (threadIdx.x == 0) s_tm = 0;
    uint32_t* left = b.left;
    while (n > 0) {
        const unsigned long long keyhi = (unsigned long long)(~epoch) << 32;
        unsigned long long* owner = b.owner;
        // CLAIM (with the kill test)
        if (threadIdx.x == 0) s_wp = 0;
        __syncthreads();
        for (uint32_t base = 0; base < n; base += blockDim.x) {
            const uint32_t i = base + threadIdx.x;
            Ent<K> e;
            if (i < n) {
                if (rounds == 0 && base == 0) e = e0;  // (nothing has been written back yet)
                else load_ent<K>(e, left + (uint64_t)i * S);
            }
            __syncthreads();
            if (i < n) {
                uint64_t lb;
                const uint32_t len = ent_len<K>(cv, e, lb);
                bool killed = false;
                for (uint32_t j = 0; j < len; ++j)
                    killed |= __hip_atomic_load(&b.cover[lit_var(ent_lit<K>(cv, e, lb, j))], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) == stamp;
                if (!killed) {
                    const unsigned long long key = keyhi | prio(b, st, e.w[0]);
                    for (uint32_t j = 0; j < len; ++j)
                        __hip_atomic_fetch_min(&owner[vmix(b, lit_var(ent_lit<K>(cv, e, lb, j)))], key, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    store_ent<K>(left + (uint64_t)atomicAdd(&s_wp, 1u) * S, e);
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
            Ent<K> e;
            if (i < n) load_ent<K>(e, left + (uint64_t)i * S);
            __syncthreads();
            if (i < n) {
                const uint32_t c = e.w[0];
                const uint32_t kc = prio(b, st, c);
                uint64_t lb;
                const uint32_t len = ent_len<K>(cv, e, lb);
                bool own = true;
                for (uint32_t j = 0; j < len; ++j)
                    own &= __hip_atomic_load(&owner[vmix(b, lit_var(ent_lit<K>(cv, e, lb, j)))], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) == (keyhi | kc);
                if (own) {
                    for (uint32_t j = 0; j < len; ++j)
                        __hip_atomic_store(&b.cover[lit_var(ent_lit<K>(cv, e, lb, j))], (uint8_t)stamp, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    b.tmis[atomicAdd(&s_tm, 1u)] = c;
                    atomicAdd(&b.tile_stats[2 * (c / TILE)], mis_weight(b, st, kc));
                    atomicAdd(&b.tile_stats[2 * (c / TILE) + 1], (unsigned long long)len);
                } else {
                    store_ent<K>(left + (uint64_t)atomicAdd(&s_wp, 1u) * S, e);
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
        if (epoch > st->round_next) st->round_next = epoch;
        st->tail_rounds = rounds;
        st->tmis_cnt = s_tm;
        const uint32_t total = first_round + rounds;
        if (total > st->max_rounds) st->max_rounds = total;
        if (b.ktime) time_slot(b, st->n_iter - 1)[3] = wall_now();
    }
}

// ------------------------------------------------------------------------------------
// Resample (resample_clauses, SATInstance.h:340-365): the variables of the MIS clauses are
// exactly those with cover[v] == stamp.  Their new values come from one Philox draw per
// assignment word: variable v takes bit v % 32 of Philox(seed, {v / 32, it_lo, 0, it_hi}).x
// (it = resample round n_iter - 1; a variable repeated inside a clause is drawn once).  A lane
// reads the 8-bit stamps of 16 variables (one 16-byte load), 2 lanes OR their halves into a
// word's covered mask, and the first of them draws and writes the word: no per-clause atomics.
// n_resamples counts every literal (SATInstance.h:363) in the joins.
__device__ __forceinline__ uint32_t resample_word(uint64_t seed, uint64_t it, uint32_t w) {
    return philox_x(w, (uint32_t)it, 0u, (uint32_t)(it >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
}

__global__ __launch_bounds__(256) void k_resample_vars(LoopBuffers b) {
    const DevState* st = b.state;
    const int lane = threadIdx.x & 63;
    const bool lead = (lane & 1) == 0;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // variables 16t .. 16t+15
    const uint32_t w = (uint32_t)(t >> 1);
    const bool live = w < b.n_words;  // (cover is padded to whole words with zeros)
    // the stamps and the word are loaded with the loop state (one round trip)
    uint32_t a = 0;
    if (lead && live) a = b.A[w];
    uint4 c = make_uint4(0u, 0u, 0u, 0u);
    if (live) c = reinterpret_cast<const uint4*>(b.cover)[t];
    const uint32_t active = st->active, stamp = st->stamp;
    const uint64_t it = st->n_iter - 1;
    spec_fence();
    if (!active) return;
    const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
    uint32_t cm = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) cm |= (uint32_t)(((cs[i >> 2] >> (8 * (i & 3))) & 0xFFu) == stamp) << i;
    cm <<= 16 * (lane & 1);
    cm |= __shfl_xor(cm, 1, 64);
    if (lead && cm) b.A[w] = (a & ~cm) | (resample_word(b.seed, it, w) & cm);
}

// Allreduce exchange (ALLL_FLAG_EXCHANGE_ALLREDUCE): each rank resamples only the MIS clauses
// of its own shard into the XOR delta (old value of v is l & 1 because the clause is
// violated; MIS clauses are variable-disjoint); the delta is summed over ranks.
template <int K>
__device__ __forceinline__ void delta_clause(const ClauseView& cv, uint32_t* delta, uint32_t c, uint64_t it,
                                             uint32_t k0, uint32_t k1) {
    uint64_t lb, le;
    if constexpr (K > 0) { lb = (uint64_t)c * K; le = lb + K; }
    else { lb = cv.offs[c]; le = cv.offs[c + 1]; }
    for (uint64_t j = lb; j < le; ++j) {
        const uint32_t l = cv.lits[j] & LIT_MASK, v = l >> 1;
        bool dup = false;
        for (uint64_t q = lb; q < j; ++q) dup |= (lvar(cv, q) == v);
        if (dup) continue;
        const uint32_t nb = (philox_x(v >> 5, (uint32_t)it, 0u, (uint32_t)(it >> 32), k0, k1) >> (v & 31u)) & 1u;
        if (nb != (l & 1u)) atomicXor(&delta[v >> 5], 1u << (v & 31u));
    }
}

template <int K>
__global__ __launch_bounds__(ROUND_THREADS) void k_resample_delta(ClauseView cv, LoopBuffers b,
                                                                  uint32_t own_begin, uint32_t own_end) {
    const DevState* st = b.state;
    if (!st->active) return;
    const uint64_t it = st->n_iter - 1;
    const uint32_t k0 = (uint32_t)b.seed, k1 = (uint32_t)(b.seed >> 32);
    const uint32_t tile = blockIdx.x;
    if (tile == b.n_tiles) {
        const uint32_t cnt = st->tmis_cnt;
        for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
            const uint32_t c = b.tmis[i];
            const uint32_t t = c / TILE;
            if (t >= own_begin && t < own_end) delta_clause<K>(cv, b.delta, c, it, k0, k1);
        }
        return;
    }
    if (tile < own_begin || tile >= own_end) return;
    const uint32_t cnt = b.mis_cnt[tile];
    const uint32_t* mis = b.mis + (uint64_t)tile * TILE;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) delta_clause<K>(cv, b.delta, mis[i], it, k0, k1);
}

__global__ void k_apply_delta(LoopBuffers b) {
    if (!b.state->active) return;
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= b.n_words) return;
    const uint32_t d = b.delta[w];
    if (d) { b.A[w] ^= d; b.delta[w] = 0; }
}

// ------------------------------------------------------------------------------------
// Round-robin MIS of T > 1 clause chunks (populate_mis_parallel with T sets,
// SATInstance.h:414-447).  The reference keeps one list U_q of violated clauses per chunk q
// and a list of live sets; turn after turn, t <- (t + 1) % |sets|: an empty set is erased
// (t is not decremented, so its successor is skipped), otherwise the set's front clause joins
// the MIS and every clause sharing a variable with it is erased from every set.  A clause is
// erased exactly when one of its variables is covered by an MIS clause, so a set is a pointer
// into its sorted list, the front is the first clause at or after it with no covered variable,
// and the sequence of turns is the whole algorithm.
//
// k_rr_mw (the fallback of the fixpoint passes below) runs the turns in speculative batches.
// B = min(|sets|, groups) consecutive sets get a group (a one-wave workgroup) each; when every
// live set has a group, each group also runs D levels (its set's next D turns).  Turn l*B + g
// belongs to group g, level l.  A group scans its list 64 clauses per step (the loads of ST
// steps in flight together) and picks its next fronts greedily, assuming that only its own
// picks and the covered variables matter.  The batch is exact up to the first turn whose pick
// shares a variable with a pick of an earlier turn, and up to the first turn a group could not
// decide; those turns are committed (cover + MIS), and the first undecided turn of an exhausted
// set is its erasure.  Skipped clauses before a group's first uncommitted pick are erased for
// certain (covered by committed picks), so no scan is repeated.
constexpr uint32_t RR_KE = 8;                 // variables stored in a scan entry (k_rr_entries)
constexpr uint32_t RR_ROUNDS = 2;             // rounds of ST scan steps (loads issued together) per group per batch
constexpr uint32_t RR_EMPTY = 0xFFFFFFFFu;
constexpr unsigned long long RR_EMPTY64 = ~0ull;

__device__ __forceinline__ uint32_t rr_hash(uint32_t v, uint32_t bits) { return (v * 0x9E3779B1u) >> (32 - bits); }

// step hash of a group (2^sbits slots): lowest lane holding variable v; returns whether v was
// already present (another lane of the step holds it)
__device__ __forceinline__ bool rr_step_insert(unsigned long long* sk, uint32_t sbits, uint32_t v, uint32_t gl) {
    const unsigned long long me = ((unsigned long long)v << 32) | gl;
    uint32_t h = rr_hash(v, sbits);
    while (true) {
        unsigned long long cur = sk[h];
        if (cur == RR_EMPTY64) {
            cur = atomicCAS(&sk[h], RR_EMPTY64, me);
            if (cur == RR_EMPTY64) return false;
        }
        if ((uint32_t)(cur >> 32) == v) { atomicMin(&sk[h], me); return true; }
        h = (h + 1) & ((1u << sbits) - 1);
    }
}

// lanes holding rv[0..n) in the step hash (RR_EMPTY if absent), probes interleaved
template <uint32_t KR>
__device__ __forceinline__ void rr_step_lanes(const unsigned long long* sk, uint32_t sbits,
                                              const uint32_t (&rv)[KR], uint32_t n, uint32_t (&ml)[KR]) {
    uint32_t h[KR];
    uint32_t act = 0;
#pragma unroll
    for (uint32_t j = 0; j < KR; ++j) {
        h[j] = rr_hash(rv[j], sbits);
        ml[j] = RR_EMPTY;
        if (j < n) act |= 1u << j;
    }
    while (act) {
#pragma unroll
        for (uint32_t j = 0; j < KR; ++j) {
            if (!((act >> j) & 1u)) continue;
            const unsigned long long cur = sk[h[j]];
            if (cur == RR_EMPTY64) {
                act &= ~(1u << j);
            } else if ((uint32_t)(cur >> 32) == rv[j]) {
                ml[j] = (uint32_t)cur;
                act &= ~(1u << j);
            } else {
                h[j] = (h[j] + 1) & ((1u << sbits) - 1);
            }
        }
    }
}

// lane holding v in the step hash, or RR_EMPTY
__device__ __forceinline__ uint32_t rr_step_lane(const unsigned long long* sk, uint32_t sbits, uint32_t v) {
    uint32_t h = rr_hash(v, sbits);
    while (true) {
        const unsigned long long cur = sk[h];
        if (cur == RR_EMPTY64) return RR_EMPTY;
        if ((uint32_t)(cur >> 32) == v) return (uint32_t)cur;
        h = (h + 1) & ((1u << sbits) - 1);
    }
}

// Violated clauses of the iteration in clause order as scan entries {id, literal start, width,
// variables 0..7} (one 256-thread workgroup per tile; tile offsets from the evaluation's
// per-tile counts), so that a scan round of k_rr_mw is two dependent loads (entry, cover).
// the fixpoint passes decided this iteration's MIS (k_rr_mw then skips it)
__device__ __forceinline__ bool fp_settled(const LoopBuffers& b) {
    return b.fp_ctl && (b.fp_ctl->state == FP_FINAL || b.fp_ctl->state == FP_DONE);
}

struct RREnt {
    uint4 a;      // {clause id, literal start, width, hot-variable mask of slots 0..7}
    uint4 v0, v1; // variables 0..RR_KE-1 (RR_EMPTY past the width)
};
static_assert(sizeof(RREnt) == 16 + 4 * RR_KE, "scan entry = header + RR_KE variables");

// Workgroup exclusive scan of one value per thread (blockDim.x <= 1024); returns the total too.
__device__ __forceinline__ uint32_t fp_block_scan(uint32_t x, uint32_t* s_w, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t incl = wave_incl_add(x);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (uint32_t w = 0; w < nw; ++w) {
        const uint32_t c = s_w[w];
        if (w < wave) before += c;
        total += c;
    }
    __syncthreads();
    return before + incl - x;
}

// the timing log of pass p (FP_LOG_RW words; nullptr past FP_LOG_PASSES) and its round records
__device__ __forceinline__ uint32_t* fp_tlog(const LoopBuffers& b, uint32_t p) {
    // (measurement: only with ALLL_FLAG_KERNEL_TIMING)
    return b.fp_log && b.ktime && p < FP_LOG_PASSES ? b.fp_log + 4 * FP_LOG_PASSES + FP_LOG_RW * p : nullptr;
}
// k_fp_bbuild's phase stamps: the row after the passes' rows
__device__ __forceinline__ uint32_t* fp_tlog_bbuild(const LoopBuffers& b) {
    return b.fp_log && b.ktime ? b.fp_log + 4 * FP_LOG_PASSES + FP_LOG_RW * FP_LOG_PASSES : nullptr;
}
__device__ __forceinline__ void fp_tround(uint32_t* t, uint32_t r, uint32_t n) {
    if (t && r < FP_LOG_RW / 2 - 8) {
        t[8 + 2 * r] = n;
        t[9 + 2 * r] = (uint32_t)wall_now();
    }
}

// literal range of clause c: fixed width k (AoS) or the CSR offsets
__device__ __forceinline__ uint32_t cl_start(const ClauseView& cv, uint32_t c) { return cv.k ? c * cv.k : cv.offs[c]; }
__device__ __forceinline__ uint32_t cl_width(const ClauseView& cv, uint32_t c) {
    return cv.k ? cv.k : cv.offs[c + 1] - cv.offs[c];
}

// Fixed-width layout (the hybrid evaluation writes its violated clauses to per-tile lists in
// evaluation order): every violated clause sets its byte of the clause-order flag array
// rr_flag (a wave per evaluation tile; k_rr_entries reads the flags in clause order and clears
// them), so the scan entries come out in clause order as from the CSR evaluation's bitmask.
template <int K>
__global__ __launch_bounds__(256) void k_rr_mark(ClauseView cv, LoopBuffers b) {
    if (!b.state->active) return;
    constexpr int S = Ent<K>::S;
    const uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (tile >= b.n_tiles) return;
    const uint32_t cnt = b.tile_cnt[tile];
    const uint32_t* lin = b.stage[0] + (uint64_t)tile * TILE * S;
    constexpr uint32_t U = 4;  // entries in flight per lane
    for (uint32_t i0 = lane; i0 < cnt; i0 += 64 * U) {
        Ent<K> e[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
            if (i0 + 64 * u < cnt) load_ent<K>(e[u], lin + (uint64_t)(i0 + 64 * u) * S);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (i0 + 64 * u >= cnt) break;
            ent_unpack<K>(cv, e[u]);
            b.rr_flag[e[u].w[0]] = 1u;
        }
    }
}

// violated clauses per clause-order tile (flag mode), a wave per tile
__global__ __launch_bounds__(256) void k_rr_count(LoopBuffers b) {
    if (!b.state->active) return;
    const uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (tile >= b.n_tiles) return;
    const uint4* f = reinterpret_cast<const uint4*>(b.rr_flag + (uint64_t)tile * TILE);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t q = 0; q < TILE / 16 / 64; ++q) {  // flags are 0 / 1 bytes
        const uint4 x = f[q * 64 + lane];
        c += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if (lane == 0) b.rr_tcnt[tile] = c;
}

__global__ __launch_bounds__(256) void k_rr_entries(ClauseView cv, LoopBuffers b) {
    const uint32_t tile = blockIdx.x, tid = threadIdx.x;
    if (!b.state->active) {
        // The evaluation sets the flags before the reduce decides whether the iteration runs
        // (k_eval_flags): the last pass of a loop that stops here (solved, or capped by max_iters)
        // leaves its flags set.  Cleared now, so that a later run (alll_set_assignment + alll_run)
        // starts from clean flags.
        if (b.rr_flag) {
            uint4* fp = reinterpret_cast<uint4*>(b.rr_flag + (uint64_t)tile * TILE) + tid;
            const uint4 f = *fp;
            if (f.x | f.y | f.z | f.w) *fp = make_uint4(0u, 0u, 0u, 0u);
        }
        return;
    }
    if (tile == 0 && tid < 2 && b.rr_ctl) b.rr_ctl[tid] = 0u;  // k_rr_mw: barrier counter, MIS count
    __shared__ uint32_t s_part[4], s_wpre[TILE_WORDS + 1];
    __shared__ uint32_t s_ids[TILE];
    // clause-order counts of the earlier tiles: the flag counts (fixed width) or the CSR
    // evaluation's own tile counts
    const uint32_t* tcnt = b.rr_flag ? b.rr_tcnt : b.tile_cnt;
    uint32_t acc = 0;
    {  // (four independent loads in flight per step, not one load-wait-add per tile)
        uint32_t t = tid;
        for (; t + 768 < tile; t += 1024) acc += tcnt[t] + tcnt[t + 256] + tcnt[t + 512] + tcnt[t + 768];
        for (; t < tile; t += 256) acc += tcnt[t];
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((tid & 63) == 0) s_part[tid >> 6] = acc;
    if (b.rr_flag) {
        // 16 flags per thread (one 16-byte load), cleared for the next iteration once read
        uint4* fp = reinterpret_cast<uint4*>(b.rr_flag + (uint64_t)tile * TILE) + tid;
        const uint4 f = *fp;
        const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
        uint32_t bits = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) bits |= ((fw[q] >> (8 * e)) & 1u) << (4 * q + e);
        if (bits) *fp = make_uint4(0u, 0u, 0u, 0u);
        const uint32_t cnt = (uint32_t)__popc(bits);
        uint32_t tot;
        __shared__ uint32_t s_w[4];
        uint32_t o = fp_block_scan(cnt, s_w, tot);
        if (tid == 0) s_wpre[TILE_WORDS] = tot;
        while (bits) {
            s_ids[o++] = tile * TILE + 16u * tid + (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1;
        }
    } else {
        uint64_t x = 0;
        uint32_t cnt = 0, excl = 0;
        if (tid < TILE_WORDS) {
            const uint64_t c0 = (uint64_t)tile * TILE + 64u * tid;
            x = c0 < cv.m ? b.vmask[(uint64_t)tile * TILE_WORDS + tid] : 0ull;
            if (c0 < cv.m && cv.m - c0 < 64) x &= (1ull << (cv.m - c0)) - 1ull;
            cnt = (uint32_t)__popcll(x);
            uint32_t incl = cnt;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if ((int)tid >= o) incl += y;
            }
            excl = incl - cnt;
            if (tid == TILE_WORDS - 1) s_wpre[TILE_WORDS] = incl;
        }
        if (tid < TILE_WORDS) {
            uint32_t o = excl;
            while (x) {
                s_ids[o++] = tile * TILE + 64u * tid + (uint32_t)__builtin_ctzll(x);
                x &= x - 1;
            }
        }
    }
    __syncthreads();
    const uint32_t base = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    const uint32_t n = s_wpre[TILE_WORDS];
    RREnt* out = reinterpret_cast<RREnt*>(b.rr_u) + base;
    if (b.fp_ctl)  // the fixpoint's set starts in the entries: those that fall in this tile
        for (uint32_t s = tid; s < b.rr_T; s += 256) {
            const uint32_t key = b.rr_sets[s];
            if (key / TILE != tile || key >= cv.m) continue;
            uint32_t lo = 0, hi = n;  // this tile's violated clauses below the set start
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_ids[mid] < key) lo = mid + 1;
                else hi = mid;
            }
            b.fp_sf[s] = base + lo;
        }
    for (uint32_t i = tid; i < n; i += 256) {
        const uint32_t c = s_ids[i], lb = cl_start(cv, c), w = cl_width(cv, c);
        uint32_t v[8], hm = 0;  // hm: slots whose variable is hot (the fixpoint's degree count)
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t raw = j < w ? cv.lits[lb + j] : 0u;
            v[j] = j < w ? lit_var(raw) : RR_EMPTY;
            hm |= ((raw & LIT_HOT) ? 1u : 0u) << j;
        }
        const uint4 a = make_uint4(c, lb, w, hm), v0 = make_uint4(v[0], v[1], v[2], v[3]);
        if (b.fp_ctl && b.rr_k >= 1 && b.rr_k <= 4) {
            // narrow instances with the passes: the header, and the variables in the 16-byte copy
            // only (every reader of a narrow entry's variables takes them there); sole bytes
            // cleared (k_fp_bbuild sets them)
            out[i].a = a;
            b.fp_v4[base + i] = v0;
            if (!b.fp_lst) reinterpret_cast<uint32_t*>(b.fp_sole)[base + i] = 0u;
        } else {
            RREnt e;
            e.a = a;
            e.v0 = v0;
            e.v1 = make_uint4(v[4], v[5], v[6], v[7]);
            out[i] = e;
            if (b.fp_ctl && !b.fp_lst) reinterpret_cast<uint2*>(b.fp_sole)[base + i] = make_uint2(0u, 0u);
        }
    }
}

// Round-robin MIS across workgroups (k_rr_mw): the batches with every lane group in
// a workgroup of its own (one wave, one CU), so that the groups' scan steps -- chains of
// dependent LDS hash operations -- no longer share one CU.  What the groups shared in LDS moves
// to global memory:
//   * the test "did my group pick this variable?" needs only the group's own picks: an LDS hash
//     per workgroup (exact, no turn arithmetic);
//   * the first conflicting turn comes from a global hash (variable -> earliest turn) that every
//     group fills with its picks after its scan (interleaved CAS / min, one pass), each insert
//     that meets another turn offering the later one to an epoch-tagged maximum of ~turn;
//   * ncand / scan_end / exh per group, set pointers, the MIS count: global words.
// Two grid barriers per batch (a monotonic counter per iteration, zeroed by k_rr_entries; every
// spin bounded by a device-clock timeout).  Every workgroup keeps the same replicated live-set
// list and turn index and takes the same decisions from the same global words, so the batch
// sequence, its exact prefix and the set erasures are the same on every workgroup.
constexpr uint32_t RR_MW_MAX = 64;        // workgroups (groups per batch)
constexpr uint32_t RR_MW_VPG = 256;       // variables of a group's picks per batch
constexpr uint32_t RR_MW_CPG = 128;       // picks of a group per batch
constexpr uint32_t RR_MW_OWN = 1024;      // own-pick hash slots (keys)
constexpr unsigned long long RR_MW_TIMEOUT = 20000000ull;  // 200 ms at 100 MHz

struct RRMwCtl {  // (b.rr_ctl: RR_MW_CTL_WORDS words, zeroed at allocation)
    uint32_t bar, tm, epoch, wide_ep;
    uint32_t pad0[12];
    unsigned long long conf;  // (ep << 32) | ~first conflicting turn, by atomicMax
    unsigned long long pad1[7];
    uint32_t ncand[RR_MW_MAX], scan_end[RR_MW_MAX], exh[RR_MW_MAX];
};

static_assert(sizeof(RRMwCtl) <= 4 * RR_MW_CTL_WORDS, "control block");
struct RRMwLds {
    uint32_t okey[RR_MW_OWN];
    unsigned long long skey[512];
    uint32_t cc[RR_MW_CPG], cpos[RR_MW_CPG];
    // the variables of this group's picks in the batch (pick index, global hash slot)
    uint32_t ivar[RR_MW_VPG], ipick[RR_MW_VPG], islot[RR_MW_VPG];
    uint32_t nvar;
    uint32_t end[RR_TMAX];
    uint16_t live[RR_TMAX];
    uint16_t moved[RR_TMAX];
};

__device__ __forceinline__ bool rr_mw_own(const RRMwLds& L, uint32_t v) {
    uint32_t h = rr_hash(v, 10);
    while (true) {
        const uint32_t k = L.okey[h];
        if (k == v) return true;
        if (k == RR_EMPTY) return false;
        h = (h + 1) & (RR_MW_OWN - 1);
    }
}

template <uint32_t KR>
__device__ __forceinline__ bool rr_mw_own_any(const RRMwLds& L, const uint32_t (&rv)[KR], uint32_t n) {
    uint32_t h[KR];
    uint32_t act = 0;
#pragma unroll
    for (uint32_t j = 0; j < KR; ++j) {
        h[j] = rr_hash(rv[j], 10);
        if (j < n) act |= 1u << j;
    }
    bool own = false;
    while (act && !own) {
#pragma unroll
        for (uint32_t j = 0; j < KR; ++j) {
            if (!((act >> j) & 1u)) continue;
            const uint32_t k = L.okey[h[j]];
            if (k == rv[j]) { own = true; act &= ~(1u << j); }
            else if (k == RR_EMPTY) act &= ~(1u << j);
            else h[j] = (h[j] + 1) & (RR_MW_OWN - 1);
        }
    }
    return own;
}

__device__ __forceinline__ void rr_mw_own_insert(RRMwLds& L, uint32_t v) {
    uint32_t h = rr_hash(v, 10);
    while (true) {
        const uint32_t k = atomicCAS(&L.okey[h], RR_EMPTY, v);
        if (k == RR_EMPTY || k == v) return;
        h = (h + 1) & (RR_MW_OWN - 1);
    }
}

// grid barrier number k over nw workgroups (one wave each); false after a timeout
__device__ __forceinline__ bool rr_mw_barrier(RRMwCtl* ctl, uint32_t target) {
    uint32_t ok = 1;
    if ((threadIdx.x & 63) == 0) {
        __threadfence();
        atomicAdd(&ctl->bar, 1u);
        const unsigned long long t0 = wall_now();
        while (__hip_atomic_load(&ctl->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (wall_now() - t0 > RR_MW_TIMEOUT) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        __threadfence();
    }
    return __shfl(ok, 0, 64) != 0;
}

template <uint32_t KR, uint32_t ST>
__global__ __launch_bounds__(64) void k_rr_mw(ClauseView cv, LoopBuffers b) {
    DevState* st = b.state;
    if (!st->active || fp_settled(b)) return;
    extern __shared__ __align__(16) unsigned char rr_mw_lds_raw[];
    RRMwLds& L = *reinterpret_cast<RRMwLds*>(rr_mw_lds_raw);
    RRMwCtl* ctl = reinterpret_cast<RRMwCtl*>(b.rr_ctl);
    uint32_t* gkey = b.rr_gkey;
    uint32_t* gmin = b.rr_gmin;
    uint32_t* gptr = b.rr_ptr;
    const uint32_t stamp = st->stamp;
    const uint32_t lane = threadIdx.x;
    const uint32_t NW = gridDim.x, g = blockIdx.x;
    const uint32_t T = b.rr_T;
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    const bool v4 = b.fp_ctl && b.rr_k >= 1 && b.rr_k <= 4;  // (k_rr_entries: variables in fp_v4)
    const auto rsC = __builtin_amdgcn_make_buffer_rsrc(b.cover, (short)0, (int)b.n_vars, 0x00020000);
    const uint32_t nu = (uint32_t)st->u_total;
    const uint32_t base = __hip_atomic_load(&ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t nbar = 0;
    bool ok = true;
    // ---- sets: [lower_bound(start q), lower_bound(start q+1)) of U, spread over the workgroups
    for (uint32_t q = g * 64 + lane; q < T; q += NW * 64) {
        uint32_t bnd[2];
        for (int e = 0; e < 2; ++e) {
            const uint32_t key = b.rr_sets[q + e];
            uint32_t lo = 0, hi = nu;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (U[mid].a.x < key) lo = mid + 1; else hi = mid;
            }
            bnd[e] = lo;
        }
        __hip_atomic_store(&gptr[q], bnd[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&b.rr_end[q], bnd[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (uint32_t i = lane; i < RR_MW_OWN; i += 64) L.okey[i] = RR_EMPTY;
    if (lane == 0) L.nvar = 0;
    ok = rr_mw_barrier(ctl, ++nbar * NW);
    for (uint32_t q = lane; q < T; q += 64) {
        L.end[q] = __builtin_amdgcn_raw_buffer_load_b32(
            __builtin_amdgcn_make_buffer_rsrc(b.rr_end, (short)0, (int)(T * 4u), 0x00020000), q * 4u, 0, 16);
        L.live[q] = (uint16_t)q;
    }
    __syncthreads();
    uint32_t n_live = T, t = 0, batches = 0;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t sbits = 9u, shs = 1u << sbits, wcap = shs / 2;
    unsigned long long* sk = L.skey;
    while (ok && n_live > 0) {
        if (++batches > 2 * nu + 2 * T + 64) {
            if (g == 0 && lane == 0) { st->error = 1; st->done = 3; }
            break;
        }
        const uint32_t ep = base + batches;
        const uint32_t B = n_live < NW ? n_live : NW;
        const uint32_t D = (B == n_live) ? RR_MW_CPG : 1u;
        const uint32_t vpg = RR_MW_VPG;
        const uint32_t t0 = t;
        uint32_t nc = 0;
        bool wide = false;
        if (g < B) {
            // ---- scan: this group decides the next D turns of set live[(t + 1 + g) % n_live]
            const uint32_t s = L.live[(t0 + 1 + g) % n_live];
            uint32_t pos = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&gptr[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            const uint32_t end = L.end[s];
            uint32_t nv = 0, scan_end = pos, exhausted = 0;
            bool stop = false;
            for (uint32_t round = 0; round < RR_ROUNDS && !stop; ++round) {
                uint32_t c[ST], lb[ST], w[ST], rv[ST][KR];
                bool alive[ST];
#pragma unroll
                for (uint32_t u = 0; u < ST; ++u) {
                    const uint32_t i = pos + u * 64 + lane;
                    alive[u] = i < end;
                    RREnt e;
                    if (alive[u]) {
                        if (KR == 4 && v4) {  // (narrow entries keep their variables in fp_v4 only)
                            e.a = U[i].a;
                            e.v0 = b.fp_v4[i];
                        } else {
                            e = U[i];
                        }
                    } else {
                        e.a = make_uint4(0u, 0u, 0u, 0u);
                        e.v0 = e.v1 = make_uint4(RR_EMPTY, RR_EMPTY, RR_EMPTY, RR_EMPTY);
                    }
                    c[u] = e.a.x; lb[u] = e.a.y; w[u] = e.a.z;
                    const uint32_t ev[8] = {e.v0.x, e.v0.y, e.v0.z, e.v0.w, e.v1.x, e.v1.y, e.v1.z, e.v1.w};
#pragma unroll
                    for (uint32_t j = 0; j < KR; ++j) rv[u][j] = ev[j];
                }
                uint32_t cs[ST][KR];
#pragma unroll
                for (uint32_t u = 0; u < ST; ++u)
#pragma unroll
                    for (uint32_t j = 0; j < KR; ++j) cs[u][j] = __builtin_amdgcn_raw_buffer_load_b8(rsC, rv[u][j], 0, 16);
#pragma unroll
                for (uint32_t u = 0; u < ST; ++u) {
#pragma unroll
                    for (uint32_t j = 0; j < KR; ++j) alive[u] &= cs[u][j] != stamp;
                }
#pragma unroll
                for (uint32_t u = 0; u < ST; ++u)
                    for (uint32_t j = KR; j < w[u]; ++j)
                        alive[u] &= __builtin_amdgcn_raw_buffer_load_b8(rsC, lit_var(cv.lits[lb[u] + j]), 0, 16) != stamp;
#pragma unroll
                for (uint32_t u = 0; u < ST; ++u) {
                    if (stop) break;
                    const uint32_t pu = pos + u * 64;
                    if (pu >= end) { exhausted = 1; scan_end = end; stop = true; break; }
                    const uint32_t i = pu + lane;
                    bool al = alive[u];
                    auto var_of = [&](uint32_t j) -> uint32_t {
                        return j < KR ? rv[u][j] : lit_var(cv.lits[lb[u] + j]);
                    };
                    if (al && nc) {  // erased by an earlier pick of this group in the batch
                        al = !rr_mw_own_any(L, rv[u], w[u] < KR ? w[u] : KR);
                        for (uint32_t j = KR; al && j < w[u]; ++j)
                            if (rr_mw_own(L, var_of(j))) al = false;
                    }
                    uint64_t und = __ballot(al);
                    if (!und) continue;
                    // greedy (lane order) subset S of the live candidates
                    uint64_t S = 0;
                    while (und) {
                        const bool me = (und >> lane) & 1ull;
                        uint32_t wsum = me ? w[u] : 0u;
                        if (b.rr_k) {
                            wsum = me ? b.rr_k * ((uint32_t)__popcll(und & below) + 1u) : 0u;
                        } else {
                            for (uint32_t o = 1; o < 64; o <<= 1) {
                                const uint32_t y = __shfl_up(wsum, o, 64);
                                if (lane >= o) wsum += y;
                            }
                        }
                        const bool inwin = me && wsum <= wcap;
                        const uint32_t first = (uint32_t)__builtin_ctzll(und);
                        bool win = false, dead = false;
                        const bool wide_first = !((__ballot(inwin) >> first) & 1ull);
                        uint64_t W;
                        if (wide_first) {
                            win = lane == first;
                            const uint32_t lb0 = __shfl(lb[u], (int)first, 64);
                            const uint32_t w0 = __shfl(w[u], (int)first, 64);
                            for (uint32_t j0 = 0; j0 < w0; ++j0) {
                                const uint32_t v0 = lit_var(cv.lits[lb0 + j0]);
                                if (me && !win && !dead)
                                    for (uint32_t j = 0; j < w[u]; ++j) dead |= var_of(j) == v0;
                            }
                            W = __ballot(win);
                        } else {
                            for (uint32_t q = lane; q < shs; q += 64) sk[q] = RR_EMPTY64;
                            __builtin_amdgcn_wave_barrier();
                            bool dup = false;
                            if (inwin)
                                for (uint32_t j = 0; j < w[u]; ++j) dup |= rr_step_insert(sk, sbits, var_of(j), lane);
                            __builtin_amdgcn_wave_barrier();
                            const uint64_t wm = __ballot(inwin);
                            if (!__ballot(dup) && wm == und) {
                                win = me;
                                W = und;
                            } else {
                                uint32_t ml[KR];
                                rr_step_lanes(sk, sbits, rv[u], me ? (w[u] < KR ? w[u] : KR) : 0u, ml);
                                win = inwin;
#pragma unroll
                                for (uint32_t j = 0; j < KR; ++j) win &= j >= w[u] || ml[j] == lane;
                                for (uint32_t j = KR; win && j < w[u]; ++j) win = rr_step_lane(sk, sbits, var_of(j)) == lane;
                                W = __ballot(win);
                                if (me && !win) {
#pragma unroll
                                    for (uint32_t j = 0; j < KR; ++j)
                                        dead |= j < w[u] && ml[j] != RR_EMPTY && ((W >> ml[j]) & 1ull);
                                    for (uint32_t j = KR; !dead && j < w[u]; ++j) {
                                        const uint32_t q = rr_step_lane(sk, sbits, var_of(j));
                                        dead = q != RR_EMPTY && ((W >> q) & 1ull);
                                    }
                                }
                            }
                        }
                        const uint64_t Dm = __ballot(dead);
                        S |= W;
                        und &= ~(W | Dm);
                    }
                    // S in lane order, up to the level and variable capacities
                    const bool inS = (S >> lane) & 1ull;
                    const uint32_t rank = (uint32_t)__popcll(S & below);
                    uint32_t wincl = inS ? w[u] : 0u;
                    if (b.rr_k) {
                        wincl = inS ? b.rr_k * (rank + 1u) : 0u;
                    } else {
                        for (uint32_t o = 1; o < 64; o <<= 1) {
                            const uint32_t y = __shfl_up(wincl, o, 64);
                            if (lane >= o) wincl += y;
                        }
                    }
                    const bool picked = inS && nc + rank < D && nv + wincl <= vpg;
                    const uint64_t pm = __ballot(picked);
                    if (picked) {
                        const uint32_t idx = nc + rank;
                        L.cc[idx] = c[u];
                        L.cpos[idx] = i;
                        const uint32_t f = atomicAdd(&L.nvar, w[u]);  // (nv + wincl <= vpg: fits)
                        for (uint32_t j = 0; j < w[u]; ++j) {
                            const uint32_t v = var_of(j);
                            L.ivar[f + j] = v;
                            L.ipick[f + j] = idx;
                            rr_mw_own_insert(L, v);
                        }
                    }
                    const uint32_t np = (uint32_t)__popcll(pm);
                    if (np) {
                        const uint32_t lastp = 63u - (uint32_t)__builtin_clzll(pm);
                        nv += __shfl(wincl, (int)lastp, 64);
                    }
                    nc += np;
                    const uint64_t rest = S & ~pm;
                    if (rest) {
                        const uint32_t i0 = (uint32_t)__builtin_ctzll(rest);
                        stop = true;
                        scan_end = pu + i0;
                        if (np == 0 && nc == 0 && g == 0) {
                            // turn 0 is always exact: a pick too wide to record is committed alone
                            if (lane == i0) { L.cc[0] = c[u]; L.cpos[0] = i; }
                            wide = true;
                            nc = 1;
                            scan_end = pu + i0 + 1;
                        }
                    } else if (nc == D) {
                        stop = true;
                        scan_end = pu + 64 < end ? pu + 64 : end;
                    }
                }
                if (!stop) { pos += ST * 64; scan_end = pos; }
            }
            if (!stop && pos >= end) { exhausted = 1; scan_end = end; }
            __syncthreads();
            // ---- the picks' variables into the global hash (turn pick * B + g), RR_MW_VPG / 64
            // per lane, their slot claims issued together, then their minima; an insert that
            // meets another turn offers the later one to ctl->conf
            if (!wide) {
                constexpr uint32_t PL = RR_MW_VPG / 64;
                const uint32_t nvv = L.nvar;
                uint32_t v[PL], h[PL], tau[PL];
                uint32_t act = 0;
#pragma unroll
                for (uint32_t q = 0; q < PL; ++q) {
                    const uint32_t f = q * 64 + lane;
                    v[q] = f < nvv ? L.ivar[f] : RR_EMPTY;
                    tau[q] = f < nvv ? L.ipick[f] * B + g : RR_EMPTY;
                    h[q] = (v[q] * 0x9E3779B1u) >> (32 - 15);
                    if (f < nvv) act |= 1u << q;
                }
                const uint32_t have = act;
                while (act) {
                    uint32_t k[PL];
#pragma unroll
                    for (uint32_t q = 0; q < PL; ++q) k[q] = ((act >> q) & 1u) ? atomicCAS(&gkey[h[q]], 0u, v[q] + 1u) : 0u;
#pragma unroll
                    for (uint32_t q = 0; q < PL; ++q) {
                        if (!((act >> q) & 1u)) continue;
                        if (k[q] == 0u || k[q] == v[q] + 1u) act &= ~(1u << q);
                        else h[q] = (h[q] + 1) & (RR_MW_GH - 1);
                    }
                }
                uint32_t old[PL];
#pragma unroll
                for (uint32_t q = 0; q < PL; ++q) old[q] = ((have >> q) & 1u) ? atomicMin(&gmin[h[q]], tau[q]) : RR_EMPTY;
                unsigned long long worst = 0;
#pragma unroll
                for (uint32_t q = 0; q < PL; ++q) {
                    if ((have >> q) & 1u) L.islot[q * 64 + lane] = h[q];
                    if (old[q] != RR_EMPTY && old[q] != tau[q]) {
                        const uint32_t loser = old[q] > tau[q] ? old[q] : tau[q];
                        const unsigned long long cand = ((unsigned long long)ep << 32) | (uint32_t)~loser;
                        worst = cand > worst ? cand : worst;
                    }
                }
                for (int o = 32; o > 0; o >>= 1) {
                    const unsigned long long y = __shfl_xor(worst, o, 64);
                    worst = y > worst ? y : worst;
                }
                if (lane == 0 && worst) atomicMax(&ctl->conf, worst);
            } else if (lane == 0) {
                __hip_atomic_store(&ctl->wide_ep, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane == 0) {
                __hip_atomic_store(&ctl->ncand[g], nc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctl->scan_end[g], scan_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctl->exh[g], exhausted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // (the own-pick hash is cleared after the commit)
            if (!(ok = rr_mw_barrier(ctl, ++nbar * NW))) break;
            // ---- the exact prefix (identical in every workgroup)
        } else {
            if (!(ok = rr_mw_barrier(ctl, ++nbar * NW))) break;
        }
        const unsigned long long cf = __hip_atomic_load(&ctl->conf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool wide_all = __hip_atomic_load(&ctl->wide_ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ep;
        uint32_t trunc = (uint32_t)(cf >> 32) == ep ? ~(uint32_t)cf : RR_EMPTY;
        const uint32_t ncl = lane < B ? __hip_atomic_load(&ctl->ncand[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : D;
        uint32_t und = ncl < D ? ncl * B + lane : RR_EMPTY;
        for (int o = 32; o > 0; o >>= 1) und = min(und, (uint32_t)__shfl_xor(und, o, 64));
        trunc = min(trunc, und);
        trunc = wide_all ? 1u : min(trunc, D * B);
        // ---- commit this group's turns < trunc: covers, MIS, its set pointer; clear its hash slots
        if (g < B) {
            const uint32_t a_raw = trunc > g ? (trunc - g + B - 1) / B : 0u;
            const uint32_t a = a_raw < nc ? a_raw : nc;
            const uint32_t s = L.live[(t0 + 1 + g) % n_live];
            if (wide) {
                if (a) {
                    const uint32_t cl = L.cc[0], lbp = cl_start(cv, cl), wp = cl_width(cv, cl);
                    for (uint32_t j = lane; j < wp; j += 64)
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)stamp, rsC, lit_var(cv.lits[lbp + j]), 0, 16);
                }
            } else {
                const uint32_t nvv = L.nvar;
                for (uint32_t f = lane; f < nvv; f += 64) {
                    const uint32_t hs = L.islot[f];
                    gkey[hs] = 0u;
                    gmin[hs] = RR_EMPTY;
                    if (L.ipick[f] < a) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)stamp, rsC, L.ivar[f], 0, 16);
                }
            }
            uint32_t mb = 0;
            if (lane == 0 && a) mb = atomicAdd(&ctl->tm, a);
            mb = __shfl(mb, 0, 64);
            for (uint32_t p = lane; p < a; p += 64) b.tmis[mb + p] = L.cc[p];
            if (lane == 0) {
                const uint32_t se = __hip_atomic_load(&ctl->scan_end[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&gptr[s], a < nc ? L.cpos[a] : se, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            for (uint32_t i = lane; i < RR_MW_OWN; i += 64) L.okey[i] = RR_EMPTY;
            if (lane == 0) L.nvar = 0;
        }
        // ---- erasure at turn trunc, or the next turn index (replicated in every workgroup)
        bool erase = false;
        uint32_t idx_e = 0;
        if (trunc < D * B) {
            const uint32_t ge = trunc % B, le = trunc / B;
            const uint32_t nge = __hip_atomic_load(&ctl->ncand[ge], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t xge = __hip_atomic_load(&ctl->exh[ge], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            erase = le == nge && xge;
            idx_e = (t0 + 1 + trunc) % n_live;
        }
        if (erase) {
            for (uint32_t i = idx_e + lane; i + 1 < n_live; i += 64) L.moved[i] = L.live[i + 1];
            __syncthreads();
            for (uint32_t i = idx_e + lane; i + 1 < n_live; i += 64) L.live[i] = L.moved[i];
            __syncthreads();
            n_live -= 1;
            t = idx_e;  // t is not decremented: the next turn skips the moved-up set
        } else {
            t = (t0 + trunc) % n_live;
        }
        if (!(ok = rr_mw_barrier(ctl, ++nbar * NW))) break;
    }
    if (!ok) {  // a grid barrier timed out: the workgroups were not all resident (error 4)
        if (lane == 0) { st->error = 4; st->done = 3; }
        return;
    }
    // statistics of the MIS (per tile, like the LFMIS kernels), spread over the workgroups
    const uint32_t tm = __hip_atomic_load(&ctl->tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = g * 64 + lane; i < tm; i += NW * 64) {
        const uint32_t c = b.tmis[i];
        atomicAdd(&b.tile_stats[2 * (c / TILE)], 1ull);
        atomicAdd(&b.tile_stats[2 * (c / TILE) + 1], (unsigned long long)cl_width(cv, c));
    }
    if (g == 0 && lane == 0) {
        st->tmis_cnt = tm;
        st->tail_rounds = batches;
        if (batches > st->max_rounds) st->max_rounds = batches;
        __hip_atomic_store(&ctl->epoch, base + batches + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (b.ktime) time_slot(b, st->n_iter - 1)[3] = wall_now();
    }
}

// ------------------------------------------------------------------------------------
// Round robin as a fixpoint of LFMIS passes (SATInstance.h:414-447).
//
// The scan entries (k_rr_entries) list the violated clauses in clause order; set s is the
// entry range [sf[s], sf[s+1]).  In the reference's loop set s picks its front clause at each
// of its turns, so it reaches the entries after its l-th pick at one step, turn(s, l), and
// those steps depend on the sets' pick counts alone: the live sets take steps in cyclic order,
// a set is erased at its first turn after its last pick, and the set that moves into its place
// loses that cycle's turn (the schedule, k_fp_sched).  A clause is picked iff no clause sharing
// a variable was picked at an earlier (turn, entry).  So the picks P are the LFMIS under the
// priority (turn(s, level_P(x)), x), level_P(x) = P's picks before x in its set, and any P
// with P = LFMIS(priority_P) is the reference's MIS (by induction over the steps: at every step
// both take the same front, or erase the same set).  The passes iterate P <- LFMIS(priority_P)
// from a guess (picks spread at the previous iteration's density) until a pass reproduces its
// input -- about ten passes at 10M clauses.  An iteration that has not settled after fp_max
// passes (or whose owner epochs ran out) is decided by k_rr_mw, so every result is exact.
//
// LFMIS pass: CLAIM(r) / JOIN(r) grid rounds as in §4 with 64-bit keys
// {~epoch | turn | entry} on fp_owner (reset every iteration), FP_G grid rounds, then the
// one-workgroup k_fp_tail.  Picks are bit 0 of fp_in (bit 1: the previous pass's).
constexpr int FP_THREADS = 256;
constexpr uint32_t FP_PER = FP_B / FP_THREADS;  // entries per thread in the count / turn passes
static_assert(FP_PER == 8, "a thread's pick bytes are one 8-byte load");
constexpr uint32_t FP_RT = 256;        // entries per round tile (one per thread): many workgroups per CU
constexpr uint32_t FP_LDS_SEG_T = 32;     // k_fp_turn keeps the schedule in LDS up to this many sets
constexpr uint32_t FP_COUNT_GRID = 1024;  // workgroups of k_fp_count / k_fp_turn (grid-stride over blocks)
constexpr uint32_t FP_HEAVY = 64;         // claimant lists longer than this are reduced by waves

constexpr uint32_t FP_SEG = 2048;         // claimants per wave of k_fp_vmin's long-list workgroups
constexpr uint32_t FP_HEAVY_GRID = 512;   // ... their number (instances with hot variables)
// workgroups of the wave-per-tile rounds (512 / 1024 / 2048: 607 / 627 / 628 iterations/s at
// M, T = 16; the workgroup-per-tile kernels for these rounds: 605)
constexpr uint32_t FP_WGRID = 1024;
constexpr uint32_t FP_SCHED_LDS_BLK = 4096;  // k_fp_sched keeps the block offsets in LDS up to this many blocks

__device__ __forceinline__ unsigned long long fp_key(const LoopBuffers& b, uint32_t ep, uint32_t turn, uint32_t i) {
    const uint32_t sh = b.fp_tb + b.fp_ib;
    const unsigned long long epmax = (1ull << (64 - sh)) - 1ull;
    return ((epmax - ep) << sh) | ((unsigned long long)turn << b.fp_ib) | i;
}
// epochs one iteration may use (keys of later epochs are smaller)
__device__ __forceinline__ uint32_t fp_ep_budget(const LoopBuffers& b) {
    const uint32_t eb = 64 - b.fp_tb - b.fp_ib;
    return eb >= 31 ? 0x7FFFFFFFu : (1u << eb) - 1u;
}

// the variables of scan entry i: the entry's first 4 (KW = 4: every clause is that narrow),
// the next 4, then the CSR literals
template <uint32_t KW, typename F>
__device__ __forceinline__ void fp_for_vars(const ClauseView& cv, const RREnt* U, uint32_t i, const uint4& a,
                                            const uint4& v0, F&& f) {
    const uint32_t w = a.z;
    if (w > 0) f(v0.x);
    if (w > 1) f(v0.y);
    if (w > 2) f(v0.z);
    if (w > 3) f(v0.w);
    if constexpr (KW == 0) {
        if (w > 4) {
            const uint4 v1 = U[i].v1;
            f(v1.x);
            if (w > 5) f(v1.y);
            if (w > 6) f(v1.z);
            if (w > 7) f(v1.w);
            for (uint32_t j = 8; j < w; ++j) f(lit_var(cv.lits[a.y + j]));
        }
    }
}

// the same over the variables another violated clause also holds (bit j of `sole`: slot j's
// variable has no other claimant this iteration, so it is always owned and never covered by
// another pick; slots past 8 are always visited)
template <uint32_t KW, typename F>
__device__ __forceinline__ void fp_for_shared(const ClauseView& cv, const RREnt* U, uint32_t i, const uint4& a,
                                              const uint4& v0, uint32_t sole, F&& f) {
    const uint32_t w = a.z;
    if (w > 0 && !(sole & 1u)) f(v0.x);
    if (w > 1 && !(sole & 2u)) f(v0.y);
    if (w > 2 && !(sole & 4u)) f(v0.z);
    if (w > 3 && !(sole & 8u)) f(v0.w);
    if constexpr (KW == 0) {
        if (w > 4 && (sole & 0xF0u) != 0xF0u) {
            const uint4 v1 = U[i].v1;
            if (!(sole & 16u)) f(v1.x);
            if (w > 5 && !(sole & 32u)) f(v1.y);
            if (w > 6 && !(sole & 64u)) f(v1.z);
            if (w > 7 && !(sole & 128u)) f(v1.w);
        }
        for (uint32_t j = 8; j < w; ++j) f(lit_var(cv.lits[a.y + j]));
    }
}

// sole mask of an entry (bit j: slot j's variable has no other violated claimant this
// iteration; the entry's sole bytes, k_fp_bbuild): such a variable is always owned by the entry
// and never covered by another pick, so the claims, ownership and kill tests skip it.  One load
// that does not wait for the entry's variables
__device__ __forceinline__ uint32_t fp_bytes_bits(uint32_t x) {  // bytes 0 / 1 -> bits 0..3
    return (x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u);
}
template <uint32_t KW>
__device__ __forceinline__ uint32_t fp_sole_mask(const LoopBuffers& b, uint32_t i) {
    if (b.fp_lst) {
        // incremental passes: a sole slot is a claimant list of one (the entry itself), read from
        // the entry's list rows (k_fp_bbuild writes them anyway; the sole bytes would be another
        // scattered store per single-claimant variable).  Bits past the width are don't-care.
        constexpr uint32_t RW = KW == 4 ? 4u : 8u;
        const uint4* rows = reinterpret_cast<const uint4*>(b.fp_lst) + (uint64_t)i * (RW / 2);
        uint32_t m = 0;
#pragma unroll
        for (uint32_t h = 0; h < RW / 2; ++h) {
            const uint4 r2 = rows[h];
            m |= (r2.y == 1u ? 1u : 0u) << (2 * h);
            m |= (r2.w == 1u ? 1u : 0u) << (2 * h + 1);
        }
        return m;
    }
    if constexpr (KW == 4) {
        return fp_bytes_bits(reinterpret_cast<const uint32_t*>(b.fp_sole)[i]);
    } else {
        const uint2 x = reinterpret_cast<const uint2*>(b.fp_sole)[i];
        return fp_bytes_bits(x.x) | (fp_bytes_bits(x.y) << 4);
    }
}

// an entry's header and first 4 variables in a pass; narrow instances (one width <= 4) read
// the 16-byte copy k_rr_entries made (a third of the 48-byte scan entry's lines)
template <uint32_t KW>
__device__ __forceinline__ void fp_ent(const LoopBuffers& b, const RREnt* U, uint32_t i, uint4& a, uint4& v0) {
    if constexpr (KW == 4) {
        v0 = b.fp_v4[i];
        a = make_uint4(0u, 0u, b.rr_k, 0u);
    } else {
        a = U[i].a;
        v0 = U[i].v0;
    }
}

// largest s < T with sf[s] <= i (sf non-decreasing, sf[0] = 0): the set of entry i < nu
__device__ __forceinline__ uint32_t fp_set_of(const uint32_t* sf, uint32_t T, uint32_t i) {
    uint32_t lo = 0, hi = T;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sf[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

// wave-aggregated append of `i` to list `out` (counter `cnt`, LDS or global); every lane of the
// wave calls it
__device__ __forceinline__ void fp_append(bool keep, uint32_t i, uint32_t* cnt, uint32_t* out) {
    const unsigned long long bal = __ballot(keep);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == 0 && bal) base = atomicAdd(cnt, (uint32_t)__popcll(bal));
    base = __shfl(base, 0, 64);
    if (keep) out[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = i;
}

// The first pass's input: picks spread evenly over every set at density num / den.
__global__ __launch_bounds__(FP_THREADS) void k_fp_guess(LoopBuffers b) {
    const RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN) return;
    if (const uint32_t rs = ctl->restart)  // (the iteration's restart of owner epochs / cover serials)
        for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < b.n_vars; v += gridDim.x * blockDim.x) {
            if (rs & 1u) b.fp_owner[v] = ~0ull;
            if (rs & 2u) b.fp_cov[v] = 0;
        }
    __shared__ uint32_t s_sf[FP_TMAX + 1];
    const uint32_t T = b.rr_T, nu = ctl->nu;
    const unsigned long long num = ctl->guess_num, den = ctl->guess_den;
    for (uint32_t s = threadIdx.x; s <= T; s += blockDim.x) s_sf[s] = b.fp_sf[s];
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nu; i += gridDim.x * blockDim.x) {
        const unsigned long long pos = i - s_sf[fp_set_of(s_sf, T, i)];
        b.fp_in[i] = (uint8_t)((pos + 1) * num / den > pos * num / den);
    }
}

// Round 0 without atomics: the violated claimants of every shared variable (two or more) in
// per-variable lists built once per iteration, by variable buckets (bkt_width variables each,
// vmix order; as the bucketed round 0 of the one-set LFMIS, §4.1 of DESIGN.md):
//   k_fp_bscatter (workgroup per FP_BS_ENT scan entries): every claim {entry, variable} is
//     ranked in an LDS histogram of its bucket, the workgroup reserves its ranges in the
//     buckets' static pair regions (fp_breg: the bucket's literal occurrences) with one global
//     atomic per bucket, and the pairs are stored there;
//   k_fp_bbuild (workgroup per bucket): LDS counters per variable place each claimant in its
//     variable's static list region (fp_soff: the variable's literal occurrences); then per
//     variable: the single claimant as its round-0 owner and its sole byte
//     (fp_own0, for the whole iteration), the shared variables' list {start, count, variable}
//     (fp_sv, per bucket) and the segments of long lists (fp_heavy).
// Each pass's round-0 owner of a shared variable is then the minimum key over its list
// (k_fp_vmin, plain stores), which CLAIM(0)'s atomics computed before.
constexpr uint32_t FP_BS_PER = 8;                          // scan entries per thread of k_fp_bscatter
constexpr uint32_t FP_BS_ENT = FP_BS_PER * FP_THREADS;     // ... per workgroup
constexpr int FP_BB_THREADS = 1024;
// a pair's entry word: the entry index (below 2^FP_SLOT_SH) and the claim's slot (8: past the
// entry's 8 variables) above it
constexpr uint32_t FP_SLOT_SH = 28;
constexpr uint32_t FP_IMASK = (1u << FP_SLOT_SH) - 1u;

// slot j < 8 of an entry (narrow instances: the 16-byte copy)
__device__ __forceinline__ uint32_t fp_slot(const uint4& v0, const uint4& v1, uint32_t j) {
    const uint32_t v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    return v[j];
}

template <uint32_t KW>
__global__ __launch_bounds__(FP_THREADS) void k_fp_bscatter(ClauseView cv, LoopBuffers b) {
    const RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN) return;
    const uint32_t nu = ctl->nu, nb = b.n_bkt, tid = threadIdx.x;
    extern __shared__ uint32_t s_bs[];
    uint32_t* s_h = s_bs;                                   // nb: claims per bucket, then their bases
    uint32_t* s_breg = s_bs + nb;                           // nb: static pair regions
    uint16_t* s_rank = reinterpret_cast<uint16_t*>(s_bs + 2 * nb);  // FP_BS_ENT x 8 ranks
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    uint2* pairs = reinterpret_cast<uint2*>(b.fp_pairs);
    for (uint32_t k = tid; k < nb; k += FP_THREADS) s_breg[k] = b.fp_breg[k];
    auto ent = [&](uint32_t i, uint4& a, uint4& v0, uint4& v1) {
        if constexpr (KW == 4) {
            v0 = b.fp_v4[i];
            v1 = make_uint4(RR_EMPTY, RR_EMPTY, RR_EMPTY, RR_EMPTY);
            a = make_uint4(0u, 0u, b.rr_k, 0u);
        } else {
            a = U[i].a;
            v0 = U[i].v0;
            v1 = U[i].v1;
        }
    };
    constexpr uint32_t FP_JM = KW == 4 ? 4u : 8u;  // slots held in the entry
    for (uint32_t i0 = blockIdx.x * FP_BS_ENT; i0 < nu; i0 += gridDim.x * FP_BS_ENT) {
        for (uint32_t k = tid; k < nb; k += FP_THREADS) s_h[k] = 0u;
        // the chunk's entries, all loads first, kept in registers for the second phase
        uint4 ea[FP_BS_PER], e0[FP_BS_PER], e1[FP_BS_PER];
#pragma unroll
        for (uint32_t e = 0; e < FP_BS_PER; ++e) {
            const uint32_t i = i0 + e * FP_THREADS + tid;
            if (i < nu) ent(i, ea[e], e0[e], e1[e]);
            else ea[e].z = 0u;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t e = 0; e < FP_BS_PER; ++e) {  // ranks of slots 0..7 within this chunk
            const uint32_t i = i0 + e * FP_THREADS + tid;
            const uint32_t w = ea[e].z, w8 = w < 8u ? w : 8u;
            uint32_t off;
#pragma unroll
            for (uint32_t j = 0; j < FP_JM; ++j)
                if (j < w8)
                    s_rank[(e * FP_THREADS + tid) * 8 + j] =
                        (uint16_t)atomicAdd(&s_h[bucket_of(b, fp_slot(e0[e], e1[e], j), off)], 1u);
            if constexpr (KW == 0) {  // slots past 8 of wide clauses (rare): a global rank each
                for (uint32_t j = 8; j < w; ++j) {
                    const uint32_t v = lit_var(cv.lits[ea[e].y + j]);
                    const uint32_t bk = bucket_of(b, v, off);
                    pairs[s_breg[bk] + atomicAdd(&b.fp_bfill[bk], 1u)] = make_uint2(i | (8u << FP_SLOT_SH), v);
                }
            }
        }
        __syncthreads();
        for (uint32_t k = tid; k < nb; k += FP_THREADS) {  // this chunk's range in every bucket region
            const uint32_t c = s_h[k];
            s_h[k] = c ? s_breg[k] + atomicAdd(&b.fp_bfill[k], c) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t e = 0; e < FP_BS_PER; ++e) {
            const uint32_t i = i0 + e * FP_THREADS + tid;
            const uint32_t w8 = ea[e].z < 8u ? ea[e].z : 8u;
            uint32_t off;
#pragma unroll
            for (uint32_t j = 0; j < FP_JM; ++j) {
                if (j >= w8) break;
                const uint32_t v = fp_slot(e0[e], e1[e], j);
                pairs[s_h[bucket_of(b, v, off)] + s_rank[(e * FP_THREADS + tid) * 8 + j]] = make_uint2(i | (j << FP_SLOT_SH), v);
            }
        }
        __syncthreads();  // (s_h is reset for the next chunk)
    }
}

__global__ __launch_bounds__(FP_BB_THREADS) void k_fp_bbuild(LoopBuffers b) {
    RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN) return;
    const uint32_t bk = blockIdx.x, W = b.bkt_width, tid = threadIdx.x;
    const uint32_t xb = bk * W;  // first vmix slot of the bucket
    const uint32_t nw = min(W, b.bkt_span - xb);  // (vmix slots [0, bkt_span))
    extern __shared__ uint32_t s_bb[];
    uint32_t* s_cnt = s_bb;
    uint32_t* s_off = s_bb + W;
    uint32_t* s_first = s_bb + 2 * W;
    __shared__ uint32_t s_ns;
    const uint32_t n = b.fp_bfill[bk];
    constexpr uint32_t U4 = 4;  // loads in flight per thread
    uint32_t* tlb = bk == 0 && tid == 0 ? fp_tlog_bbuild(b) : nullptr;  // (phase stamps: measurement)
    if (tlb) tlb[0] = (uint32_t)wall_now();
    for (uint32_t w = tid; w < nw; w += FP_BB_THREADS) s_cnt[w] = 0u;
    if (tid == 0) s_ns = 0;
    __syncthreads();
    if (tlb) tlb[1] = (uint32_t)wall_now();
    if (tid == 0) b.fp_bfill[bk] = 0u;  // (read by every thread above; the next iteration's count)
    const uint2* P = reinterpret_cast<const uint2*>(b.fp_pairs) + b.fp_breg[bk];
    // The bucket's lists packed at the start of its region (the pairs' region bounds: fp_breg):
    // claims counted per variable, the counts scanned into list starts, then every claim placed.
    // (At static per-variable offsets -- every literal occurrence's slot -- the lists were sparse
    // and each claim's store a line of its own: the placement cost three times as much.)
    // rank / place: the lanes that share the first valid lane's variable take theirs from one
    // atomic (a hub's claims would serialise on one LDS word)
    auto grouped_add = [&](uint32_t* ctr, bool valid, uint32_t w) -> uint32_t {
        const unsigned long long vb = __ballot(valid);
        if (!vb) return 0u;
        const int fl = __ffsll((long long)vb) - 1;
        const uint32_t wl = __shfl(w, fl, 64);
        const bool grp = valid && w == wl;
        const unsigned long long same = __ballot(grp);
        uint32_t base = 0;
        if ((int)(tid & 63) == fl) base = atomicAdd(&ctr[wl], (uint32_t)__popcll(same));
        base = __shfl(base, fl, 64);
        if (!valid) return 0u;
        return grp ? base + (uint32_t)__popcll(same & ((1ull << (tid & 63)) - 1ull)) : atomicAdd(&ctr[w], 1u);
    };
    for (uint32_t k0 = tid; k0 < n; k0 += U4 * FP_BB_THREADS) {  // counts, first claimants
        uint2 p[U4];
#pragma unroll
        for (uint32_t u = 0; u < U4; ++u) {
            const uint32_t k = k0 + u * FP_BB_THREADS;
            p[u] = k < n ? P[k] : make_uint2(0u, ~0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < U4; ++u) {
            const bool valid = p[u].y != ~0u;
            const uint32_t w = valid ? vmix(b, p[u].y) - xb : 0u;
            const uint32_t r = grouped_add(s_cnt, valid, w);
            if (valid && r == 0) s_first[w] = p[u].x;
        }
    }
    __syncthreads();
    {  // list starts: a contiguous range of variables per thread, one workgroup scan
        const uint32_t per = (nw + FP_BB_THREADS - 1) / FP_BB_THREADS;
        const uint32_t w0 = min(nw, tid * per), w1 = min(nw, w0 + per);
        uint32_t sum = 0;
        for (uint32_t w = w0; w < w1; ++w) sum += s_cnt[w];
        __shared__ uint32_t s_sw[FP_BB_THREADS / 64];
        uint32_t tot;
        uint32_t o = b.fp_breg[bk] + fp_block_scan(sum, s_sw, tot);
        for (uint32_t w = w0; w < w1; ++w) {
            s_off[w] = o;
            o += s_cnt[w];
        }
    }
    __syncthreads();
    for (uint32_t k0 = tid; k0 < n; k0 += U4 * FP_BB_THREADS) {  // placement
        uint2 p[U4];
#pragma unroll
        for (uint32_t u = 0; u < U4; ++u) {
            const uint32_t k = k0 + u * FP_BB_THREADS;
            p[u] = k < n ? P[k] : make_uint2(0u, ~0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < U4; ++u) {
            const bool valid = p[u].y != ~0u;
            const uint32_t w = valid ? vmix(b, p[u].y) - xb : 0u;
            const uint32_t pos = grouped_add(s_off, valid, w);
            if (valid) b.fp_vlist[pos] = p[u].x & FP_IMASK;
        }
    }
    __syncthreads();
    for (uint32_t w = tid; w < nw; w += FP_BB_THREADS) s_off[w] -= s_cnt[w];  // (back to the starts)
    __syncthreads();
    if (tlb) tlb[2] = (uint32_t)wall_now();
    if (b.fp_lst) {
        // incremental passes: every claim's list {start, length} at its entry's slot (the repair
        // reads an entry's lists with its first load; slots past the list rows keep the rolled path)
        const uint32_t rw = b.rr_k >= 1 && b.rr_k <= 4 ? 4u : 8u;
        for (uint32_t k0 = tid; k0 < n; k0 += U4 * FP_BB_THREADS) {
            uint2 p[U4];
#pragma unroll
            for (uint32_t u = 0; u < U4; ++u) {
                const uint32_t k = k0 + u * FP_BB_THREADS;
                p[u] = k < n ? P[k] : make_uint2(0u, ~0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < U4; ++u) {
                const uint32_t j = p[u].x >> FP_SLOT_SH;
                if (p[u].y == ~0u || j >= rw) continue;
                const uint32_t w = vmix(b, p[u].y) - xb;
                reinterpret_cast<uint2*>(b.fp_lst)[(uint64_t)(p[u].x & FP_IMASK) * rw + j] = make_uint2(s_off[w], s_cnt[w]);
            }
        }
    }
    if (tlb) tlb[3] = (uint32_t)wall_now();
    // per variable (vmix slot order): the single claimant's ownership and sole byte, the shared
    // list and the long lists' segments
    uint4* sv = reinterpret_cast<uint4*>(b.fp_sv) + (uint64_t)bk * W;
    const uint32_t sw = b.rr_k >= 1 && b.rr_k <= 4 ? 4u : 8u;  // sole bytes per entry
    for (uint32_t w0 = 0; w0 < nw; w0 += FP_BB_THREADS) {  // (every thread runs every step: wave appends)
        const uint32_t w = w0 + tid;
        const uint32_t c = w < nw ? s_cnt[w] : 0u;
        const uint32_t v = c ? vunmix(b, xb + w) : 0u;
        // shared variables: one LDS atomic per wave for the list positions
        const bool shared = c > 1u;
        const unsigned long long bal = __ballot(shared);
        const uint32_t lane = tid & 63;
        uint32_t base = 0;
        if (lane == 0 && bal) base = atomicAdd(&s_ns, (uint32_t)__popcll(bal));
        base = __shfl(base, 0, 64);
        if (c && b.fp_sc) b.fp_sc[v] = make_uint2(s_off[w], c);  // (incremental passes: the list)
        if (c == 1u) {
            // (the ownership is read for slots past the sole bytes only: wide entries; the sole
            // byte, when there are no list rows to tell it: fp_sole_mask)
            const uint32_t x = s_first[w], i = x & FP_IMASK, j = x >> FP_SLOT_SH;
            if (sw == 8u) b.fp_own0[v] = i;
            if (j < sw && !b.fp_lst) b.fp_sole[(uint64_t)i * sw + j] = 1u;
        } else if (shared) {
            sv[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = make_uint4(s_off[w], c, v, 0u);
            if (c > FP_HEAVY) {  // long lists (hubs of skewed instances): a wave per FP_SEG claimants
                // (hot instances: their round claims go through LDS; from 16 or 32 claimants on
                // instead of 64: 173 vs 177 it/s at C5, T = 16)
                if (b.fp_hv) b.fp_hv[v] = (uint8_t)b.state->stamp;
                const uint32_t ns = (c + FP_SEG - 1) / FP_SEG;
                const uint32_t h0 = atomicAdd(&ctl->nheavy, ns);
                for (uint32_t k = 0; k < ns; ++k)
                    reinterpret_cast<uint4*>(b.fp_heavy)[h0 + k] =
                        make_uint4(v, s_off[w] + k * FP_SEG, s_off[w] + min(c, (k + 1) * FP_SEG), 0u);
            }
        }
    }
    __syncthreads();
    if (tlb) tlb[4] = (uint32_t)wall_now();
    if (tid == 0) b.fp_sbcnt[bk] = s_ns;
}

// Round 0 of a pass: the minimum key over every shared variable's claimants, FP_VS workgroups
// per bucket striding its shared list.  Variables with more than FP_HEAVY claimants (hubs of
// skewed instances) are left to the workgroups past the buckets: a wave per segment of FP_SEG
// claimants, lanes striding it; segments meet in the owner key by atomicMin (keys of this pass
// are below every earlier one), and JOIN(0) compares keys for such variables (own0 = ~0).
constexpr uint32_t FP_VS = 4;  // (1, 2, 4, 8: 444, 464, 461, 462 iterations/s at M, T = 16)
__global__ __launch_bounds__(FP_THREADS) void k_fp_vmin(LoopBuffers b) {
    const RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN || ctl->inc) return;  // (a full pass)
    const uint32_t ep = ctl->ep_base, nbw = b.n_bkt * FP_VS;
    if (blockIdx.x >= nbw) {
        const uint32_t nh = ctl->nheavy, lane = threadIdx.x & 63, hw = gridDim.x - nbw;
        for (uint32_t h = (blockIdx.x - nbw) * (FP_THREADS / 64) + (threadIdx.x >> 6); h < nh;
             h += hw * (FP_THREADS / 64)) {
            const uint4 sg = reinterpret_cast<const uint4*>(b.fp_heavy)[h];
            unsigned long long best = ~0ull;
            for (uint32_t o = sg.y + lane; o < sg.z; o += 64) {
                const uint32_t i = b.fp_vlist[o];
                const unsigned long long k = fp_key(b, ep, b.fp_turn[i], i);
                best = k < best ? k : best;
            }
            for (int sh = 32; sh > 0; sh >>= 1) {
                const unsigned long long y = __shfl_xor(best, sh, 64);
                best = y < best ? y : best;
            }
            if (lane == 0) {
                b.fp_own0[sg.x] = ~0u;
                atomicMin(&b.fp_owner[sg.x], best);
            }
        }
        return;
    }
    // the slices of bucket bk are workgroups bk + k n_bkt: one XCD for the bucket's lists when
    // n_bkt is a multiple of the 8 XCDs (workgroups are dealt to the XCDs round robin)
    const uint32_t bk = blockIdx.x % b.n_bkt, sl = blockIdx.x / b.n_bkt;
    const uint32_t ns = b.fp_sbcnt[bk];
    const uint4* sv = reinterpret_cast<const uint4*>(b.fp_sv) + (uint64_t)bk * b.bkt_width;
    for (uint32_t k = sl * FP_THREADS + threadIdx.x; k < ns; k += FP_VS * FP_THREADS) {
        const uint4 e = sv[k];
        if (e.y > FP_HEAVY) continue;
        // two claimants at a time (every list here has two or more)
        unsigned long long best = ~0ull;
        uint32_t o = e.x;
        const uint32_t end = e.x + e.y;
        for (; o + 1 < end; o += 2) {
            const uint32_t i0 = b.fp_vlist[o], i1 = b.fp_vlist[o + 1];
            const uint32_t t0 = b.fp_turn[i0], t1 = b.fp_turn[i1];
            const unsigned long long k0 = fp_key(b, ep, t0, i0), k1 = fp_key(b, ep, t1, i1);
            const unsigned long long k01 = k0 < k1 ? k0 : k1;
            best = k01 < best ? k01 : best;
        }
        if (o < end) {
            const uint32_t i = b.fp_vlist[o];
            const unsigned long long key = fp_key(b, ep, b.fp_turn[i], i);
            best = key < best ? key : best;
        }
        // JOIN(0) reads the winning entry from a 4-byte array (half the footprint of the keys;
        // marking the losers instead, a byte per entry, measured 4% slower).  The owner key
        // itself is not needed: the later rounds' claims are of later epochs, below any key
        // left here
        b.fp_own0[e.z] = (uint32_t)best & ((1u << b.fp_ib) - 1u);
    }
}

// One entry of CLAIM(r), r >= 1: out when a pick of this pass covers one of its shared
// variables, else it claims them (keep).
// Claims on the long lists' variables (hot instances) go through a workgroup's LDS table
// first (bounded probing; a claim that finds no slot goes to memory): a hub's claimants would
// otherwise serialise on one owner word.  fp_ht_flush sends one claim per variable, and only
// one that can still lower the owner key (keys only decrease).
struct FpHotTable {
    uint32_t* k;
    unsigned long long* v;
};
__device__ __forceinline__ void fp_ht_init(const FpHotTable& t) {
    for (uint32_t q = threadIdx.x; q < HOT_SLOTS; q += blockDim.x) { t.k[q] = 0xFFFFFFFFu; t.v[q] = ~0ull; }
}
__device__ __forceinline__ void fp_ht_claim(const FpHotTable& t, unsigned long long* owner, uint32_t var,
                                            unsigned long long key) {
    uint32_t h = (var * 2654435761u) & (HOT_SLOTS - 1);
    for (int probe = 0; probe < 32; ++probe) {
        const uint32_t prev = atomicCAS(&t.k[h], 0xFFFFFFFFu, var);
        if (prev == 0xFFFFFFFFu || prev == var) {
            __hip_atomic_fetch_min(&t.v[h], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        h = (h + 1) & (HOT_SLOTS - 1);
    }
    atomicMin(&owner[var], key);
}
__device__ __forceinline__ void fp_ht_flush(const FpHotTable& t, unsigned long long* owner) {
    for (uint32_t q = threadIdx.x; q < HOT_SLOTS; q += blockDim.x) {
        const uint32_t var = t.k[q];
        if (var == 0xFFFFFFFFu) continue;
        unsigned long long* o = &owner[var];
        if (t.v[q] < __hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(o, t.v[q]);
    }
}

template <uint32_t KW>
__device__ __forceinline__ bool fp_claim_one(const ClauseView& cv, const LoopBuffers& b, const RREnt* U, uint32_t i,
                                             uint32_t ep, uint32_t serial, uint32_t* hk, unsigned long long* hv,
                                             uint8_t stamp) {
    uint4 a, v0;
    fp_ent<KW>(b, U, i, a, v0);
    const uint32_t sole = fp_sole_mask<KW>(b, i);
    const uint32_t turn = b.fp_turn[i];
    bool dead = false;
    uint32_t dv = 0;  // a covered variable (its pick is the entry's blocker: incremental passes)
    fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
        const bool c = b.fp_cov[v] == (uint8_t)serial;
        if (c && !dead) dv = v;
        dead |= c;
    });
    if (dead) {
        if (b.fp_blocker) b.fp_blocker[i] = b.fp_covby[dv];
        return false;
    }
    const unsigned long long key = fp_key(b, ep, turn, i);
    fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
        if (hk && b.fp_hv[v] == stamp) fp_ht_claim(FpHotTable{hk, hv}, b.fp_owner, v, key);
        else atomicMin(&b.fp_owner[v], key);
    });
    return true;
}

// One entry of JOIN(r): picked when it holds every variable it claimed (its variables covered
// by this pass's serial); returns whether it survives to round r + 1.
template <uint32_t KW>
__device__ __forceinline__ bool fp_join_one(const ClauseView& cv, const LoopBuffers& b, const RREnt* U, uint32_t i,
                                            uint32_t r, uint32_t ep, uint32_t serial, uint32_t tpre) {
    uint4 a, v0;
    fp_ent<KW>(b, U, i, a, v0);
    // (a sole slot's variable is owned by the entry and covered by no other pick)
    const uint32_t sole = fp_sole_mask<KW>(b, i);
    const uint32_t turn = b.fp_turn[i];
    bool own = true, pre = false;
    if (r == 0 && turn < tpre) {  // decided as in the last pass (bit 1)
        pre = true;
        own = (b.fp_in[i] >> 1) & 1u;
    } else if (r == 0) {
        fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
            const uint32_t w = b.fp_own0[v];  // (~0: a long list, reduced into the key)
            own &= w == i || (w == ~0u && b.fp_owner[v] == fp_key(b, ep, turn, i));
        });
    } else {
        const unsigned long long key = fp_key(b, ep, turn, i);
        fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) { own &= b.fp_owner[v] == key; });
    }
    if (own) {
        fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
            b.fp_cov[v] = (uint8_t)serial;
            if (b.fp_covby) b.fp_covby[v] = i;
        });
        b.fp_in[i] = (uint8_t)(b.fp_in[i] | 1u);
    }
    return !own && !pre;
}

// JOIN(0), a workgroup per round tile of FP_RT entries (every entry of the pass): the
// survivors go to the tile's list (slots [tile * FP_RT, +count), counted in LDS: no global
// counter).
template <uint32_t KW>
__global__ __launch_bounds__(FP_THREADS) void k_fp_join0(ClauseView cv, LoopBuffers b) {
    constexpr uint32_t r = 0;
    RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN || ctl->inc) return;  // (a full pass)
    const uint32_t nu = ctl->nu;
    __shared__ uint32_t s_cnt;
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    const uint32_t ntile = (nu + FP_RT - 1) / FP_RT;
    const uint32_t ep = ctl->ep_base + r, serial = ctl->serial, tpre = ctl->tpre;
    for (uint32_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const uint32_t i0 = tile * FP_RT;
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
        const uint32_t n = min(FP_RT, nu - i0);
        uint32_t* lout = b.fp_list + i0;
        for (uint32_t j0 = 0; j0 < n; j0 += blockDim.x) {
            const uint32_t j = j0 + threadIdx.x;
            bool keep = false;
            uint32_t i = 0;
            if (j < n) {
                i = i0 + j;
                keep = fp_join_one<KW>(cv, b, U, i, r, ep, serial, tpre);
            }
            fp_append(keep, i, &s_cnt, lout);
        }
        __syncthreads();
        if (threadIdx.x == 0) b.fp_tcnt[tile] = s_cnt;
        __syncthreads();
    }
}

// Rounds r >= 1 (round 1: ~100 of a tile's 256 entries, then a few): CLAIM(r) / JOIN(r) with a
// wave per tile, no workgroup barriers; list positions from the wave's ballots.  (A workgroup
// per tile measured the same in round 1 and 3.5% slower overall.)
__device__ __forceinline__ uint32_t fp_wave_append(bool keep, uint32_t i, uint32_t kept, uint32_t* out) {
    const unsigned long long bal = __ballot(keep);
    const uint32_t lane = threadIdx.x & 63;
    if (keep) out[kept + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = i;
    return kept + (uint32_t)__popcll(bal);
}

template <uint32_t KW>
__global__ __launch_bounds__(FP_THREADS) void k_fp_wclaim(ClauseView cv, LoopBuffers b, uint32_t r) {
    const RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN || ctl->inc) return;  // (a full pass)
    const uint32_t nu = ctl->nu, lane = threadIdx.x & 63, wpb = FP_THREADS / 64;
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    const uint32_t ntile = (nu + FP_RT - 1) / FP_RT;
    const uint32_t ep = ctl->ep_base + r, serial = ctl->serial;
    __shared__ uint32_t s_hk[HOT_SLOTS];
    __shared__ unsigned long long s_hv[HOT_SLOTS];
    const bool hot = b.fp_hv != nullptr;
    const uint8_t stamp = hot ? (uint8_t)b.state->stamp : 0;
    if (hot) {
        fp_ht_init(FpHotTable{s_hk, s_hv});
        __syncthreads();
    }
    for (uint32_t tile = blockIdx.x * wpb + (threadIdx.x >> 6); tile < ntile; tile += gridDim.x * wpb) {
        const uint32_t i0 = tile * FP_RT;
        const uint32_t n = __builtin_amdgcn_readfirstlane(b.fp_tcnt[(2 * (r - 1)) * ntile + tile]);
        const uint32_t* lin = b.fp_list + i0;
        uint32_t* lout = b.fp_list + b.m + i0;
        uint32_t kept = 0;
        for (uint32_t j0 = 0; j0 < n; j0 += 64) {
            const uint32_t j = j0 + lane;
            bool keep = false;
            uint32_t i = 0;
            if (j < n) {
                i = lin[j];
                keep = fp_claim_one<KW>(cv, b, U, i, ep, serial, hot ? s_hk : nullptr, s_hv, stamp);
            }
            kept = fp_wave_append(keep, i, kept, lout);
        }
        if (lane == 0) b.fp_tcnt[(2 * r - 1) * ntile + tile] = kept;
    }
    if (hot) {  // (every wave of the workgroup reaches this barrier)
        __syncthreads();
        fp_ht_flush(FpHotTable{s_hk, s_hv}, b.fp_owner);
    }
}

template <uint32_t KW>
__global__ __launch_bounds__(FP_THREADS) void k_fp_wjoin(ClauseView cv, LoopBuffers b, uint32_t r) {
    // (the last grid round's lists are compacted by k_fp_tail: no contended counter)
    RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN || ctl->inc) return;  // (a full pass)
    const uint32_t nu = ctl->nu, lane = threadIdx.x & 63, wpb = FP_THREADS / 64;
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    const uint32_t ntile = (nu + FP_RT - 1) / FP_RT;
    const uint32_t ep = ctl->ep_base + r, serial = ctl->serial, tpre = ctl->tpre;
    for (uint32_t tile = blockIdx.x * wpb + (threadIdx.x >> 6); tile < ntile; tile += gridDim.x * wpb) {
        const uint32_t i0 = tile * FP_RT;
        const uint32_t n = __builtin_amdgcn_readfirstlane(b.fp_tcnt[(2 * r - 1) * ntile + tile]);
        const uint32_t* lin = b.fp_list + b.m + i0;
        uint32_t* lout = b.fp_list + i0;
        uint32_t kept = 0;
        for (uint32_t j0 = 0; j0 < n; j0 += 64) {
            const uint32_t j = j0 + lane;
            bool keep = false;
            uint32_t i = 0;
            if (j < n) {
                i = lin[j];
                keep = fp_join_one<KW>(cv, b, U, i, r, ep, serial, tpre);
            }
            kept = fp_wave_append(keep, i, kept, lout);
        }
        if (lane == 0) b.fp_tcnt[(2 * r) * ntile + tile] = kept;
    }
}

// The pass's remaining rounds in one workgroup (the lists are short by now).  Reads that other
// threads' atomics or stores of this launch decide go around L1 (agent-scope loads).
template <uint32_t KW>
__global__ __launch_bounds__(1024) void k_fp_tail(ClauseView cv, LoopBuffers b, uint32_t rg) {
    RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN || ctl->inc) return;  // (a full pass)
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    __shared__ uint32_t s_cnt, s_w[16];
    // the last grid round (rg - 1) left its survivors in per-tile lists (fp_list + tile * FP_RT,
    // counts in fp_tcnt): compacted into the other half of fp_list, a range of tiles per thread
    uint32_t* la = b.fp_list + b.m;
    uint32_t* lb = b.fp_list;
    uint32_t n;
    {
        const uint32_t ntile = (ctl->nu + FP_RT - 1) / FP_RT;
        const uint32_t* tc = b.fp_tcnt + (2 * (rg - 1)) * ntile;
        const uint32_t per = (ntile + blockDim.x - 1) / blockDim.x;
        const uint32_t t0 = min(ntile, threadIdx.x * per), t1 = min(ntile, t0 + per);
        uint32_t sum = 0;
        for (uint32_t t = t0; t < t1; ++t) sum += tc[t];
        uint32_t pos = fp_block_scan(sum, s_w, n);
        for (uint32_t t = t0; t < t1; ++t) {
            const uint32_t c = tc[t];
            for (uint32_t k = 0; k < c; ++k) la[pos + k] = lb[t * FP_RT + k];
            pos += c;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const uint32_t serial = ctl->serial, budget = fp_ep_budget(b);
    uint32_t ep = ctl->ep_base + rg;
    bool failed = false;
    while (n > 0) {
        if (ep >= budget) { failed = true; break; }
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
        for (uint32_t j0 = 0; j0 < n; j0 += blockDim.x) {  // CLAIM: la -> lb
            const uint32_t j = j0 + threadIdx.x;
            bool keep = false;
            uint32_t i = 0;
            if (j < n) {
                i = la[j];
                uint4 a, v0;
                fp_ent<KW>(b, U, i, a, v0);
                const uint32_t sole = fp_sole_mask<KW>(b, i);
                bool dead = false;
                uint32_t dv = 0;
                fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
                    const bool c = __hip_atomic_load(&b.fp_cov[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint8_t)serial;
                    if (c && !dead) dv = v;
                    dead |= c;
                });
                if (dead && b.fp_blocker)
                    b.fp_blocker[i] = __hip_atomic_load(&b.fp_covby[dv], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!dead) {
                    const unsigned long long key = fp_key(b, ep, b.fp_turn[i], i);
                    fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) { atomicMin(&b.fp_owner[v], key); });
                    keep = true;
                }
            }
            fp_append(keep, i, &s_cnt, lb);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const uint32_t nc = s_cnt;
        __syncthreads();
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
        for (uint32_t j0 = 0; j0 < nc; j0 += blockDim.x) {  // JOIN: lb -> la
            const uint32_t j = j0 + threadIdx.x;
            bool keep = false;
            uint32_t i = 0;
            if (j < nc) {
                i = lb[j];
                uint4 a, v0;
                fp_ent<KW>(b, U, i, a, v0);
                const uint32_t sole = fp_sole_mask<KW>(b, i);
                const unsigned long long key = fp_key(b, ep, b.fp_turn[i], i);
                bool own = true;
                fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
                    own &= __hip_atomic_load(&b.fp_owner[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key;
                });
                if (own) {
                    fp_for_shared<KW>(cv, U, i, a, v0, sole, [&](uint32_t v) {
                        if (b.fp_covby) __hip_atomic_store(&b.fp_covby[v], i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&b.fp_cov[v], (uint8_t)serial, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    });
                    b.fp_in[i] = (uint8_t)(b.fp_in[i] | 1u);
                }
                keep = !own;
            }
            fp_append(keep, i, &s_cnt, la);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        n = s_cnt;
        ++ep;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        ctl->ep_next = ep;
        ctl->ran = 1;
        if (failed) ctl->state = FP_FAIL;
    }
}

// Incremental passes.  A pass takes the last pass's picks P (the LFMIS of the
// last turns) to the LFMIS of the turns P implies.  The two differ only where the new turns change
// the order of an entry and a pick below it: every entry out of P keeps a *blocker* (a pick below
// it sharing a variable: the cover its full pass killed it by, or the pick its repair found), and
// it stays out for certain while that blocker stays below it and in P.  So the pass
//   * marks the entries whose blocker is no longer below them (k_fp_detect, every entry), then
//   * re-decides them in Jacobi rounds (k_fp_repair, one workgroup): an entry is in iff no pick of
//     the current decisions shares a variable with it and lies below it; a changed decision marks
//     the entries above it that share a variable with it for the next round.
// Decisions depend only on entries below, so the rounds end after the longest chain of changes
// (at M: a few thousand entries in at most ~8 rounds per pass, against ~800k entries and ~10
// kernels of a full pass).  Instances with hot variables keep the full passes (a hub's claimant
// list would be scanned per decision).
constexpr uint32_t FP_REP_QMAX = 1u << 20;  // entries whose decisions the repair keeps in LDS (128 KiB of bits):
                                            // iterations with more violated clauses keep the full passes
constexpr uint32_t FP_REP_MAXR = 4096;      // repair rounds per pass before it gives up

__device__ __forceinline__ unsigned long long fp_order_key(const LoopBuffers& b, uint32_t i) {
    return ((unsigned long long)b.fp_turn[i] << 32) | i;
}

// The incremental passes' buffers exist (alll_create allocates them only for instances without hot
// variables, b.fp_inc).  k_fp_detect and k_fp_repair load from them before they read the pass state
// (one round trip less): without them they stop the loop (state error 5, reported by the host)
// instead of dereferencing a null buffer.  (Round 5's fault: a hoisted fp_pbits load of k_fp_turn
// without its null test, on a power-law instance)
__device__ __forceinline__ bool fp_inc_buffers(const LoopBuffers& b) {
    return b.fp_inc && b.fp_blocker && b.fp_covby && b.fp_sc && b.fp_dl && b.fp_dmark && b.fp_pbits && b.fp_lst;
}
__device__ __forceinline__ void fp_inc_missing(const LoopBuffers& b) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        b.state->error = 5;
        b.state->done = 3;
        b.fp_ctl->state = FP_FAIL;
    }
}

__global__ __launch_bounds__(FP_THREADS) void k_fp_detect(LoopBuffers b) {
    RRFpCtl* ctl = b.fp_ctl;
    if (!fp_inc_buffers(b)) { fp_inc_missing(b); return; }  // (kernel arguments: a uniform branch)
    // (the first entry's pick byte, blocker and turn loaded before the state is read -- in bounds
    // of their buffers, independent of each other: one round trip less per pass)
    const uint32_t i1 = blockIdx.x * FP_THREADS + threadIdx.x;
    uint32_t p_in = 1, p_bk = 0, p_t = 0;
    if (i1 < b.m) {  // (the kernel runs with incremental passes only: fp_blocker exists)
        p_in = b.fp_in[i1];
        p_bk = b.fp_blocker[i1];
        p_t = b.fp_turn[i1];
    }
    // (the control words read together: no chain of scalar loads behind the branches)
    const uint32_t state = ctl->state, inc = ctl->inc, nu = ctl->nu, stamp = ctl->rep_serial;
    if ((state != FP_RUN) | (inc == 0)) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // (the wide rounds' barrier counter, k_fp_repair)
        if (uint32_t* t = fp_tlog(b, ctl->fp_iter)) t[0] = (uint32_t)wall_now();
        ctl->wlist = 0;
        ctl->wrounds = 0;
        ctl->wwork = 0;
        ctl->wfail = 0;
        ctl->wbar = 0;
    }
    for (uint32_t i0 = blockIdx.x * FP_THREADS; i0 < nu; i0 += gridDim.x * FP_THREADS) {
        const uint32_t i = i0 + threadIdx.x;
        const bool first = i == i1;
        bool d = false;
        if (i < nu && !((first ? p_in : b.fp_in[i]) & 1u)) {
            const uint32_t bk = first ? p_bk : b.fp_blocker[i];
            const unsigned long long ki = ((unsigned long long)(first ? p_t : b.fp_turn[i]) << 32) | i;
            d = bk >= nu || fp_order_key(b, bk) > ki;
            if (d) b.fp_dmark[i] = stamp;
        }
        fp_append(d, i, &ctl->ndirty, b.fp_dl);  // (every lane of the wave calls it)
    }
}

// The repair's view of an entry x: the claimant lists of its variables (fp_vlist; the entry's
// list rows {start, length} in fp_lst, k_fp_bbuild) hold its neighbours y != x.  A group of
// FP_LPE lanes decides one entry: lane u takes slots u and u + FP_LPE of the concatenated lists
// (FP_RN slots in all), so a decision is three dependent round trips (x's turn and list rows,
// the list slots, their turns and decisions) and a few dozen instructions per lane; the rare
// entry with more slots (or wider than its rows) has its group stride every list in turn.
// (One lane per entry with all FP_RN slots unrolled ran ~4x the instructions: a one-entry
// round took ~5 us; 16 lanes of one slot each: half the entries per step of a workgroup.  The
// rows loaded per decision from the variables and fp_sc instead of fp_lst: one more round trip,
// the same iteration time as the rows' scattered stores in k_fp_bbuild.)
constexpr uint32_t FP_RN = 16;   // list slots decided at once (the entry's own included: ~99.9% of the
                                 // dirty entries at M fit)
constexpr uint32_t FP_LPE = 8;        // lanes per entry in the one-workgroup rounds (2 slots per lane)
constexpr uint32_t FP_LPE_WIDE = 16;  // ... in the wide rounds (one step of the grid holds a round anyway;
                                      // 8 lanes per entry: ~1 us slower per wide round)

// decision of entry y in the repair's bits
__device__ __forceinline__ uint32_t fp_q(const uint32_t* sq, uint32_t y) { return (sq[y >> 5] >> (y & 31u)) & 1u; }
__device__ __forceinline__ unsigned long long fp_tkey(uint32_t t, uint32_t y) {
    return ((unsigned long long)t << 32) | y;
}

// One entry per group of FP_LPE lanes (x == ~0u: an idle group; every lane of the wave calls it).
// Decides x against the current decisions (pol.q), records its blocker, stores a changed
// decision (pol.set) and pushes the neighbours above a changed entry
// (pol.push, pol.push1: the next round's list).  Policies: FpPolLds (one workgroup, LDS bits and
// lists), FpPolWide (the wide rounds, global bits).
template <uint32_t KW, uint32_t LPE, typename P>
__device__ __forceinline__ void fp_grp_step(const ClauseView& cv, const LoopBuffers& b, const RREnt* U, uint32_t x,
                                            P& pol) {
    constexpr uint32_t RW = KW == 4 ? 4u : 8u;
    constexpr uint32_t FP_SPL = FP_RN / LPE;  // slots per lane
    const uint32_t lane = threadIdx.x & 63, gl = lane & (LPE - 1), g0 = lane & ~(LPE - 1);
    const bool act = x != ~0u;
    unsigned long long kx = 0;
    uint32_t w = 0, tot = 0, so[RW], cn[RW];
#pragma unroll
    for (uint32_t k = 0; k < RW; ++k) so[k] = cn[k] = 0;
    if (act) {
        // x's turn and list rows (every lane of the group loads the same words)
        kx = fp_tkey(b.fp_turn[x], x);
        w = KW == 4 ? b.rr_k : U[x].a.z;
        const uint4* rows = reinterpret_cast<const uint4*>(b.fp_lst) + (uint64_t)x * (RW / 2);
#pragma unroll
        for (uint32_t h = 0; h < RW / 2; ++h) {
            const uint4 r2 = rows[h];
            so[2 * h] = r2.x;
            cn[2 * h] = r2.y;
            so[2 * h + 1] = r2.z;
            cn[2 * h + 1] = r2.w;
        }
#pragma unroll
        for (uint32_t k = 0; k < RW; ++k) {
            if (k >= w) cn[k] = 0;
            tot += cn[k];
        }
    }
    const bool fast = act && w <= RW && tot <= FP_RN, slow = act && !fast;
    // fast: slots gl + t FP_LPE of the lists (all loads of a level in flight together)
    uint32_t y[FP_SPL];
#pragma unroll
    for (uint32_t t = 0; t < FP_SPL; ++t) {
        const uint32_t u = gl + t * LPE;
        y[t] = ~0u;
        if (fast && u < tot) {
            uint32_t r = u, pos = 0;
            bool found = false;
#pragma unroll
            for (uint32_t k = 0; k < RW; ++k) {
                if (!found && r < cn[k]) {
                    pos = so[k] + r;
                    found = true;
                } else if (!found) {
                    r -= cn[k];
                }
            }
            y[t] = b.fp_vlist[pos];
        }
    }
    bool above[FP_SPL];
    uint32_t by = ~0u;  // a pick below x sharing a variable (this lane's)
#pragma unroll
    for (uint32_t t = 0; t < FP_SPL; ++t) {
        above[t] = false;
        if (y[t] != ~0u && y[t] != x) {
            const unsigned long long ky = fp_tkey(b.fp_turn[y[t]], y[t]);
            if (ky < kx && pol.q(y[t])) by = y[t];
            above[t] = ky > kx;
        }
    }
    // slow: the group strides every list of the entry
    auto each = [&](auto f) {
        uint4 a, v0;
        fp_ent<KW>(b, U, x, a, v0);
        fp_for_vars<KW>(cv, U, x, a, v0, [&](uint32_t v) {
            const uint2 sc = b.fp_sc[v];
            const uint32_t s0 = sc.x, c = sc.y;
#pragma unroll 1
            for (uint32_t q = gl; q < c; q += LPE) {
                const uint32_t z = b.fp_vlist[s0 + q];
                if (z != x) f(z, fp_tkey(b.fp_turn[z], z));
            }
        });
    };
    if (slow)
        each([&](uint32_t z, unsigned long long kz) {
            if (kz < kx && pol.q(z)) by = z;
        });
    const uint32_t gm = (uint32_t)(__ballot(by != ~0u) >> g0) & ((1u << LPE) - 1u);
    const bool in = gm == 0;
    const uint32_t bky = __shfl(by, (int)(g0 + (gm ? (uint32_t)__ffs(gm) - 1u : 0u)), 64);
    bool ch = false;
    if (act && gl == 0) {
        if (!in) b.fp_blocker[x] = bky;
        ch = in != (pol.q(x) != 0);
        if (ch) pol.set(x, in);
    }
    const bool gch = (__ballot(ch) >> g0) & 1ull;
#pragma unroll
    for (uint32_t t = 0; t < FP_SPL; ++t) pol.push(gch && above[t], y[t]);
    if (__ballot(gch && slow))
        if (gch && slow)
            each([&](uint32_t z, unsigned long long kz) {
                if (kz > kx) pol.push1(z);
            });
}

constexpr uint32_t FP_RH_BITS = 12;  // LDS dedupe table of a repair round (4096 entry ids)
constexpr uint32_t FP_RL = 1024;     // dirty entries of a round kept in LDS (more: the global list; 128 + 16 + 8 KiB of LDS)

// true for the first caller with y since the table hk was cleared: an LDS hash (linear probing,
// slots only ever filled, so every caller with y sees the same window), the global stamp fp_dmark
// (rid) when y's probe window is full
__device__ __forceinline__ bool fp_rep_first(const LoopBuffers& b, uint32_t* hk, uint32_t y, uint32_t rid) {
    uint32_t h = (y * 0x9E3779B1u) >> (32 - FP_RH_BITS);
    bool fresh = false, found = false;
#pragma unroll 1
    for (int probe = 0; probe < 32 && !found; ++probe) {
        const uint32_t prev = atomicCAS(&hk[h], 0xFFFFFFFFu, y);
        fresh = prev == 0xFFFFFFFFu;
        found = fresh || prev == y;
        h = (h + 1) & ((1u << FP_RH_BITS) - 1u);
    }
    if (!found) fresh = atomicExch(&b.fp_dmark[y], rid) != rid;
    return fresh;
}

// cnt (< 32) consecutive slots of a list (LDS or global counter) for each active lane: one atomic per wave
// (thousands of lanes appending to one word serialise at the memory side otherwise); the lane's
// offset in the wave's range from one ballot per bit of cnt.  Returns the lane's first slot.
__device__ __forceinline__ uint32_t fp_wave_slots(uint32_t* ctr, uint32_t cnt) {
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t excl = 0, tot = 0;
#pragma unroll
    for (uint32_t bit = 0; bit < 5; ++bit) {
        const unsigned long long m = __ballot((cnt >> bit) & 1u);
        excl += (uint32_t)__popcll(m & below) << bit;
        tot += (uint32_t)__popcll(m) << bit;
    }
    const unsigned long long act = __ballot(true);
    const uint32_t leader = (uint32_t)__ffsll((long long)act) - 1u;
    uint32_t base = 0;
    if (lane == leader && tot) base = atomicAdd(ctr, tot);
    base = __shfl(base, (int)leader, 64);
    return base + excl;
}

struct FpPolLds {  // the one-workgroup rounds: decisions in LDS bits, LDS dedupe table and lists
    const LoopBuffers* b;
    uint32_t *sq, *hk, *nb, *lb, *gb;
    uint32_t rid;
    bool sp;  // (a push went to the global part of the list, read next round once this wave's stores completed)
    __device__ uint32_t q(uint32_t y) const { return fp_q(sq, y); }
    __device__ void set(uint32_t x, bool in) {
        if (in) atomicOr(&sq[x >> 5], 1u << (x & 31u));
        else atomicAnd(&sq[x >> 5], ~(1u << (x & 31u)));
    }
    __device__ void put(uint32_t i, uint32_t y) {
        if (i < FP_RL) {
            lb[i] = y;
        } else {
            gb[i] = y;
            sp = true;
        }
    }
    __device__ void push(bool c, uint32_t y) {  // (wave op)
        const bool f = c && fp_rep_first(*b, hk, y, rid);
        const uint32_t i = fp_wave_slots(nb, f ? 1u : 0u);
        if (f) put(i, y);
    }
    __device__ void push1(uint32_t y) {
        if (fp_rep_first(*b, hk, y, rid)) put(atomicAdd(nb, 1u), y);
    }
};

struct FpPolWide {  // the wide rounds: decisions in global bits; per workgroup an LDS dedupe table
                    // and its own segment of the next list
    const LoopBuffers* b;
    uint32_t *qg, *hk, *nb, *seg;
    uint32_t rid, cap;
    bool over;  // (the segment is full: the pass fails over to a full one)
    __device__ uint32_t q(uint32_t y) const { return fp_q(qg, y); }
    __device__ void set(uint32_t x, bool in) {
        if (in) atomicOr(&qg[x >> 5], 1u << (x & 31u));
        else atomicAnd(&qg[x >> 5], ~(1u << (x & 31u)));
    }
    __device__ void put(uint32_t i, uint32_t y) {
        if (i < cap) seg[i] = y;
        else over = true;
    }
    __device__ void push(bool c, uint32_t y) {  // (wave op)
        const bool f = c && fp_rep_first(*b, hk, y, rid);
        const uint32_t i = fp_wave_slots(nb, f ? 1u : 0u);
        if (f) put(i, y);
    }
    __device__ void push1(uint32_t y) {
        if (fp_rep_first(*b, hk, y, rid)) put(atomicAdd(nb, 1u), y);
    }
};

// the last pass's picks behind the working bits of fp_pbits (16-byte aligned)
__device__ __forceinline__ uint8_t* fp_pold(const LoopBuffers& b) {
    return b.fp_pbits + ((b.m / 8 + 64 + 15) & ~15u);
}

// The large early rounds of a repair across FP_RW_GRID workgroups (a single CU's memory-level
// parallelism bounds a round of thousands of decisions: ~34 us per 1,000 at M).  The decisions
// live in the global bits fp_pbits (atomic updates; every round starts after a grid barrier whose
// acquire fence drops stale L1 lines, within a round stale reads are allowed as in the one-
// workgroup rounds), the lists in fp_dl, dedup by the round stamps fp_dmark.  The kernel stops
// once a round holds at most FP_RW_MIN entries and hands the list, the change log and the round
// stamp over to k_fp_repair; a grid barrier that times out (workgroups not all resident) hands
// over as well, at a round boundary, so the result is the same either way.

__device__ __forceinline__ bool fp_rw_barrier(const LoopBuffers& b, RRFpCtl* ctl, uint32_t target) {
    __shared__ uint32_t s_ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t ok = 1;
        // release (the XCD L2's dirty lines written back: this workgroup's decisions and list
        // entries), then the arrival; acquire (the CU's L1 invalidated) after the poll.  (Two
        // __threadfence() -- each both -- cost more per round.)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the write-back completes before the arrival)
        atomicAdd(&ctl->wbar, 1u);
        const unsigned long long t0 = wall_now();
        while (__hip_atomic_load(&ctl->wbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (wall_now() - t0 > b.fp_rw_timeout) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the invalidate completes before the barrier below)
        if (!ok) atomicAdd(&ctl->rw_timeouts, 1u);  // (a slowdown the host can report: the pass gives up)
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// The wide rounds, by every workgroup of k_fp_repair's grid (groups of FP_LPE lanes, per-workgroup
// list segments; see above).  In: n, the detect list's length (list 0 of fp_dl); out: n, the
// rounds' last list (segments of list `cur`, starts s_pre) or the detect list when no round ran,
// the round stamp, rounds and entries decided.  Returns false when a barrier timed out or a
// segment overflowed (the pass gives up).
template <uint32_t KW>
__device__ bool fp_wide_rounds(const ClauseView& cv, const LoopBuffers& b, RRFpCtl* ctl, uint32_t* s_hk, uint32_t* s_pre,
                               uint32_t& n, uint32_t& rid, uint32_t& r, uint32_t& work, uint32_t& cur, uint32_t* tl) {
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    uint32_t* Q = reinterpret_cast<uint32_t*>(b.fp_pbits);  // the decisions, a bit per entry
    uint32_t* cnts = b.fp_dl + 3 * (size_t)b.m;  // [2][FP_RW_GRID]: the segments' lengths of a list
    const uint32_t G = gridDim.x, g = blockIdx.x, cap = b.m / G;  // (segment g of a list: cap entries at g cap)
    const uint32_t gpw = blockDim.x / FP_LPE_WIDE;  // groups per workgroup
    __shared__ uint32_t s_nb, s_over;
    bool ok = true;
    if (tl) tl[1] = (uint32_t)wall_now();
    if (threadIdx.x == 0) s_over = 0;
    while (n > b.fp_rw_min && n <= b.fp_rep_cap && ok && r < FP_REP_MAXR) {
        ++rid;
        work += n;
        const uint32_t* A = b.fp_dl + (size_t)cur * b.m;
        uint32_t* B = b.fp_dl + (size_t)(cur ^ 1) * b.m;
        for (uint32_t q = threadIdx.x; q < (1u << FP_RH_BITS); q += blockDim.x) s_hk[q] = 0xFFFFFFFFu;
        if (threadIdx.x == 0) s_nb = 0;
        __syncthreads();
        // a group of FP_LPE_WIDE lanes per entry (fp_grp_step); every lane runs every step
        FpPolWide pol{&b, Q, s_hk, &s_nb, B + (size_t)g * cap, rid, cap, false};
        const uint32_t ng = G * gpw;
        for (uint32_t j0 = 0; j0 < n; j0 += ng) {
            const uint32_t j = j0 + g * gpw + threadIdx.x / FP_LPE_WIDE;
            uint32_t x = ~0u;
            if (j < n) {
                if (r == 0) {
                    x = A[j];  // (k_fp_detect's list)
                } else {       // entry j of the segmented list
                    uint32_t lo = 0, hi = G;
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_pre[mid] <= j) lo = mid;
                        else hi = mid;
                    }
                    x = A[(size_t)lo * cap + (j - s_pre[lo])];
                }
            }
            fp_grp_step<KW, FP_LPE_WIDE>(cv, b, U, x, pol);
        }
        if (pol.over) s_over = 1;
        __syncthreads();
        if (threadIdx.x == 0) cnts[(size_t)((r + 1) & 1) * FP_RW_GRID + g] = s_over ? 0xFFFFFFFFu : s_nb;
        if (tl && r < 4) tl[56 + 2 * r] = (uint32_t)wall_now();  // (the round's decisions issued: measurement)
        ++r;
        ok = fp_rw_barrier(b, ctl, r * G);
        fp_tround(tl, r - 1, n);
        if (!ok) break;  // (the round is complete on this workgroup; the others may not be: fail)
        // the next list's segment starts (a full segment fails the pass)
        if (threadIdx.x < 64) {
            const uint32_t c = threadIdx.x < G ? cnts[(size_t)(r & 1) * FP_RW_GRID + threadIdx.x] : 0u;
            const bool bad = __ballot(c == 0xFFFFFFFFu) != 0;
            const uint32_t incl = wave_incl_add(bad ? 0u : c);
            if (threadIdx.x < G) s_pre[threadIdx.x + 1] = incl;
            if (threadIdx.x == 0) {
                s_pre[0] = 0;
                if (bad) s_over = 2;
            }
        }
        __syncthreads();
        if (s_over == 2) { ok = false; break; }
        n = s_pre[G];
        cur ^= 1;
    }
    return ok;
}

__device__ __forceinline__ void fp_sched_core(const LoopBuffers& b, RRFpCtl* ctl, int test, bool bail, uint32_t ch,
                                              uint32_t tmin, uint32_t* s_off, const uint32_t* sfp,
                                              const uint32_t* bndp, const uint32_t* blkp, uint32_t* tl);

// The end of an incremental pass: the rounds, then (as k_fp_count + k_fp_sched after a full
// pass) the pass test and the next pass's schedule, in this same workgroup: the block pick counts
// and the sets' in-block counts move by the pass's net changes only.
// One launch of FP_RW_GRID workgroups (all resident: one per CU by its LDS): every workgroup
// takes part in the wide rounds (fp_wide_rounds), then workgroup 0 alone runs the small rounds,
// the write-back, the pass test and the schedule.  (The wide rounds as a kernel of their own cost
// a launch per pass even when there was nothing for them: ~4.5 us.)
template <uint32_t KW>
__global__ __launch_bounds__(1024) void k_fp_repair(ClauseView cv, LoopBuffers b) {
    RRFpCtl* ctl = b.fp_ctl;
    if (!fp_inc_buffers(b)) { fp_inc_missing(b); return; }
    const uint32_t state = ctl->state;
    if (state == FP_FINAL) {  // (as k_fp_sched: the finalizing k_fp_turn has run)
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl->state = FP_DONE;
        return;
    }
    if (state != FP_RUN) return;
    if (!ctl->inc) {  // a full pass is due (one of the other kind in the graph): nothing to test
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl->skip = 1;
        return;
    }
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    extern __shared__ uint32_t s_q[];  // the current decisions, a bit per entry
    __shared__ uint32_t s_nb;
    __shared__ uint32_t s_hk[1u << FP_RH_BITS];
    __shared__ uint32_t s_l[2][FP_RL];  // the rounds' dirty lists (their first FP_RL entries)
    __shared__ uint32_t s_pre[FP_RW_GRID + 1];  // (the wide rounds' list segments)
    // global spill of the lists past FP_RL: index i of list c lives at s_l[c][i] or fp_dl[c m + i]
    const uint32_t nu = ctl->nu, nw = (nu + 31) / 32;
    const uint32_t n0 = ctl->ndirty;
    uint32_t n = n0, rid = ctl->rep_serial, rounds = 0, work = 0, cur = 0, wcur = 0;
    uint32_t* tl = blockIdx.x == 0 && threadIdx.x == 0 ? fp_tlog(b, ctl->fp_iter) : nullptr;
    bool bail = nu > FP_REP_QMAX;
    if (!bail) bail = !fp_wide_rounds<KW>(cv, b, ctl, s_hk, s_pre, n, rid, rounds, work, wcur, tl);
    if (blockIdx.x != 0) return;
    // (a wide round leaves at most fp_rw_min (<= FP_RL) entries unless the pass gives up: all in LDS below)
    if (rounds > 0 && n > FP_RL) bail = true;
    if (tl) tl[2] = (uint32_t)wall_now();
    if (n0 == 0 && rounds == 0 && !bail) {
        // nothing to repair: the picks repeat, the pass converged, and the counts and the
        // schedule (k_fp_turn finalizes with it) are the last pass's
        if (threadIdx.x == 0) {
            ctl->state = FP_FINAL;
            ctl->guess_num = ctl->total;
            ctl->guess_den = nu ? nu : 1u;
            ctl->changes = 0;
            ctl->pbsrc = 1;
            if (b.fp_log && ctl->fp_iter < FP_LOG_PASSES) {
                uint32_t* lg = b.fp_log + 4 * ctl->fp_iter;
                lg[0] = lg[1] = lg[2] = lg[3] = 0;
            }
            if (tl) tl[4] = (uint32_t)wall_now();
        }
        return;
    }
    // the block pick counts, set starts and their in-block counts (one each per thread: nblk <=
    // FP_REP_QMAX / FP_B, T < blockDim.x), loaded now, kept in LDS for the write-back and schedule
    const uint32_t T = b.rr_T, nblk = (nu + FP_B - 1) / FP_B;
    const bool lds_cnt = nu <= FP_REP_QMAX;
    uint32_t r_blk = 0, r_sf = 0, r_bnd = 0;
    if (lds_cnt) {
        if (threadIdx.x < nblk) r_blk = b.fp_blk[threadIdx.x];
        if (threadIdx.x <= T) { r_sf = b.fp_sf[threadIdx.x]; r_bnd = b.fp_bnd[threadIdx.x]; }
    }
    if (!bail) {
        // the decisions (the last pass's picks as packed by k_fp_turn, updated by the wide rounds)
        // into LDS (8 loads in flight per thread: up to 2^20 entries in one step of the
        // workgroup); k_fp_detect's list into the first list
        const uint4* src = reinterpret_cast<const uint4*>(b.fp_pbits);
        const uint32_t n4 = (nw + 3) / 4;
        for (uint32_t q0 = 0; q0 < n4; q0 += 8 * blockDim.x) {
            uint4 w[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                w[u] = q < n4 ? src[q] : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                const uint32_t e[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k)
                    if (4 * q + k < nw) s_q[4 * q + k] = e[k];
            }
        }
        // the list the wide rounds left (segments of list wcur) or k_fp_detect's (list 0) becomes
        // list 0 (LDS part + global part)
        if (rounds > 0) {
            const uint32_t* A = b.fp_dl + (size_t)wcur * b.m;
            const uint32_t G = gridDim.x, cap = b.m / G;
            for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
                uint32_t lo = 0, hi = G;
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_pre[mid] <= j) lo = mid;
                    else hi = mid;
                }
                s_l[0][j] = A[(size_t)lo * cap + (j - s_pre[lo])];  // (n <= FP_RL)
            }
        } else {
            for (uint32_t j = threadIdx.x; j < n && j < FP_RL; j += blockDim.x) s_l[0][j] = b.fp_dl[j];
        }
        __syncthreads();
        if (tl) tl[5] = (uint32_t)wall_now();
    }
    // Rounds over the dirty entries.  An entry's new decision is stored at once (the others of
    // the round may read it or the old one): whatever it read, an entry is dirty again in the
    // next round after any change of a neighbour below it, and decisions depend only on the
    // entries below, so the rounds settle on the exact LFMIS (the lowest dirty entry is final
    // after its first decision, and so on up).
    while (n > 0 && !bail) {
        if (n > b.fp_rep_cap || rounds >= FP_REP_MAXR) { bail = true; break; }
        ++rounds;
        ++rid;
        work += n;
        for (uint32_t q = threadIdx.x; q < (1u << FP_RH_BITS); q += blockDim.x) s_hk[q] = 0xFFFFFFFFu;
        if (threadIdx.x == 0) s_nb = 0;
        __syncthreads();
        const uint32_t* la = s_l[cur];
        const uint32_t* ga = b.fp_dl + (size_t)cur * b.m;
        uint32_t* lb = s_l[cur ^ 1];
        uint32_t* gb = b.fp_dl + (size_t)(cur ^ 1) * b.m;
        // a group of FP_LPE lanes per entry (fp_grp_step); every lane runs every step
        FpPolLds pol{&b, s_q, s_hk, &s_nb, lb, gb, rid, false};
        constexpr uint32_t NG = 1024 / FP_LPE;
        for (uint32_t j0 = 0; j0 < n; j0 += NG) {
            const uint32_t j = j0 + threadIdx.x / FP_LPE;
            fp_grp_step<KW, FP_LPE>(cv, b, U, j < n ? (j < FP_RL ? la[j] : ga[j]) : ~0u, pol);
        }
        const bool sp = pol.sp;
        // (only the next list's global part crosses waves within the rounds: the blockers are
        // read by the next pass)
        if (__ballot(sp)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        fp_tround(tl, rounds - 1, n);
        n = s_nb;
        cur ^= 1;
        __syncthreads();  // (the counters and the table are reset at the top of the next round)
    }
    // The net changes, word by word against the last pass's picks (the copy behind the working
    // bits); the blocks they fall in recounted from the decisions, with the in-block counts of
    // the set starts in them (LDS; the lists' space is free now); the decisions back into the
    // working bits, where k_fp_turn reads the picks (ctl->pbsrc); then the test and the next
    // schedule from the counts.
    __shared__ uint32_t s_ch;
    if (tl) tl[3] = (uint32_t)wall_now();
    uint32_t* s_blk = s_l[0];
    uint32_t* s_sf = s_l[1];
    uint32_t* s_bnd = s_l[1] + 512;  // (T + 1 <= 257)
    __shared__ uint8_t s_touch[FP_REP_QMAX / FP_B];  // blocks with changed decisions
    __syncthreads();  // (the last round's lists are read)
    if (threadIdx.x == 0) s_ch = 0;
    if (lds_cnt) {
        if (threadIdx.x < nblk) s_blk[threadIdx.x] = r_blk;
        if (threadIdx.x <= T) { s_sf[threadIdx.x] = r_sf; s_bnd[threadIdx.x] = r_bnd; }
    }
    for (uint32_t k = threadIdx.x; k < nblk; k += blockDim.x) s_touch[k] = 0;
    __syncthreads();  // (the rounds' blocker stores are for the next pass: no wait)
    if (!bail) {
        const uint4* old4 = reinterpret_cast<const uint4*>(fp_pold(b));
        uint4* wk4 = reinterpret_cast<uint4*>(b.fp_pbits);
        const uint32_t n4 = (nw + 3) / 4, tail = (nu & 31u) ? (1u << (nu & 31u)) - 1u : ~0u;
        uint32_t my_ch = 0;
        for (uint32_t q0 = 0; q0 < n4; q0 += 8 * blockDim.x) {  // (8 loads in flight per thread)
            uint4 o[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                o[u] = q < n4 ? old4[q] : make_uint4(0u, 0u, 0u, 0u);
            }
            // (stores after every load is consumed: a store between them made each step wait for
            // the previous store to complete)
            uint4 nqs[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                nqs[u] = make_uint4(0u, 0u, 0u, 0u);
                if (q >= n4) continue;
                // (a 16-byte group of words lies in one block: FP_B / 32 == 64 words)
                uint4 nq = make_uint4(s_q[4 * q], s_q[4 * q + 1], s_q[4 * q + 2], s_q[4 * q + 3]), oq = o[u];
                if (4 * q + 3 >= nw - 1) {  // (the last group: words past the entries masked)
                    const uint32_t m0 = 4 * q < nw - 1 ? ~0u : (4 * q == nw - 1 ? tail : 0u);
                    const uint32_t m1 = 4 * q + 1 < nw - 1 ? ~0u : (4 * q + 1 == nw - 1 ? tail : 0u);
                    const uint32_t m2 = 4 * q + 2 < nw - 1 ? ~0u : (4 * q + 2 == nw - 1 ? tail : 0u);
                    const uint32_t m3 = 4 * q + 3 == nw - 1 ? tail : 0u;
                    nq = make_uint4(nq.x & m0, nq.y & m1, nq.z & m2, nq.w & m3);
                    oq = make_uint4(oq.x & m0, oq.y & m1, oq.z & m2, oq.w & m3);
                }
                const uint4 d = make_uint4(nq.x ^ oq.x, nq.y ^ oq.y, nq.z ^ oq.z, nq.w ^ oq.w);
                if (d.x | d.y | d.z | d.w) {
                    s_touch[q / (FP_B / 128)] = 1;
                    my_ch += (uint32_t)(__popc(d.x) + __popc(d.y) + __popc(d.z) + __popc(d.w));
                }
                nqs[u] = nq;
            }
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t q = q0 + u * blockDim.x + threadIdx.x;
                if (q < n4) wk4[q] = nqs[u];
            }
        }
        const uint32_t wch = wave_incl_add(my_ch);
        if ((threadIdx.x & 63) == 63 && wch) atomicAdd(&s_ch, wch);
        __syncthreads();
        if (tl) tl[57] = (uint32_t)wall_now();  // (measurement: the comparison done)
        // the marked blocks' pick counts recounted from the decisions (a thread per block, its 64
        // words read in an order rotated by the block index so the threads' LDS reads spread over
        // the banks), and the in-block counts of the set starts in them (a thread per set, from the
        // top of the workgroup)
        for (uint32_t k = threadIdx.x; k < nblk; k += blockDim.x) {
            if (!s_touch[k]) continue;
            const uint32_t w0 = k * (FP_B / 32);  // (FP_B / 32 == 64 words per block)
            uint32_t c = 0;
#pragma unroll 8
            for (uint32_t i = 0; i < FP_B / 32; ++i) {
                const uint32_t wd = w0 + ((i + k) & (FP_B / 32 - 1u));
                uint32_t bits = wd < nw ? s_q[wd] : 0u;
                if (wd == nw - 1) bits &= tail;
                c += (uint32_t)__popc(bits);
            }
            s_blk[k] = c;
        }
        const uint32_t ts = blockDim.x - 1u - threadIdx.x;
        if (ts <= T) {
            const uint32_t f = s_sf[ts];
            if (f < nu && s_touch[f / FP_B]) {
                const uint32_t w0 = (f / FP_B) * (FP_B / 32), we = f / 32;
                uint32_t c = 0;
#pragma unroll 8
                for (uint32_t i = 0; i < FP_B / 32; ++i) {
                    const uint32_t wd = w0 + ((i + ts) & (FP_B / 32 - 1u));
                    if (wd < we) c += (uint32_t)__popc(s_q[wd]);
                }
                if (f & 31u) c += (uint32_t)__popc(s_q[we] & ((1u << (f & 31u)) - 1u));
                s_bnd[ts] = c;
            }
        }
        __syncthreads();  // (the working bits' stores are for the next kernels: no wait)
        if (tl) tl[59] = (uint32_t)wall_now();  // (measurement: the recount done)
    }
    if (threadIdx.x == 0) {
        ctl->rep_serial = rid + 1;
        ctl->rep_rounds += rounds;
        if (bail) ctl->bail = 1;
        ctl->pbsrc = bail ? 0u : 1u;
        if (b.fp_log && ctl->fp_iter < FP_LOG_PASSES) {
            uint32_t* lg = b.fp_log + 4 * ctl->fp_iter;
            lg[0] = n0;
            lg[1] = bail ? 0xFFFFFFFFu : rounds;
            lg[2] = work;
            lg[3] = bail ? 0u : s_ch;
        }
    }
    if (lds_cnt) {
        // (tmin 0: an incremental pass is followed by another, or by a full one after giving up; the
        // earliest changed turn serves full passes only)
        fp_sched_core(b, ctl, 1, bail, threadIdx.x == 0 ? s_ch : 0u, 0u, s_hk, s_sf, s_bnd, s_blk, tl);
        // (the counts for the next repair / k_fp_count's successor passes)
        if (threadIdx.x < nblk) b.fp_blk[threadIdx.x] = s_blk[threadIdx.x];
        if (threadIdx.x <= T) b.fp_bnd[threadIdx.x] = s_bnd[threadIdx.x];
    } else {
        fp_sched_core(b, ctl, 1, bail, threadIdx.x == 0 ? s_ch : 0u, 0u, nullptr, b.fp_sf, b.fp_bnd, b.fp_blk, tl);
    }
    if (tl) tl[4] = (uint32_t)wall_now();
}



// Picks per block of FP_B entries, picks before every set start that falls in the block, and
// (test) the picks that changed since the previous pass.
__global__ __launch_bounds__(FP_THREADS) void k_fp_count(LoopBuffers b, int test) {
    RRFpCtl* ctl = b.fp_ctl;
    if (ctl->state != FP_RUN || (test && !ctl->ran)) return;  // (no pass ran: nothing to test)
    __shared__ uint32_t s_w[FP_THREADS / 64], s_ex[FP_THREADS], s_bits[FP_THREADS];
    const uint32_t nu = ctl->nu, T = b.rr_T, nblk = (nu + FP_B - 1) / FP_B;
    uint32_t changed = 0, tmin = ~0u;
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const uint32_t i0 = blk * FP_B + threadIdx.x * FP_PER;
        unsigned long long x = 0;
        if (i0 < nu) {
            x = *reinterpret_cast<const unsigned long long*>(b.fp_in + i0);
            if (nu - i0 < FP_PER) x &= (1ull << (8 * (nu - i0))) - 1ull;
        }
        const unsigned long long b0 = x & 0x0101010101010101ull, b1 = (x >> 1) & 0x0101010101010101ull;
        const uint32_t cnt = (uint32_t)__popcll(b0);
        changed += (uint32_t)__popcll(b0 ^ b1);
        if (test && (b0 ^ b1)) {  // the earliest turn (of the last pass) whose decision changed
            const unsigned long long d = b0 ^ b1;
            for (uint32_t e = 0; e < FP_PER; ++e)
                if ((d >> (8 * e)) & 1ull) tmin = min(tmin, b.fp_turn[i0 + e]);
        }
        uint32_t total;
        const uint32_t ex = fp_block_scan(cnt, s_w, total);
        s_ex[threadIdx.x] = ex;
        s_bits[threadIdx.x] = (uint32_t)((b0 * 0x0102040810204080ull) >> 56);  // bit e = entry i0 + e
        __syncthreads();
        if (threadIdx.x == 0) b.fp_blk[blk] = total;
        for (uint32_t s = threadIdx.x; s <= T; s += blockDim.x) {
            const uint32_t f = b.fp_sf[s];
            if (f >= nu || f / FP_B != blk) continue;
            const uint32_t t = (f % FP_B) / FP_PER, e = f % FP_PER;
            b.fp_bnd[s] = s_ex[t] + (uint32_t)__popc(s_bits[t] & ((1u << e) - 1u));
        }
        __syncthreads();
    }
    if (test) {  // per workgroup (k_fp_sched sums them): no contended counter
        for (int o = 32; o > 0; o >>= 1) changed += __shfl_down(changed, o, 64);
        if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = changed;
        __syncthreads();
        if (threadIdx.x == 0) b.fp_blk[2 * (b.m / FP_B + 2) + blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        for (int o = 32; o > 0; o >>= 1) tmin = min(tmin, (uint32_t)__shfl_down(tmin, o, 64));
        __syncthreads();
        if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = tmin;
        __syncthreads();
        if (threadIdx.x == 0)
            b.fp_blk[2 * (b.m / FP_B + 2) + FP_COUNT_GRID + blockIdx.x] = min(min(s_w[0], s_w[1]), min(s_w[2], s_w[3]));
    }
}

// One workgroup: convergence, block offsets, picks per set, the schedule, the next pass.
// The schedule of the next pass from the block pick counts (fp_blk) and the set starts' in-block
// counts (fp_bnd), with the pass test: ch / tmin = this thread's share of the picks the pass
// changed and their earliest turn (OR / min over the workgroup here).  One workgroup; k_fp_sched
// (after k_fp_count) or the end of k_fp_repair (which updates the counts itself).  s_off: LDS
// for the block offsets (FP_SCHED_LDS_BLK words) or nullptr; sfp / bndp / blkp: the set starts,
// their in-block counts and the block counts (fp_sf, fp_bnd, fp_blk or LDS copies of them).
__device__ __forceinline__ void fp_sched_core(const LoopBuffers& b, RRFpCtl* ctl, int test, bool bail, uint32_t ch,
                                              uint32_t tmin, uint32_t* s_off, const uint32_t* sfp,
                                              const uint32_t* bndp, const uint32_t* blkp, uint32_t* tl) {
    __shared__ uint32_t s_w[16], s_e0;
    __shared__ uint32_t s_n[FP_TMAX], s_nseg[FP_TMAX], s_pf[FP_TMAX + 1];
    const uint32_t nu = ctl->nu, T = b.rr_T, nblk = (nu + FP_B - 1) / FP_B;
    uint32_t* blkoff = b.fp_blk + (b.m / FP_B + 2);
    const bool lds_off = s_off && nblk <= FP_SCHED_LDS_BLK;
    uint32_t sf[2], bnd[2];
    for (uint32_t q = 0; q < 2; ++q) {  // (T + 1 <= 2 * blockDim.x)
        const uint32_t s = threadIdx.x + q * blockDim.x;
        sf[q] = s <= T ? sfp[s] : 0u;
        bnd[q] = s <= T ? bndp[s] : 0u;
    }
    ch = __syncthreads_or(ch != 0);
    for (int o = 32; o > 0; o >>= 1) tmin = min(tmin, (uint32_t)__shfl_down(tmin, o, 64));
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = tmin;
    __syncthreads();
    tmin = s_w[0];
    for (uint32_t w = 1; w < (blockDim.x >> 6); ++w) tmin = min(tmin, s_w[w]);
    __syncthreads();
    const bool conv = test && ch == 0 && !bail;
    // exclusive scan of the block counts: a contiguous range per thread (independent loads),
    // one workgroup scan of the range sums
    const uint32_t per = (nblk + blockDim.x - 1) / blockDim.x;
    const uint32_t kb = min(nblk, threadIdx.x * per), ke = min(nblk, kb + per);
    uint32_t rsum = 0;
    for (uint32_t k = kb; k < ke; ++k) rsum += blkp[k];
    uint32_t total;
    uint32_t ex = fp_block_scan(rsum, s_w, total);
    for (uint32_t k = kb; k < ke; ++k) {
        const uint32_t x = blkp[k];
        blkoff[k] = ex;
        if (lds_off) s_off[k] = ex;
        ex += x;
    }
    __syncthreads();
    // picks before every set's first entry, picks per set
    for (uint32_t q = 0; q < 2; ++q) {
        const uint32_t s = threadIdx.x + q * blockDim.x;
        if (s > T) continue;
        const uint32_t f = sf[q];
        const uint32_t pf = f >= nu ? total : (lds_off ? s_off[f / FP_B] : blkoff[f / FP_B]) + bnd[q];
        s_pf[s] = pf;
        b.fp_pf[s] = pf;
    }
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < T; s += blockDim.x) {
        s_n[s] = s_pf[s + 1] - s_pf[s];
        s_nseg[s] = 0;
    }
    __syncthreads();
    if (tl) tl[6] = (uint32_t)wall_now();
    // schedule (wave 0): phases between erasures.  With L live sets and the turn index t, live
    // index x takes its j-th turn of the phase at step + j L + o(x), o(x) = (x - t - 1) mod L;
    // the first set to run out of picks is erased at its next turn E = step + min(r L + o), r =
    // picks left; then t = its index (the reference's t is not decremented).
    if (T <= 64) {
        // up to 64 sets: lane s keeps set s's state in registers, the live list is a lane mask
        // (live index = the lanes below it), and a phase is one wave minimum
        if (threadIdx.x < 64) {
            const uint32_t lane = threadIdx.x;
            const uint32_t n = s_n[lane < T ? lane : 0];
            // every key ((picks left) L + o) << 6 | lane fits 32 bits (a live key is never ~0u)
            const bool k32 = ((unsigned long long)nu + 1) * T * 64 + 64 < (1ull << 32);
            uint32_t done = 0, nseg = 0, t = 0, step = 0;
            unsigned long long alive = T == 64 ? ~0ull : (1ull << T) - 1ull;
            for (uint32_t p = 0; p < T; ++p) {
                const uint32_t L = (uint32_t)__popcll(alive);
                const bool live = (alive >> lane) & 1ull;
                const uint32_t x = (uint32_t)__popcll(alive & ((1ull << lane) - 1ull));
                // o = (x - t - 1) mod L, x < L; t <= L (the erased set's index among L + 1)
                uint32_t o = x + L - (t == L ? 0u : t) - 1;
                if (o >= L) o -= L;
                const uint32_t left = n - done;
                uint32_t ls;
                if (k32) {  // the wave minimum in 32 bits (DPP moves)
                    ls = wave_min_u32(live ? ((left * L + o) << 6 | lane) : ~0u) & 63u;
                } else {
                    unsigned long long best = live ? (((unsigned long long)left * L + o) << 6 | lane) : ~0ull;
                    for (int q = 32; q > 0; q >>= 1) {
                        const unsigned long long y = __shfl_xor(best, q, 64);
                        best = y < best ? y : best;
                    }
                    ls = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(best & 63u));
                }
                // the first set out: picks left r*, offset o*; it is erased at step + r* L + o*,
                // every other live set takes r* or r* + 1 turns before (no division)
                const uint32_t rs = (uint32_t)__builtin_amdgcn_readlane((int)left, (int)ls);
                const uint32_t os = (uint32_t)__builtin_amdgcn_readlane((int)o, (int)ls);
                const unsigned long long d = (unsigned long long)rs * L + os;
                if (live) {
                    const uint32_t cnt = lane == ls ? left : rs + (o < os ? 1u : 0u);
                    b.fp_seg[(uint64_t)lane * T + nseg] = make_uint4(done, step, L, o);
                    nseg += 1;
                    done += cnt;
                }
                const uint32_t E = step + (uint32_t)d;
                if (lane == 0) {
                    b.fp_erase[p] = E;
                    if (p == 0) s_e0 = E;
                }
                t = (uint32_t)__popcll(alive & ((1ull << ls) - 1ull));
                alive &= ~(1ull << ls);
                step = E + 1;
            }
            if (lane < T) s_nseg[lane] = nseg;
            if (lane == 0) ctl->n_steps = step;
        }
    } else if (threadIdx.x < 64) {
        // up to FP_TMAX sets: lane l keeps sets l, l + 64, l + 128, l + 192 in registers, the
        // live list is a mask of FP_TMAX / 64 words; a set that is not the phase's winner takes
        // r* or r* + 1 turns before the erasure (r* L + o* = the winner's key), no division
        constexpr uint32_t Q = FP_TMAX / 64;
        const uint32_t lane = threadIdx.x;
        uint32_t n[Q], done[Q], nseg[Q];
        unsigned long long alive[Q];
#pragma unroll
        for (uint32_t q = 0; q < Q; ++q) {
            const uint32_t s = lane + 64 * q;
            n[q] = s < T ? s_n[s] : 0u;
            done[q] = 0;
            nseg[q] = 0;
            alive[q] = T >= 64 * (q + 1) ? ~0ull : (T > 64 * q ? (1ull << (T - 64 * q)) - 1ull : 0ull);
        }
        const unsigned long long lt = (1ull << lane) - 1ull;
        uint32_t t = 0, step = 0;
        for (uint32_t p = 0; p < T; ++p) {
            uint32_t L = 0;
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) L += (uint32_t)__popcll(alive[q]);
            const uint32_t tl = t % L;
            unsigned long long best = ~0ull;
            uint32_t o[Q], below = 0;
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) {
                const uint32_t x = below + (uint32_t)__popcll(alive[q] & lt);
                o[q] = x + L - tl - 1;  // (x < L)
                if (o[q] >= L) o[q] -= L;
                if ((alive[q] >> lane) & 1ull) {
                    const unsigned long long key = (((unsigned long long)(n[q] - done[q]) * L + o[q]) << 8) | (lane + 64 * q);
                    best = key < best ? key : best;
                }
                below += (uint32_t)__popcll(alive[q]);
            }
            for (int sh = 32; sh > 0; sh >>= 1) {
                const unsigned long long y = __shfl_xor(best, sh, 64);
                best = y < best ? y : best;
            }
            const uint32_t ls = (uint32_t)(best & 255u);
            const unsigned long long d = best >> 8;
            const uint32_t rs = (d >> 32) ? (uint32_t)(d / L) : (uint32_t)d / L;
            const uint32_t os = (uint32_t)(d - (unsigned long long)rs * L);
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) {
                if (!((alive[q] >> lane) & 1ull)) continue;
                const uint32_t s = lane + 64 * q;
                const uint32_t cnt = s == ls ? n[q] - done[q] : rs + (o[q] < os ? 1u : 0u);
                b.fp_seg[(uint64_t)s * T + nseg[q]] = make_uint4(done[q], step, L, o[q]);
                nseg[q] += 1;
                done[q] += cnt;
            }
            const uint32_t E = step + (uint32_t)d;
            if (lane == 0) {
                b.fp_erase[p] = E;
                if (p == 0) s_e0 = E;
            }
            // t = the erased set's live index; then erase it
            uint32_t ti = 0;
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) {
                if ((ls >> 6) > q) ti += (uint32_t)__popcll(alive[q]);
                else if ((ls >> 6) == q) {
                    ti += (uint32_t)__popcll(alive[q] & ((1ull << (ls & 63u)) - 1ull));
                    alive[q] &= ~(1ull << (ls & 63u));
                }
            }
            t = ti;
            step = E + 1;
        }
#pragma unroll
        for (uint32_t q = 0; q < Q; ++q)
            if (lane + 64 * q < T) s_nseg[lane + 64 * q] = nseg[q];
        if (lane == 0) ctl->n_steps = step;
    }
    __syncthreads();
    if (tl) tl[7] = (uint32_t)wall_now();
    for (uint32_t s = threadIdx.x; s < T; s += blockDim.x) b.fp_nseg[s] = s_nseg[s];
    if (threadIdx.x == 0) {
        ctl->total = total;
        ctl->changes = 0;
        // The next pass keeps the decisions below min(earliest changed turn, both schedules'
        // first erasure): there the turns did not change, so neither did the sub-problem.
        const uint32_t e0 = s_e0;
        ctl->tpre = test && !bail ? min(tmin, min(e0, ctl->e0)) : 0u;
        ctl->e0 = e0;
        // the next pass: incremental once a full pass has run (test), unless this one gave up
        ctl->inc = test && b.fp_inc && !bail && nu <= FP_REP_QMAX && ctl->fp_iter + 1 >= b.fp_inc_after ? 1u : 0u;
        ctl->bail = 0;
        ctl->ndirty = 0;
        ctl->ran = 0;
        ctl->skip = 0;
        if (conv) {
            ctl->state = FP_FINAL;
            ctl->guess_num = total;
            ctl->guess_den = nu ? nu : 1u;
        } else {
            if (test) ctl->fp_iter += 1;
            ctl->ep_base = ctl->ep_next;
            ctl->serial = ctl->serial + 1u;  // 8-bit cover serials: at most 255 passes per iteration
            if (ctl->ep_base + FP_G_MAX + 1u >= fp_ep_budget(b) || ctl->serial > 255u) ctl->state = FP_FAIL;
        }
    }
}

// One workgroup after k_fp_count: convergence, block offsets, picks per set, the schedule, the
// next pass.
__global__ __launch_bounds__(256) void k_fp_sched(LoopBuffers b, int test) {
    RRFpCtl* ctl = b.fp_ctl;
    const uint32_t state = ctl->state;
    if (state == FP_FINAL) {  // the finalizing k_fp_turn has run
        if (threadIdx.x == 0) ctl->state = FP_DONE;
        return;
    }
    if (state != FP_RUN) return;
    if (test && !ctl->ran) {  // no pass ran (one of the other kind in the graph): nothing to test
        if (threadIdx.x == 0) ctl->skip = 1;
        return;
    }
    const bool bail = test && ctl->bail;  // the incremental pass gave up: its picks are no fixpoint test
    if (threadIdx.x == 0) ctl->pbsrc = 0;  // (a full pass: its picks are bit 0 of fp_in)
    __shared__ uint32_t s_off[FP_SCHED_LDS_BLK];  // block offsets (when they fit)
    const uint32_t nblk = (ctl->nu + FP_B - 1) / FP_B;
    // change counts and earliest changes of the k_fp_count workgroups
    uint32_t ch = 0, tmin = ~0u;
    if (test)
        for (uint32_t k = threadIdx.x; k < min(nblk, FP_COUNT_GRID); k += blockDim.x) {
            ch += b.fp_blk[2 * (b.m / FP_B + 2) + k];
            tmin = min(tmin, b.fp_blk[2 * (b.m / FP_B + 2) + FP_COUNT_GRID + k]);
        }
    fp_sched_core(b, ctl, test, bail, ch, tmin, s_off, b.fp_sf, b.fp_bnd, b.fp_blk, nullptr);
}

// a thread's MIS statistics of one clause tile into the block's LDS tally (tiles s_t0 ..
// s_t0 + 63; others straight to tile_stats)
__device__ __forceinline__ void fp_stat_add(const LoopBuffers& b, uint32_t t0, uint32_t* sn, uint32_t* sw, uint32_t tile,
                                            uint32_t n, unsigned long long w) {
    if (tile >= t0 && tile - t0 < 64 && w < (1ull << 31)) {
        atomicAdd(&sn[tile - t0], n);
        atomicAdd(&sw[tile - t0], (uint32_t)w);
    } else {
        atomicAdd(&b.tile_stats[2 * tile], (unsigned long long)n);
        atomicAdd(&b.tile_stats[2 * tile + 1], w);
    }
}

// Turns of every block of entries (grid-stride) for the next pass, or (fin) the MIS: picks in
// step order into tmis (step minus the erasures before it), their variables covered with the
// iteration's stamp, and the statistics of k_rr_mw.  blk_off(blk): picks before block blk.
// the first block's words of a thread (its picks both ways and the block's offset), loaded by
// k_fp_turn before it reads the state
struct FpTurnPre {
    uint32_t in, by, off;
    bool ok;
};

// k_fp_turn: FP_TPER entries per thread (half the count kernel's: twice the threads per block,
// half the per-thread chain of set and phase lookups; 10.1 -> 9.1 us per pass at M.  Two per
// thread, 1024-thread blocks: 13 us)
constexpr uint32_t FP_TPER = 4;
constexpr int FP_TURN_THREADS = FP_B / FP_TPER;

template <uint32_t KW, typename BlkOff>
__device__ __forceinline__ void fp_turn_blocks(const ClauseView& cv, const LoopBuffers& b, bool fin, bool inc, bool pb, uint32_t nu,
                                               uint32_t T, uint32_t stamp, const uint32_t* s_sf,
                                               const uint32_t* s_pf, const uint32_t* s_nseg, const uint32_t* s_er,
                                               const uint4* segs, uint32_t* s_w, BlkOff blk_off, FpTurnPre pre) {
    const RREnt* U = reinterpret_cast<const RREnt*>(b.rr_u);
    const uint32_t nblk = (nu + FP_B - 1) / FP_B;
    // (fin: the block's MIS statistics per clause tile in LDS -- its entries span a few
    // consecutive tiles from s_t0 on -- then one global add per tile; past FP_ST_TILES, direct)
    constexpr uint32_t FP_ST_TILES = 64;
    __shared__ uint32_t s_t0, s_stn[FP_ST_TILES], s_stw[FP_ST_TILES];
    for (uint32_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const uint32_t i0 = blk * FP_B + threadIdx.x * FP_TPER;
        if (fin) {
            if (threadIdx.x == 0) s_t0 = U[blk * FP_B].a.x / TILE;
            if (threadIdx.x < FP_ST_TILES) s_stn[threadIdx.x] = s_stw[threadIdx.x] = 0;
        }
        const bool first = pre.ok && blk == blockIdx.x;
        static_assert(FP_TPER == 2 || FP_TPER == 4, "FP_TPER pick bits and bytes of fp_in per thread");
        constexpr uint32_t TMASK = (1u << FP_TPER) - 1u;
        uint32_t x = 0;
        if (i0 < nu) {
            if (pb) {  // (after an incremental pass: its picks are bits; bits -> bit 0 of FP_TPER bytes)
                const uint32_t by = first ? pre.by : b.fp_pbits[i0 / 8];
                x = (((by >> (i0 & 7u)) & TMASK) * 0x00204081u) & 0x01010101u;
            } else {
                x = first ? pre.in : (FP_TPER == 4 ? *reinterpret_cast<const uint32_t*>(b.fp_in + i0)
                                                   : (uint32_t)*reinterpret_cast<const uint16_t*>(b.fp_in + i0));
            }
            if (nu - i0 < FP_TPER) x &= (1u << (8 * (nu - i0))) - 1u;
        }
        const unsigned long long b0 = x & 0x01010101u;
        uint32_t tot;
        uint32_t P = (first ? pre.off : blk_off(blk)) + fp_block_scan((uint32_t)__popcll(b0), s_w, tot);
        // the next pass sets bit 0 of its picks; these become bit 1 (k_fp_count compares them); an
        // incremental pass starts from them (bit 0 too), packed: the working bits it repairs and
        // the copy its net changes are taken against
        if (!fin) {
            const uint32_t fv = (uint32_t)((b0 << 1) | (inc ? b0 : 0ull));
            if (i0 < nu) {
                if (FP_TPER == 4) *reinterpret_cast<uint32_t*>(b.fp_in + i0) = fv;
                else *reinterpret_cast<uint16_t*>(b.fp_in + i0) = (uint16_t)fv;
            }
            if (inc) {  // (the first thread of each 8 entries stores their byte, OR-ed over the lanes)
                constexpr uint32_t TPB = 8 / FP_TPER;  // threads per byte
                uint32_t v = ((uint32_t)((b0 * 0x0102040810204080ull) >> 56) & TMASK) << (FP_TPER * (threadIdx.x % TPB));
#pragma unroll
                for (uint32_t o = 1; o < TPB; o <<= 1) v |= (uint32_t)__shfl_xor((int)v, (int)o, 64);
                if (threadIdx.x % TPB == 0 && i0 < nu) {
                    b.fp_pbits[i0 / 8] = (uint8_t)v;
                    fp_pold(b)[i0 / 8] = (uint8_t)v;
                }
            }
        }
        if (i0 < nu) {
            uint32_t s = fp_set_of(s_sf, T, i0);
            const uint32_t e1 = min(nu - i0, FP_TPER);
            uint32_t st_tile = ~0u, st_n = 0;  // MIS statistics of this thread's picks, per clause tile
            unsigned long long st_w = 0;
            // the phase record of the current set: found by binary search at the thread's first
            // entry of a set, then walked forward (levels do not decrease within a set)
            uint32_t rs = ~0u, lo = 0, ns = 0;
            const uint4* rec = segs;
            // (fin: the picks' headers and variables loaded together up front, not one pick's
            // chain after the other)
            uint4 pa[FP_TPER], pv[FP_TPER];
            if (fin) {
#pragma unroll
                for (uint32_t e = 0; e < FP_TPER; ++e) {
                    pa[e] = pv[e] = make_uint4(0u, 0u, 0u, 0u);
                    if (e < e1 && ((b0 >> (8 * e)) & 1ull)) {
                        pa[e] = U[i0 + e].a;
                        pv[e] = KW == 4 ? b.fp_v4[i0 + e] : U[i0 + e].v0;
                    }
                }
            }
#pragma unroll
            for (uint32_t e = 0; e < FP_TPER; ++e) {
                if (e >= e1) break;
                const uint32_t i = i0 + e;
                while (i >= s_sf[s + 1]) ++s;
                const bool pick = (b0 >> (8 * e)) & 1ull;
                if (!fin || pick) {
                    const uint32_t lev = P - s_pf[s];
                    // last phase record of s whose first level <= lev
                    if (s != rs) {
                        rs = s;
                        rec = segs + (uint64_t)s * T;
                        ns = s_nseg[s];
                        lo = 0;
                        uint32_t hi = ns;
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (rec[mid].x <= lev) lo = mid;
                            else hi = mid;
                        }
                    } else {
                        while (lo + 1 < ns && rec[lo + 1].x <= lev) ++lo;
                    }
                    const uint4 g = rec[lo];
                    const uint32_t turn = g.y + (lev - g.x) * g.z + g.w;
                    if (!fin) {
                        b.fp_turn[i] = turn;
                    } else {
                        uint32_t a = 0, z = T;  // erasures before the turn
                        while (a < z) {
                            const uint32_t mid = (a + z) >> 1;
                            if (s_er[mid] < turn) a = mid + 1;
                            else z = mid;
                        }
                        const uint4 ea = pa[e];
                        b.tmis[turn - a] = ea.x;
                        const uint4 v0 = pv[e];
                        fp_for_vars<KW>(cv, U, i, ea, v0, [&](uint32_t v) { b.cover[v] = (uint8_t)stamp; });
                        if (ea.x / TILE != st_tile) {
                            if (st_n) fp_stat_add(b, s_t0, s_stn, s_stw, st_tile, st_n, st_w);
                            st_tile = ea.x / TILE;
                            st_n = 0;
                            st_w = 0;
                        }
                        st_n += 1;
                        st_w += ea.z;
                    }
                }
                P += pick ? 1u : 0u;
            }
            if (st_n) fp_stat_add(b, s_t0, s_stn, s_stw, st_tile, st_n, st_w);
        }
        __syncthreads();
        if (fin) {
            if (threadIdx.x < FP_ST_TILES && s_stn[threadIdx.x]) {
                atomicAdd(&b.tile_stats[2 * (s_t0 + threadIdx.x)], (unsigned long long)s_stn[threadIdx.x]);
                atomicAdd(&b.tile_stats[2 * (s_t0 + threadIdx.x) + 1], (unsigned long long)s_stw[threadIdx.x]);
            }
            __syncthreads();  // (s_t0 and the tally are rewritten for the next block)
        }
    }
}

// Turns of every entry for the next pass (RUN), or, after the converged pass (FINAL), the MIS
// (fp_turn_blocks), from the schedule k_fp_sched wrote.
template <uint32_t KW>
__global__ __launch_bounds__(FP_TURN_THREADS) void k_fp_turn(ClauseView cv, LoopBuffers b) {
    const RRFpCtl* ctl = b.fp_ctl;
    const uint32_t T = b.rr_T;
    const uint32_t* blkoff = b.fp_blk + (b.m / FP_B + 2);
    // The first block's words and the schedule's tables are loaded before the state is read (each
    // load within its buffer, none depending on another): one round trip before the first block
    // instead of three.
    FpTurnPre pre{0u, 0u, 0u, false};
    if (blockIdx.x < (b.m + FP_B - 1) / FP_B) {
        const uint32_t i1 = blockIdx.x * FP_B + threadIdx.x * FP_TPER;
        pre.in = FP_TPER == 4 ? *reinterpret_cast<const uint32_t*>(b.fp_in + i1)  // (fp_in: m + FP_B bytes)
                              : (uint32_t)*reinterpret_cast<const uint16_t*>(b.fp_in + i1);
        pre.by = b.fp_pbits && i1 < b.m ? b.fp_pbits[i1 / 8] : 0u;  // (fp_pbits: incremental passes only)
        pre.off = blkoff[blockIdx.x];
        pre.ok = true;
    }
    const uint32_t s1 = threadIdx.x;  // (set s1 <= T; sets past the block below)
    uint32_t t_sf = 0, t_pf = 0, t_ns = 0, t_er = 0;
    if (s1 <= T) {
        t_sf = b.fp_sf[s1];
        t_pf = b.fp_pf[s1];
        if (s1 < T) { t_ns = b.fp_nseg[s1]; t_er = b.fp_erase[s1]; }
    }
    const bool lds_seg = T <= FP_LDS_SEG_T;
    constexpr uint32_t SEG_PT = FP_LDS_SEG_T * FP_LDS_SEG_T / FP_TURN_THREADS;  // phase records per thread
    uint4 t_seg[SEG_PT];
#pragma unroll
    for (uint32_t u = 0; u < SEG_PT; ++u) {
        const uint32_t q = threadIdx.x + u * FP_TURN_THREADS;
        t_seg[u] = lds_seg && q < T * T ? b.fp_seg[q] : make_uint4(0u, 0u, 0u, 0u);
    }
    DevState* st = b.state;
    // (the control words read together: no chain of scalar loads behind the branches)
    const uint32_t state = ctl->state, skip = ctl->skip, nu = ctl->nu, inc = ctl->inc, pbsrc = ctl->pbsrc;
    const uint32_t stamp = st->stamp;
    if ((state != FP_RUN) & (state != FP_FINAL)) return;
    if ((state == FP_RUN) & (skip != 0)) return;  // (k_fp_sched found no pass to test)
    const bool fin = state == FP_FINAL;
    __shared__ uint32_t s_w[FP_TURN_THREADS / 64];
    __shared__ uint32_t s_sf[FP_TMAX + 1], s_pf[FP_TMAX + 1], s_nseg[FP_TMAX], s_er[FP_TMAX];
    __shared__ uint4 s_seg[FP_LDS_SEG_T * FP_LDS_SEG_T];  // the schedule itself when T is small
    if (s1 <= T) {
        s_sf[s1] = t_sf;
        s_pf[s1] = t_pf;
        if (s1 < T) { s_nseg[s1] = t_ns; s_er[s1] = t_er; }
    }
    for (uint32_t s = threadIdx.x + blockDim.x; s <= T; s += blockDim.x) {
        s_sf[s] = b.fp_sf[s];
        s_pf[s] = b.fp_pf[s];
        if (s < T) { s_nseg[s] = b.fp_nseg[s]; s_er[s] = b.fp_erase[s]; }
    }
    if (lds_seg) {
#pragma unroll
        for (uint32_t u = 0; u < SEG_PT; ++u) {
            const uint32_t q = threadIdx.x + u * FP_TURN_THREADS;
            if (q < T * T) s_seg[q] = t_seg[u];
        }
    }
    __syncthreads();
    // (the incremental passes' picks live in fp_pbits, which exists only with b.fp_inc)
    const bool has_pb = b.fp_pbits != nullptr;
    fp_turn_blocks<KW>(cv, b, fin, inc != 0 && has_pb, pbsrc != 0 && has_pb, nu, T, stamp, s_sf, s_pf, s_nseg, s_er, lds_seg ? s_seg : b.fp_seg, s_w,
                       [&](uint32_t blk) { return blkoff[blk]; }, pre);
    if (fin && blockIdx.x == 0 && threadIdx.x == 0) {
        st->tmis_cnt = ctl->total;
        st->tail_rounds = ctl->fp_iter;
        if (ctl->fp_iter > st->max_rounds) st->max_rounds = ctl->fp_iter;
        if (b.ktime) time_slot(b, st->n_iter - 1)[3] = wall_now();
    }
}


// ------------------------------------------------------------------------------------
// Launchers.
hipError_t launch_init_assignment(const LoopBuffers& b, hipStream_t s) {
    if (b.rrng_mask) return launch_refrng_init(b, s);  // (reference-RNG mode)
    if (b.n_words == 0) return hipSuccess;
    k_init_assignment<<<(b.n_words + 255) / 256, 256, 0, s>>>(b.A, b.n_words, b.n_vars, b.seed);
    return hipGetLastError();
}

__global__ void k_set_limits(DevState* st, uint64_t n) {
    if (threadIdx.x != 0) return;
    st->limit_eval = st->n_iter + n;
    st->limit_nores = ~0ull;
    if (st->done == 2) st->done = 0;
}

hipError_t launch_set_limits(const LoopBuffers& b, uint64_t n, hipStream_t s) {
    k_set_limits<<<1, 64, 0, s>>>(b.state, n);
    return hipGetLastError();
}

hipError_t launch_eval(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                       uint32_t tile_end, bool gated, hipStream_t s) {
    if (tile_end <= tile_begin) return hipSuccess;
    const dim3 grid(tile_end - tile_begin);
    const int g = gated ? 1 : 0;
    if (cv.k == 0) {
        k_eval_csr<<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g);
    } else {
        ALLL_DISPATCH_K(cv.k, (k_eval_fixed<(K > 0 ? K : 1)><<<grid, EVAL_THREADS, 0, s>>>(cv, b, tile_begin, g)));
    }
    return hipGetLastError();
}

// Kernel attributes (dynamic LDS above the default) are per device: one bit per kernel group
// and device records what is set (contexts on several devices may share a process).
constexpr int ATTR_MAX_DEV = 64;
static std::atomic<uint32_t> g_attr_done[ATTR_MAX_DEV];
enum : uint32_t { ATTR_HYBRID = 0, ATTR_BUCKETS = 9, ATTR_FP = 18, ATTR_RAGGED = 30 };  // + k for per-width groups
static bool attr_pending(uint32_t bit, int& dev) {
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= ATTR_MAX_DEV) {
        dev = -1;
        return true;
    }
    return !(g_attr_done[dev].load(std::memory_order_acquire) & (1u << bit));
}
static void attr_mark(uint32_t bit, int dev) {
    if (dev >= 0) g_attr_done[dev].fetch_or(1u << bit, std::memory_order_release);
}

// Kernel attributes of the loop (dynamic LDS above the default), set once per device and
// kernel group by alll_create, before any stream capture: a capture then holds launches only
// (the launchers set no attributes; a kernel whose attribute is missing fails its launch).
hipError_t prepare_kernels(const ClauseView& cv, const LoopBuffers& b) {
    int dev;
    if (cv.k >= 1 && cv.k <= (uint32_t)MAX_FIXED_K && attr_pending(ATTR_HYBRID + cv.k, dev)) {
        hipError_t e = hipSuccess;
        ALLL_DISPATCH_K(cv.k, (e = hipFuncSetAttribute((const void*)k_eval_hybrid<(K > 0 ? K : 1)>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)(LDS_WORDS * 4 + 16))));
        if (e != hipSuccess) return e;
        ALLL_DISPATCH_K(cv.k, (e = hipFuncSetAttribute((const void*)k_eval_scatter<(K > 0 ? K : 1)>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)std::max<size_t>(LDS_WORDS * 4 + 16, SCATTER_LDS_BYTES))));
        if (e != hipSuccess) return e;
        ALLL_DISPATCH_K(cv.k, (e = hipFuncSetAttribute((const void*)k_eval_flags<(K > 0 ? K : 1)>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)(LDS_WORDS * 4 + 16))));
        if (e != hipSuccess) return e;
        attr_mark(ATTR_HYBRID + cv.k, dev);
    }
    if (cv.rg_off && attr_pending(ATTR_RAGGED, dev)) {
        hipError_t e = hipFuncSetAttribute((const void*)k_eval_ragged, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)(LDS_WORDS * 4 + 16));
        if (e != hipSuccess) return e;
        attr_mark(ATTR_RAGGED, dev);
    }
    if (b.pairs) {
        if (cv.k <= (uint32_t)MAX_FIXED_K && attr_pending(ATTR_BUCKETS + cv.k, dev)) {
            hipError_t e = hipFuncSetAttribute((const void*)k_bresolve<BRS_UNROLL_WIDE, BRS_THREADS>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4u << BKT_SHIFT_MAX));
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_bresolve<BRS_UNROLL_NARROW, BRS_THREADS>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4u << BKT_SHIFT_MAX));
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_bresolve<BRS_UNROLL_DEEP, BRS_THREADS_DEEP>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)(4u << BKT_SHIFT_MAX));
            if (e != hipSuccess) return e;
            ALLL_DISPATCH_K(cv.k, (e = hipFuncSetAttribute((const void*)k_bscatter<(K > 0 ? K : 1)>,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                                           (int)(BKT_STAGE * 8))));
            if (e != hipSuccess) return e;
            ALLL_DISPATCH_K(cv.k, (e = hipFuncSetAttribute((const void*)k_bjoin<(K > 0 ? K : 1)>,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                                           (int)(RUN_TILES_MAX * TILE))));
            if (e != hipSuccess) return e;
            attr_mark(ATTR_BUCKETS + cv.k, dev);
        }
    }
    if (b.fp_ctl) {
        if (attr_pending(ATTR_FP, dev)) {
            hipError_t e = hipFuncSetAttribute((const void*)k_fp_bscatter<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(8ull * BKT_MAX + 2ull * FP_BS_ENT * 8));
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_fp_bscatter<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)(8ull * BKT_MAX + 2ull * FP_BS_ENT * 8));
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_fp_bbuild, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024 - 1024);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_fp_repair<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)(FP_REP_QMAX / 8));
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_fp_repair<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)(FP_REP_QMAX / 8));
            if (e != hipSuccess) return e;
            attr_mark(ATTR_FP, dev);
        }
    }
    return hipSuccess;
}

hipError_t launch_eval_hybrid(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                              uint32_t tile_end, bool gated, int n_blocks, bool scatter, hipStream_t s, bool flags) {
    if (flags && (scatter || !b.rr_flag)) return hipErrorInvalidValue;
    if (tile_end <= tile_begin) return hipSuccess;
    const uint32_t nt = tile_end - tile_begin;
    const dim3 grid(std::min<uint32_t>(nt, (uint32_t)std::max(1, n_blocks)));
    if (scatter && (!b.pairs || b.n_runs % grid.x != 0)) return hipErrorInvalidValue;  // runs per workgroup
    // window words (a multiple of 4) + the zero word (a 16-byte slot); the scatter reuses it
    size_t lds = ((size_t)(std::min(b.n_words, b.win_words) + 3) / 4 * 4 + 4) * 4;
    if (scatter) lds = std::max(lds, SCATTER_LDS_BYTES);
    const int g = gated ? 1 : 0;
    if (cv.k < 1 || cv.k > (uint32_t)MAX_FIXED_K) return hipErrorInvalidValue;
    if (scatter) {
        ALLL_DISPATCH_K(cv.k, (k_eval_scatter<(K > 0 ? K : 1)><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g)));
    } else if (flags) {
        ALLL_DISPATCH_K(cv.k, (k_eval_flags<(K > 0 ? K : 1)><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g)));
    } else {
        ALLL_DISPATCH_K(cv.k, (k_eval_hybrid<(K > 0 ? K : 1)><<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, g)));
    }
    return hipGetLastError();
}

hipError_t launch_eval_ragged(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                              uint32_t tile_end, bool gated, int n_blocks, hipStream_t s) {
    if (tile_end <= tile_begin) return hipSuccess;
    const uint32_t nt = tile_end - tile_begin;
    const dim3 grid(std::min<uint32_t>(nt, (uint32_t)std::max(1, n_blocks)));
    const size_t lds = ((size_t)(std::min(b.n_words, b.win_words) + 3) / 4 * 4 + 4) * 4;
    k_eval_ragged<<<grid, HYB_THREADS, lds, s>>>(cv, b, tile_begin, tile_end, gated ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_collect(const ClauseView& cv, const LoopBuffers& b, uint32_t own_begin,
                          uint32_t own_end, hipStream_t s) {
    if (b.n_tiles == 0) return hipSuccess;
    ALLL_DISPATCH_K(cv.k, (k_collect<K><<<b.n_tiles, EVAL_THREADS, 0, s>>>(cv, b, own_begin, own_end)));
    return hipGetLastError();
}

hipError_t launch_cmark(const ClauseView& cv, const LoopBuffers& b, size_t words_per_rank, int rank, bool gated,
                        hipStream_t s) {
    if (!b.cmask || !b.cflag || words_per_rank >= (1ull << 32)) return hipErrorInvalidValue;
    // violated clauses → a byte each (k_cmark), packed into this rank's mask words (k_cpack);
    // 64-bit atomicOr per clause instead: 34.6 µs per iteration at M on one rank
    const uint64_t base = (uint64_t)words_per_rank * (uint64_t)rank * 64u;
    if (b.own_end > b.own_begin) {
        const uint32_t g = (b.own_end - b.own_begin + 3) / 4;
        ALLL_DISPATCH_K(cv.k, (k_cmark<K><<<g, 256, 0, s>>>(cv, b, base, gated ? 1 : 0)));
    }
    if (words_per_rank) {
        uint64_t* w = reinterpret_cast<uint64_t*>(b.cmask) + words_per_rank * (size_t)rank;
        k_cpack<<<(uint32_t)((words_per_rank + 255) / 256), 256, 0, s>>>(b, w, (uint32_t)words_per_rank, gated ? 1 : 0);
    }
    return hipGetLastError();
}

hipError_t launch_reduce(const LoopBuffers& b, int mode, hipStream_t s) {
    k_reduce<<<1, 1024, 0, s>>>(b, mode);
    return hipGetLastError();
}

hipError_t launch_round(const ClauseView& cv, const LoopBuffers& b, uint32_t r, bool last, hipStream_t s) {
    // buffers: eval -> stage[0]; CLAIM(0) in place; JOIN(r) stage[0] -> stage[1];
    // CLAIM(r>0) stage[1] -> stage[0]
    if (b.n_tiles == 0) return hipSuccess;
    uint32_t* s0 = b.stage[0];
    uint32_t* s1 = b.stage[1];
    const int l = last ? 1 : 0;
    if (r >= WAVE_ROUND_MIN) {  // rounds >= 1: a wave per tile
        const uint32_t grid = (b.n_tiles + ROUND_THREADS / 64 - 1) / (ROUND_THREADS / 64);
        ALLL_DISPATCH_K(cv.k, (k_wclaim<K><<<grid, ROUND_THREADS, 0, s>>>(cv, b, r, s1, s0)));
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        ALLL_DISPATCH_K(cv.k, (k_wjoin<K><<<grid, ROUND_THREADS, 0, s>>>(cv, b, r, s0, s1, l)));
        return hipGetLastError();
    }
    ALLL_DISPATCH_K(cv.k, (k_claim<K><<<b.n_tiles, ROUND_THREADS, 0, s>>>(cv, b, s0)));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    ALLL_DISPATCH_K(cv.k, (k_join<K><<<b.n_tiles, JOIN_THREADS, 0, s>>>(cv, b, r, s0, s1, l)));
    return hipGetLastError();
}

hipError_t launch_round0_buckets(const ClauseView& cv, const LoopBuffers& b, bool last, bool fused_reduce,
                                 bool scattered, hipStream_t s) {
    // buffers as CLAIM(0) + JOIN(0): eval -> stage[0] (ids translated in place); JOIN stage[0] -> stage[1]
    if (b.n_tiles == 0 || cv.k == 0 || !b.pairs) return hipErrorInvalidValue;
    const uint64_t run_cap = (uint64_t)b.run_tiles * TILE * cv.k;
    const size_t lds = (size_t)4 * b.bkt_width;  // k_bresolve minima
    // fused_reduce: the loop's reduce has not run; it runs in an extra workgroup of k_bresolve
    // (the scatter uses the pre-reduce epoch).  scattered: k_eval_hybrid has scattered the runs.
    const int fr = fused_reduce ? 1 : 0;
    hipError_t e;
    if (!scattered) {
        ALLL_DISPATCH_K(cv.k, (k_bscatter<(K > 0 ? K : 1)><<<b.n_runs, BSC_THREADS, BKT_STAGE * 8, s>>>(
                                  cv, b, b.stage[0], fr)));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const uint32_t nb = b.n_bkt;
    if (b.n_bkt <= b.n_cu)
        k_bresolve<BRS_UNROLL_WIDE, BRS_THREADS><<<nb, BRS_THREADS, lds, s>>>(b, (uint32_t)run_cap, fr);
    else if (lds > (size_t)BRS_DEEP_LDS)  // minima too large for two workgroups per CU
        k_bresolve<BRS_UNROLL_DEEP, BRS_THREADS_DEEP><<<nb, BRS_THREADS_DEEP, lds, s>>>(b, (uint32_t)run_cap, fr);
    else
        k_bresolve<BRS_UNROLL_NARROW, BRS_THREADS><<<nb, BRS_THREADS, lds, s>>>(b, (uint32_t)run_cap, fr);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int l = last ? 1 : 0;
    ALLL_DISPATCH_K(cv.k, (k_bjoin<(K > 0 ? K : 1)><<<b.n_runs, BJN_THREADS, (size_t)b.run_tiles * TILE, s>>>(
                              cv, b, b.stage[0], b.stage[1], l)));
    return hipGetLastError();
}

hipError_t launch_tail(const ClauseView& cv, const LoopBuffers& b, uint32_t first_round, hipStream_t s) {
    ALLL_DISPATCH_K(cv.k, (k_tail<K><<<1, TAIL_THREADS, 0, s>>>(cv, b, first_round)));
    return hipGetLastError();
}

// grids of the fixpoint kernels
struct FpGrids {
    uint32_t gb, gl, gr, gw;
    uint32_t rounds;  // grid rounds before the one-workgroup tail
    bool narrow;
};
static FpGrids fp_grids(const LoopBuffers& b) {
    FpGrids g;
    g.narrow = b.rr_k >= 1 && b.rr_k <= 4;
    g.rounds = b.fp_hot ? FP_G_HOT : FP_G;
    g.gb = (uint32_t)std::min<uint64_t>((b.m + FP_B - 1) / FP_B + 1, FP_COUNT_GRID);
    g.gl = (uint32_t)std::min<uint64_t>((b.m + FP_THREADS - 1) / FP_THREADS + 1, 2048);
    // workgroups of the grid-stride round kernels (2048)
    g.gr = (uint32_t)std::min<uint64_t>((b.m + FP_RT - 1) / FP_RT + 1, 2048);
    // wave-per-tile rounds: four tiles per workgroup
    g.gw = (uint32_t)std::min<uint64_t>(((b.m + FP_RT - 1) / FP_RT + 4) / 4, FP_WGRID);
    return g;
}

static void fp_turns(const ClauseView& cv, const LoopBuffers& b, const FpGrids& g, int test, hipStream_t s) {
    k_fp_count<<<g.gb, FP_THREADS, 0, s>>>(b, test);
    // (the schedule computed redundantly by every workgroup of the turn kernel, the last one to
    // finish advancing the pass: 615 -> 527 it/s at M, T = 16; 50 KB of LDS per workgroup and
    // the schedule's latency in every one of them cost more than the launch saved)
    k_fp_sched<<<1, 256, 0, s>>>(b, test);
    if (g.narrow) k_fp_turn<4><<<g.gb, FP_TURN_THREADS, 0, s>>>(cv, b);
    else k_fp_turn<0><<<g.gb, FP_TURN_THREADS, 0, s>>>(cv, b);
}

hipError_t launch_rr_prep(const ClauseView& cv, const LoopBuffers& b, bool marked, hipStream_t s) {
    if (!b.rr_u || b.rr_T < 2 || b.rr_T > RR_TMAX) return hipErrorInvalidValue;
    if (b.rr_flag) {  // fixed width: violated flags in clause order from the evaluation's lists
        if (cv.k == 0 || !b.rr_tcnt) return hipErrorInvalidValue;
        const uint32_t gw = (b.n_tiles + 3) / 4;
        if (gw) {
            // (marked: the evaluation set the flags itself, k_eval_flags)
            if (!marked) ALLL_DISPATCH_K(cv.k, (k_rr_mark<(K > 0 ? K : 1)><<<gw, 256, 0, s>>>(cv, b)));
            k_rr_count<<<gw, 256, 0, s>>>(b);
        }
    } else if (cv.k != 0) {
        return hipErrorInvalidValue;
    }
    if (b.n_tiles) k_rr_entries<<<b.n_tiles, 256, 0, s>>>(cv, b);
    if (!b.fp_ctl) return hipGetLastError();
    // the fixpoint passes: iteration set-up, claimant lists, first guess
    if (b.rr_T > FP_TMAX) return hipErrorInvalidValue;
    if (!b.fp_pairs || !b.fp_soff || b.n_bkt == 0 || b.n_bkt > BKT_MAX) return hipErrorInvalidValue;
    const FpGrids g = fp_grids(b);
    const size_t lds_bs = 8ull * b.n_bkt + 2ull * FP_BS_ENT * 8;
    const size_t lds_bb = fp_bbuild_lds_bytes(b.bkt_width);
    // (the iteration's start ran with the reduce: fp_begin_body; the owner / cover restart runs in k_fp_guess)
    const uint32_t gbs = (uint32_t)std::min<uint64_t>((b.m + FP_BS_ENT - 1) / FP_BS_ENT + 1, 512);
    if (g.narrow) k_fp_bscatter<4><<<gbs, FP_THREADS, lds_bs, s>>>(cv, b);
    else k_fp_bscatter<0><<<gbs, FP_THREADS, lds_bs, s>>>(cv, b);
    k_fp_guess<<<g.gl, FP_THREADS, 0, s>>>(b);
    k_fp_bbuild<<<b.n_bkt, FP_BB_THREADS, lds_bb, s>>>(b);
    fp_turns(cv, b, g, 0, s);
    return hipGetLastError();
}

hipError_t launch_rr_passes(const ClauseView& cv, const LoopBuffers& b, uint32_t n, bool full, hipStream_t s) {
    if (!b.fp_ctl) return hipSuccess;
    const FpGrids g = fp_grids(b);
    // (the incremental kernels need their buffers: never enqueued without them)
    if (b.fp_inc && (!b.fp_blocker || !b.fp_covby || !b.fp_sc || !b.fp_dl || !b.fp_dmark || !b.fp_pbits || !b.fp_lst))
        return hipErrorInvalidValue;
    for (uint32_t p = 0; p < n; ++p) {
        if (b.fp_inc && !(full && p == 0)) {
            // an incremental pass (its kernels run only when the device state asks for one)
            k_fp_detect<<<g.gl, FP_THREADS, 0, s>>>(b);
            const size_t lq = ((size_t)std::min<uint64_t>(b.m, FP_REP_QMAX) + 127) / 128 * 16;  // (uint4 rows)
            // (all resident: one workgroup per CU by its LDS)
            const uint32_t gw = std::min<uint32_t>(FP_RW_GRID, std::max<uint32_t>(1, b.n_cu));
            if (g.narrow) k_fp_repair<4><<<gw, 1024, lq, s>>>(cv, b);
            else k_fp_repair<0><<<gw, 1024, lq, s>>>(cv, b);
            // (the repair ran the pass test and the schedule: the turns follow)
            if (g.narrow) k_fp_turn<4><<<g.gb, FP_TURN_THREADS, 0, s>>>(cv, b);
            else k_fp_turn<0><<<g.gb, FP_TURN_THREADS, 0, s>>>(cv, b);
            continue;
        }
        // round 0: the claimant-list minima, then JOIN(0) (a workgroup per tile); rounds 1..:
        // a wave per tile.  (Instances with hot variables get FP_HEAVY_GRID more k_fp_vmin
        // workgroups for the long lists.)
        k_fp_vmin<<<b.n_bkt * FP_VS + (cv.n_hot ? FP_HEAVY_GRID : 16u), FP_THREADS, 0, s>>>(b);
        if (g.narrow) k_fp_join0<4><<<g.gr, FP_THREADS, 0, s>>>(cv, b);
        else k_fp_join0<0><<<g.gr, FP_THREADS, 0, s>>>(cv, b);
        for (uint32_t r = 1; r < g.rounds; ++r) {
            if (g.narrow) {
                k_fp_wclaim<4><<<g.gw, FP_THREADS, 0, s>>>(cv, b, r);
                k_fp_wjoin<4><<<g.gw, FP_THREADS, 0, s>>>(cv, b, r);
            } else {
                k_fp_wclaim<0><<<g.gw, FP_THREADS, 0, s>>>(cv, b, r);
                k_fp_wjoin<0><<<g.gw, FP_THREADS, 0, s>>>(cv, b, r);
            }
        }
        if (g.narrow) k_fp_tail<4><<<1, 1024, 0, s>>>(cv, b, g.rounds);
        else k_fp_tail<0><<<1, 1024, 0, s>>>(cv, b, g.rounds);
        fp_turns(cv, b, g, 1, s);
    }
    return hipGetLastError();
}

hipError_t launch_rr_finish(const ClauseView& cv, const LoopBuffers& b, hipStream_t s) {
    // the batch kernel decides an iteration the fixpoint passes did not settle (or every
    // iteration without them); clause variables held in registers: 4 for widths <= 4
    if (!b.rr_ctl || b.rr_mw == 0 || b.rr_mw > RR_MW_MAX) return hipErrorInvalidValue;
    if (b.rr_k >= 1 && b.rr_k <= 4) k_rr_mw<4, 4><<<b.rr_mw, 64, sizeof(RRMwLds), s>>>(cv, b);
    else k_rr_mw<8, 2><<<b.rr_mw, 64, sizeof(RRMwLds), s>>>(cv, b);
    return hipGetLastError();
}

hipError_t launch_resample(const ClauseView& cv, const LoopBuffers& b, uint32_t own_begin,
                           uint32_t own_end, bool to_delta, hipStream_t s) {
    if (to_delta) {
        if (b.n_tiles == 0) return hipSuccess;
        ALLL_DISPATCH_K(cv.k, (k_resample_delta<K><<<b.n_tiles + 1, ROUND_THREADS, 0, s>>>(cv, b, own_begin, own_end)));
        return hipGetLastError();
    }
    if (b.rrng_mask) return launch_refrng_resample(cv, b, s);  // (reference-RNG mode)
    if (b.n_vars == 0) return hipSuccess;
    const uint64_t blocks = ((uint64_t)b.n_words * 2 + 255) / 256;  // a thread per 16 variables
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    k_resample_vars<<<(uint32_t)blocks, 256, 0, s>>>(b);
    return hipGetLastError();
}

hipError_t fp_repair_occupancy(const ClauseView& cv, const LoopBuffers& b, int* blocks_per_cu) {
    const size_t lq = ((size_t)std::min<uint64_t>(b.m, FP_REP_QMAX) + 127) / 128 * 16;
    const bool narrow = b.rr_k >= 1 && b.rr_k <= 4;
    return narrow ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_fp_repair<4>, 1024, lq)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_fp_repair<0>, 1024, lq);
}

hipError_t launch_apply_delta(const LoopBuffers& b, hipStream_t s) {
    if (b.n_words == 0) return hipSuccess;
    k_apply_delta<<<(b.n_words + 255) / 256, 256, 0, s>>>(b);
    return hipGetLastError();
}

}  // namespace alll
