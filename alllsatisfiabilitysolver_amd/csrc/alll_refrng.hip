// alll_refrng.hip -- CDNA4 (gfx950) kernels of the reference-RNG mode (ALLL_FLAG_REFERENCE_RNG).
//
// The reference draws every resampled bit from RBG<default_random_engine> (RandomBoolGenerator.h:
// 29-52): a 64-bit uniform_int_distribution<unsigned long long> draw with bit 63 set serves 63
// bits, lowest first.  default_random_engine is libstdc++'s minstd_rand0 (x <- 16807 x mod
// 2^31 - 1; min 1, max 2^31 - 2), and the 64-bit draw comes from libstdc++'s upscaling (GCC 11
// bits/uniform_int_dist.h): a 64-bit value is UR * (a draw in [0, Q1]) + one more engine value,
// that draw in turn UR * (a draw in [0, Q2]) + one more, the innermost by rejection-downscaling,
// every level redrawn when it overflows its range.  Each engine is seeded with one
// std::random_device value: one for the initial fill (VariablesArray.h:23-34), one per resample
// round with T = 1 (SATInstance.h:340-365), whose bits go to the MIS clauses' literals in pick
// order -- ascending clause index for the one-set MIS, yield order in the streaming solve.  random_device is replaced by the 64-bit
// LCG of oracle/ref_probe.cpp, so a run here equals the reference run the probe records, bit for
// bit (oracle: orc_solve_refrng; tests/test_gpu_refrng.py).
//
// Per resample round:
//   k_rrng_mark   the MIS (per-tile lists and the tail's list) as a bitmask in pick order (clause
//                 index; streaming: window offset, with the clause of every position), and per
//                 64-position word the literal count of its MIS clauses;
//   k_rrng_scan1  per 1024-word block: exclusive offsets of the words, the block total;
//   k_rrng_scan2  one workgroup: the blocks' offsets, the round's bit count, the engine's seed;
//   k_rrng_pos / k_rrng_lift / k_rrng_collect
//                 the round's ceil(bits / 63) RBG draws in parallel (below);
//   k_rrng_apply  a thread per mask word: its MIS clauses in order, each literal's variable set to
//                 the next bit (a repeated variable keeps the last, as in the reference).
// Integer work, latency bound: no MFMA.
#include "alll_internal.h"

namespace alll {
namespace {

constexpr uint32_t RRNG_LIT_MASK = 0x7FFFFFFFu;  // (bit 31 of the AoS literals: hot-variable flag)
constexpr int RRNG_BLOCK = 1024;                  // mask words per scan block

// minstd_rand0 and the upscaling constants of uniform_int_distribution<unsigned long long>{}
constexpr uint64_t MS_M = 2147483647ull;
constexpr uint64_t MS_MIN = 1ull;
constexpr uint64_t MS_RANGE = MS_M - 1ull - MS_MIN;  // urng.max() - urng.min()
constexpr uint64_t UR = MS_RANGE + 1ull;             // __uerngrange
constexpr uint64_t Q1 = ~0ull / UR;                  // range of the middle draw
constexpr uint64_t Q2 = Q1 / UR;                     // range of the innermost draw
static_assert(MS_RANGE < Q1 && MS_RANGE > Q2, "two upscaling levels, then downscaling");
constexpr uint64_t C_UE = Q2 + 1ull;                 // innermost: __uerange
constexpr uint64_t C_SCALING = MS_RANGE / C_UE;
constexpr uint64_t C_PAST = C_UE * C_SCALING;

__device__ __forceinline__ uint32_t rd_next(uint64_t& s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(s >> 33);
}
// x <- 16807 x mod (2^31 - 1), Mersenne reduction (x < 2^31: the product is < 2^46)
__device__ __forceinline__ uint64_t ms_next(uint64_t& x) {
    const uint64_t p = x * 16807ull;
    uint64_t r = (p & MS_M) + (p >> 31);
    if (r >= MS_M) r -= MS_M;
    x = r;
    return r;
}
__device__ __forceinline__ uint64_t ms_seed(uint32_t s) {
    const uint64_t r = (uint64_t)s % MS_M;
    return r ? r : 1ull;
}
__device__ __forceinline__ uint64_t uid_inner(uint64_t& x) {
    uint64_t r;
    do r = ms_next(x) - MS_MIN;
    while (r >= C_PAST);
    return r / C_SCALING;
}
__device__ __forceinline__ uint64_t uid_middle(uint64_t& x) {
    uint64_t ret, tmp;
    do {
        tmp = UR * uid_inner(x);
        ret = tmp + (ms_next(x) - MS_MIN);
    } while (ret > Q1 || ret < tmp);
    return ret;
}
// uniform_int_distribution<unsigned long long>{}(engine): [0, 2^64 - 1]
__device__ __forceinline__ uint64_t uid_u64(uint64_t& x) {
    uint64_t ret, tmp;
    do {
        tmp = UR * uid_middle(x);
        ret = tmp + (ms_next(x) - MS_MIN);
    } while (ret < tmp);  // (ret > 2^64 - 1 cannot happen)
    return ret;
}

// (x * y) mod (2^31 - 1) for x, y < 2^31
__device__ __forceinline__ uint64_t ms_mul(uint64_t x, uint64_t y) {
    const uint64_t p = x * y;
    uint64_t r = (p & MS_M) + (p >> 31);
    r = (r & MS_M) + (r >> 31);
    return r >= MS_M ? r - MS_M : r;
}
// 16807^e mod (2^31 - 1): the engine e steps ahead (jump-ahead of the LCG)
__device__ __forceinline__ uint64_t ms_pow(uint64_t e) {
    uint64_t r = 1, base = 16807ull;
    while (e) {
        if (e & 1ull) r = ms_mul(r, base);
        base = ms_mul(base, base);
        e >>= 1;
    }
    return r;
}
// uid_u64 counting the engine values it takes
__device__ __forceinline__ uint64_t ms_next_cnt(uint64_t& x, uint32_t& n) {
    ++n;
    return ms_next(x);
}
__device__ __forceinline__ uint64_t uid_u64_cnt(uint64_t& x, uint32_t& n) {
    uint64_t ret, tmp;
    do {
        uint64_t mid, mtmp;
        do {
            uint64_t r;
            do r = ms_next_cnt(x, n) - MS_MIN;
            while (r >= C_PAST);
            mtmp = UR * (r / C_SCALING);
            mid = mtmp + (ms_next_cnt(x, n) - MS_MIN);
        } while (mid > Q1 || mid < mtmp);
        tmp = UR * mid;
        ret = tmp + (ms_next_cnt(x, n) - MS_MIN);
    } while (ret < tmp);
    return ret;
}

__device__ __forceinline__ uint32_t clause_len(const ClauseView& cv, uint32_t c) {
    return cv.k ? cv.k : (uint32_t)(cv.offs[c + 1] - cv.offs[c]);
}
__device__ __forceinline__ uint64_t clause_start(const ClauseView& cv, uint32_t c) {
    return cv.k ? (uint64_t)c * cv.k : (uint64_t)cv.offs[c];
}

// VariablesArray(n): one engine seeded by random_device, one RBG bit per variable in index order
__global__ void k_rrng_init(LoopBuffers b) {
    if (threadIdx.x != 0) return;
    DevState* st = b.state;
    uint64_t rd = st->rd_state;
    uint64_t x = ms_seed(rd_next(rd));
    st->rd_state = rd;
    uint64_t buf = 0;
    uint32_t nb = 0;  // unused bits of the current draw (lowest first)
    for (uint32_t w = 0; w < b.n_words; ++w) {
        const uint32_t need = min(32u, b.n_vars - 32u * w);
        uint32_t word = 0, filled = 0;
        while (filled < need) {
            if (nb == 0) {
                buf = uid_u64(x) & ~(1ull << 63);  // (bit 63: RBG's sentinel, never served)
                nb = 63;
            }
            const uint32_t take = min(nb, need - filled);
            word |= (uint32_t)(buf & ((1ull << take) - 1ull)) << filled;
            buf >>= take;
            nb -= take;
            filled += take;
        }
        b.A[w] = word;
    }
}

// Pick position of MIS clause c: its clause index, or in the streaming solve its offset in the
// iteration's window of generator steps (the LFMIS key - 1, alll_kernels.hip prio(): the clause
// generator yields clause j*P mod m at step j, ClauseGenerator.h:47)
__device__ __forceinline__ uint32_t pick_pos(const LoopBuffers& b, const DevState* st, uint32_t c) {
    if (!b.stream_batch) return c;
    const uint64_t m = b.m;
    uint64_t pos = ((uint64_t)c * b.stream_pinv) % m;
    if (pos == 0) pos = m;
    return (uint32_t)((pos - 1 + m - st->win_start % m) % m);
}

__global__ __launch_bounds__(256) void k_rrng_mark(ClauseView cv, LoopBuffers b) {
    const DevState* st = b.state;
    if (!st->active) return;
    const uint32_t t = blockIdx.x;
    const uint32_t* list = t < b.n_tiles ? b.mis + (uint64_t)t * TILE : b.tmis;
    const uint32_t cnt = t < b.n_tiles ? b.mis_cnt[t] : st->tmis_cnt;
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
        const uint32_t c = list[i], p = pick_pos(b, st, c);
        atomicOr(&b.rrng_mask[p >> 6], 1ull << (p & 63));
        atomicAdd(&b.rrng_woff[p >> 6], clause_len(cv, c));
        if (b.rrng_map) b.rrng_map[p] = c;
    }
}

// workgroup exclusive scan of one value per thread (1024 threads); returns the total too
__device__ __forceinline__ uint32_t block_excl_1024(uint32_t x, uint32_t* s_w, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (uint32_t w = 0; w < RRNG_BLOCK / 64; ++w) {
        const uint32_t c = s_w[w];
        if (w < wave) before += c;
        total += c;
    }
    __syncthreads();
    return before + incl - x;
}

__global__ __launch_bounds__(RRNG_BLOCK) void k_rrng_scan1(LoopBuffers b, uint32_t n_mask_words) {
    if (!b.state->active) return;
    __shared__ uint32_t s_w[RRNG_BLOCK / 64];
    const uint32_t w = blockIdx.x * RRNG_BLOCK + threadIdx.x;
    const uint32_t x = w < n_mask_words ? b.rrng_woff[w] : 0u;
    uint32_t total;
    const uint32_t e = block_excl_1024(x, s_w, total);
    if (w < n_mask_words) b.rrng_woff[w] = e;
    if (threadIdx.x == 0) b.rrng_bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(RRNG_BLOCK) void k_rrng_scan2(LoopBuffers b, uint32_t n_blocks) {
    DevState* st = b.state;
    if (!st->active) return;
    __shared__ uint32_t s_w[RRNG_BLOCK / 64];
    __shared__ uint32_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t q0 = 0; q0 < n_blocks; q0 += RRNG_BLOCK) {  // (uniform loop)
        const uint32_t q = q0 + threadIdx.x;
        const uint32_t x = q < n_blocks ? b.rrng_bsum[q] : 0u;
        uint32_t total;
        const uint32_t e = block_excl_1024(x, s_w, total);
        const uint32_t carry = s_carry;
        if (q < n_blocks) b.rrng_bsum[q] = carry + e;
        __syncthreads();
        if (threadIdx.x == 0) s_carry = carry + total;
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    // the round's engine: seeded by the next random_device value (resample_clauses,
    // SATInstance.h:343-350, T = 1); ceil(bits / 63) 64-bit draws serve every bit
    const uint64_t bits = s_carry;
    uint64_t rd = st->rd_state;
    st->rd_x0 = ms_seed(rd_next(rd));
    st->rd_state = rd;
    st->rd_bits = bits;
    const uint64_t draws = (bits + 62) / 63;
    if (draws > b.rrng_cap) {  // (the host sizes the buffer for every literal: never taken)
        st->error = 7;
        st->done = 3;
        return;
    }
    st->rd_draws = (uint32_t)draws;
    st->rd_n = (uint32_t)min<uint64_t>(draws * RRNG_POS_PER_DRAW + 64, b.rrng_nmax);
    st->rd_fail = 0;
}

// The round's draws in parallel.  Engine position i (1-based: the i-th value the seeded engine
// returns) holds x0 * 16807^i mod (2^31 - 1), so every position's value is known without the
// ones before it; a draw that starts at position i takes n(i) values (3, plus 2 per redrawn
// middle level, ~1 in 5) and yields v(i), both functions of the values from i on:
//   k_rrng_pos      a thread per position: jump[0][i] = i + n(i) (the next draw's start), val[i];
//   k_rrng_lift(t)  jump[t + 1][i] = jump[t][jump[t][i]]: 2^(t+1) draws on;
//   k_rrng_collect  a thread per draw k: its start = position 1 advanced by the bits of k, its
//                   value val[start];
//   k_rrng_seq      the one-thread chain, only when the draws ran past the positions considered
//                   (more than RRNG_POS_PER_DRAW values per draw on average: not seen).
__global__ __launch_bounds__(256) void k_rrng_pos(LoopBuffers b) {
    const DevState* st = b.state;
    if (!st->active || st->done == 3) return;
    const uint32_t n = st->rd_n;
    const uint64_t x0 = st->rd_x0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i <= (uint64_t)n + 1; i += stride) {
        if (i == (uint64_t)n + 1) {
            b.rrng_jump[i] = n + 1;  // (the sentinel past the positions)
            continue;
        }
        uint64_t x = ms_mul(x0, ms_pow(i - 1));  // the state whose next value is position i's
        uint32_t used = 0;
        b.rrng_val[i] = uid_u64_cnt(x, used);
        b.rrng_jump[i] = (uint32_t)min<uint64_t>(i + used, (uint64_t)n + 1);
    }
}

__global__ __launch_bounds__(256) void k_rrng_lift(LoopBuffers b, uint32_t t) {
    const DevState* st = b.state;
    if (!st->active || st->done == 3) return;
    const uint32_t d = st->rd_draws;
    if (d < 2 || (uint64_t)(d - 1) >> (t + 1) == 0) return;  // (level t + 1 is not needed for k < d)
    const uint32_t n = st->rd_n, w = b.rrng_nmax + 2;
    const uint32_t* j0 = b.rrng_jump + (uint64_t)t * w;
    uint32_t* j1 = b.rrng_jump + (uint64_t)(t + 1) * w;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i <= (uint64_t)n + 1; i += stride)
        j1[i] = j0[j0[i]];
}

__global__ __launch_bounds__(256) void k_rrng_collect(LoopBuffers b) {
    DevState* st = b.state;
    if (!st->active || st->done == 3) return;
    const uint32_t d = st->rd_draws, n = st->rd_n, w = b.rrng_nmax + 2;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < d; k += stride) {
        uint32_t pos = 1;
        for (uint32_t t = 0; (k >> t) != 0; ++t)
            if ((k >> t) & 1ull) pos = b.rrng_jump[(uint64_t)t * w + pos];
        if (pos > n) st->rd_fail = 1u;
        else b.rrng_stream[k] = b.rrng_val[pos];
    }
}

__global__ void k_rrng_seq(LoopBuffers b) {
    const DevState* st = b.state;
    if (threadIdx.x != 0 || !st->active || st->done == 3 || !st->rd_fail) return;
    uint64_t x = st->rd_x0;
    const uint32_t d = st->rd_draws;
    for (uint32_t k = 0; k < d; ++k) b.rrng_stream[k] = uid_u64(x);
}

__global__ __launch_bounds__(RRNG_BLOCK) void k_rrng_apply(ClauseView cv, LoopBuffers b, uint32_t n_mask_words) {
    const DevState* st = b.state;
    if (!st->active || st->done == 3) return;
    const uint32_t w = blockIdx.x * RRNG_BLOCK + threadIdx.x;
    if (w >= n_mask_words) return;
    unsigned long long bits = b.rrng_mask[w];
    uint64_t o = (uint64_t)b.rrng_bsum[blockIdx.x] + b.rrng_woff[w];  // this word's first bit
    b.rrng_woff[w] = 0u;  // (every word: the scan wrote them all; for the next round)
    if (!bits) return;
    while (bits) {
        const uint32_t p = 64u * w + (uint32_t)__builtin_ctzll(bits);
        const uint32_t c = b.rrng_map ? b.rrng_map[p] : p;  // (the clause picked p-th)
        bits &= bits - 1ull;
        const uint64_t lb = clause_start(cv, c);
        const uint32_t len = clause_len(cv, c);
        for (uint32_t j = 0; j < len; ++j, ++o) {
            const uint32_t v = (cv.lits[lb + j] & RRNG_LIT_MASK) >> 1;
            const uint32_t bit = (uint32_t)(b.rrng_stream[o / 63] >> (o % 63)) & 1u;
            if (bit) atomicOr(&b.A[v >> 5], 1u << (v & 31));
            else atomicAnd(&b.A[v >> 5], ~(1u << (v & 31)));
        }
    }
    b.rrng_mask[w] = 0ull;  // (for the next round)
}

}  // namespace

hipError_t launch_refrng_init(const LoopBuffers& b, hipStream_t s) {
    if (b.n_words == 0) return hipSuccess;
    k_rrng_init<<<1, 64, 0, s>>>(b);
    return hipGetLastError();
}

hipError_t launch_refrng_resample(const ClauseView& cv, const LoopBuffers& b, hipStream_t s) {
    const uint64_t nmw = (b.m + 63) / 64;
    if (nmw == 0) return hipSuccess;
    if (nmw > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t nblk = (uint32_t)((nmw + RRNG_BLOCK - 1) / RRNG_BLOCK);
    k_rrng_mark<<<b.n_tiles + 1, 256, 0, s>>>(cv, b);
    k_rrng_scan1<<<nblk, RRNG_BLOCK, 0, s>>>(b, (uint32_t)nmw);
    k_rrng_scan2<<<1, RRNG_BLOCK, 0, s>>>(b, nblk);
    const uint32_t gp = (uint32_t)std::min<uint64_t>(((uint64_t)b.rrng_nmax + 2 + 255) / 256, 2048);
    k_rrng_pos<<<gp, 256, 0, s>>>(b);
    for (uint32_t t = 0; t + 1 < b.rrng_levels; ++t) k_rrng_lift<<<gp, 256, 0, s>>>(b, t);
    k_rrng_collect<<<(uint32_t)std::min<uint64_t>((b.rrng_cap + 255) / 256, 2048), 256, 0, s>>>(b);
    k_rrng_seq<<<1, 64, 0, s>>>(b);
    k_rrng_apply<<<nblk, RRNG_BLOCK, 0, s>>>(cv, b, (uint32_t)nmw);
    return hipGetLastError();
}

}  // namespace alll
