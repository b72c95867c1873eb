// alll_stream.hip -- CDNA4 (gfx950) kernels of the streaming solve with T > 1 threads,
// SATInstance::solve(getEnumeratedClause, n_clauses, batch_size) (reference SATInstance.h:70-153).
//
// The reference keeps T ClauseGenerators (SATInstance.h:74-86), each walking its own clause range
// with c <- (c + P) % n_t (ClauseGenerator.h:44-47).  An iteration is a sequence of batch steps: every
// generator yields its next batch of walk steps and keeps the violated clauses, then
// populate_mis_parallel (SATInstance.h:391-451) drops the clauses that share a variable with the MIS
// accumulated so far and extends it by the T-set round robin; after the step at which all
// generators finish together the MIS is resampled.  Here the host plans the iteration from the
// generators' states (SrrGen, alll_runtime.cpp) and the device
//   k_srr_first   finds the end-of-iteration check's first violated offset in every generator's range
//                 (where the lock-step check stops, oracle/alll_oracle.c orc_solve_stream_rr);
//   k_srr_count / k_srr_scan / k_srr_fill
//                 lists every generator's violated walk steps in walk order (a thread per 16 steps,
//                 violated bits from the clause-order bitmask of k_eval_csr), with each clause's
//                 variables inline, and the first list entry of every (batch step, generator);
//   k_srr_mis     runs the batch steps' round robins in order, one 1024-thread workgroup, a cycle
//                 of turns at a time: every set's next uncovered entries are gathered, the turn
//                 sequence they would give is laid out in closed form, and an LDS hash of first
//                 uses finds the first turn whose candidate an earlier pick covers; the turns
//                 before it are the reference's (the filter against the MIS so far and the round
//                 robin's erasures are both the "first entry with no covered variable" rule).
// k_resample_vars (alll_kernels.hip) then resamples the covered variables.  Integer work, latency
// bound: no MFMA.
#include "alll_internal.h"

namespace alll {
namespace {

constexpr uint32_t S_LIT_MASK = 0x7FFFFFFFu;  // (bit 31 of the AoS literals: hot-variable flag)
constexpr int SRR_THREADS = 1024;
constexpr int SRR_WALK = 16;                  // walk steps per thread of k_srr_count / k_srr_fill
static_assert(256 * SRR_WALK == SRR_BLK, "a 256-thread block per virtual block");

__device__ __forceinline__ uint32_t s_var(uint32_t raw) { return (raw & S_LIT_MASK) >> 1; }

// generator of virtual block blk: the t with vblk[t] <= blk < vblk[t + 1] (generators without walk
// steps have no blocks)
__device__ uint32_t srr_block_gen(const LoopBuffers& b, uint32_t blk) {
    uint32_t lo = 0, hi = b.srr_T;  // vblk[lo] <= blk < vblk[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (b.srr_gen[mid].vblk <= blk) lo = mid; else hi = mid;
    }
    return lo;
}

// Walk steps j0 .. j0 + 15 of generator g: clause of step j = base + (c0 + (j + 1) pt) mod n; bit k of
// the result = step j0 + k is one of the iteration's steps and its clause is violated.
__device__ __forceinline__ uint32_t srr_walk16(const LoopBuffers& b, const SrrGen& g, uint64_t j0,
                                               uint32_t (&cl)[SRR_WALK]) {
    if (j0 >= g.yields) return 0;
    const uint64_t n = g.n;
    uint64_t c = (g.c0 + ((j0 % n) * g.pt) % n) % n;  // (both factors < 2^32) position after step j0 - 1
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < SRR_WALK; ++k) {
        c += g.pt;
        if (c >= n) c -= n;
        const uint64_t id = g.base + c;
        cl[k] = (uint32_t)id;
        const bool v = j0 + k < g.yields && ((b.vmask[id >> 6] >> (id & 63)) & 1ull);
        bits |= (uint32_t)v << k;
    }
    return bits;
}

// 256-thread block: exclusive prefix of x over the block, and the total
__device__ __forceinline__ uint32_t block256_excl(uint32_t x, uint32_t* s_w, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = x;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t pre = 0;
    total = 0;
    for (int w = 0; w < 4; ++w) {
        if (w < wave) pre += s_w[w];
        total += s_w[w];
    }
    return pre + incl - x;
}

}  // namespace

// ------------------------------------------------------------------------------------
// End-of-iteration check (SATInstance.h:129-147): first violated clause offset in every generator's
// range (the generators' ranges of SATInstance.h:74-86: t * (m / T), the last one the remainder).
__global__ __launch_bounds__(256) void k_srr_first(LoopBuffers b) {
    if (!b.state->active) return;
    const uint32_t t = blockIdx.x, T = b.srr_T;
    const uint64_t m = b.m, tn = m / T, base = (uint64_t)t * tn, n = (t == T - 1) ? m - base : tn;
    __shared__ unsigned long long s_min;
    if (threadIdx.x == 0) s_min = ~0ull;
    __syncthreads();
    if (n) {
        const uint64_t w_lo = base >> 6, w_hi = (base + n - 1) >> 6;
        for (uint64_t w0 = w_lo; w0 <= w_hi; w0 += blockDim.x) {
            const uint64_t w = w0 + threadIdx.x;
            if (w <= w_hi) {
                uint64_t x = b.vmask[w];
                if (w == w_lo) x &= ~0ull << (base & 63);
                const uint32_t e = (uint32_t)((base + n) & 63);
                if (w == w_hi && e) x &= (1ull << e) - 1ull;
                if (x) atomicMin(&s_min, (unsigned long long)((w << 6) + (uint64_t)__builtin_ctzll(x) - base));
            }
            __syncthreads();
            const bool found = s_min != ~0ull;
            __syncthreads();
            if (found) break;
        }
    }
    if (threadIdx.x == 0) b.srr_first[t] = s_min;
}

// Violated walk steps per virtual block.
__global__ __launch_bounds__(256) void k_srr_count(LoopBuffers b) {
    const uint32_t blk = blockIdx.x;
    const SrrGen g = b.srr_gen[srr_block_gen(b, blk)];
    const uint64_t j0 = (uint64_t)(blk - g.vblk) * SRR_BLK + threadIdx.x * SRR_WALK;
    uint32_t cl[SRR_WALK];
    const uint32_t cnt = (uint32_t)__popc(srr_walk16(b, g, j0, cl));
    __shared__ uint32_t s_w[4];
    uint32_t total;
    (void)block256_excl(cnt, s_w, total);
    if (threadIdx.x == 0) b.srr_bcnt[blk] = total;
}

// Exclusive prefix of the block counts (one workgroup), every generator's first entry, the end row
// of the step table, and the rows of generators without walk steps.
__global__ __launch_bounds__(1024) void k_srr_scan(LoopBuffers b) {
    const SrrPlan pl = *b.srr_plan;
    const uint32_t nblk = pl.nblk, T = pl.T;
    uint32_t* off = b.srr_bcnt + nblk;
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t base = 0; base < nblk; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t x = i < nblk ? b.srr_bcnt[i] : 0u;
        uint32_t incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        uint32_t pre = s_carry, tot = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wave) pre += s_w[w];
            tot += s_w[w];
        }
        if (i < nblk) off[i] = pre + incl - x;
        __syncthreads();
        if (threadIdx.x == 0) s_carry += tot;
        __syncthreads();
    }
    const uint32_t total = s_carry;
    if (threadIdx.x == 0) off[nblk] = total;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < T; t += blockDim.x) {
        const uint64_t v0 = b.srr_gen[t].vblk, v1 = b.srr_gen[t + 1].vblk;
        const uint32_t e0 = v0 < nblk ? off[v0] : total, e1 = v1 < nblk ? off[v1] : total;
        b.srr_gen[t].e0 = e0;
        b.srr_step[pl.steps * T + t] = e1;
        if (v0 == v1)  // (no walk steps: an empty set at every batch step)
            for (uint64_t s = 0; s < pl.steps; ++s) b.srr_step[s * T + t] = e0;
    }
}

// The lists: entry {clause id, width, literal start, 0, first 8 variables (~0 past the width)} of
// every violated walk step, and the first entry of every (batch step, generator).  Step of walk step
// j: the first window's r steps come in batches from step 0; after it, whole walks of p batches.
__global__ __launch_bounds__(256) void k_srr_fill(ClauseView cv, LoopBuffers b) {
    const uint32_t blk = blockIdx.x;
    const SrrPlan pl = *b.srr_plan;
    const uint32_t t = srr_block_gen(b, blk), T = pl.T;
    const SrrGen g = b.srr_gen[t];
    const uint64_t j0 = (uint64_t)(blk - g.vblk) * SRR_BLK + threadIdx.x * SRR_WALK;
    uint32_t cl[SRR_WALK];
    const uint32_t bits = srr_walk16(b, g, j0, cl);
    __shared__ uint32_t s_w[4];
    uint32_t total;
    uint32_t e = b.srr_bcnt[pl.nblk + blk] + block256_excl((uint32_t)__popc(bits), s_w, total);
    const uint64_t B = pl.batch;
    for (int k = 0; k < SRR_WALK; ++k) {
        const uint64_t j = j0 + k;
        if (j >= g.yields) break;
        uint64_t s, w;
        if (j < g.r) { s = j / B; w = j; }
        else {
            const uint64_t q = j - g.r;
            w = q % g.n;
            s = g.b + (q / g.n) * g.p + w / B;
        }
        if (w % B == 0) b.srr_step[s * T + t] = e;  // (the first walk step of the generator's batch)
        if ((bits >> k) & 1u) {
            const uint32_t id = cl[k];
            const uint32_t lb = cv.offs[id], wd = cv.offs[id + 1] - lb;
            uint32_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = (uint32_t)q < wd ? s_var(cv.lits[lb + q]) : 0xFFFFFFFFu;
            uint4* d = reinterpret_cast<uint4*>(b.srr_ent + (uint64_t)e * SRR_ENT_WORDS);
            d[0] = make_uint4(id, wd, lb, 0u);
            d[1] = make_uint4(v[0], v[1], v[2], v[3]);
            d[2] = make_uint4(v[4], v[5], v[6], v[7]);
            ++e;
        }
    }
}

namespace {
constexpr uint32_t SRR_WAVES = SRR_THREADS / 64;
constexpr uint32_t SRR_CAND = 512;          // candidate slots of one gather (all sets)
constexpr uint32_t SRR_KMAX = 256;          // candidates per set
constexpr uint32_t SRR_HASH = 8192;         // >= 2 x SRR_CAND x 8 variables: never more than half full
constexpr uint32_t SRR_COMPLETE = 1u << 31; // (s_cnt) the set's list holds every uncovered entry left
constexpr uint32_t SRR_NONE = ~0u;
constexpr int SRR_GU = 1;                   // list entries per lane in a gather's window (2: 5.8 vs 3.5 us per window, 4% slower overall)

__device__ __forceinline__ uint32_t srr_hslot(uint32_t v) { return (v * 2654435761u) >> 19; }

// Inserts variable v used at sequence position p; returns a position that shares v with an
// earlier one, or SRR_NONE.  The minimum over every insert of a segment is exactly the first
// position q* with a variable some earlier position uses: for a variable with users p1 < p2 < ...,
// whichever of p1, p2 arrives second finds the other (or a larger user) as the slot's minimum and
// reports max(old, p) = p2; every report is the later of two users.  (A clause repeating a
// variable finds its own position: not a conflict.)
__device__ __forceinline__ uint32_t srr_hins(uint32_t* key, uint32_t* pos, uint32_t v, uint32_t p) {
    uint32_t h = srr_hslot(v);
    for (;;) {
        const uint32_t k = atomicCAS(&key[h], SRR_NONE, v);
        if (k == SRR_NONE || k == v) {
            const uint32_t old = atomicMin(&pos[h], p);
            return old == SRR_NONE || old == p ? SRR_NONE : max(old, p);
        }
        h = (h + 1) & (SRR_HASH - 1);
    }
}

// The cover stamps of list entries {id, width, literal start, 0, 8 variables}.  Every stamp read
// here was stored either before this launch or by a wave of this workgroup (one CU), which waits
// for its stores (vmcnt(0)) ahead of the barrier before a gather: workgroup scope, so plain loads
// and stores (no sc1: agent-scope stores drop the cover lines from L2, agent-scope loads bypass
// L1 and were waited one by one).  All of a lane's loads are issued before the first is used, and
// only slots below the wave's widest clause are loaded (each lane's scattered byte load costs the
// CU's address unit a cycle; a 3-SAT list needs 3 of the 8).
template <int U>
__device__ __forceinline__ void srr_cover_test(const ClauseView& cv, const LoopBuffers& b, const uint4 (&hd)[U],
                                               const uint32_t (&v)[U][8], uint32_t stamp, bool (&alive)[U]) {
    uint32_t wmax = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) wmax = max(wmax, alive[u] ? min(hd[u].y, 8u) : 0u);
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
    uint8_t cs[U][8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if ((uint32_t)q < wmax) {
#pragma unroll
            for (int u = 0; u < U; ++u) cs[u][q] = alive[u] && (uint32_t)q < hd[u].y ? b.cover[v[u][q]] : (uint8_t)0;
        }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        bool cov = false;
#pragma unroll
        for (int q = 0; q < 8; ++q) cov |= (uint32_t)q < wmax && cs[u][q] == stamp;
        for (uint32_t q = 8; alive[u] && q < hd[u].y && !cov; ++q)  // (clauses wider than 8: rare)
            cov = b.cover[s_var(cv.lits[hd[u].z + q])] == stamp;
        alive[u] &= !cov;
    }
}

// the first sequence position recorded for variable v, or SRR_NONE
__device__ __forceinline__ uint32_t srr_hget(const uint32_t* key, const uint32_t* pos, uint32_t v) {
    uint32_t h = srr_hslot(v);
    for (;;) {
        const uint32_t k = key[h];
        if (k == v) return pos[h];
        if (k == SRR_NONE) return SRR_NONE;
        h = (h + 1) & (SRR_HASH - 1);
    }
}

// workgroup exclusive scan of one value per thread (SRR_THREADS)
__device__ __forceinline__ uint32_t srr_block_excl(uint32_t x, uint32_t* s_w) {
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
    for (uint32_t w = 0; w < wave; ++w) before += s_w[w];
    __syncthreads();
    return before + incl - x;
}

__device__ __forceinline__ uint32_t srr_wave_min(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o, 64));
    return x;
}
}  // namespace

// The batch steps of the iteration in order; in each, the round robin of populate_mis_parallel
// (SATInstance.h:414-447) over the T lists of the step: t <- (t + 1) % |sets|; a set with no entry
// left whose variables are all uncovered is erased (t is not decremented, so the set moving into
// its place loses its turn), else its first such entry joins the MIS and stamps its variables.
// The MIS size after every step adds to the statistic (SATInstance.h:113-114), then `extra` times more.
//
// The turns run a cycle at a time instead of one by one:
//   gather   every live set's first uncovered entries (up to K; the sets in turn order from the next
//            turn share SRR_CAND slots), with a flag when the list holds all of them;
//   segment  were no turn to find its candidate covered by an earlier pick of the cycle, the turns
//            would take the sets' candidates in order until the first set out of candidates (E
//            turns, closed form over the live list).  The candidates' variables go into an LDS hash
//            with the first sequence position using them; the first turn q* whose candidate has a
//            variable used earlier is where that assumption breaks.  Turns [0, min(q*, E)) are
//            exactly the reference's (each candidate was uncovered at the gather and shares nothing
//            with the cycle's earlier picks, and entries the gather skipped were covered): their picks
//            are committed in order.  At q* the cycle ends (the turn re-runs after a new gather,
//            where the candidate is covered); at E the set out of candidates is erased when its list
//            was complete (then the next segment follows on the same gather) or a new gather runs.
// A clause wider than 8 variables is a candidate only as the first turn of a cycle, alone.
__global__ __launch_bounds__(SRR_THREADS) void k_srr_mis(ClauseView cv, LoopBuffers b) {
    DevState* st = b.state;
    if (!st->active) return;
    const SrrPlan pl = *b.srr_plan;
    const uint32_t T = pl.T, stamp = st->stamp;
    __shared__ uint32_t s_live[RR_TMAX], s_ptr[RR_TMAX], s_end[RR_TMAX];
    __shared__ uint32_t s_base[RR_TMAX], s_cnt[RR_TMAX];  // per set id, this gather
    __shared__ uint32_t s_use[2][RR_TMAX];  // candidates consumed: by segment parity
    __shared__ uint32_t s_cent[SRR_CAND], s_cid[SRR_CAND], s_cw[SRR_CAND], s_cv[SRR_CAND * 8];
    __shared__ uint32_t s_hkey[SRR_HASH], s_hpos[SRR_HASH];
    __shared__ uint32_t s_gcur[SRR_WAVES], s_gcnt[SRR_WAVES], s_gst[SRR_WAVES];
    __shared__ uint32_t s_wc[SRR_WAVES], s_wwide[SRR_WAVES];
    __shared__ uint32_t s_red[4], s_wide, s_tot[2];  // (s_red: {E, q*} by segment parity)
    __shared__ uint32_t s_slotset[SRR_CAND], s_rank[SRR_CAND], s_kc[SRR_CAND];  // (compaction)
    __shared__ uint32_t s_scan[SRR_WAVES];
    __shared__ unsigned long long s_lits;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    if (tid == 0) {
        s_lits = 0;
        s_tot[0] = 0;
        for (int q = 0; q < 4; ++q) s_red[q] = SRR_NONE;
    }
    __syncthreads();
    uint32_t seg = 0;  // segments so far (parity: s_red, s_use)
    uint32_t nm = 0, all_gathers = 0;
    unsigned long long weighted = 0, lits = 0;
#ifdef SRR_PROFILE  // (development: phase clocks of thread 0, printed at the end)
    unsigned long long p_t0 = __builtin_amdgcn_s_memrealtime(), p_g = 0, p_x;
    uint32_t p_segs = 0, p_conf = 0, p_wit = 0, p_cmp = 0;
    unsigned long long p_a = 0, p_b = 0, p_y, p_ph[5] = {0, 0, 0, 0, 0}, p_z;
#define SRR_PH(k) { const unsigned long long z_ = __builtin_amdgcn_s_memrealtime(); p_ph[k] += z_ - p_z; p_z = z_; }
#else
#define SRR_PH(k)
#endif
    for (uint64_t s = 0; s < pl.steps; ++s) {
        uint32_t ent = 0;
        for (uint32_t t = tid; t < T; t += SRR_THREADS) {
            s_ptr[t] = b.srr_step[s * T + t];
            s_end[t] = b.srr_step[(s + 1) * T + t];
            s_live[t] = t;
            ent += s_end[t] - s_ptr[t];
        }
        if (ent) atomicAdd(&s_tot[s & 1], ent);
        if (tid == 0) s_tot[(s + 1) & 1] = 0;
        uint32_t sz = T, tt = 0;  // block-uniform
        __syncthreads();
        // every gather is followed by a pick or an erasure, or by one at the next gather: a step
        // needs at most 2 (entries + T) gathers (a guard against a wrong plan, error 6)
        const uint64_t max_gathers = 2ull * ((uint64_t)s_tot[s & 1] + T) + 8;
        uint64_t gathers = 0;
        while (sz > 0) {
            ++all_gathers;
            if (++gathers > max_gathers) {
                if (tid == 0) { st->error = 6; st->done = 3; }
                return;
            }
            // ---- gather
#ifdef SRR_PROFILE
            p_x = __builtin_amdgcn_s_memrealtime();
#endif
            const uint32_t t0 = (tt + 1) % sz;
            const uint32_t K = max(1u, min(SRR_KMAX, SRR_CAND / sz));
            const uint32_t nsl = min(sz, SRR_CAND / K);  // sets with slots: turn-order offsets [0, nsl)
            for (uint32_t i = tid; i < sz; i += SRR_THREADS) {
                const uint32_t g = s_live[i], d = (i + sz - t0) % sz;
                s_base[g] = d * K;
                s_cnt[g] = 0;
                s_use[seg & 1][g] = 0;
                if (d < nsl) s_slotset[d] = g;
            }
            for (uint32_t h = tid; h < SRR_HASH; h += SRR_THREADS) { s_hkey[h] = SRR_NONE; s_hpos[h] = SRR_NONE; }
            if (tid == 0) s_wide = 0;
            const uint32_t wps = nsl >= SRR_WAVES ? 1u : SRR_WAVES / nsl;  // waves per set
            const uint32_t G = SRR_WAVES / wps;                             // sets per pass
            const uint32_t h = wave / wps, sub = wave % wps;
#ifdef SRR_PROFILE
            p_y = __builtin_amdgcn_s_memrealtime();
            p_a += p_y - p_x;
#endif
            for (uint32_t d0 = 0; d0 < nsl; d0 += G) {
                const uint32_t d = d0 + h;
                const bool mine = h < G && d < nsl;
                const uint32_t g = mine ? s_live[(t0 + d) % sz] : 0u;
                const uint32_t e = mine ? s_end[g] : 0u;
                // (the previous pass's last "more" reads; and every commit's cover stamps must
                // have reached the L2 before the cover loads below: a barrier does not wait for
                // outstanding stores)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (mine && sub == 0 && lane == 0) { s_gcur[h] = s_ptr[g]; s_gcnt[h] = 0; s_gst[h] = 0; }
                __syncthreads();
#ifdef SRR_PROFILE
                { const unsigned long long z = __builtin_amdgcn_s_memrealtime(); p_b += z - p_y; p_y = z; }
#endif
                for (;;) {
                    const bool active = mine && s_gst[h] == 0;
                    const uint32_t i0 = (active ? s_gcur[h] : 0u) + sub * (64u * SRR_GU) + lane;
                    bool alive[SRR_GU];
                    uint4 hd[SRR_GU];
                    uint32_t v[SRR_GU][8];
#pragma unroll
                    for (int u = 0; u < SRR_GU; ++u) {
                        const uint32_t i = i0 + 64u * u;
                        alive[u] = active && i < e;
                        hd[u] = make_uint4(0, 0, 0, 0);
                        uint4 x = make_uint4(0, 0, 0, 0), y = x;
                        if (alive[u]) {
                            const uint4* dp = reinterpret_cast<const uint4*>(b.srr_ent + (uint64_t)i * SRR_ENT_WORDS);
                            hd[u] = dp[0];
                            x = dp[1];
                            y = dp[2];
                        }
                        v[u][0] = x.x; v[u][1] = x.y; v[u][2] = x.z; v[u][3] = x.w;
                        v[u][4] = y.x; v[u][5] = y.y; v[u][6] = y.z; v[u][7] = y.w;
                    }
                    srr_cover_test<SRR_GU>(cv, b, hd, v, stamp, alive);
                    // candidate order: entry u = 0's 64 lanes, then u = 1's
                    unsigned long long bal[SRR_GU];
                    uint32_t wcnt = 0, wwide = SRR_NONE;
#pragma unroll
                    for (int u = 0; u < SRR_GU; ++u) {
                        bal[u] = __ballot(alive[u]);
                        const unsigned long long wb = __ballot(alive[u] && hd[u].y > 8);
                        if (wb && wwide == SRR_NONE)
                            wwide = wcnt + (uint32_t)__popcll(bal[u] & ((1ull << __builtin_ctzll(wb)) - 1ull));
                        wcnt += (uint32_t)__popcll(bal[u]);
                    }
                    if (lane == 0) {
                        s_wc[wave] = wcnt;
                        s_wwide[wave] = wwide;
                    }
                    __syncthreads();
                    if (active) {
                        // this wave's first candidate index, the group's first wide one, the group total
                        uint32_t pre = s_gcnt[h], off = 0, fw = SRR_NONE;
                        for (uint32_t u = 0; u < wps; ++u) {
                            const uint32_t wv = h * wps + u;
                            if (u == sub) off = pre;
                            if (fw == SRR_NONE && s_wwide[wv] != SRR_NONE) fw = pre + s_wwide[wv];
                            pre += s_wc[wv];
                        }
                        const bool takewide = fw == 0 && d == 0;
                        const uint32_t lim = takewide ? 1u : min(K, fw);
                        uint32_t r = off;
#pragma unroll
                        for (int u = 0; u < SRR_GU; ++u) {
                            const uint32_t ru = r + (uint32_t)__popcll(bal[u] & lt_mask);
                            if (alive[u] && ru < lim) {
                                const uint32_t slot = d * K + ru;
                                s_cent[slot] = i0 + 64u * u;
                                s_cid[slot] = hd[u].x;
                                s_cw[slot] = hd[u].y;
                                if (hd[u].y <= 8) {
#pragma unroll
                                    for (int q = 0; q < 8; ++q) s_cv[slot * 8 + q] = v[u][q];
                                } else {
                                    s_cv[slot * 8] = hd[u].z;
                                }
                            }
                            r += (uint32_t)__popcll(bal[u]);
                        }
                        if (sub == 0 && lane == 0) {
                            const uint32_t cur = s_gcur[h] + wps * 64u * SRR_GU, n = min(pre, lim);
                            uint32_t stt = 0;
                            if (fw != SRR_NONE || pre > K) stt = 2;        // truncated
                            else if (cur >= e) stt = 1;                    // complete
                            else if (pre == K) stt = 2;
                            if (takewide) s_wide = 1;
                            s_gcnt[h] = n;
                            s_gcur[h] = cur;
                            s_gst[h] = stt;
                            if (stt) s_cnt[g] = n | (stt == 1 ? SRR_COMPLETE : 0u);
                        }
                    }
                    __syncthreads();
#ifdef SRR_PROFILE
                    ++p_wit;
#endif
                    bool more = false;
                    for (uint32_t u = 0; u < G && d0 + u < nsl; ++u) more |= s_gst[u] == 0;
                    if (!more) break;
                }
            }
            __syncthreads();
            if (s_wide) {  // a wide first candidate runs alone: every other set stops at its turn
                for (uint32_t i = tid; i < sz; i += SRR_THREADS)
                    if (i != t0) s_cnt[s_live[i]] = 0;
                __syncthreads();
            }
            // ---- segments on this gather
#ifdef SRR_PROFILE
            { const unsigned long long y = __builtin_amdgcn_s_memrealtime(); p_g += y - p_x; p_x = y; }
#endif
            uint32_t qb = 0;
            for (;;) {
#ifdef SRR_PROFILE
                p_z = __builtin_amdgcn_s_memrealtime();
#endif
                const uint32_t ts = (tt + 1) % sz, pr = seg & 1u;
                uint32_t* use = s_use[pr];
                uint32_t* red = s_red + 2 * pr;  // (reset during the previous segment)
                uint32_t em = SRR_NONE;
                for (uint32_t i = tid; i < sz; i += SRR_THREADS) {
                    const uint32_t g = s_live[i], d = (i + sz - ts) % sz;
                    em = min(em, d + ((s_cnt[g] & ~SRR_COMPLETE) - use[g]) * sz);
                }
                em = srr_wave_min(em);
                if (lane == 0 && em != SRR_NONE) atomicMin(&red[0], em);
                __syncthreads();
                const uint32_t E = red[0];
                SRR_PH(0)
                if (tid == 0) { s_red[2 * (pr ^ 1u)] = SRR_NONE; s_red[2 * (pr ^ 1u) + 1] = SRR_NONE; }
                uint32_t qm = SRR_NONE;  // (positions are relative to the cycle: qb + j)
                for (uint32_t j = tid; j < E; j += SRR_THREADS) {
                    const uint32_t g = s_live[(ts + j) % sz], slot = s_base[g] + use[g] + j / sz;
                    const uint32_t w = s_cw[slot];
                    if (w <= 8)
                        for (uint32_t q = 0; q < w; ++q) qm = min(qm, srr_hins(s_hkey, s_hpos, s_cv[slot * 8 + q], qb + j));
                }
                SRR_PH(1)
                qm = srr_wave_min(qm);
                if (lane == 0 && qm != SRR_NONE) atomicMin(&red[1], qm - qb);
                __syncthreads();
                const uint32_t A = min(red[1], E);  // turns taken in this segment
                SRR_PH(2)
                for (uint32_t j = tid; j < A; j += SRR_THREADS) {
                    const uint32_t g = s_live[(ts + j) % sz], slot = s_base[g] + use[g] + j / sz;
                    const uint32_t w = s_cw[slot];
                    for (uint32_t q = 0; q < w; ++q) {
                        const uint32_t var = w <= 8 ? s_cv[slot * 8 + q] : s_var(cv.lits[s_cv[slot * 8] + q]);
                        b.cover[var] = (uint8_t)stamp;  // (workgroup scope: srr_cover_test)
                    }
                    b.tmis[nm + j] = s_cid[slot];
                    lits += w;
                }
                // consumed counts into the other parity (the commits above still read this one)
                for (uint32_t i = tid; i < sz; i += SRR_THREADS) {
                    const uint32_t d = (i + sz - ts) % sz, g = s_live[i];
                    const uint32_t u = use[g] + (A > d ? (A - d + sz - 1) / sz : 0u);
                    s_use[pr ^ 1u][g] = u;
                    if (A > d) s_ptr[g] = s_cent[s_base[g] + u - 1] + 1;
                }
                __syncthreads();
                SRR_PH(3)
                ++seg;
                nm += A;
                qb += A;
#ifdef SRR_PROFILE
                ++p_segs;
                p_conf += A < E;
#endif
                if (A > 0) tt = (ts + A - 1) % sz;
                if (A < E) {
                    // a covered candidate (the turn at q* re-runs): instead of a new gather, the
                    // sets' unconsumed candidates minus those an accepted pick of this cycle covers
                    // (a variable with a position below qb in the hash) become their lists, and the
                    // hash starts afresh.  Every candidate left was uncovered at the gather and
                    // shares nothing with the picks since; the candidate at q* is dropped.
                    if (s_wide) break;  // (a wide first candidate's cycle: new gather)
                    uint32_t* use2 = s_use[seg & 1];
                    const uint32_t ns = nsl * K;
                    bool keep = false;
                    uint32_t d = 0, kent = 0, kid = 0, kw = 0, kv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    if (tid < ns) {
                        d = tid / K;
                        const uint32_t r = tid - d * K, g = s_slotset[d];
                        if (r >= use2[g] && r < (s_cnt[g] & ~SRR_COMPLETE)) {
                            kent = s_cent[tid];
                            kid = s_cid[tid];
                            kw = s_cw[tid];
#pragma unroll
                            for (int q = 0; q < 8; ++q) kv[q] = s_cv[tid * 8 + q];
                            keep = true;
                            for (uint32_t q = 0; q < kw && q < 8; ++q) keep &= srr_hget(s_hkey, s_hpos, kv[q]) >= qb;
                        }
                    }
                    if (tid < nsl) s_kc[tid] = 0;
                    const uint32_t ex = srr_block_excl(keep ? 1u : 0u, s_scan);
                    if (tid < ns) s_rank[tid] = ex;
                    __syncthreads();
                    if (keep) {
                        const uint32_t slot = d * K + (ex - s_rank[d * K]);
                        s_cent[slot] = kent;
                        s_cid[slot] = kid;
                        s_cw[slot] = kw;
#pragma unroll
                        for (int q = 0; q < 8; ++q) s_cv[slot * 8 + q] = kv[q];
                        atomicAdd(&s_kc[d], 1u);
                    }
                    for (uint32_t hh = tid; hh < SRR_HASH; hh += SRR_THREADS) { s_hkey[hh] = SRR_NONE; s_hpos[hh] = SRR_NONE; }
                    __syncthreads();
                    if (tid < nsl) {
                        const uint32_t g = s_slotset[tid];
                        s_cnt[g] = s_kc[tid] | (s_cnt[g] & SRR_COMPLETE);
                        use2[g] = 0;
                    }
                    __syncthreads();
                    qb = 0;
#ifdef SRR_PROFILE
                    ++p_cmp;
#endif
                    continue;
                }
                const uint32_t te = (tt + 1) % sz, ge = s_live[te];
                if (!(s_cnt[ge] & SRR_COMPLETE)) break;  // out of gathered candidates: new gather
                // the set has no uncovered entry left: erase live[te]
                for (uint32_t q0 = te; q0 + 1 < sz; q0 += SRR_THREADS) {
                    const uint32_t q = q0 + tid;
                    const uint32_t x = q + 1 < sz ? s_live[q + 1] : 0u;
                    __syncthreads();
                    if (q + 1 < sz) s_live[q] = x;
                }
                __syncthreads();
                --sz;
                tt = te;
                SRR_PH(4)
                if (sz == 0) break;
            }
        }
        weighted += nm;
        __syncthreads();
    }
#ifdef SRR_PROFILE
    if (tid == 0)
        printf("srr_prof T %u steps %llu picks %u gathers %u window_iters %u segs %u conflicts %u compactions %u ticks total %llu gather %llu reset %llu firstbar %llu seg E %llu ins %llu det %llu com %llu erase %llu\n",
               T, (unsigned long long)pl.steps, nm, all_gathers, p_wit, p_segs, p_conf, p_cmp,
               __builtin_amdgcn_s_memrealtime() - p_t0, p_g, p_a, p_b, p_ph[0], p_ph[1], p_ph[2], p_ph[3], p_ph[4]);
#endif
    weighted += (unsigned long long)nm * pl.extra;
    if (lits) atomicAdd(&s_lits, lits);
    __syncthreads();
    if (tid == 0) {
        st->tmis_cnt = nm;
        st->tail_rounds = all_gathers;  // (the statistics' lfmis_tail_rounds: gathers of the iteration)
        if (all_gathers > st->max_rounds) st->max_rounds = all_gathers;
        b.tile_stats[0] += weighted;
        b.tile_stats[1] += s_lits;
    }
}

hipError_t launch_srr_first(const LoopBuffers& b, hipStream_t s) {
    hipLaunchKernelGGL(k_srr_first, dim3(b.srr_T), dim3(256), 0, s, b);
    return hipGetLastError();
}

hipError_t launch_srr_lists(const ClauseView& cv, const LoopBuffers& b, uint32_t nblk, hipStream_t s) {
    if (nblk) hipLaunchKernelGGL(k_srr_count, dim3(nblk), dim3(256), 0, s, b);
    hipLaunchKernelGGL(k_srr_scan, dim3(1), dim3(1024), 0, s, b);
    if (nblk) hipLaunchKernelGGL(k_srr_fill, dim3(nblk), dim3(256), 0, s, cv, b);
    return hipGetLastError();
}

hipError_t launch_srr_mis(const ClauseView& cv, const LoopBuffers& b, hipStream_t s) {
    hipLaunchKernelGGL(k_srr_mis, dim3(1), dim3(SRR_THREADS), 0, s, cv, b);
    return hipGetLastError();
}

}  // namespace alll
