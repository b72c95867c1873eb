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
//   k_srr_mis     runs the batch steps' round robins in order, one 1024-thread workgroup: a turn is
//                 one parallel scan of the set's next entries against the cover stamps (the filter
//                 against the MIS so far and the round robin's erasures are both the "first entry
//                 with no covered variable" rule), the pick stamps its variables.
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
// entry i has a variable covered by the MIS of this iteration (cover stamps read at agent scope: the
// picks of this workgroup's earlier turns are stored the same way)
__device__ __forceinline__ bool srr_covered(const ClauseView& cv, const LoopBuffers& b, uint32_t i, uint32_t stamp) {
    const uint4* d = reinterpret_cast<const uint4*>(b.srr_ent + (uint64_t)i * SRR_ENT_WORDS);
    const uint4 h = d[0], x = d[1], y = d[2];
    const uint32_t wd = h.y;
    bool cov = false;
    if (wd <= 8) {
        const uint32_t v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if ((uint32_t)q < wd)
                cov |= __hip_atomic_load(&b.cover[v[q]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == stamp;
    } else {
        for (uint32_t q = 0; q < wd && !cov; ++q)
            cov = __hip_atomic_load(&b.cover[s_var(cv.lits[h.z + q])], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == stamp;
    }
    return cov;
}
}  // namespace

// The batch steps of the iteration in order; in each, the round robin of populate_mis_parallel
// (SATInstance.h:414-447) over the T lists of the step: t <- (t + 1) % |sets|; a set with no entry
// left whose variables are all uncovered is erased (t is not decremented, so the set moving into
// its place loses its turn), else its first such entry joins the MIS and stamps its variables.
// The MIS size after every step adds to the statistic (SATInstance.h:113-114), then `extra` times more.
__global__ __launch_bounds__(SRR_THREADS) void k_srr_mis(ClauseView cv, LoopBuffers b) {
    DevState* st = b.state;
    if (!st->active) return;
    const SrrPlan pl = *b.srr_plan;
    const uint32_t T = pl.T, stamp = st->stamp;
    __shared__ uint32_t s_live[RR_TMAX], s_ptr[RR_TMAX], s_end[RR_TMAX];
    __shared__ uint32_t s_wmin[SRR_THREADS / 64];
    __shared__ unsigned long long s_lits;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_lits = 0;
    uint32_t nm = 0;
    unsigned long long weighted = 0;
    for (uint64_t s = 0; s < pl.steps; ++s) {
        for (uint32_t t = tid; t < T; t += SRR_THREADS) {
            s_ptr[t] = b.srr_step[s * T + t];
            s_end[t] = b.srr_step[(s + 1) * T + t];
            s_live[t] = t;
        }
        __syncthreads();
        uint32_t size = T, tt = 0;
        while (size > 0) {
            tt = (tt + 1) % size;
            const uint32_t g = s_live[tt];
            const uint32_t e = s_end[g];
            uint32_t p0 = s_ptr[g], front = ~0u;
            while (p0 < e) {
                const uint32_t i = p0 + tid;
                const bool alive = i < e && !srr_covered(cv, b, i, stamp);
                const unsigned long long bal = __ballot(alive);
                if (lane == 0) s_wmin[wave] = bal ? p0 + wave * 64u + (uint32_t)__builtin_ctzll(bal) : ~0u;
                __syncthreads();
                uint32_t f = ~0u;
#pragma unroll
                for (int w = 0; w < SRR_THREADS / 64; ++w) f = min(f, s_wmin[w]);
                __syncthreads();
                if (f != ~0u) { front = f; break; }
                p0 += SRR_THREADS;
            }
            if (front == ~0u) {  // erase live[tt]
                for (uint32_t q0 = tt; q0 + 1 < size; q0 += SRR_THREADS) {
                    const uint32_t q = q0 + tid;
                    const uint32_t x = q + 1 < size ? s_live[q + 1] : 0u;
                    __syncthreads();
                    if (q + 1 < size) s_live[q] = x;
                    __syncthreads();
                }
                --size;
                continue;
            }
            if (tid == front - p0) {
                const uint4* d = reinterpret_cast<const uint4*>(b.srr_ent + (uint64_t)front * SRR_ENT_WORDS);
                const uint4 h = d[0], x = d[1], y = d[2];
                const uint32_t v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
                for (uint32_t q = 0; q < h.y; ++q) {
                    const uint32_t var = q < 8 ? v[q] : s_var(cv.lits[h.z + q]);
                    __hip_atomic_store(&b.cover[var], (uint8_t)stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                b.tmis[nm] = h.x;
                s_lits += h.y;
                s_ptr[g] = front + 1;
                // the stamps must have reached the L2 before any wave's next cover load: the
                // barrier below does not wait for this thread's outstanding stores (a missed stamp
                // lets a later front share a variable with this pick -- seen once in 550 cases)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            ++nm;
            __syncthreads();
        }
        weighted += nm;
        // (a step can end with a turn that passed no barrier -- the last set erased without a scan:
        // every thread must be done reading this step's set bounds before they are rewritten)
        __syncthreads();
    }
    weighted += (unsigned long long)nm * pl.extra;
    __syncthreads();
    if (tid == 0) {
        st->tmis_cnt = nm;
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
