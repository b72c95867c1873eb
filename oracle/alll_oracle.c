/*
 * alll_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference's serial Moser-Tardos resample loop
 * (xmif1/ALLLSatisfiabilitySolver).  It is the parity checker for the HIP product
 * path and must never be linked into, or called by, the product
 * (alllsatisfiabilitysolver_amd/).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.
 *
 * Parity pinning: every deterministic function here (eval, LFMIS, round-robin
 * MIS, chunking, statistics arithmetic, DIMACS semantics) is checked against
 * golden vectors produced by the reference's own code (oracle/ref_probe.cpp
 * compiled from /root/reference sources, fixtures in tests/golden/).  The product
 * RNG is Philox4x32-10 (pinned against the Random123 known-answer vectors) in place
 * of std::random_device; the reference's own stream (RBG over libstdc++'s
 * minstd_rand0 and uniform_int_distribution, engines seeded from the probe's
 * random_device stand-in) is restated too (orc_solve_refrng) and pinned to the
 * reference's recorded T = 1 trajectories.
 *
 * Citations are to files under the reference repository.
 */
#include "alll_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 reference constants).      */
/* Replaces RBG<default_random_engine>::sample (RandomBoolGenerator.h:35-44). */
/* ------------------------------------------------------------------------- */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* A0 word w (variables 32w..32w+31) = Philox(key=seed, ctr={w, 0, 0xFFFFFFFF, 0}).x.
 * Replaces the random_device-seeded fill of VariablesArray (VariablesArray.h:23-34). */
void orc_init_assignment(uint64_t seed, uint32_t n_vars, uint32_t* A) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t nw = (n_vars + 31) / 32;
    for (uint32_t w = 0; w < nw; ++w) {
        uint32_t ctr[4] = {w, 0u, 0xFFFFFFFFu, 0u}, o[4];
        orc_philox4x32_10(ctr, key, o);
        uint32_t word = o[0];
        if (w == nw - 1 && (n_vars & 31)) word &= (1u << (n_vars & 31)) - 1u;
        A[w] = word;
    }
}

/* Resampled value of variable v in resample round `iter` (0-based): bit v % 32 of
 * Philox(key=seed, ctr={v / 32, iter_lo, 0, iter_hi}).x -- one draw per assignment word and
 * round, like the initial assignment (ctr c2 = 0 here, 0xFFFFFFFF there: disjoint streams).
 * Replaces `vars[l>>1] = rbg.sample()` (SATInstance.h:358-360). */
uint32_t orc_resample_bit(uint64_t seed, uint64_t iter, uint32_t v) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {v >> 5, (uint32_t)iter, 0u, (uint32_t)(iter >> 32)}, o[4];
    orc_philox4x32_10(ctr, key, o);
    return (o[0] >> (v & 31u)) & 1u;
}

/* ------------------------------------------------------------------------- */
/* The reference's own RNG, for the reference-RNG mode:       */
/* RBG<default_random_engine> (RandomBoolGenerator.h:29-52) over libstdc++'s   */
/* (GCC 11, the toolchain here; unpinned by the reference) default_random_    */
/* engine = minstd_rand0 = linear_congruential_engine<uint_fast32_t, 16807, 0, */
/* 2147483647> and uniform_int_distribution<unsigned long long> (bits/         */
/* uniform_int_dist.h: downscaling by rejection, upscaling by recursion), each */
/* engine seeded with one std::random_device{}() value (VariablesArray.h:24,   */
/* SATInstance.h:346).  random_device is the reference's only nondeterminism:  */
/* the probe (oracle/ref_probe.cpp) replaces it with a 64-bit LCG, restated     */
/* here, so the reference's whole T = 1 trajectory is reproducible.            */
/* ------------------------------------------------------------------------- */
uint32_t orc_refrng_rd_next(uint64_t* state) {
    *state = *state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*state >> 33);
}

#define MINSTD_M 2147483647ull
#define MINSTD_MIN 1ull
#define MINSTD_RANGE (MINSTD_M - 1ull - MINSTD_MIN) /* max() - min() */

static void minstd_seed(uint64_t* x, uint64_t s) {
    const uint64_t r = s % MINSTD_M;
    *x = r ? r : 1ull;
}
static uint64_t minstd_next(uint64_t* x) {
    *x = (*x * 16807ull) % MINSTD_M;
    return *x;
}

/* uniform_int_distribution<unsigned long long>(0, urange)(engine) */
static uint64_t uid_u64(uint64_t* x, uint64_t urange) {
    uint64_t ret;
    if (MINSTD_RANGE > urange) {
        const uint64_t uerange = urange + 1, scaling = MINSTD_RANGE / uerange, past = uerange * scaling;
        do ret = minstd_next(x) - MINSTD_MIN;
        while (ret >= past);
        ret /= scaling;
    } else if (MINSTD_RANGE < urange) {
        uint64_t tmp;
        do {
            const uint64_t uerngrange = MINSTD_RANGE + 1;
            tmp = uerngrange * uid_u64(x, urange / uerngrange);
            ret = tmp + (minstd_next(x) - MINSTD_MIN);
        } while (ret > urange || ret < tmp);
    } else {
        ret = minstd_next(x) - MINSTD_MIN;
    }
    return ret;
}

void orc_rbg_seed(orc_rbg* g, uint32_t seed) {
    minstd_seed(&g->x, seed);
    g->m = 1;
}
/* RBG::sample: a 64-bit draw | bit 63 serves 63 bits, lowest first */
uint32_t orc_rbg_sample(orc_rbg* g) {
    if (g->m == 1) g->m = uid_u64(&g->x, ~0ull) | (1ull << 63);
    const uint32_t b = (uint32_t)(g->m & 1u);
    g->m >>= 1;
    return b;
}

/* VariablesArray(n) (VariablesArray.h:23-34): one random_device value seeds the engine, then
 * one RBG bit per variable in index order */
void orc_refrng_init(uint64_t* rd_state, uint32_t n_vars, uint32_t* A) {
    orc_rbg g;
    orc_rbg_seed(&g, orc_refrng_rd_next(rd_state));
    memset(A, 0, sizeof(uint32_t) * ((n_vars + 31) / 32));
    for (uint32_t v = 0; v < n_vars; ++v) A[v >> 5] |= orc_rbg_sample(&g) << (v & 31);
}

/* ------------------------------------------------------------------------- */
/* Synthetic instance generator (shared specification with the product's      */
/* generator; both are checked equal in tests).  Counter-based per clause.     */
/* ------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Draw variable index in [0,n): uniform (kind 0) or power-law P(v) ~ (v+1)^-0.8
 * (kind 1: v = floor(n * u^5), u a 32-bit fixed-point uniform). */
static inline uint32_t draw_var(uint64_t r, uint32_t n, int kind) {
    uint64_t u = r >> 32;
    if (kind == 1) {
        uint64_t p = u;
        for (int i = 0; i < 4; ++i) p = (p * u) >> 32;
        u = p;
    }
    return (uint32_t)((u * (uint64_t)n) >> 32);
}

int orc_generate_ksat(uint64_t gen_seed, uint32_t n_vars, uint64_t n_clauses, uint32_t k,
                      int kind, uint64_t c_begin, uint64_t c_end, uint32_t* lits) {
    if (k == 0 || k > 64 || n_vars < k || c_end > n_clauses || c_begin > c_end) return -1;
    for (uint64_t c = c_begin; c < c_end; ++c) {
        uint64_t s = mix64(gen_seed ^ mix64(c + 0x632BE59BD9B4E019ull));
        uint32_t* out = lits + (c - c_begin) * k;
        for (uint32_t j = 0; j < k; ++j) {
            for (;;) {
                s += 0x9E3779B97F4A7C15ull;
                uint64_t r = mix64(s);
                uint32_t v = draw_var(r, n_vars, kind);
                int dup = 0;
                for (uint32_t q = 0; q < j; ++q) dup |= ((out[q] >> 1) == v);
                if (!dup) { out[j] = 2u * v + (uint32_t)(r & 1u); break; }
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Clause evaluation: Clause<T>::is_not_satisfied (Clause.h:34-46); literal l   */
/* is true iff vars[l>>1] XOR (l&1); a clause is violated iff no literal true. */
/* ------------------------------------------------------------------------- */
static inline uint32_t abit(const uint32_t* A, uint32_t v) { return (A[v >> 5] >> (v & 31)) & 1u; }

int orc_clause_violated(const uint64_t* offs, const uint32_t* lits, const uint32_t* A, uint64_t c) {
    for (uint64_t j = offs[c]; j < offs[c + 1]; ++j) {
        uint32_t l = lits[j];
        if (abit(A, l >> 1) != (l & 1u)) return 0;
    }
    return 1;
}

/* Violated collection (SATInstance.h:264-280) as a bitmask (bit c of word c/64). */
uint64_t orc_eval(uint64_t m, const uint64_t* offs, const uint32_t* lits, const uint32_t* A,
                  uint64_t* vmask) {
    uint64_t cnt = 0, nw = (m + 63) / 64;
    memset(vmask, 0, nw * sizeof(uint64_t));
    for (uint64_t c = 0; c < m; ++c) {
        if (orc_clause_violated(offs, lits, A, c)) {
            vmask[c >> 6] |= 1ull << (c & 63);
            ++cnt;
        }
    }
    return cnt;
}

uint64_t orc_mask_to_list(uint64_t m, const uint64_t* vmask, uint32_t* U) {
    uint64_t n = 0;
    for (uint64_t c = 0; c < m; ++c)
        if ((vmask[c >> 6] >> (c & 63)) & 1ull) U[n++] = (uint32_t)c;
    return n;
}

/* ------------------------------------------------------------------------- */
/* MIS.  T=1: populate_mis_parallel (SATInstance.h:391-451) with one set is the */
/* lexicographically-first MIS of U in clause order under dependent_clauses    */
/* (shares a variable, sign ignored; SATInstance.h:369-389).                   */
/* ------------------------------------------------------------------------- */
static int touches(const uint64_t* offs, const uint32_t* lits, const uint8_t* used, uint32_t c) {
    for (uint64_t j = offs[c]; j < offs[c + 1]; ++j)
        if (used[lits[j] >> 1]) return 1;
    return 0;
}
static void mark(const uint64_t* offs, const uint32_t* lits, uint8_t* used, uint32_t c, uint8_t val) {
    for (uint64_t j = offs[c]; j < offs[c + 1]; ++j) used[lits[j] >> 1] = val;
}

uint64_t orc_lfmis(uint32_t n_vars, const uint64_t* offs, const uint32_t* lits,
                   const uint32_t* U, uint64_t nu, uint32_t* M, uint8_t* scratch_used) {
    uint64_t nm = 0;
    for (uint64_t i = 0; i < nu; ++i) {
        uint32_t c = U[i];
        if (!touches(offs, lits, scratch_used, c)) {
            M[nm++] = c;
            mark(offs, lits, scratch_used, c, 1);
        }
    }
    for (uint64_t i = 0; i < nm; ++i) mark(offs, lits, scratch_used, M[i], 0); /* restore */
    (void)n_vars;
    return nm;
}

/* Chunk of clause c under example/main.cpp:149-178 (chunk_size = ceil(m/T);
 * t advances by one whenever c > (t+1)*chunk_size -- chunk 0 holds chunk+1). */
void orc_chunk_bounds(uint64_t m, uint32_t T, uint64_t* starts /* T+1 */) {
    uint64_t chunk = (m + T - 1) / T; /* ceil(c_num / (double) n_threads) for int ranges */
    uint32_t t = 0;
    for (uint32_t q = 0; q <= T; ++q) starts[q] = m;
    starts[0] = 0;
    for (uint64_t c = 0; c < m; ++c) {
        if (c > (uint64_t)(t + 1) * chunk) { t += 1; starts[t] = c; }
    }
    /* chunks that received no clause start at m (empty) */
    for (uint32_t q = 1; q <= T; ++q)
        if (starts[q] < starts[q - 1]) starts[q] = starts[q - 1];
}

/* T>1 round-robin MIS (SATInstance.h:414-447): t starts at 0; loop while sets
 * remain: t=(t+1)%|sets|; an empty set is erased (and, because t is not
 * decremented, its successor is skipped); otherwise its front clause is popped
 * into M and every dependent clause is erased from every set.  Dependents are
 * removed lazily here (skipped at the front), which yields the same fronts and
 * the same emptiness tests as the eager vector::erase of the reference. */
uint64_t orc_rr_mis(uint32_t n_vars, const uint64_t* offs, const uint32_t* lits,
                    const uint32_t* U, uint64_t nu, uint32_t T, const uint64_t* chunk_starts,
                    uint32_t* M, uint8_t* scratch_used) {
    uint64_t* head = (uint64_t*)malloc(sizeof(uint64_t) * T);
    uint64_t* tail = (uint64_t*)malloc(sizeof(uint64_t) * T);
    uint32_t* live = (uint32_t*)malloc(sizeof(uint32_t) * T);
    /* split U (sorted) into per-chunk ranges */
    uint64_t p = 0;
    for (uint32_t q = 0; q < T; ++q) {
        head[q] = p;
        while (p < nu && U[p] < chunk_starts[q + 1]) ++p;
        tail[q] = p;
        live[q] = q;
    }
    uint32_t nlive = T;
    uint64_t nm = 0;
    uint32_t t = 0;
    while (nlive > 0) {
        t = (t + 1) % nlive;
        uint32_t s = live[t];
        while (head[s] < tail[s] && touches(offs, lits, scratch_used, U[head[s]])) ++head[s];
        if (head[s] == tail[s]) {
            for (uint32_t q = t; q + 1 < nlive; ++q) live[q] = live[q + 1];
            --nlive;
            continue;
        }
        uint32_t c = U[head[s]++];
        M[nm++] = c;
        mark(offs, lits, scratch_used, c, 1);
    }
    for (uint64_t i = 0; i < nm; ++i) mark(offs, lits, scratch_used, M[i], 0);
    free(head); free(tail); free(live);
    (void)n_vars;
    return nm;
}

/* ------------------------------------------------------------------------- */
/* Resample loop (parallel_solve, SATInstance.h:217-320; T=1 or T chunks) with */
/* Philox resampling.  Statistics semantics (SATInstance.h:25-32, 313-317):    */
/* n_iterations counts every eval pass including the final zero pass;          */
/* n_resamples = sum of clause lengths over all MIS clauses; avg_mis_size =    */
/* floor(sum|M| / n_iterations).                                               */
/* max_iters (0 = unlimited) caps eval passes; a capped pass does not resample. */
/* ------------------------------------------------------------------------- */
/* rd_state != NULL: the reference-RNG mode -- every resample round draws from a fresh
 * RBG<default_random_engine> seeded by the next random_device value (resample_clauses,
 * SATInstance.h:340-365, with T = 1: bits in MIS pick order, literal order) instead of Philox */
static int solve_sets(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
                      uint64_t seed, uint64_t max_iters, uint32_t T, const uint64_t* chunk_starts,
                      uint32_t* A, orc_stats* st, orc_iter_cb cb, void* cb_user, uint64_t* rd_state) {
    uint64_t nw = (m + 63) / 64;
    uint64_t* vmask = (uint64_t*)calloc(nw ? nw : 1, sizeof(uint64_t));
    uint32_t* U = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint32_t* M = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint8_t* used = (uint8_t*)calloc(n_vars ? n_vars : 1, 1);
    memset(st, 0, sizeof(*st));
    uint64_t sum_mis = 0;
    int solved = 0;
    for (;;) {
        st->n_iterations += 1;
        uint64_t nu = orc_eval(m, offs, lits, A, vmask);
        st->last_violated = nu;
        if (nu == 0) { solved = 1; break; }
        if (max_iters && st->n_iterations >= max_iters) break;
        orc_mask_to_list(m, vmask, U);
        uint64_t nm = T > 1 ? orc_rr_mis(n_vars, offs, lits, U, nu, T, chunk_starts, M, used)
                            : orc_lfmis(n_vars, offs, lits, U, nu, M, used);
        sum_mis += nm;
        uint64_t dres = 0, iter = st->n_iterations - 1;
        orc_rbg g;
        if (rd_state) orc_rbg_seed(&g, orc_refrng_rd_next(rd_state));
        for (uint64_t i = 0; i < nm; ++i) {
            uint32_t c = M[i];
            for (uint64_t j = offs[c]; j < offs[c + 1]; ++j) {
                uint32_t v = lits[j] >> 1;
                uint32_t b = rd_state ? orc_rbg_sample(&g) : orc_resample_bit(seed, iter, v);
                A[v >> 5] = (A[v >> 5] & ~(1u << (v & 31))) | (b << (v & 31));
            }
            dres += offs[c + 1] - offs[c];
        }
        st->n_resamples += dres;
        if (cb) cb(cb_user, st->n_iterations, nu, nm, dres, A);
    }
    st->sum_mis_size = sum_mis;
    st->avg_mis_size = st->n_iterations ? sum_mis / st->n_iterations : 0;
    st->solved = solved;
    free(vmask); free(U); free(M); free(used);
    return solved ? 0 : 1;
}

int orc_solve(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
              uint64_t seed, uint64_t max_iters, uint32_t* A, orc_stats* st,
              orc_iter_cb cb, void* cb_user) {
    return solve_sets(n_vars, m, offs, lits, seed, max_iters, 1, 0, A, st, cb, cb_user, NULL);
}

/* orc_solve in the reference-RNG mode: A is initialised here (orc_refrng_init) from the
 * random_device stand-in seeded with rd_seed, then every resample round takes the next value */
int orc_solve_refrng(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
                     uint64_t rd_seed, uint64_t max_iters, uint32_t* A, orc_stats* st,
                     orc_iter_cb cb, void* cb_user) {
    uint64_t rd = rd_seed;
    orc_refrng_init(&rd, n_vars, A);
    return solve_sets(n_vars, m, offs, lits, 0, max_iters, 1, 0, A, st, cb, cb_user, &rd);
}

/* parallel_solve with T > 1 clause chunks (chunk q = clauses [chunk_starts[q],
 * chunk_starts[q+1])): the MIS of every iteration is the round-robin greedy of
 * populate_mis_parallel (orc_rr_mis); everything else as orc_solve. */
int orc_solve_rr(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
                 uint64_t seed, uint64_t max_iters, uint32_t T, const uint64_t* chunk_starts,
                 uint32_t* A, orc_stats* st, orc_iter_cb cb, void* cb_user) {
    return solve_sets(n_vars, m, offs, lits, seed, max_iters, T, chunk_starts, A, st, cb, cb_user, NULL);
}

/* ------------------------------------------------------------------------- */
/* Streaming solve, SATInstance::solve(getEnumeratedClause, n_clauses,       */
/* batch_size) (SATInstance.h:70-153) with one thread.                        */
/*  - ClauseGenerator (ClauseGenerator.h:33-70) yields clause indices         */
/*    c <- (c + P) % m, P = 9223372036854775783, c starting at 0 and never    */
/*    reset: over the whole run the yield sequence is s_j = j*P mod m,        */
/*    j = 1, 2, ...;                                                           */
/*  - iteration 1 takes m steps.  The end-of-iteration check (:130-147) calls */
/*    yieldNextClause() for clauses 0, 1, ... in index order only until the   */
/*    first violated one (later loop turns `continue`), which leaves the      */
/*    generator at n_yielded = k0 = (first violated index) + 1 with           */
/*    finished = false; the next iteration therefore takes only m - k0 steps  */
/*    (all m when k0 == m: the generator finished and resets).  Clauses       */
/*    outside that window of the sequence are not yielded at all;             */
/*  - batches of batch_size steps from the window start (the last shorter);   */
/*    the violated clauses of a batch extend the MIS greedily in yield order  */
/*    (populate_mis_parallel with the current MIS, :391-451); the MIS is      */
/*    resampled after the last batch (parallel_solve, resample =              */
/*    finishedYielding, :217-320);                                            */
/*  - avg_mis_size accumulates the MIS size after EVERY batch (:113-114), and */
/*    is divided by n_iterations at the end;                                  */
/*  - an already satisfied start still counts one iteration.                  */
/* Restated with Philox resampling (iteration i uses round i-1).  max_iters   */
/* caps the number of iterations (the reference has no cap).                  */
/* ------------------------------------------------------------------------- */
#define ORC_STREAM_P 9223372036854775783ULL

void orc_stream_order(uint64_t m, uint32_t* order) {
    uint64_t c = 0;
    for (uint64_t k = 0; k < m; ++k) {
        c = (c + ORC_STREAM_P) % m;  /* ClauseGenerator.h:47 (c < m, no overflow) */
        order[k] = (uint32_t)c;
    }
}

/* rd_state != NULL: the reference-RNG mode (a fresh RBG per iteration, seeded by the next
 * random_device value; bits in pick order, SATInstance.h:340-365 with T = 1) */
static int stream_impl(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
                       uint64_t max_iters, uint64_t batch, uint32_t* A, orc_stats* st, orc_iter_cb cb,
                       void* cb_user, uint64_t* rd_state) {
    uint32_t* M = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint8_t* used = (uint8_t*)calloc(n_vars ? n_vars : 1, 1);
    uint64_t nw = (m + 63) / 64;
    uint64_t* vmask = (uint64_t*)calloc(nw ? nw : 1, sizeof(uint64_t));
    memset(st, 0, sizeof(*st));
    if (batch == 0) batch = 1;
    uint64_t weighted = 0, c = 0, window = m;
    int solved = 0;
    uint64_t nu = orc_eval(m, offs, lits, A, vmask);
    for (;;) {
        st->n_iterations += 1;
        st->last_violated = nu;
        /* greedy MIS over the window's violated clauses in yield order; a clause picked in
           batch b counts in the cumulative sizes of batches b .. nb-1 */
        const uint64_t nb = window ? (window + batch - 1) / batch : 0;
        uint64_t nm = 0;
        for (uint64_t k = 0; k < window; ++k) {
            c = m ? (c + ORC_STREAM_P) % m : 0;
            if (!((vmask[c >> 6] >> (c & 63)) & 1)) continue;
            int dep = 0;
            for (uint64_t j = offs[c]; j < offs[c + 1]; ++j) dep |= used[lits[j] >> 1];
            if (dep) continue;
            for (uint64_t j = offs[c]; j < offs[c + 1]; ++j) used[lits[j] >> 1] = 1;
            M[nm++] = (uint32_t)c;
            weighted += nb - k / batch;
        }
        uint64_t dres = 0;
        const uint64_t iter = st->n_iterations - 1;
        orc_rbg g;
        if (rd_state) orc_rbg_seed(&g, orc_refrng_rd_next(rd_state));
        for (uint64_t i = 0; i < nm; ++i) {
            const uint32_t cl = M[i];
            for (uint64_t j = offs[cl]; j < offs[cl + 1]; ++j) {
                const uint32_t v = lits[j] >> 1;
                const uint32_t b = rd_state ? orc_rbg_sample(&g) : orc_resample_bit(seed, iter, v);
                A[v >> 5] = (A[v >> 5] & ~(1u << (v & 31))) | (b << (v & 31));
                used[v] = 0;
            }
            dres += offs[cl + 1] - offs[cl];
        }
        st->n_resamples += dres;
        if (cb) cb(cb_user, st->n_iterations, nu, nm, dres, A);
        nu = orc_eval(m, offs, lits, A, vmask);
        if (nu == 0) { solved = 1; st->last_violated = 0; break; }
        if (max_iters && st->n_iterations >= max_iters) { st->last_violated = nu; break; }
        uint64_t first = 0;  /* first violated index: the check stops there */
        while (!((vmask[first >> 6] >> (first & 63)) & 1)) ++first;
        window = (first + 1 == m) ? m : m - (first + 1);
    }
    st->sum_mis_size = weighted;
    st->avg_mis_size = st->n_iterations ? weighted / st->n_iterations : 0;
    st->solved = solved;
    free(M); free(used); free(vmask);
    return solved ? 0 : 1;
}

int orc_solve_stream(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
                     uint64_t max_iters, uint64_t batch, uint32_t* A, orc_stats* st, orc_iter_cb cb,
                     void* cb_user) {
    return stream_impl(n_vars, m, offs, lits, seed, max_iters, batch, A, st, cb, cb_user, NULL);
}

/* orc_solve_stream in the reference-RNG mode: A initialised here from the random_device stand-in
 * seeded with rd_seed, every iteration's resample from the stand-in's next value */
int orc_solve_stream_refrng(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
                            uint64_t rd_seed, uint64_t max_iters, uint64_t batch, uint32_t* A, orc_stats* st,
                            orc_iter_cb cb, void* cb_user) {
    uint64_t rd = rd_seed;
    orc_refrng_init(&rd, n_vars, A);
    return stream_impl(n_vars, m, offs, lits, 0, max_iters, batch, A, st, cb, cb_user, &rd);
}

/* ------------------------------------------------------------------------- */
/* Streaming solve with T > 1 threads (SATInstance.h:70-153).                  */
/*  - T generators (:74-86): generator t owns clauses [t*tn, t*tn + n_t),      */
/*    tn = m / T, the last one the remainder; each walks its own range with    */
/*    c <- (c + P) % n_t from c = 0 (ClauseGenerator.h:44-47), never reset;    */
/*  - a batch step (:98-125) asks every generator for a batch                  */
/*    (yieldRandomUNSATClauseBatch, ClauseGenerator.h:32-71: a finished        */
/*    generator first resets n_yielded to 0; min(batch, n_t - n_yielded)      */
/*    steps; finished when n_yielded == n_t) and keeps the violated ones;      */
/*    populate_mis_parallel (:391-451) then drops every set's clauses that     */
/*    share a variable with the MIS accumulated so far and runs the T-set      */
/*    round robin from t = 0 (first turn: set 1), extending the MIS; the       */
/*    batch steps repeat until every generator finished at the same step,      */
/*    then the MIS is resampled (parallel_solve resample = finishedYielding);  */
/*  - avg_mis_size accumulates the MIS size after every batch step;            */
/*  - the end-of-iteration check (:129-147) runs T threads over their ranges   */
/*    in index order sharing one `solved` flag, so where each thread stops is  */
/*    a race in the reference.  Restated with the lock-step schedule: step k   */
/*    checks clause base_t + k of every generator with k < n_t, and the steps  */
/*    stop after the first one that finds a violated clause (f = the smallest  */
/*    first-violated offset over the generators); generator t is left at       */
/*    n_yielded = min(n_t, f + 1), finished iff that is n_t.  With T = 1 this  */
/*    is the one-thread window rule of orc_solve_stream.                       */
/* An empty clause is refused (-2): it is violated forever and, never sharing */
/* a variable, joins the MIS at every batch step.  A loop whose generators    */
/* never finish together (the reference would not return) stops at step_cap   */
/* batch steps in one iteration (-1).  Returns 0 solved, 1 capped.             */
/* ------------------------------------------------------------------------- */
typedef struct { uint64_t base, n, c, ny; int fin; } orc_sgen;

static uint64_t sgen_yield(orc_sgen* g, uint64_t batch, const uint64_t* vmask, uint32_t* out) {
    if (g->fin) { g->ny = 0; g->fin = 0; }  /* ClauseGenerator.h:33-35 (reset) */
    const uint64_t n = (g->ny + batch >= g->n) ? g->n - g->ny : batch;
    uint64_t k = 0;
    for (uint64_t i = 0; i < n; ++i) {
        g->c = (g->c + ORC_STREAM_P) % g->n;  /* c < n_t < 2^32: no overflow */
        const uint64_t cl = g->base + g->c;
        if ((vmask[cl >> 6] >> (cl & 63)) & 1ull) out[k++] = (uint32_t)cl;
        g->ny++;
    }
    if (g->ny == g->n) g->fin = 1;
    return k;
}

int orc_solve_stream_rr(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
                        uint64_t max_iters, uint64_t batch, uint32_t T, uint64_t step_cap, uint32_t* A,
                        orc_stats* st, orc_iter_cb cb, void* cb_user) {
    memset(st, 0, sizeof(*st));
    if (T < 1) T = 1;
    if (batch == 0) batch = 1;
    for (uint64_t c = 0; c < m; ++c)
        if (offs[c + 1] == offs[c]) return -2;
    const uint64_t nw = (m + 63) / 64, tn = m / T;
    orc_sgen* g = (orc_sgen*)calloc(T, sizeof(orc_sgen));
    uint64_t *seg = (uint64_t*)malloc(sizeof(uint64_t) * (T + 1)), *cnt = (uint64_t*)malloc(sizeof(uint64_t) * T),
             *head = (uint64_t*)malloc(sizeof(uint64_t) * T);
    uint32_t* live = (uint32_t*)malloc(sizeof(uint32_t) * T);
    uint64_t* vmask = (uint64_t*)calloc(nw ? nw : 1, sizeof(uint64_t));
    uint8_t* used = (uint8_t*)calloc(n_vars ? n_vars : 1, 1);
    uint32_t* M = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    seg[0] = 0;
    for (uint32_t t = 0; t < T; ++t) {  /* SATInstance.h:74-86 */
        g[t].base = (uint64_t)t * tn;
        g[t].n = (t == T - 1) ? m - g[t].base : tn;
        seg[t + 1] = seg[t] + (g[t].n < batch ? g[t].n : batch);  /* a batch holds at most this many */
    }
    uint32_t* lists = (uint32_t*)malloc(sizeof(uint32_t) * (seg[T] ? seg[T] : 1));
    uint64_t weighted = 0, nu = orc_eval(m, offs, lits, A, vmask);
    int rc = 0;
    for (;;) {
        st->n_iterations += 1;
        st->last_violated = nu;
        uint64_t nm = 0, steps = 0;
        int all_fin = 0;
        while (!all_fin) {
            if (++steps > step_cap) { rc = -1; goto out; }
            all_fin = 1;
            for (uint32_t t = 0; t < T; ++t) {
                cnt[t] = sgen_yield(&g[t], batch, vmask, lists + seg[t]);
                head[t] = 0;
                live[t] = t;
                all_fin &= g[t].fin;
            }
            /* populate_mis_parallel: the filter against the MIS so far and the erasures of the
               round robin are both lazy (a front touching a used variable is skipped) */
            uint32_t nlive = T, t = 0;
            while (nlive > 0) {
                t = (t + 1) % nlive;
                const uint32_t s = live[t];
                const uint32_t* L = lists + seg[s];
                while (head[s] < cnt[s] && touches(offs, lits, used, L[head[s]])) ++head[s];
                if (head[s] == cnt[s]) {
                    for (uint32_t q = t; q + 1 < nlive; ++q) live[q] = live[q + 1];
                    --nlive;
                    continue;
                }
                const uint32_t c = L[head[s]++];
                M[nm++] = c;
                mark(offs, lits, used, c, 1);
            }
            weighted += nm;  /* SATInstance.h:113-114 (avg_mis_size after every batch) */
        }
        uint64_t dres = 0;
        const uint64_t iter = st->n_iterations - 1;
        for (uint64_t i = 0; i < nm; ++i) {
            const uint32_t cl = M[i];
            for (uint64_t j = offs[cl]; j < offs[cl + 1]; ++j) {
                const uint32_t v = lits[j] >> 1;
                const uint32_t bb = orc_resample_bit(seed, iter, v);
                A[v >> 5] = (A[v >> 5] & ~(1u << (v & 31))) | (bb << (v & 31));
                used[v] = 0;
            }
            dres += offs[cl + 1] - offs[cl];
        }
        st->n_resamples += dres;
        if (cb) cb(cb_user, st->n_iterations, nu, nm, dres, A);
        nu = orc_eval(m, offs, lits, A, vmask);
        if (nu == 0) { st->solved = 1; st->last_violated = 0; break; }
        if (max_iters && st->n_iterations >= max_iters) { st->last_violated = nu; rc = 1; break; }
        /* lock-step check: f = smallest first-violated offset over the generators */
        uint64_t f = ~0ull;
        for (uint32_t t = 0; t < T; ++t)
            for (uint64_t k = 0; k < g[t].n && k < f; ++k) {
                const uint64_t cl = g[t].base + k;
                if ((vmask[cl >> 6] >> (cl & 63)) & 1ull) { f = k; break; }
            }
        for (uint32_t t = 0; t < T; ++t) {
            g[t].ny = g[t].n < f + 1 ? g[t].n : f + 1;
            g[t].fin = g[t].ny == g[t].n;
        }
    }
out:
    st->sum_mis_size = weighted;
    st->avg_mis_size = st->n_iterations ? weighted / st->n_iterations : 0;
    free(g); free(seg); free(cnt); free(head); free(live); free(vmask); free(used); free(M); free(lists);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* DIMACS semantics of cnf_header_read / cnf_data_read (example/cnf_io/        */
/* cnf_io.cpp:487-705, 126-328) plus the encoding of example/main.cpp:157-178. */
/* Restated over an in-memory buffer:                                          */
/*  - lines are split at '\n'; a final line with no '\n' is dropped (getline   */
/*    then eof -> break, cnf_io.cpp:277-281);                                  */
/*  - lines whose first char is 'c'/'C' and lines of only ' ' are skipped;     */
/*  - words are separated by ' ' only (s_word_extract_first, :1419-1486);      */
/*  - s_to_i4 (:1305-1416): optional sign, digits, stops at first non-digit;   */
/*    a word that does not start with a sign/digit ends the line;              */
/*  - non-zero -> literal, 0 -> closes the clause.                             */
/* Header: first non-comment non-blank line must be 'p'<ws>'cnf'<ws> V C.       */
/* Returns 0 ok, -1 bad header, -2 fewer clauses than the header, -3 literal   */
/* out of [1,V].                                                                */
/* ------------------------------------------------------------------------- */
static int is_ws(char c) { return c == ' ' || c == '\f' || c == '\n' || c == '\r' || c == '\t' || c == '\v'; }

/* s_to_i4 on a word [w, we): returns 0 ok / 1 error; *val set */
static int s_to_i4(const char* w, const char* we, long long* val) {
    int st = 0, sgn = 1;
    long long iv = 0;
    for (const char* p = w;; ++p) {
        char c = (p < we) ? *p : '\0';
        if (st == 0) {
            if (c == ' ') {}
            else if (c == '-') { st = 1; sgn = -1; }
            else if (c == '+') { st = 1; sgn = 1; }
            else if (c >= '0' && c <= '9') { st = 2; iv = c - '0'; }
            else return 1;
        } else if (st == 1) {
            if (c == ' ') {}
            else if (c >= '0' && c <= '9') { st = 2; iv = c - '0'; }
            else return 1;
        } else {
            if (c >= '0' && c <= '9') iv = 10 * iv + (c - '0');
            else { *val = sgn * iv; return 0; }
        }
    }
}

int orc_dimacs_parse(const char* buf, uint64_t len, uint32_t* v_num, uint64_t* c_num,
                     uint64_t* offs /* c_num+1, may be NULL */, uint32_t* lits /* may be NULL */,
                     uint64_t* l_num) {
    uint64_t pos = 0;
    int have_header = 0;
    long long V = 0, C = 0;
    uint64_t nclauses = 0, nlits = 0, cur = 0;
    int rc = 0;
    if (offs) offs[0] = 0;
    while (pos < len) {
        const char* ls = buf + pos;
        const char* nl = memchr(ls, '\n', len - pos);
        if (!nl) break; /* last line without newline: dropped */
        const char* le = nl;
        pos = (uint64_t)(nl - buf) + 1;
        uint64_t L = (uint64_t)(le - ls);
        if (L > 0 && (ls[0] == 'c' || ls[0] == 'C')) continue;
        /* s_len_trim: trailing ' ' only */
        uint64_t tl = L;
        while (tl > 0 && ls[tl - 1] == ' ') --tl;
        if (tl == 0) continue;
        if (!have_header) {
            /* 'p', whitespace, adjustl, 'cnf' (case-insensitive), whitespace, V, C */
            if (!(ls[0] == 'p' || ls[0] == 'P')) return -1;
            if (L < 2 || !is_ws(ls[1])) return -1;
            const char* p = ls + 2;
            while (p < le && (*p == ' ' || *p == '\t')) ++p;
            if (le - p < 4) return -1;
            if (!((p[0] | 32) == 'c' && (p[1] | 32) == 'n' && (p[2] | 32) == 'f')) return -1;
            if (!is_ws(p[3])) return -1;
            p += 4;
            while (p < le && (*p == ' ' || *p == '\t')) ++p;
            /* two words separated by ' ' */
            const char* w = p; while (w < le && *w == ' ') ++w;
            const char* we = w; while (we < le && *we != ' ') ++we;
            if (we == w || s_to_i4(w, we, &V)) return -1;
            w = we; while (w < le && *w == ' ') ++w;
            we = w; while (we < le && *we != ' ') ++we;
            if (we == w || s_to_i4(w, we, &C)) return -1;
            if (V < 0 || C < 0) return -1;
            have_header = 1;
            continue;
        }
        /* data line: words separated by ' ' */
        const char* p = ls;
        for (;;) {
            while (p < le && *p == ' ') ++p;
            const char* we = p; while (we < le && *we != ' ') ++we;
            if (we == p) break;
            long long x;
            if (s_to_i4(p, we, &x)) break;
            p = we;
            if (x != 0) {
                if (nclauses < (uint64_t)C) {
                    if (x > V || -x > V) rc = rc ? rc : -3;
                    if (lits) lits[nlits] = (x > 0) ? (uint32_t)(2 * x - 2) : (uint32_t)(-2 * x - 1);
                    ++nlits;
                }
                ++cur;
            } else {
                if (nclauses < (uint64_t)C && offs) offs[nclauses + 1] = nlits;
                ++nclauses;
                cur = 0;
            }
        }
    }
    (void)cur;
    if (!have_header) return -1;
    *v_num = (uint32_t)V;
    *c_num = (uint64_t)C;
    if (l_num) *l_num = nlits;
    if (nclauses < (uint64_t)C) return -2;
    return rc;
}
