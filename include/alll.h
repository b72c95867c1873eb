/*
 * alll.h -- C-ABI of the MI355X-native Moser-Tardos (ALLL) resample loop.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference exposes a
 * header-only C++ API (xmif1/ALLLSatisfiabilitySolver, library/include/SATInstance.h);
 * the compatibility headers in include/alll_compat/ keep that API and call the entry
 * points below.  Every entry point cites the reference interface it replaces.
 *
 * Conventions: plain pointers and sizes only; no exceptions cross this boundary; every
 * function returns an alll_status (0 = ok) and alll_last_error() describes the last
 * failure on the calling thread.  Literals use the reference encoding of
 * example/main.cpp:168: DIMACS x>0 -> 2(x-1), -x -> 2(x-1)+1 (variable = l >> 1).
 */
#ifndef ALLL_H
#define ALLL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALLL_ABI_VERSION 1

typedef enum alll_status {
    ALLL_OK = 0,
    ALLL_ERR_INVALID_ARG = 1,   /* null pointer, bad size, bad option */
    ALLL_ERR_BAD_INPUT = 2,     /* malformed CSR or DIMACS (header, missing clauses) */
    ALLL_ERR_LITERAL_RANGE = 3, /* literal variable >= n_vars (reference: UB, Clause.h:40) */
    ALLL_ERR_HIP = 4,           /* HIP runtime failure */
    ALLL_ERR_RCCL = 5,          /* RCCL failure */
    ALLL_ERR_MAX_ITERS = 6,     /* max_iters eval passes done, instance not solved */
    ALLL_ERR_NO_DEVICE = 7,     /* no usable gfx950 device */
    ALLL_ERR_OOM = 8,           /* device or host allocation failed */
    ALLL_ERR_IO = 9,            /* file could not be opened / read */
    ALLL_ERR_UNSUPPORTED = 10   /* size beyond the implementation limits */
} alll_status;

/* Instance in CSR form (replaces vector<ClauseArray*> of Clause<T>*, Clause.h:17-28;
 * the chunking of example/main.cpp:149-178 is irrelevant to the T=1 semantics). */
typedef struct alll_problem {
    uint32_t n_vars;            /* VariablesArray<T>::n_vars (VariablesArray.h:20) */
    uint32_t pad;
    uint64_t n_clauses;
    const uint64_t* offsets;    /* n_clauses+1, offsets[0] = 0, non-decreasing */
    const uint32_t* literals;   /* offsets[n_clauses] encoded literals */
} alll_problem;

/* flags */
#define ALLL_FLAG_NO_GRAPH          (1u << 0) /* launch eagerly instead of replaying a hipGraph */
#define ALLL_FLAG_EXCHANGE_ALLREDUCE (1u << 1) /* multi-GPU: shard resample + allreduce of the
                                                 bit-packed assignment delta (north_star form) */
#define ALLL_FLAG_GENERIC_CSR       (1u << 2) /* disable the fixed-width clause layout */
#define ALLL_FLAG_NO_RANGED         (1u << 3) /* use the L2-gather eval kernel instead of the
                                                 persistent LDS/L2 hybrid */
#define ALLL_FLAG_KERNEL_TIMING     (1u << 4) /* stamp every loop iteration with device wall-clock
                                                 times (alll_loop_times) */
#define ALLL_FLAG_ATOMIC_CLAIMS     (1u << 5) /* LFMIS round 0 by global atomicMin claims instead of
                                                 the variable-bucketed LDS resolution */
#define ALLL_FLAG_LFMIS             (1u << 6) /* n_threads > 1: keep the one-set MIS (the
                                                 lexicographically-first MIS in clause order, fast)
                                                 instead of the reference's T-set round robin */
#define ALLL_FLAG_REFERENCE_RNG     (1u << 7) /* the reference's own random stream instead of Philox:
                                                 RBG<default_random_engine> (RandomBoolGenerator.h,
                                                 libstdc++ minstd_rand0 + uniform_int_distribution
                                                 <unsigned long long>), every engine seeded with the
                                                 next value of std::random_device, for which `seed`
                                                 is the state of the 64-bit LCG stand-in of
                                                 oracle/ref_probe.cpp (x = x*6364136223846793005 +
                                                 1442695040888963407, value x >> 33): the initial
                                                 fill (VariablesArray.h:23-34) and every resample
                                                 round (SATInstance.h:340-365, T = 1) then equal the
                                                 reference's, bit for bit (the draws in parallel by
                                                 jump-ahead; about half the Philox loop's rate at
                                                 10M clauses).  n_threads = 1 (also for the streaming
                                                 solve: bits in yield order), one GPU:
                                                 ALLL_ERR_UNSUPPORTED otherwise */

typedef struct alll_options {
    uint64_t seed;          /* Philox4x32-10 key; replaces std::random_device (SATInstance.h:346) */
    uint64_t max_iters;     /* cap on eval passes (n_iterations); 0 = unlimited like the reference */
    int32_t device;         /* HIP device ordinal; -1 = current device */
    int32_t n_threads;      /* the reference's n_threads T (SATInstance.h:51): T > 1 makes the MIS
                               the round-robin greedy over T clause chunks (populate_mis_parallel,
                               SATInstance.h:414-447; at most 4096 chunks) unless ALLL_FLAG_LFMIS */
    int32_t rank;           /* clause shard of this process (0 .. world-1) */
    int32_t world;          /* number of GPUs the clauses are sharded over (1 = single GPU) */
    uint8_t comm_id[128];   /* RCCL unique id from alll_comm_unique_id() on rank 0 (world > 1);
                               all zero: no RCCL, alll_set_host_exchange() is required.  With
                               world == 1 a non-zero id creates a one-rank communicator and runs
                               the clause-sharded exchange path on one GPU (a rehearsal of the
                               multi-GPU path; the results are the same) */
    uint32_t flags;         /* ALLL_FLAG_* */
    uint32_t grid_rounds;   /* full-grid LFMIS rounds before the tail kernel (0 = default) */
    uint64_t stream_batch;  /* 0: SATInstance::solve(vector<ClauseArray*>*) semantics.  > 0: the
                               streaming solve SATInstance::solve(getEnumeratedClause, n_clauses,
                               batch_size) (SATInstance.h:70-153) with this batch size and
                               n_threads clause generators (ClauseGenerator.h:32-71): with one
                               thread the MIS follows the generator's yield order; with n_threads
                               = T > 1 every batch step runs the T-set round robin over the T
                               generators' violated lists, filtered by the MIS so far
                               (SATInstance.h:98-125, 391-447), and the end-of-iteration check
                               runs in lock step.  T > 1 returns
                               ALLL_ERR_UNSUPPORTED for an empty clause, for world > 1, and from
                               alll_solve / alll_run at an iteration whose generators would never
                               finish at the same batch step (the reference's loop does not end
                               there).  ALLL_FLAG_LFMIS keeps the one-thread order for any T.
                               alll_stats reports the reference's statistics (n_iterations =
                               stream iterations, avg_mis_size summed per batch step); max_iters
                               then caps stream iterations */
    const uint64_t* set_starts; /* n_threads > 1: n_threads + 1 non-decreasing clause indices,
                               chunk q = [set_starts[q], set_starts[q+1]), set_starts[0] = 0,
                               set_starts[n_threads] = n_clauses (the sizes of the caller's
                               vector<ClauseArray*>); NULL = the chunking of example/main.cpp:
                               149-178.  Read by alll_create only */
} alll_options;

#define ALLL_MAX_GPU_STATS 64

/* Replaces struct Statistics (SATInstance.h:25-32). */
typedef struct alll_stats {
    uint64_t n_iterations;   /* eval passes, including the final zero-violation pass */
    uint64_t n_resamples;    /* sum of clause lengths over every MIS clause */
    uint64_t avg_mis_size;   /* floor(sum |MIS_i| / n_iterations) (SATInstance.h:317) */
    uint64_t sum_mis_size;
    uint64_t n_violated;     /* violated clauses found by the last eval pass */
    int32_t solved;          /* 1 if the last eval pass found no violated clause */
    int32_t n_gpus;          /* entries used in gpu_resamples */
    uint32_t lfmis_rounds_max;  /* most LFMIS rounds one iteration needed (grid + tail) */
    uint32_t lfmis_tail_rounds; /* rounds run by the tail kernel in the last iteration */
    uint64_t gpu_resamples[ALLL_MAX_GPU_STATS]; /* per clause-shard share of n_resamples */
} alll_stats;

/* Per-phase device time (ms, averaged over the profiled iterations), from HIP events on
 * the solver's stream. */
typedef struct alll_phase_times {
    double eval_ms;          /* clause evaluation + compaction kernel */
    double exchange_ms;      /* RCCL collectives + collect (0 on one GPU) */
    double mis_ms;           /* count reduction + LFMIS rounds + tail */
    double resample_ms;      /* Philox resample kernel */
    double total_ms;         /* whole iteration */
    uint64_t iterations;
} alll_phase_times;

typedef struct alll_ctx alll_ctx;

const char* alll_version(void);
const char* alll_last_error(void);
void alll_default_options(alll_options* opt);

/* Number of visible HIP devices (0 without a GPU; never fails). */
int alll_device_count(void);

/* RCCL unique id for a multi-GPU solver (rank 0 creates it, all ranks pass it in
 * alll_options.comm_id). */
int alll_comm_unique_id(uint8_t out[128]);

/* Host-staged exchange for the clause-sharded mode (alternative to RCCL, e.g. several
 * ranks sharing one GPU, or CPU-side collectives): op ALLL_XCHG_ALLGATHER -- `buf` holds
 * world * `bytes` bytes, this rank's piece at rank * bytes is filled, gather the others in
 * place; op ALLL_XCHG_ALLREDUCE_SUM_U32 -- element-wise sum of `bytes`/4 uint32 in place.
 * Return 0 on success. */
#define ALLL_XCHG_ALLGATHER 0
#define ALLL_XCHG_ALLREDUCE_SUM_U32 1
typedef int (*alll_exchange_fn)(void* user, int op, void* buf, uint64_t bytes);

/* Replaces SATInstance<T>(VariablesArray<T>*, int n_threads) (SATInstance.h:51-56) plus the
 * random initial assignment of VariablesArray<T>(n_vars) (VariablesArray.h:23-34).  Copies
 * the caller's CSR to the device; keeps no caller pointer. */
int alll_create(const alll_problem* prob, const alll_options* opt, alll_ctx** out);
int alll_destroy(alll_ctx* ctx);

/* Use a host-staged exchange instead of RCCL (world > 1; create with an all-zero comm_id). */
int alll_set_host_exchange(alll_ctx* ctx, alll_exchange_fn fn, void* user);

/* Replaces Statistics* SATInstance::solve(vector<ClauseArray*>*) (SATInstance.h:60-66 ->
 * parallel_solve :217-320).  Runs until no clause is violated (ALLL_OK) or max_iters
 * eval passes were done (ALLL_ERR_MAX_ITERS).  Statistics accumulate over calls. */
int alll_solve(alll_ctx* ctx, alll_stats* stats);

/* Fixed-iteration mode (benchmarks, step-by-step parity tests): run n_iters more full
 * iterations (eval + MIS + resample); stops early only when an eval pass finds no
 * violated clause.  Asynchronous unless stats != NULL. */
int alll_run(alll_ctx* ctx, uint64_t n_iters, alll_stats* stats);

int alll_get_stats(alll_ctx* ctx, alll_stats* stats);

/* Replaces bool SATInstance::verify_validity(vector<ClauseArray*>*) const
 * (SATInstance.h:156-173): one device eval pass over the current assignment. */
int alll_verify(alll_ctx* ctx, int* valid, uint64_t* n_violated);

/* Current assignment as n_vars bytes of 0/1 (the bool vars[] of VariablesArray.h:21). */
int alll_get_assignment(alll_ctx* ctx, uint8_t* out, uint64_t n);
int alll_set_assignment(alll_ctx* ctx, const uint8_t* in, uint64_t n);
/* Bit-packed form: ceil(n_vars/32) words, bit v%32 of word v/32. */
int alll_get_assignment_words(alll_ctx* ctx, uint32_t* out, uint64_t n_words);
int alll_set_assignment_words(alll_ctx* ctx, const uint32_t* in, uint64_t n_words);

/* Introspection of the last iteration (parity tests): violated bitmask of the last eval
 * pass (ceil(n_clauses/64) words) and the MIS picked from it (ascending clause order). */
int alll_get_violated_mask(alll_ctx* ctx, uint64_t* out, uint64_t n_words);
int alll_get_mis(alll_ctx* ctx, uint32_t* out, uint64_t cap, uint64_t* n_out);

/* Benchmark helpers.  eval-only launches time the evaluation kernel alone on the current
 * assignment; profile runs n_iters iterations eagerly with HIP events around each phase. */
int alll_bench_eval(alll_ctx* ctx, int reps, double* avg_ms, uint64_t* n_violated);
int alll_profile(alll_ctx* ctx, uint64_t n_iters, alll_phase_times* out);
/* In-loop phase times of iterations [first_iter, first_iter + n_iters) as they ran (graph
 * replay included), from device wall-clock stamps taken by the kernels themselves; needs
 * ALLL_FLAG_KERNEL_TIMING at create.  eval_ms = evaluation kernel (first workgroup start to
 * last workgroup end); exchange_ms = evaluation end to reduce start (collectives + collect on
 * several GPUs, a launch gap on one); mis_ms = reduce start to LFMIS tail end; resample_ms =
 * tail end to the next evaluation start; total_ms = evaluation start to the next one.  Only
 * the last 4096 iterations are kept.  (No reference counterpart: measurement) */
int alll_loop_times(alll_ctx* ctx, uint64_t first_iter, uint64_t n_iters, alll_phase_times* out);
/* Block the host until all work queued on the solver's stream finished. */
int alll_synchronize(alll_ctx* ctx);
/* Bytes the evaluation kernel reads/writes per pass (algorithmic). */
uint64_t alll_eval_bytes(alll_ctx* ctx);
/* Layout in use: 0 generic CSR, k>0 fixed-width-k layout. */
int alll_layout(alll_ctx* ctx);
/* Name of the evaluation kernel the loop launches (e.g. "k_eval_hybrid<3>"). */
const char* alll_eval_kernel(alll_ctx* ctx);
/* 1 when the loop replays captured hipGraphs, 0 when it launches eagerly (ALLL_FLAG_NO_GRAPH, a
 * host-staged exchange, or a capture / instantiation that failed: the loop then falls back to
 * eager launches with the same results); *why (may be NULL) names the reason.  -1: null ctx.
 * (No reference counterpart: measurement honesty of the benchmark) */
int alll_uses_graphs(alll_ctx* ctx, const char** why);
/* Round robin (n_threads > 1): the pass log of the last iteration, 4 words per pass {dirty
 * entries, repair rounds (0xFFFFFFFF: the incremental pass gave up), entries decided, decisions
 * changed} for the incremental passes (zeros for full ones), at most 64 passes, then -- written
 * only with ALLL_FLAG_KERNEL_TIMING, zeros otherwise -- 64 words per pass of repair clock stamps
 * (100 MHz; words 0..5: detect, wide repair, repair, rounds end, repair end, decisions loaded;
 * from word 8 {round entries, stamp} pairs) and one 64-word row of k_fp_bbuild's phase stamps;
 * returns the words written (0 without incremental passes).  (No reference counterpart:
 * measurement) */
int alll_rr_pass_log(alll_ctx* ctx, uint32_t* out, uint32_t n_words);
/* Round robin: grid barriers of the incremental passes' wide repair rounds that timed out since
 * alll_create (each makes its pass give up and a full pass follow: correct, slower); -1 on failure.
 * Non-zero means the repair's workgroups were not all resident (the GPU shared with other work).
 * (No reference counterpart: measurement) */
int64_t alll_rr_barrier_timeouts(alll_ctx* ctx);
/* Ranks taking part in the clause-sharded solve: ncclCommCount of the RCCL communicator, or
 * alll_options.world with a host-staged exchange (1 on one GPU); -1 on failure.  (The
 * reference counterpart is the thread count of the -p path, example/main.cpp:76-84.) */
int alll_comm_size(alll_ctx* ctx);

/* ---- host-side helpers (no GPU needed) ---------------------------------------------- */

/* DIMACS loader with the clause semantics of example/cnf_io (cnf_header_read
 * cnf_io.cpp:487-705 + cnf_data_read :126-328) and the encoding of main.cpp:157-178.
 * Two calls: first with offsets/literals NULL to get the sizes, then with buffers. */
int alll_dimacs_parse(const char* buf, uint64_t len, uint32_t* n_vars, uint64_t* n_clauses,
                      uint64_t* offsets, uint32_t* literals, uint64_t* n_literals);
/* Same from a file path (mmap). */
int alll_dimacs_read(const char* path, uint32_t* n_vars, uint64_t* n_clauses, uint64_t* offsets,
                     uint32_t* literals, uint64_t* n_literals);

/* Clause sharding of the multi-GPU mode (host-only): rank `rank` of `world` owns the clause
 * range [*clause_begin, *clause_end) (contiguous, 4096-clause tile aligned, so rank-major
 * concatenation is clause order) and contributes *mask_words_per_rank 64-bit words to the
 * per-iteration all-gather of the violated bitmask. */
int alll_shard_plan(uint64_t n_clauses, int world, int rank, uint64_t* clause_begin,
                    uint64_t* clause_end, uint64_t* mask_words_per_rank);

/* Multi-GPU plan for one instance on `world` GPUs of one node.  The exact
 * LFMIS and the resample run on every rank whatever the plan (their per-round minima over all
 * clauses would cost ~2 collectives per round), so only the evaluation can shard, and the
 * sharded plan (alll_shard_plan + the RCCL all-gather of the violated bitmask) pays an exchange
 * every iteration.  From the instance's size, the model predicts the evaluation time on one GPU,
 * what sharding saves of it, and the exchange's cost (marking, all-gather, collection of the
 * other shards' violated clauses, the round-0 scatter and reduce the exchange path cannot fuse),
 * with rates measured on one MI355X; `plan` is ALLL_PLAN_SHARD when the saving
 * exceeds the exchange, else ALLL_PLAN_REPLICATE: every rank runs the whole one-GPU loop (no
 * exchange; the trajectories are identical by construction, Philox keyed by seed, iteration
 * and word).  k_avg = literals / clauses. */
#define ALLL_PLAN_REPLICATE 0
#define ALLL_PLAN_SHARD 1
typedef struct {
    double eval_us_1gpu;   /* evaluation of the whole instance on one GPU */
    double eval_saved_us;  /* eval_us_1gpu * (1 - 1/world) */
    double exchange_us;    /* the sharded plan's per-iteration exchange */
    double violated_est;   /* violated clauses per iteration assumed: n_clauses * 2^-k_avg */
    int plan;              /* ALLL_PLAN_REPLICATE or ALLL_PLAN_SHARD */
    int pad;
} alll_multi_plan;
int alll_plan_multi_gpu(uint64_t n_clauses, uint64_t n_literals, uint32_t n_vars, int world,
                        alll_multi_plan* out);

/* The solver's initial assignment for `seed` as n_vars bytes of 0/1 (word w of the packed
 * form = Philox4x32-10(key=seed, ctr={w, 0, 0xFFFFFFFF, 0}).x); used by the compatibility
 * VariablesArray (replaces the random_device fill of VariablesArray.h:23-34). */
int alll_initial_assignment(uint64_t seed, uint32_t n_vars, uint8_t* out);

/* The reference's own initial assignment (VariablesArray.h:23-34) in the reference-RNG mode
 * (ALLL_FLAG_REFERENCE_RNG): `rd_state` is the random_device stand-in's state
 * before the fill draws its one value; the bytes equal the device fill of a context created
 * with that seed and the flag.  Used by the compatibility VariablesArray (env ALLL_REFERENCE_RNG). */
int alll_reference_initial_assignment(uint64_t rd_state, uint32_t n_vars, uint8_t* out);

/* Synthetic random k-SAT with k distinct variables per clause (kind 0 uniform, kind 1
 * power-law P(v) ~ (v+1)^-0.8); clauses [c_begin, c_end) of the instance, fixed width k. */
int alll_generate_ksat(uint64_t gen_seed, uint32_t n_vars, uint64_t n_clauses, uint32_t k,
                       int kind, uint64_t c_begin, uint64_t c_end, uint32_t* literals);

#ifdef __cplusplus
}
#endif
#endif /* ALLL_H */
