// alll_internal.h -- shared between the HIP kernels (alll_kernels.hip) and the host runtime
// (alll_runtime.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace alll {

// Clauses per tile.  A tile is the unit of evaluation (one 256-thread workgroup), of the
// violated-clause staging lists and of the LFMIS round kernels.
constexpr uint32_t TILE = 4096;
constexpr uint32_t TILE_WORDS = TILE / 64;   // violated-bitmask words per tile
constexpr uint32_t CHUNK = 256;              // clauses per transposed literal chunk
constexpr int EVAL_THREADS = 256;
constexpr int ROUND_THREADS = 256;
constexpr int JOIN_THREADS = 128;  // k_join: ~230 entries per tile in round 1, all tiles resident at once
constexpr int TAIL_THREADS = 1024;
// grid rounds from here on run a wave per tile (instances with hot variables: one round later,
// their round 2 still holds ~10% of the violated clauses)
constexpr uint32_t WAVE_ROUND_MIN = 1;  // grid rounds >= 1 run a wave per tile
constexpr int MAX_FIXED_K = 8;
// Persistent hybrid evaluation: LDS window of at most LDS_VARS variables' assignment words.
constexpr uint32_t LDS_WORDS = 38912;              // 152 KiB of LDS
constexpr uint32_t LDS_VARS = LDS_WORDS * 32;      // 1,245,184 variables
constexpr int HYB_THREADS = 1024;
constexpr uint32_t HYB_MAX_TILES = 256;            // per-tile LDS counters per pass
// Hot variables (skewed degree): at most HOT_MAX are flagged; LDS hash slots per claim block.
constexpr uint32_t HOT_MAX = 512;  // (256, 128: same C5 throughput)
constexpr uint32_t HOT_SLOTS = 1024;
// hot: degree >= max(HOT_THR_MIN, HOT_MEAN_X x mean degree) (round 4 at C5: 1024 hot variables
// from degree 16 x mean on, 2048 LDS slots: 3508 -> 3437 it/s)
constexpr uint32_t HOT_THR_MIN = 1024;
constexpr uint32_t HOT_MEAN_X = 32;
constexpr uint32_t RANGED_MAX_TILES = 16;          // tiles per block pass (64-bit sat mask/lane)
// Every LFMIS round decides at least the lowest undecided clause, so rounds <= |U|; the cap
// only bounds a kernel that would otherwise run away on a bug or an adversarial chain.
constexpr uint32_t MAX_TAIL_ROUNDS = 1u << 20;
// Bucketed LFMIS round 0 (fixed width K): every claim of round 0 becomes a 64-bit pair
// {clause id:32 | lose:1 | entry index in its run:16 | variable offset in its bucket:15},
// written grouped by variable bucket (bkt_width variables) inside its run (run_tiles
// consecutive tiles); per-bucket minima are then resolved in LDS instead of by global atomics.
constexpr uint32_t BKT_MAX = 4096;            // buckets (LDS histogram of k_bscatter)
constexpr uint32_t BKT_SHIFT_MIN = 10;
constexpr uint32_t BKT_SHIFT_MAX = 15;        // LDS minima of k_bresolve: 4 << 15 = 128 KiB
constexpr uint32_t RUN_TILES_MAX = 16;        // entry index within a run < 16 * TILE = 2^16
constexpr int BKT_THREADS = 512;
constexpr uint32_t BKT_RUN_BATCH = 1024;        // runs per segment-table batch of k_bresolve
constexpr unsigned long long PAIR_LOSE = 1ull << 31;
// Round-robin MIS of T > 1 clause chunks (the reference's n_threads > 1): at most RR_TMAX sets.
constexpr uint32_t RR_TMAX = 2048;
constexpr uint32_t RR_MW_GH = 1u << 15;  // k_rr_mw global hash slots
constexpr uint32_t RR_MW_CTL_WORDS = 1024; // k_rr_mw control block (words)
// Round robin as a fixpoint: the round-robin MIS is the LFMIS of the
// violated clauses under the priority (turn, clause order), where a clause's turn is the step
// at which its set's scan reaches it -- a function of how many clauses its set picked before
// it.  The pick sets are iterated, LFMIS(turns(P)) -> P, until they repeat.
constexpr uint32_t FP_TMAX = 256;          // sets (the schedule keeps T x T phase records)
constexpr uint32_t FP_B = 2048;            // entries per block of the count / turn passes
constexpr uint32_t FP_G = 4;       // grid LFMIS rounds before the one-workgroup tail (2, 3, 5: slower)
constexpr uint32_t FP_G_HOT = 6;   // ... on instances with hot variables (5, 7, 8, 10: slower)
constexpr uint32_t FP_G_MAX = FP_G_HOT > FP_G ? FP_G_HOT : FP_G;
constexpr uint32_t FP_MAX_DEFAULT = 64;    // LFMIS passes per iteration before k_rr_mw decides it
// incremental passes: defaults of LoopBuffers::fp_rep_cap / fp_rw_min / fp_rw_timeout
constexpr uint32_t FP_REP_CAP = 1u << 16;   // dirty entries per round before the pass gives up (a full pass follows)
constexpr uint32_t FP_RW_GRID = 64;         // workgroups of the wide repair (one per CU, all resident)
constexpr uint32_t FP_RW_MIN = 256;         // rounds this small are left to the one-workgroup repair
constexpr unsigned long long FP_RW_TIMEOUT = 2000000ull;  // wide-round barrier timeout: 20 ms at 100 MHz
constexpr uint32_t FP_LOG_PASSES = 64;     // passes of an iteration in the pass log (fp_log)
constexpr uint32_t FP_LOG_RW = 64;         // words per pass of the timing log behind it: {detect, wide, repair,
                                           //   rounds end, repair end, LDS loaded, schedule, phases} clock
                                           //   stamps, {round entries, stamp} pairs (24 rounds), then the
                                           //   first 4 wide rounds' pre-barrier stamps (words 56, 58, 60, 62)
// (one timing row per pass and one more for k_fp_bbuild's phase stamps; the rows are written and
// cleared only with ALLL_FLAG_KERNEL_TIMING, the per-pass counts always)
constexpr uint32_t FP_LOG_WORDS = 4 * FP_LOG_PASSES + FP_LOG_RW * (FP_LOG_PASSES + 1);
enum : uint32_t { FP_RUN = 0, FP_FINAL = 1, FP_DONE = 2, FP_OFF = 3, FP_FAIL = 4 };
struct RRFpCtl {
    uint32_t state;      // FP_*: RUN iterating; FINAL the last pass converged (finalize now);
                         // DONE finalized; OFF inactive iteration; FAIL fall back to k_rr_mw
    uint32_t nu;         // violated clauses (scan entries) of the iteration
    uint32_t fp_iter;    // LFMIS passes so far in this iteration
    uint32_t changes;    // picks that differ between the last two passes
    uint32_t serial;     // cover serial of the current LFMIS pass (fp_cov, 8-bit), never 0; carries over
                         // from iteration to iteration and restarts at 0 (k_fp_reset clears fp_cov)
                         // only when fewer than fp_max + 2 serials are left (fp_serial_restart)
    uint32_t ep_base;    // owner epoch of round 0 of the current pass; epochs carry over from iteration
                         // to iteration (keys of later epochs are smaller, so fp_owner needs no reset)
                         // and restart at 0 (k_fp_reset clears fp_owner) once half the epoch budget
                         // is used (fp_ep_restart)
    uint32_t ep_next;    // first epoch after the current pass
    uint32_t total;      // picks of the last pass
    uint32_t guess_num, guess_den;  // previous iteration's |M| / |U| (initial pick density)
    uint32_t n_steps;    // schedule length (turns + erasures)
    uint32_t tpre;       // entries whose turn is below this keep the last pass's decision
    uint32_t e0;         // first erasure step of the last schedule
    uint32_t nheavy;     // variables with more than FP_HEAVY claimants (fp_heavy)
    // incremental passes: after a full pass, a pass re-decides only the entries
    // whose blocker no longer lies below them (k_fp_detect) and what their changes reach (k_fp_repair)
    uint32_t inc;        // the next pass is incremental (1) or a full LFMIS pass (0)
    uint32_t bail;       // an incremental pass gave up (its dirty set outgrew FP_REP_CAP): the next
                         // pass is a full one, with no settled prefix (tpre = 0)
    uint32_t ndirty;     // entries k_fp_detect marked for the repair
    uint32_t rep_serial; // repair round stamps (fp_dmark), never reset
    uint32_t rep_rounds; // repair rounds of the iteration (statistics)
    uint32_t ran;        // the pass's last kernel ran (k_fp_tail or k_fp_repair): k_fp_count / k_fp_sched
                         // test a pass only then (a pass of the other kind in a graph is a no-op)
    uint32_t skip;       // k_fp_sched found no pass to test: k_fp_turn leaves the turns as they are
    uint32_t restart;    // iteration start: bit 0 the owner epochs restart (fp_owner cleared), bit 1 the
                         // cover serials (fp_cov cleared) -- decided with the reduce, done by k_fp_guess
    // the wide repair (k_fp_repair_wide, the large early rounds across workgroups) hands over to
    // the one-workgroup repair: the list (wlist: 0 / 1 of fp_dl, ndirty entries), the rounds and
    // entries decided; its grid barrier
    uint32_t wlist, wrounds, wwork, wfail;
    uint32_t wbar;
    uint32_t pbsrc;      // the last pass was incremental: its picks are the bits fp_pbits (k_fp_turn reads
                         // them there), not bit 0 of fp_in
    uint32_t rw_timeouts;  // wide-round grid barriers that timed out (never reset; alll_rr_barrier_timeouts)
    uint32_t spare[3];
};
static_assert(sizeof(RRFpCtl) == 128, "RRFpCtl: 32 words");
// Streaming solve with T > 1 threads (SATInstance::solve(getEnumeratedClause, n, batch),
// SATInstance.h:70-153).  The host plans every iteration from the generators'
// states (alll_runtime.cpp, srr_plan); the device lists each generator's violated clauses in walk
// order (k_srr_count / k_srr_scan / k_srr_fill) and runs the batch steps' round robins
// (k_srr_mis).  Generator t of an iteration:
struct SrrGen {
    uint64_t base;    // first clause of its range
    uint64_t n;       // clauses in its range (0: it yields nothing)
    uint64_t pt;      // P mod n (P = 9223372036854775783, ClauseGenerator.h:109)
    uint64_t c0;      // walk position c at the iteration start (ClauseGenerator.h:110, never reset)
    uint64_t r;       // walk steps of its first batches: n - n_yielded, or n after a reset
    uint64_t b;       // batch steps of those, ceil(r / batch) (it finishes at step b)
    uint64_t p;       // batch steps of a whole walk, ceil(n / batch) (it finishes every p steps after)
    uint64_t yields;  // its walk steps in the iteration's materialised batch steps
    uint64_t vblk;    // its first virtual block of SRR_BLK walk steps (entry T: the block count)
    uint64_t e0;      // first entry of its violated list (k_srr_scan)
};
struct SrrPlan {
    uint32_t T;
    uint32_t nblk;    // virtual blocks
    uint64_t batch;
    uint64_t steps;   // materialised batch steps (every generator has walked its whole range by then)
    uint64_t extra;   // later batch steps, up to the one where all generators finish together: they
                      // re-yield only clauses already seen, so each adds the MIS size to the statistic
};
constexpr uint32_t SRR_BLK = 4096;      // walk steps per virtual block (k_srr_count / k_srr_fill)
constexpr uint32_t SRR_ENT_WORDS = 12;  // list entry {clause id, width, literal start, 0, 8 variables}

// In-loop kernel timing (ALLL_FLAG_KERNEL_TIMING): per iteration i, slot i % TIME_SLOTS holds
// device wall-clock stamps (s_memrealtime) {eval start (min over workgroups), eval end (max),
// reduce start, LFMIS tail end}.
constexpr uint32_t TIME_SLOTS = 4096;
constexpr uint32_t TIME_FIELDS = 4;

// Device-resident loop state.  Written only by the single-block reduce / tail kernels,
// read by every other kernel at entry (kernel boundaries order the accesses).
struct DevState {
    uint64_t n_iter;       // eval passes executed (Statistics::n_iterations)
    uint64_t limit_eval;   // eval passes allowed (kernels skip once n_iter >= limit_eval)
    uint64_t limit_nores;  // an eval pass with n_iter == limit_nores does not resample
    uint64_t u_total;      // violated clauses of the last eval pass
    uint64_t count_out;    // standalone eval count (verify / bench_eval)
    uint32_t done;         // 0 running, 1 solved, 2 stopped at limit_nores
    uint32_t active;       // the current iteration runs MIS + resample
    uint32_t stamp;        // cover stamp of the current iteration: 1 .. 255, cycling (never 0)
    uint32_t round_base;   // owner-key epoch of grid round 0 of the current iteration
    uint32_t round_next;   // first unused epoch
    uint32_t tail_rounds;  // rounds the tail kernel needed in the last iteration
    uint32_t max_rounds;   // max total rounds seen in one iteration
    uint32_t error;        // loop stopped (done = 3): 1 LFMIS exceeded MAX_TAIL_ROUNDS or the round
                           // robin its batch cap; 4 a k_rr_mw grid barrier timed out; 5 an incremental
                           // round-robin pass kernel found its buffers missing; 6 the streaming
                           // round robin exceeded its gather bound
    uint32_t left_cnt;     // undecided entries handed from the last grid round to the tail
    uint32_t tmis_cnt;     // MIS entries decided by the tail kernel (list b.tmis)
    uint64_t win_start;    // streaming solve: generator steps taken before this iteration
    uint64_t win_len;      // streaming solve: steps (clauses yielded) in this iteration
    uint64_t rd_state;     // reference-RNG mode: state of the random_device stand-in (alll_refrng.hip)
    uint64_t rd_bits;      // reference-RNG mode: bits the current resample round draws
    uint64_t rd_x0;        // reference-RNG mode: the round's engine state after seeding
    uint32_t rd_draws;     // reference-RNG mode: the round's draws
    uint32_t rd_n;         // reference-RNG mode: engine positions the parallel draws consider
    uint32_t rd_fail;      // reference-RNG mode: the parallel draws ran past rd_n (sequential redo)
    uint32_t rd_pad;
};

// Clause storage on the device.
struct ClauseView {
    const uint32_t* offs;   // generic CSR: m+1 offsets (uint32); nullptr in fixed-k layout
    const uint32_t* lits;   // AoS literals (CSR order; fixed-k: lits[c*k + j])
    const uint32_t* lits_t; // fixed-k only: chunk-transposed [c/256][j][c%256]
    uint64_t m;             // clauses
    uint32_t k;             // fixed width, 0 = generic CSR
    uint32_t n_hot;         // variables flagged hot (bit 31 of their literals in `lits`)
    const uint32_t* perm;   // fixed-k: evaluation position -> clause id (nullptr = identity or
                            // ids packed into lits_t)
    // Packed clause ids (fixed k): the literals of lits_t use their low id_shift bits, and
    // slot j carries bits [j * id_bits, (j + 1) * id_bits) of the clause id above them (below
    // the hot flag, bit 31), so that the evaluation emits clause ids without reading perm.
    uint32_t lit_mask;      // lits_t literal bits (LIT_MASK when ids are not packed)
    uint32_t id_shift;      // = bit width of the literals when packed
    uint32_t id_bits;       // id bits per slot; 0 = not packed (entries carry positions)
    uint32_t lits_nt;       // hybrid eval: non-temporal loads of lits_t (a stream larger than
                            // the Infinity Cache)
    // Ragged widths (generic CSR entries, T = 1, not streaming): the evaluation reads a
    // chunk-transposed copy instead of the CSR arrays.  Clauses are evaluated sorted by width
    // (then by the block of their smallest variable and their largest variable; perm maps
    // positions to clause ids), chunk g of 256 positions holds w_g = rg_off[g+1] - rg_off[g]
    // slots [slot j][256] from word 256 * rg_off[g] of rg_lits, each clause's literals by
    // descending variable and padded with an always-false literal (variable 32 * n_words,
    // past the assignment: its buffer load is out of range and reads 0).  nullptr = CSR eval.
    const uint32_t* rg_off;
    const uint32_t* rg_lits;
};

struct LoopBuffers {
    uint32_t* A;            // bit-packed assignment, ceil(n/32) words
    uint64_t* vmask;        // violated bitmask in evaluation order, n_tiles_padded * TILE_WORDS words:
                            // CSR: bit i of word w = position 64w + i; fixed width: word w = the
                            // ballot of slot w % 4 of chunk w / 4, bit i = position
                            // (w / 4) * CHUNK + 4i + w % 4
    uint64_t* cmask;        // clause-sharded runs whose evaluation order is not clause order (fixed
                            // width, ragged): the violated bitmask in clause order, bit c % 64 of
                            // word c / 64 (k_cmark sets the own shard's bits; the all-gathered
                            // mask gives the other shards' lists, k_collect); nullptr = vmask
    uint8_t* cflag;         // clause-sharded exchange: a byte per clause of this rank's mask words
                            //   (k_cmark marks, k_cpack packs into cmask and clears)
    uint32_t* xcount;       // clause-sharded verify: the own shard's violated count (u32), summed
    uint32_t own_begin, own_end;  // this rank's tiles
    uint32_t* tile_cnt;     // undecided violated entries per tile
    uint32_t* stage[2];     // per tile: TILE entries of undecided violated clauses, double
                            // buffered across LFMIS rounds.  Entry = {id, K literals} (fixed
                            // width K) or {id} (CSR); id = evaluation position until round 0
                            // translates it to the clause id
    uint32_t* mis_cnt;      // MIS entries per tile (current iteration)
    uint32_t* mis;          // per tile: TILE slots of MIS clause ids
    uint32_t* left;         // compact list of undecided entries handed to the tail kernel
    uint32_t* tmis;         // MIS clauses decided by the tail kernel
    unsigned long long* owner; // n_vars 64-bit owner keys (epoch-tagged, never reset)
    uint8_t* cover;         // per variable: stamp of the iteration whose MIS covers it (the
                            // reduce clears it when the stamp cycles back to 1)
    unsigned long long* tile_stats; // per tile: [2t] sum |MIS|, [2t+1] sum resampled literals
    uint32_t* delta;        // allreduce exchange: per-iteration assignment XOR delta
    DevState* state;
    unsigned long long* ktime; // TIME_SLOTS x TIME_FIELDS stamps, nullptr = timing off
    unsigned long long* pairs;  // bucketed round 0: n_runs x run_tiles*TILE*K pairs (nullptr = atomics)
    unsigned long long* runtab; // [bucket][run]: start | count << 32 of the bucket's pairs in the run
    uint32_t* run_pairs;        // pairs per run
    const uint32_t* win_base;   // hybrid eval: per tile, first assignment word of its LDS window
                                // (nullptr: words [0, win_words) for every tile)
    uint32_t win_words;         // hybrid eval: LDS window size in words (<= LDS_WORDS)
    // Variable spread of skewed instances (power-law hubs have the lowest ids): the owner slot
    // and the round-0 bucket of variable v are taken from vmix(v) = (v * vmix_mul) & vmix_mask,
    // a bijection onto [0, vmix_mask] (odd multiplier mod 2^k), so that the hubs' owner keys
    // fall in different memory channels and their pairs in different buckets.  Identity
    // (mul 1, mask ~0) otherwise.
    uint32_t vmix_mul;
    uint32_t vmix_mask;
    uint32_t vmix_inv;          // vmix_mul's inverse mod 2^32 (vunmix)
    uint32_t bkt_span;          // vmix slots [0, bkt_span) that the buckets cover (round robin)
    uint32_t bkt_width;         // bucket = vmix(variable) / bkt_width (<= 2^BKT_SHIFT_MAX)
    uint32_t bkt_magic;         // floor(2^32 / bkt_width): bucket by multiply-high
    uint32_t n_cu;              // compute units of the device
    uint32_t n_bkt;
    uint32_t run_tiles;         // tiles per run at most (a run's pair area holds run_tiles * TILE * K)
    uint32_t n_runs;
    const uint32_t* run_t0;     // n_runs + 1: first tile of every run (runs split the tile range of
                                // every evaluation workgroup, so one GPU scatters inside k_eval_hybrid)
    // streaming solve (SATInstance::solve(getEnumeratedClause, ...), T = 1): LFMIS priority =
    // position in the clause generator's yield window (alll_options.stream_batch > 0)
    uint64_t m;                 // clauses
    uint64_t stream_batch;      // 0: clause-order LFMIS
    uint64_t stream_pinv;       // inverse of P mod m (P = 9223372036854775783, ClauseGenerator.h:110)
    // round-robin MIS (T = rr_T > 1 clause chunks, SATInstance.h:414-447; CSR layout)
    uint32_t* rr_u;             // violated clauses in clause order: m scan entries of 12 words
    uint8_t* rr_flag;           // fixed width (hybrid evaluation): m clause-order violated flags
                                // (k_rr_mark sets, k_rr_entries clears); nullptr = CSR bitmask
    uint32_t* rr_tcnt;          // fixed width: violated clauses per clause-order tile
    const uint32_t* rr_sets;    // rr_T + 1 chunk starts (clause ids)
    uint32_t rr_T;
    uint32_t rr_k;              // common clause width (<= 8), 0 = ragged
    // multi-workgroup round robin (k_rr_mw): control words, global batch hash (keys = variable
    // + 1, 0 empty; minima = earliest turn, ~0 empty), per-set scan pointers and ends
    uint32_t* rr_ctl;
    uint32_t* rr_gkey;
    uint32_t* rr_gmin;
    uint32_t* rr_ptr;
    uint32_t* rr_end;
    uint32_t rr_mw;             // workgroups of k_rr_mw (one wave each, at most 64)
    // round robin by fixpoint (nullptr = off; k_rr_mw then decides every iteration,
    // otherwise only those whose fixpoint failed)
    RRFpCtl* fp_ctl;
    uint8_t* fp_in;             // per scan entry: bit 0 picked by the last pass, bit 1 by the one before
    uint32_t* fp_turn;          // per scan entry: turn = LFMIS priority of the next pass
    uint4* fp_v4;               // per scan entry of narrow instances: its variables (16-byte copy)
    uint32_t* fp_list;          // 2 x m: round lists per tile of FP_B entries (JOIN output, CLAIM output)
    uint32_t* fp_tcnt;          // 2 FP_G_MAX x tiles: list lengths per round and tile
    unsigned long long* fp_owner; // n_vars claim keys {epoch | turn | entry}, cleared only at an epoch restart
    uint32_t* fp_own0;          // n_vars: round-0 winner (entry) of every claimed variable (single
                                // claimants: for the whole iteration, k_fp_bbuild; shared: per pass)
    uint8_t* fp_cov;            // n_vars: serial of the pass whose pick covers the variable (cleared only at a
                                //   serial restart)
    // per-iteration claimant lists (k_fp_bscatter / k_fp_bbuild): variable v's violated
    // claimants are fp_vlist[fp_soff[v] ..), fp_soff = prefix of the static literal counts
    const uint32_t* fp_soff;    // n_vars + 1
    const uint32_t* fp_breg;    // n_bkt + 1: static pair region of every bucket (its literal count)
    unsigned long long* fp_pairs;  // L pairs {entry, variable} grouped by bucket
    uint32_t* fp_bfill;         // n_bkt: pairs in each bucket's region (this iteration)
    uint8_t* fp_hv;             // per variable (hot instances): the iteration stamp when it has > FP_HEAVY
                                //   violated claimants (its round claims are reduced in LDS first)
    uint8_t* fp_sole;           // per scan entry, byte j = 1: slot j's variable has no other violated
                                //   claimant this iteration (4 bytes per entry when every width <= 4, else 8)
    uint4* fp_sv;               // per bucket (bkt_width slots): shared variables {list start, count, v}
    uint32_t* fp_sbcnt;         // n_bkt: shared variables per bucket
    uint32_t* fp_vlist;         // violated claimants per variable (scan entries)
    uint32_t* fp_heavy;         // uint4 {v, start, end} segments of long lists (a wave each in round 0)
    uint32_t* fp_blk;           // 2 x blocks: pick counts, then their exclusive prefix
    uint32_t* fp_sf;            // T + 1: first scan entry of every set (entries past the last: nu)
    uint32_t* fp_bnd;           // T + 1: picks before the set's first entry inside its block
    uint32_t* fp_pf;            // T + 1: picks before the set's first entry (global)
    uint32_t* fp_nseg;          // T: schedule phases the set lives through
    uint4* fp_seg;              // T x T: {first level, first step, stride, offset} per (set, phase)
    uint32_t* fp_erase;         // T: erasure steps, ascending
    // incremental passes (fp_inc != 0; nullptr otherwise)
    uint32_t* fp_blocker;       // per scan entry out of the last pass's picks: a pick below it that shares a
                                //   variable with it (the pass's cover of that variable, fp_covby)
    uint32_t* fp_covby;         // n_vars: the pick that covered the variable in the current pass
    uint32_t* fp_lst;           // per scan entry, 4 slots (widths <= 4) or 8: {start, length} of the slot's
                                //   variable's claimant list (uint2; k_fp_bbuild)
    uint2* fp_sc;               // n_vars: {fp_soff, violated claimants this iteration}: a variable's claimant
                                //   list (written for the claimed variables only)
    uint32_t* fp_dl;            // 3 x m + 16 min(m, 2^16): the repair's dirty lists (two), its change log and
                                //   its raw push list
    uint32_t* fp_dmark;         // per scan entry: repair round stamp of its last dirty-list insertion
    uint8_t* fp_pbits;          // 2 x (m / 8 + 80) bytes: the picks, a bit per scan entry -- the working copy
                                //   (k_fp_turn writes it, the wide repair updates it, the repair keeps it in LDS
                                //   and writes its result back) and the last pass's picks behind it
    uint32_t* fp_log;           // FP_LOG_PASSES x 4: per pass of the current iteration {dirty entries, repair
                                //   rounds, entries decided, changes}, then the timing log (FP_LOG_RW per
                                //   pass; alll_rr_pass_log; measurement)
    uint32_t fp_inc;            // incremental passes enabled (no hot variables)
    uint32_t fp_rep_cap;        // dirty entries per repair round before the pass gives up (FP_REP_CAP; tests lower it)
    uint32_t fp_rw_min;         // wide repair rounds run while a round holds more entries than this (FP_RW_MIN;
                                // ~0u: no wide rounds, e.g. when its workgroups cannot all be resident)
    unsigned long long fp_rw_timeout;  // wide-round grid barrier timeout, 100 MHz ticks (FP_RW_TIMEOUT; tests)
    uint32_t fp_inc_after;      // full passes of an iteration before the incremental ones
    uint32_t fp_ib, fp_tb;      // key bits of the entry index and of the turn
    uint32_t fp_hot;            // the instance has hot variables (more grid rounds per pass)
    uint32_t fp_max;            // LFMIS passes per iteration
    // streaming solve with T > 1 threads (srr_T > 0; nullptr otherwise)
    uint32_t srr_T;
    SrrGen* srr_gen;            // srr_T + 1 generator plans of the iteration
    SrrPlan* srr_plan;
    unsigned long long* srr_first; // srr_T: first violated offset in every generator's range (~0: none)
    uint32_t* srr_bcnt;         // 2 x virtual blocks: violated walk steps per block, then their exclusive prefix
    uint32_t* srr_ent;          // violated walk steps of every generator in walk order (SRR_ENT_WORDS each)
    uint32_t* srr_step;         // (steps + 1) x srr_T: first entry of generator t's batch at step s; row
                                // `steps` = the ends of the lists
    // reference-RNG mode (ALLL_FLAG_REFERENCE_RNG, alll_refrng.hip; nullptr otherwise)
    unsigned long long* rrng_mask;   // ceil(m/64) words: this round's MIS clauses, clause order
    uint32_t* rrng_woff;             // per mask word: its clauses' literal count, then their bit offset in the block
    uint32_t* rrng_bsum;             // per 1024-word block: bit total, then the block's bit offset
    unsigned long long* rrng_stream; // the round's RBG draws (63 bits each)
    uint32_t* rrng_map;              // streaming solve: pick position -> clause id (the mask is by position)
    uint64_t rrng_cap;               // draws rrng_stream holds
    uint32_t* rrng_jump;             // rrng_levels x (rrng_nmax + 2): successor draw start, 2^t draws on
    unsigned long long* rrng_val;    // rrng_nmax + 2: the draw a start at each engine position yields
    uint32_t rrng_nmax;              // engine positions the parallel draws can consider
    uint32_t rrng_levels;            // jump levels: 2^levels > rrng_cap
    uint32_t n_vars;
    uint32_t n_words;
    uint32_t n_tiles;       // tiles covering [0, m)
    uint64_t seed;
};

// LDS of k_fp_bbuild for a bucket of `width` variables: counters, list starts, first claimants
inline size_t fp_bbuild_lds_bytes(uint32_t width) { return (size_t)12 * width + 16; }

// Launchers (alll_kernels.hip).  All asynchronous on `s`.
hipError_t launch_init_assignment(const LoopBuffers& b, hipStream_t s);
hipError_t launch_init_state(const LoopBuffers& b, hipStream_t s);
// limit_eval = n_iter + n, limit_nores = none, a stop at limit_nores is lifted (alll_run)
hipError_t launch_set_limits(const LoopBuffers& b, uint64_t n, hipStream_t s);
hipError_t launch_eval(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                       uint32_t tile_end, bool gated, hipStream_t s);
// scatter: also the bucket scatter of LFMIS round 0 (one GPU; runs split the workgroups' tiles)
// flags: the one-GPU round robin's evaluation (clause-order violated flags, no lists)
hipError_t launch_eval_hybrid(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                              uint32_t tile_end, bool gated, int n_blocks, bool scatter, hipStream_t s,
                              bool flags = false);
hipError_t launch_eval_ragged(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                              uint32_t tile_end, bool gated, int n_blocks, hipStream_t s);
hipError_t launch_collect(const ClauseView& cv, const LoopBuffers& b, uint32_t own_begin,
                          uint32_t own_end, hipStream_t s);
// clause-sharded: the own shard's violated clauses into cmask (own words cleared first); gated: the
// loop's (skipped once the loop state closes the evaluation), else a standalone pass (alll_verify)
hipError_t launch_cmark(const ClauseView& cv, const LoopBuffers& b, size_t words_per_rank, int rank, bool gated,
                        hipStream_t s);
hipError_t launch_reduce(const LoopBuffers& b, int mode, hipStream_t s);
hipError_t launch_round(const ClauseView& cv, const LoopBuffers& b, uint32_t r, bool last, hipStream_t s);
hipError_t launch_round0_buckets(const ClauseView& cv, const LoopBuffers& b, bool last, bool fused_reduce,
                                 bool scattered, hipStream_t s);
hipError_t launch_tail(const ClauseView& cv, const LoopBuffers& b, uint32_t first_round,
                       hipStream_t s);
// round robin: scan entries and the fixpoint's iteration set-up (when b.fp_ctl); n fixpoint
// passes; k_rr_mw for an iteration the passes did not settle
// marked: the evaluation set the clause-order violated flags itself (k_eval_flags)
hipError_t launch_rr_prep(const ClauseView& cv, const LoopBuffers& b, bool marked, hipStream_t s);
hipError_t prepare_kernels(const ClauseView& cv, const LoopBuffers& b);  // attributes, before any capture
// n passes: the first full (an LFMIS pass over every entry) when `full`, the others incremental
// when b.fp_inc (each kernel is gated on the pass kind the device state asks for)
hipError_t launch_rr_passes(const ClauseView& cv, const LoopBuffers& b, uint32_t n, bool full, hipStream_t s);
hipError_t launch_rr_finish(const ClauseView& cv, const LoopBuffers& b, hipStream_t s);
hipError_t launch_resample(const ClauseView& cv, const LoopBuffers& b, uint32_t tile_begin,
                           uint32_t tile_end, bool to_delta, hipStream_t s);
hipError_t launch_apply_delta(const LoopBuffers& b, hipStream_t s);
// resident workgroups of k_fp_repair per CU (its wide rounds need all FP_RW_GRID of them at once)
hipError_t fp_repair_occupancy(const ClauseView& cv, const LoopBuffers& b, int* blocks_per_cu);
// streaming solve with T > 1 threads (alll_stream.hip): the check's first violated offset of every
// generator (gated on the loop state), then the iteration's lists and round robins (b.srr_plan)
// reference-RNG mode (alll_refrng.hip): the initial fill and the resample round
hipError_t launch_refrng_init(const LoopBuffers& b, hipStream_t s);
hipError_t launch_refrng_resample(const ClauseView& cv, const LoopBuffers& b, hipStream_t s);
constexpr uint32_t RRNG_POS_PER_DRAW = 4;  // engine positions per draw the parallel draws allow (3.5 on average)
hipError_t launch_srr_first(const LoopBuffers& b, hipStream_t s);
hipError_t launch_srr_lists(const ClauseView& cv, const LoopBuffers& b, uint32_t nblk, hipStream_t s);
hipError_t launch_srr_mis(const ClauseView& cv, const LoopBuffers& b, hipStream_t s);

}  // namespace alll
