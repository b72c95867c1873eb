// alll_runtime.cpp -- host side of the C-ABI (include/alll.h): device memory layout,
// the per-iteration launch sequence (captured once into a hipGraph), the RCCL exchange of
// the clause-sharded multi-GPU mode, statistics.
//
// Reference correspondence: alll_create ~ SATInstance(var_arr, n_threads) +
// VariablesArray(n_vars) (SATInstance.h:51-56, VariablesArray.h:23-34); alll_solve ~
// SATInstance::solve -> parallel_solve (SATInstance.h:60-66, 217-320); alll_verify ~
// verify_validity (SATInstance.h:156-173).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <sched.h>
#include <thread>
#include <string>
#include <vector>

#include "alll.h"
#include "alll_internal.h"

using namespace alll;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess)                                                            \
            return fail(ALLL_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                        __FILE__, __LINE__);                                             \
    } while (0)

#define NCCL_TRY(expr)                                                                    \
    do {                                                                                  \
        ncclResult_t _r = (expr);                                                         \
        if (_r != ncclSuccess)                                                            \
            return fail(ALLL_ERR_RCCL, "%s failed: %s", #expr, ncclGetErrorString(_r));  \
    } while (0)

constexpr uint32_t DEFAULT_GRID_ROUNDS = 4;
// captured graphs of 1, 2, 4 and 8 iterations: a batch of n iterations replays n / 8 eight-
// iteration graphs and at most one of each smaller size (one launch gap per graph)
constexpr int GRAPH_SIZES = 4;
constexpr uint64_t SMALL_U_DEFAULT = 8192;
constexpr uint32_t GRAPH_UNROLL = 1u << (GRAPH_SIZES - 1);
constexpr uint32_t SKEWED_GRID_ROUNDS = 7;  // instances with hot variables

}  // namespace

struct alll_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    alll_options opt{};
    uint32_t n_vars = 0;
    uint64_t m = 0;
    uint64_t n_lits = 0;
    ClauseView cv{};
    LoopBuffers b{};
    uint32_t tiles_per_rank = 0, own_begin = 0, own_end = 0, n_tiles_padded = 0;
    uint32_t grid_rounds = DEFAULT_GRID_ROUNDS;
    // One GPU, bucketed round 0: the evaluation workgroups scatter their runs' claims themselves
    // (k_eval_scatter<K>, no k_bscatter launch; +2.6% iterations/s at M in round 4).  The
    // evaluation alone keeps its own kernel (k_eval_hybrid<K>: alll_bench_eval, verify, the
    // other variants) for its roofline.  env ALLL_FUSE_SCATTER=0: the separate k_bscatter
    bool fuse_scatter = true;
    std::vector<uint32_t> run_t0;  // bucketed round 0: first tile of every run (+ end)
    int rank = 0, world = 1;
    bool allreduce = false;
    ncclComm_t comm = nullptr;
    // device allocations
    std::vector<void*> allocs;
    DevState* h_state = nullptr;  // pinned mirror
    // captured iterations per LFMIS variant (0: atomic round 0, 1: bucketed round 0, 2: one grid
    // round + tail for few violated clauses): [v][j]
    // holds 2^j iterations
    hipGraph_t graph[3][GRAPH_SIZES] = {};
    hipGraphExec_t graph_exec[3][GRAPH_SIZES] = {};
    bool use_graph = true;
    std::string graph_note;      // why the loop launches eagerly (empty: graphs replay)
    // Hint for the LFMIS variant of the next launch batch (round0_variant): the violated count
    // and pass count of the last pass the host knows of.  read_state refreshes it; every
    // launch batch ends with an asynchronous copy of the device state into h_async, adopted
    // by the next batch once its event has completed (so a run(sync=False) loop follows the
    // device a batch behind instead of freezing at the last read); an assignment set by the
    // caller makes it unknown (treated as large).
    uint64_t hint_u = ~0ull, hint_iter = 0;
    // Round robin with the fixpoint passes: every iteration is a graph of the evaluation, the
    // set-up and rr_p passes, then (host-driven, after reading the pass state) single-pass
    // graphs until the passes settle (at most fp_max), then the finishing graph (k_rr_mw when
    // they did not, resample).  rr_p = the passes the last iteration needed.
    uint32_t rr_p = 8;
    std::vector<hipGraph_t> rr_graph;         // every captured round-robin graph (destroyed at the end)
    std::vector<hipGraphExec_t> rr_pre;       // [P]: evaluation .. set-up + P passes
    hipGraphExec_t rr_more = nullptr, rr_full = nullptr, rr_post = nullptr;
    uint32_t* h_fp = nullptr;                 // pinned copy of RRFpCtl's first words {state, nu, fp_iter, .., inc}
    DevState* h_async = nullptr;  // pinned
    hipEvent_t ev_async = nullptr;
    bool async_pending = false;
    uint64_t small_u = 0;       // one grid round (then the tail) when the last pass found at most
                                // this many violated clauses (variant 2)
    uint64_t bucket_min_u = 0;  // bucketed round 0 when the last pass found at least this many
    hipEvent_t ev[8] = {};
    int n_cu = 256;
    bool hybrid = false;
    alll_exchange_fn xfn = nullptr;  // host-staged exchange (instead of RCCL)
    void* xuser = nullptr;
    std::vector<uint8_t> xbuf;
    std::vector<uint32_t> perm;  // evaluation position -> clause id (fixed-k layout)
    std::string eval_name;
    int wall_khz = 100000;       // s_memrealtime rate (ALLL_FLAG_KERNEL_TIMING)
    // Streaming solve with T > 1 threads (b.srr_T > 0): the reference's
    // ClauseGenerator states (ClauseGenerator.h:104-113) between iterations, the plan of the next
    // one (pinned, uploaded per iteration) and the device lists, grown on demand
    struct SGen { uint64_t base = 0, n = 0, c = 0, ny = 0; bool fin = false; };
    std::vector<SGen> sgen;
    bool srr_started = false;   // an iteration ran: the next one starts where its check stopped
    uint64_t srr_batch = 1;
    SrrGen* h_srr = nullptr;
    SrrPlan* h_plan = nullptr;
    unsigned long long* h_first = nullptr;
    size_t srr_cap_blk = 0, srr_cap_ent = 0, srr_cap_step = 0;
    int rw_occupancy = 0;       // resident k_fp_repair workgroups per CU found at create (-1: query failed)
};

namespace {

// Host threads for the layout work of alll_create: the process's CPU affinity, at most 16
// (the CPU share of one GPU on the MI355X boxes) or OMP_NUM_THREADS when set.
unsigned host_threads() {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = std::max(1, CPU_COUNT(&cs));
    unsigned cap = 16;
    if (const char* e = getenv("OMP_NUM_THREADS")) { const int v = atoi(e); if (v > 0) cap = (unsigned)v; }
    return std::min(n, cap);
}

// Runs f(i) for i in [0, n) on up to nt threads (contiguous blocks of indices).
template <typename F>
void parallel_for(uint64_t n, unsigned nt, F f) {
    nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nt, n / 4096 + 1));
    if (nt <= 1) { for (uint64_t i = 0; i < n; ++i) f(i); return; }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] { for (uint64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) f(i); });
    for (auto& x : th) x.join();
}

// f(t, begin, end) on up to nt threads over contiguous blocks of [0, n); returns the threads used
template <typename F>
unsigned parallel_chunks(uint64_t n, unsigned nt, F f) {
    nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nt, n / 65536 + 1));
    if (nt <= 1) { f(0u, (uint64_t)0, n); return 1; }
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t) th.emplace_back([&, t] { f(t, n * t / nt, n * (t + 1) / nt); });
    for (auto& x : th) x.join();
    return nt;
}

// std::sort of a[0, n) on nt threads: sorted blocks, then pairwise merges level by level.
template <typename T, typename Cmp>
void parallel_sort(T* a, size_t n, Cmp cmp, unsigned nt) {
    if (nt <= 1 || n < (1u << 16)) { std::sort(a, a + n, cmp); return; }
    std::vector<size_t> cut(nt + 1);
    for (unsigned i = 0; i <= nt; ++i) cut[i] = n * i / nt;
    {
        std::vector<std::thread> th;
        for (unsigned i = 0; i < nt; ++i) th.emplace_back([&, i] { std::sort(a + cut[i], a + cut[i + 1], cmp); });
        for (auto& x : th) x.join();
    }
    for (unsigned w = 1; w < nt; w *= 2) {
        std::vector<std::thread> th;
        for (unsigned i = 0; i + w < nt; i += 2 * w)
            th.emplace_back([&, i, w] { std::inplace_merge(a + cut[i], a + cut[i + w], a + cut[std::min(i + 2 * w, nt)], cmp); });
        for (auto& x : th) x.join();
    }
}

template <typename T>
int dalloc(alll_ctx* c, T** p, size_t count, int fill = 0) {
    size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess)
        return fail(ALLL_ERR_OOM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
    c->allocs.push_back(q);
    e = hipMemsetAsync(q, fill, bytes, c->stream);
    if (e != hipSuccess) return fail(ALLL_ERR_HIP, "hipMemsetAsync failed: %s", hipGetErrorString(e));
    *p = static_cast<T*>(q);
    return ALLL_OK;
}

// Ragged-width evaluation layout (ClauseView::rg_off, k_eval_ragged): inside every shard the
// clauses are evaluated sorted by (width, block of the smallest variable, largest variable),
// so a chunk's 256 clauses share one width and the slot-0 lookups of a wave fall on few
// lines; every clause's literals are stored by descending variable (its smallest variable,
// looked up last, lies in the tile's LDS window) and padded to its chunk's width with an
// always-false literal.  perm maps positions to clause ids (CLAIM(0) translates the
// evaluation's positions; alll_get_violated_mask reorders the bitmask on the host).
int build_ragged(alll_ctx* c, const alll_problem* prob) {
    const uint64_t m = c->m;
    const uint64_t* offs = prob->offsets;
    const uint32_t* lits = prob->literals;
    LoopBuffers& b = c->b;
    ClauseView& cv = c->cv;
    const uint64_t win_vars = (uint64_t)b.win_words * 32;
    bool windows = c->n_vars > win_vars;
    if (const char* e = getenv("ALLL_EVAL_WINDOWS")) windows = atoi(e) != 0;
    const unsigned nt = host_threads();
    std::vector<uint32_t>& perm = c->perm;
    perm.resize(m);
    struct Key { uint64_t k1; uint32_t id; };
    auto key_of = [&](uint64_t cl) -> Key {
        uint32_t hi = 0, lo = ~0u;
        for (uint64_t j = offs[cl]; j < offs[cl + 1]; ++j) {
            const uint32_t v = lits[j] >> 1;
            hi = std::max(hi, v);
            lo = std::min(lo, v);
        }
        const uint64_t w = std::min<uint64_t>(offs[cl + 1] - offs[cl], (1u << 20) - 1);
        const uint64_t blk = (windows && lo != ~0u) ? std::min<uint64_t>(lo / win_vars, 1023) : 0;
        return {(w << 40) | (blk << 30) | (hi & ((1u << 30) - 1)), (uint32_t)cl};
    };
    // the own shard only (a clause range; the other ranks' shards keep clause order here: their
    // lists come from the all-gathered clause-order mask, k_collect)
    parallel_for(m, nt, [&](uint64_t i) { perm[i] = (uint32_t)i; });
    {
        const uint64_t cb0 = std::min<uint64_t>(m, (uint64_t)c->own_begin * TILE);
        const uint64_t ce0 = std::min<uint64_t>(m, (uint64_t)c->own_end * TILE);
        std::vector<Key> kv(ce0 - cb0);
        parallel_for(ce0 - cb0, nt, [&](uint64_t i) { kv[i] = key_of(cb0 + i); });
        parallel_sort(kv.data(), kv.size(), [](const Key& x, const Key& y) {
            return x.k1 != y.k1 ? x.k1 < y.k1 : x.id < y.id;
        }, nt);
        parallel_for(kv.size(), nt, [&](uint64_t i) { perm[cb0 + i] = kv[i].id; });
    }
    // chunk widths and offsets (units of CHUNK words)
    const uint64_t n_chunks = (m + CHUNK - 1) / CHUNK;
    std::vector<uint32_t> off(n_chunks + 1, 0u);
    uint64_t acc = 0;
    for (uint64_t g = 0; g < n_chunks; ++g) {
        uint64_t w = 0;
        for (uint64_t p = g * CHUNK; p < std::min<uint64_t>(m, (g + 1) * CHUNK); ++p)
            w = std::max<uint64_t>(w, offs[perm[p] + 1] - offs[perm[p]]);
        off[g] = (uint32_t)acc;
        acc += w;
        if (acc >= (1ull << 32)) return fail(ALLL_ERR_UNSUPPORTED, "ragged layout exceeds 2^32 chunk slots");
    }
    off[n_chunks] = (uint32_t)acc;
    static_assert(sizeof(b.n_words) == 4, "n_words");
    if (b.n_words >= (1u << 25)) return fail(ALLL_ERR_UNSUPPORTED, "ragged layout needs n_words < 2^25");
    const uint32_t false_lit = 64u * b.n_words;  // variable 32 * n_words: its word is out of range
    std::vector<uint32_t> t((size_t)acc * CHUNK, false_lit);
    const uint64_t own_p0 = std::min<uint64_t>(m, (uint64_t)c->own_begin * TILE);
    const uint64_t own_p1 = std::min<uint64_t>(m, (uint64_t)c->own_end * TILE);
    parallel_for(own_p1 - own_p0, nt, [&](uint64_t q) {
        const uint64_t p = own_p0 + q;
        const uint64_t cl = perm[p], g = p / CHUNK, r = p % CHUNK;
        const uint64_t w = offs[cl + 1] - offs[cl];
        std::vector<uint32_t> tmp(lits + offs[cl], lits + offs[cl] + w);
        std::sort(tmp.begin(), tmp.end(), [](uint32_t x, uint32_t y) { return (x >> 1) > (y >> 1); });
        uint32_t* dst = t.data() + (size_t)off[g] * CHUNK + r;
        for (uint64_t j = 0; j < w; ++j) dst[j * CHUNK] = tmp[j];
    });
    uint32_t *d_off = nullptr, *d_lits = nullptr, *d_perm = nullptr, *d_wb = nullptr;
    int rc;
    if ((rc = dalloc(c, &d_off, n_chunks + 1)) || (rc = dalloc(c, &d_lits, t.size())) || (rc = dalloc(c, &d_perm, m)))
        return rc;
    std::vector<uint32_t> wb;
    if (windows) {
        const uint32_t lds_words = std::min<uint32_t>(b.n_words, b.win_words);
        wb.assign(b.n_tiles, 0u);
        for (uint32_t tt = c->own_begin; tt < c->own_end; ++tt) {
            const uint64_t p = (uint64_t)tt * TILE;
            if (p >= m) break;
            const uint64_t cl = perm[p];
            uint32_t lo = ~0u;
            for (uint64_t j = offs[cl]; j < offs[cl + 1]; ++j) lo = std::min(lo, lits[j] >> 1);
            if (lo == ~0u) lo = 0;
            wb[tt] = std::min<uint64_t>((uint64_t)(lo / win_vars) * b.win_words, b.n_words - lds_words);
        }
        if ((rc = dalloc(c, &d_wb, b.n_tiles))) return rc;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(d_off, off.data(), off.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (!t.empty() && hipMemcpy(d_lits, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(d_perm, perm.data(), m * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (d_wb && hipMemcpy(d_wb, wb.data(), wb.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
        return fail(ALLL_ERR_HIP, "ragged layout upload failed");
    cv.rg_off = d_off;
    cv.rg_lits = d_lits;
    cv.perm = d_perm;
    if (d_wb) b.win_base = d_wb;
    return ALLL_OK;
}

int read_state(alll_ctx* c) {
    HIP_TRY(hipMemcpyAsync(c->h_state, c->b.state, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->hint_u = c->h_state->u_total;
    c->hint_iter = c->h_state->n_iter;
    c->async_pending = false;  // (the stream is drained: this read is newer)
    if (c->h_state->error == 4)
        return fail(ALLL_ERR_HIP, "round-robin MIS: a grid barrier of k_rr_mw timed out (its %u workgroups "
                                  "were not all resident)", c->b.rr_mw);
    if (c->h_state->error == 5)
        return fail(ALLL_ERR_HIP, "round-robin MIS: an incremental-pass kernel ran without its buffers (DESIGN.md §10)");
    if (c->h_state->error == 7)
        return fail(ALLL_ERR_HIP, "reference-RNG mode: a resample round needed more draws than its buffer holds");
    if (c->h_state->error == 6)
        return fail(ALLL_ERR_HIP, "streaming round robin: k_srr_mis made no progress (DESIGN.md §4.2.1)");
    if (c->h_state->error)
        return fail(ALLL_ERR_UNSUPPORTED, c->b.rr_T ? "round-robin MIS exceeded its batch cap in one iteration"
                                                    : "LFMIS needed more than %u rounds in one iteration",
                    MAX_TAIL_ROUNDS);
    return ALLL_OK;
}

int write_limits(alll_ctx* c, uint64_t limit_eval, uint64_t limit_nores) {
    // called only with the stream drained (after read_state)
    c->h_state->limit_eval = limit_eval;
    c->h_state->limit_nores = limit_nores;
    if (c->h_state->done == 2) c->h_state->done = 0;
    HIP_TRY(hipMemcpyAsync(c->b.state, c->h_state, sizeof(DevState), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ALLL_OK;
}

hipError_t eval_launch(alll_ctx* c, uint32_t tb, uint32_t te, bool gated, bool scatter = false, bool flags = false) {
    if (c->cv.rg_off) return launch_eval_ragged(c->cv, c->b, tb, te, gated, c->n_cu, c->stream);
    if (c->hybrid) return launch_eval_hybrid(c->cv, c->b, tb, te, gated, c->n_cu, scatter, c->stream, flags);
    return launch_eval(c->cv, c->b, tb, te, gated, c->stream);
}

// Host-staged collective: drain the stream, move the device buffer through host memory and
// the user's exchange function.  Allgather: `bytes` per rank, own piece at `own_off`.
int host_exchange(alll_ctx* c, int op, void* dev, size_t bytes, size_t own_off) {
    if (!c->xfn) return fail(ALLL_ERR_INVALID_ARG, "world > 1 without RCCL needs alll_set_host_exchange");
    const size_t total = op == ALLL_XCHG_ALLGATHER ? bytes * c->world : bytes;
    c->xbuf.resize(total);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (op == ALLL_XCHG_ALLGATHER)
        HIP_TRY(hipMemcpy(c->xbuf.data() + own_off, (uint8_t*)dev + own_off, bytes, hipMemcpyDeviceToHost));
    else
        HIP_TRY(hipMemcpy(c->xbuf.data(), dev, bytes, hipMemcpyDeviceToHost));
    if (c->xfn(c->xuser, op, c->xbuf.data(), bytes) != 0)
        return fail(ALLL_ERR_RCCL, "host exchange callback failed");
    HIP_TRY(hipMemcpy(dev, c->xbuf.data(), total, hipMemcpyHostToDevice));
    return ALLL_OK;
}

// Clause-sharded exchange after the evaluation: the violated bitmask pieces are all-gathered
// (clause order: cmask, marked from the own lists, when the evaluation order is not clause
// order; else the evaluation's own bitmask), then the other shards' lists are collected.
int enqueue_exchange(alll_ctx* c, hipStream_t s) {
    const size_t words = (size_t)c->tiles_per_rank * TILE_WORDS;
    uint64_t* mask = c->b.cmask ? c->b.cmask : c->b.vmask;
    if (c->b.cmask) HIP_TRY(launch_cmark(c->cv, c->b, words, c->rank, true, s));
    if (c->comm) {
        NCCL_TRY(ncclAllGather(mask + (size_t)c->rank * words, mask, words, ncclUint64, c->comm, s));
    } else {
        int rc = host_exchange(c, ALLL_XCHG_ALLGATHER, mask, words * 8, (size_t)c->rank * words * 8);
        if (rc) return rc;
    }
    HIP_TRY(launch_collect(c->cv, c->b, c->own_begin, c->own_end, s));
    return ALLL_OK;
}

// The launch sequence of one iteration (SATInstance.h:260-311).  Every kernel is gated on
// the device state, so replaying it after convergence is a no-op.
// Round-0 variant for the next iterations, from the last state read: the bucketed kernels
// have a fixed cost that only pays off on large violated sets (and they are not built for
// skewed instances, see create).
int round0_variant(const alll_ctx* c) {
    const uint64_t u = c->hint_u;
    if (c->b.rr_T) return 0;  // (round robin: launch_rr_iteration)
    if (c->b.pairs && (c->hint_iter == 0 || u >= c->bucket_min_u)) return 1;
    // few violated clauses (the end of a converging solve): round 0 on the grid, the rest in
    // the one-workgroup tail -- 6 launches per iteration instead of 12, each ~4.5 us even
    // when it has almost nothing to do
    if (c->hint_iter > 0 && u <= c->small_u && !c->b.rr_T) return 2;
    return 0;
}

// Adopt the asynchronous state copy of the last launch batch once it has landed.
// Ranks of a sharded run keep the hint of the synchronous state reads only (which they make at
// the same points of the loop), so that they pick the same graph variants at the same batches
// and capture their collectives in lockstep.
void refresh_hint(alll_ctx* c) {
    if (!c->async_pending) return;
    const hipError_t q = hipEventQuery(c->ev_async);
    if (q != hipSuccess) {
        // (hipErrorNotReady would stay the thread's last error and fail the next launch check)
        if (q == hipErrorNotReady) (void)hipGetLastError();
        return;
    }
    c->hint_u = c->h_async->u_total;
    c->hint_iter = c->h_async->n_iter;
    c->async_pending = false;
}

int post_state_copy(alll_ctx* c) {
    if (c->world > 1 || c->comm) return ALLL_OK;  // (sharded: synchronous hints only, refresh_hint)
    HIP_TRY(hipMemcpyAsync(c->h_async, c->b.state, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->ev_async, c->stream));
    c->async_pending = true;
    return ALLL_OK;
}

int enqueue_iteration(alll_ctx* c, hipEvent_t* marks, int variant) {
    hipStream_t s = c->stream;
    if (marks) HIP_TRY(hipEventRecord(marks[0], s));
    // one GPU, bucketed round 0: the evaluation workgroups scatter their runs' claims
    // themselves (no k_bscatter), before the reduce (pre-reduce epoch)
    const bool xchg = c->world > 1 || c->comm;  // the clause-sharded exchange path
    const bool scatter = variant == 1 && !xchg && c->hybrid && c->fuse_scatter && !c->b.rr_T;
    HIP_TRY(eval_launch(c, c->own_begin, c->own_end, true, scatter));
    if (marks) HIP_TRY(hipEventRecord(marks[1], s));
    if (xchg) {
        int rc = enqueue_exchange(c, s);
        if (rc) return rc;
    }
    if (marks) HIP_TRY(hipEventRecord(marks[2], s));
    // the bucketed round 0 runs the reduce in an extra k_bscatter workgroup (one GPU, no hot
    // variables, not the round robin): one launch less
    const bool fused = variant == 1 && !xchg && !c->b.rr_T;
    if (!fused) HIP_TRY(launch_reduce(c->b, 0, s));
    if (c->b.rr_T) {  // (without the fixpoint passes: k_rr_mw decides every iteration)
        HIP_TRY(launch_rr_prep(c->cv, c->b, false, s));
        HIP_TRY(launch_rr_finish(c->cv, c->b, s));
    } else {
        const uint32_t rounds = variant == 2 ? 1u : c->grid_rounds;
        for (uint32_t r = 0; r < rounds; ++r) {
            if (r == 0 && variant == 1)
                HIP_TRY(launch_round0_buckets(c->cv, c->b, rounds == 1, fused, scatter, s));
            else HIP_TRY(launch_round(c->cv, c->b, r, r + 1 == rounds, s));
        }
        HIP_TRY(launch_tail(c->cv, c->b, rounds, s));
    }
    if (marks) HIP_TRY(hipEventRecord(marks[3], s));
    if (c->allreduce && xchg) {
        HIP_TRY(launch_resample(c->cv, c->b, c->own_begin, c->own_end, true, s));
        if (c->comm) {
            NCCL_TRY(ncclAllReduce(c->b.delta, c->b.delta, c->b.n_words, ncclUint32, ncclSum, c->comm, s));
        } else {
            int rc = host_exchange(c, ALLL_XCHG_ALLREDUCE_SUM_U32, c->b.delta, (size_t)c->b.n_words * 4, 0);
            if (rc) return rc;
        }
        HIP_TRY(launch_apply_delta(c->b, s));
    } else {
        HIP_TRY(launch_resample(c->cv, c->b, c->own_begin, c->own_end, false, s));
    }
    if (marks) HIP_TRY(hipEventRecord(marks[4], s));
    return ALLL_OK;
}

// Round robin with the fixpoint passes: the pieces of one iteration.
//   pre(P):  evaluation [+ exchange] + reduce + scan entries + set-up + P passes
//   more:    one pass
//   post:    k_rr_mw (only if the passes did not settle) + resample
int enqueue_rr_piece(alll_ctx* c, hipEvent_t* marks, int piece, uint32_t passes) {
    hipStream_t s = c->stream;
    const bool xchg = c->world > 1 || c->comm;
    // one GPU, hybrid evaluation: the evaluation writes the clause-order violated flags itself
    const bool flags = !xchg && c->hybrid && c->b.rr_flag;
    if (piece == 0) {
        if (marks) HIP_TRY(hipEventRecord(marks[0], s));
        HIP_TRY(eval_launch(c, c->own_begin, c->own_end, true, false, flags));
        if (marks) HIP_TRY(hipEventRecord(marks[1], s));
        if (xchg) {
            int rc = enqueue_exchange(c, s);
            if (rc) return rc;
        }
        if (marks) HIP_TRY(hipEventRecord(marks[2], s));
        HIP_TRY(launch_reduce(c->b, 0, s));
        HIP_TRY(launch_rr_prep(c->cv, c->b, flags, s));
        HIP_TRY(launch_rr_passes(c->cv, c->b, passes, true, s));
    } else if (piece == 1 || piece == 3) {  // one incremental (1) or full (3) pass
        HIP_TRY(launch_rr_passes(c->cv, c->b, passes, piece == 3, s));
    } else {
        HIP_TRY(launch_rr_finish(c->cv, c->b, s));
        if (marks) HIP_TRY(hipEventRecord(marks[3], s));
        if (c->allreduce && xchg) {
            HIP_TRY(launch_resample(c->cv, c->b, c->own_begin, c->own_end, true, s));
            if (c->comm) {
                NCCL_TRY(ncclAllReduce(c->b.delta, c->b.delta, c->b.n_words, ncclUint32, ncclSum, c->comm, s));
            } else {
                int rc = host_exchange(c, ALLL_XCHG_ALLREDUCE_SUM_U32, c->b.delta, (size_t)c->b.n_words * 4, 0);
                if (rc) return rc;
            }
            HIP_TRY(launch_apply_delta(c->b, s));
        } else {
            HIP_TRY(launch_resample(c->cv, c->b, c->own_begin, c->own_end, false, s));
        }
        if (marks) HIP_TRY(hipEventRecord(marks[4], s));
    }
    return ALLL_OK;
}

// captured once per (piece, passes); nullptr when the loop launches eagerly
int rr_graph_of(alll_ctx* c, int piece, uint32_t passes, hipGraphExec_t* out) {
    *out = nullptr;
    hipGraphExec_t* slot = piece == 0 ? &c->rr_pre[passes] : piece == 1 ? &c->rr_more : piece == 3 ? &c->rr_full
                                                                                               : &c->rr_post;
    if (!c->use_graph) return ALLL_OK;
    if (*slot) { *out = *slot; return ALLL_OK; }
    hipError_t e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
        c->use_graph = false;
        c->graph_note = std::string("hipStreamBeginCapture: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        return ALLL_OK;
    }
    const int rc = enqueue_rr_piece(c, nullptr, piece, passes);
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(c->stream, &g);
    if (rc != ALLL_OK || e != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        c->graph_note = rc != ALLL_OK ? "capture of the iteration failed: " + g_err
                                      : std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        c->use_graph = false;
        return ALLL_OK;
    }
    c->rr_graph.push_back(g);
    e = hipGraphInstantiate(slot, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        *slot = nullptr;
        c->use_graph = false;
        c->graph_note = std::string("hipGraphInstantiate: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        return ALLL_OK;
    }
    (void)hipGraphUpload(*slot, c->stream);
    *out = *slot;
    return ALLL_OK;
}

int launch_rr_piece(alll_ctx* c, hipEvent_t* marks, int piece, uint32_t passes) {
    hipGraphExec_t g = nullptr;
    int rc;
    if (!marks && (rc = rr_graph_of(c, piece, passes, &g))) return rc;
    if (g) {
        HIP_TRY(hipGraphLaunch(g, c->stream));
        return ALLL_OK;
    }
    return enqueue_rr_piece(c, marks, piece, passes);
}

// One round-robin iteration with host-driven passes: pre(rr_p) (a full pass, then incremental
// ones), then one pass at a time while the pass state (read back) is still running -- an
// incremental one, or a full one after an incremental pass gave up -- at most fp_max in all, then
// post.  The host reads the pass state per decision instead of the GPU running passes after
// convergence.
int launch_rr_iteration(alll_ctx* c, hipEvent_t* marks) {
    const uint32_t cap = c->b.fp_max;
    uint32_t done = std::min(c->rr_p, cap);
    int rc;
    if ((rc = launch_rr_piece(c, marks, 0, done))) return rc;
    constexpr size_t ctl_words = offsetof(RRFpCtl, inc) / 4 + 1;  // {state, nu, fp_iter, ..., inc}
    for (;;) {
        HIP_TRY(hipMemcpyAsync(c->h_fp, c->b.fp_ctl, ctl_words * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->h_fp[0] != FP_RUN || done >= cap) break;
        const bool inc = c->h_fp[offsetof(RRFpCtl, inc) / 4] != 0;
        if ((rc = launch_rr_piece(c, marks, inc ? 1 : 3, 1))) return rc;
        ++done;
    }
    // next iteration: the passes this one needed (fp_iter = passes that changed the picks)
    // (two or four passes fewer, with more host-driven passes after them: within noise at M
    // and C5)
    if (c->h_fp[0] == FP_FINAL || c->h_fp[0] == FP_DONE) c->rr_p = std::max<uint32_t>(1, std::min(cap, c->h_fp[2] + 1));
    return launch_rr_piece(c, marks, 2, 0);
}

// ---- streaming solve with T > 1 threads ------------------------------------
// Device lists grown on demand (the stream is drained: the caller has just read the state).
int srr_grow(alll_ctx* c, uint32_t** p, size_t& cap, size_t need) {
    if (need <= cap) return ALLL_OK;
    need = std::max<size_t>(need + need / 4, 1024);
    if (*p) { (void)hipFree(*p); *p = nullptr; cap = 0; }
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, need * 4);
    if (e != hipSuccess) return fail(ALLL_ERR_OOM, "hipMalloc(%zu bytes) failed: %s", need * 4, hipGetErrorString(e));
    *p = static_cast<uint32_t*>(q);
    cap = need;
    return ALLL_OK;
}

// smallest s >= 1 with s = b_t (mod p_t) for every generator: the batch step at which all of them
// finish together (1 <= b_t <= p_t); false when there is none, or it lies beyond 2^62
bool srr_common_finish(const std::vector<uint64_t>& bs, const std::vector<uint64_t>& ps, uint64_t* S) {
    __int128 a = 0, mod = 1;  // s = a (mod mod)
    for (size_t t = 0; t < bs.size(); ++t) {
        const __int128 n2 = ps[t], a2 = bs[t] % ps[t];
        // a + mod k = a2 (mod n2)
        __int128 r0 = mod, r1 = n2, x0 = 1, x1 = 0;  // extended Euclid: x0 mod = r0 (mod n2)
        while (r1) {
            const __int128 q = r0 / r1, r = r0 - q * r1, x = x0 - q * x1;
            r0 = r1; r1 = r; x0 = x1; x1 = x;
        }
        const __int128 g = r0, d = a2 - a;
        if (d % g != 0) return false;
        const __int128 n2g = n2 / g;
        __int128 k = ((d / g) % n2g) * (x0 % n2g) % n2g;
        if (k < 0) k += n2g;
        a = a + mod * k;
        mod = mod * n2g;
        if (mod > ((__int128)1 << 62)) return false;
        a %= mod;
    }
    *S = a == 0 ? (uint64_t)mod : (uint64_t)a;
    return true;
}

// One iteration: evaluation + reduce (the previous iteration's check) + the check's stop offsets;
// then, while the loop is active, the plan from the generators' states, the lists, the round robins
// and the resample.  Host-synchronous (one state read per iteration).
int launch_srr_iteration(alll_ctx* c, hipEvent_t* marks) {
    hipStream_t s = c->stream;
    LoopBuffers& b = c->b;
    const uint32_t T = b.srr_T;
    if (marks) HIP_TRY(hipEventRecord(marks[0], s));
    HIP_TRY(eval_launch(c, c->own_begin, c->own_end, true));
    if (marks) { HIP_TRY(hipEventRecord(marks[1], s)); HIP_TRY(hipEventRecord(marks[2], s)); }
    HIP_TRY(launch_reduce(b, 0, s));
    HIP_TRY(launch_srr_first(b, s));
    HIP_TRY(hipMemcpyAsync(c->h_first, b.srr_first, T * 8ull, hipMemcpyDeviceToHost, s));
    int rc = read_state(c);
    if (rc) return rc;
    if (!c->h_state->active) {
        if (marks) { HIP_TRY(hipEventRecord(marks[3], s)); HIP_TRY(hipEventRecord(marks[4], s)); }
        return ALLL_OK;
    }
    std::vector<alll_ctx::SGen>& gens = c->sgen;
    if (c->srr_started) {
        // the lock-step check stopped after its first step that found a violated clause: every
        // generator has yielded min(n_t, f + 1) clauses (oracle/alll_oracle.c orc_solve_stream_rr)
        unsigned long long f = ~0ull;
        for (uint32_t t = 0; t < T; ++t) f = std::min(f, c->h_first[t]);
        for (auto& g : gens) {
            g.ny = std::min<uint64_t>(g.n, f + 1);
            g.fin = g.ny == g.n;
        }
    }
    // ---- plan: every generator's first window (r steps, finished at batch step b) and walks (p
    // steps each); the step S at which all finish together; the lists stop at the step by which
    // every generator has walked its whole range (later steps re-yield seen clauses only)
    const uint64_t B = c->srr_batch;
    std::vector<uint64_t> bs(T), ps(T), zs(T);
    for (uint32_t t = 0; t < T; ++t) {
        const auto& g = gens[t];
        SrrGen& d = c->h_srr[t];
        d.base = g.base;
        d.n = g.n;
        d.pt = g.n ? 9223372036854775783ull % g.n : 0;
        d.c0 = g.c;
        if (g.n == 0) { d.r = 0; d.b = 1; d.p = 1; zs[t] = 1; }
        else {
            d.r = g.fin ? g.n : g.n - g.ny;
            d.b = (d.r + B - 1) / B;
            d.p = (g.n + B - 1) / B;
            zs[t] = d.r == g.n ? d.b : d.b + d.p;
        }
        bs[t] = d.b;
        ps[t] = d.p;
    }
    uint64_t S = 0;
    if (!srr_common_finish(bs, ps, &S))
        return fail(ALLL_ERR_UNSUPPORTED, "streaming solve, %u threads: the generators never finish at the same "
                                          "batch step (the reference's loop, SATInstance.h:98-125, would not end)", T);
    const uint64_t steps = std::min<uint64_t>(S, *std::max_element(zs.begin(), zs.end()));
    uint64_t nblk = 0, total = 0;
    for (uint32_t t = 0; t < T; ++t) {
        SrrGen& d = c->h_srr[t];
        uint64_t y = 0;
        if (d.n) {
            if (steps <= d.b) y = std::min<uint64_t>(d.r, steps * B);
            else {
                const uint64_t q = steps - d.b;
                y = d.r + (q / d.p) * d.n + std::min<uint64_t>(d.n, (q % d.p) * B);
            }
        }
        d.yields = y;
        d.vblk = nblk;
        d.e0 = 0;
        nblk += (y + SRR_BLK - 1) / SRR_BLK;
        total += y;
    }
    c->h_srr[T] = SrrGen{};
    c->h_srr[T].vblk = nblk;
    if (total >= 0xFFFFFFFFull || nblk >= (1ull << 31) || (steps + 1) * T >= (1ull << 40))
        return fail(ALLL_ERR_UNSUPPORTED, "streaming solve: %llu walk steps in one iteration (limit 2^32)",
                    (unsigned long long)total);
    *c->h_plan = SrrPlan{T, (uint32_t)nblk, B, steps, S - steps};
    if ((rc = srr_grow(c, &b.srr_bcnt, c->srr_cap_blk, 2 * nblk + 1)) ||
        (rc = srr_grow(c, &b.srr_ent, c->srr_cap_ent, std::max<uint64_t>(total, 1) * SRR_ENT_WORDS)) ||
        (rc = srr_grow(c, &b.srr_step, c->srr_cap_step, (steps + 1) * T)))
        return rc;
    HIP_TRY(hipMemcpyAsync(b.srr_gen, c->h_srr, (T + 1) * sizeof(SrrGen), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(b.srr_plan, c->h_plan, sizeof(SrrPlan), hipMemcpyHostToDevice, s));
    HIP_TRY(launch_srr_lists(c->cv, b, (uint32_t)nblk, s));
    HIP_TRY(launch_srr_mis(c->cv, b, s));
    if (marks) HIP_TRY(hipEventRecord(marks[3], s));
    HIP_TRY(launch_resample(c->cv, b, c->own_begin, c->own_end, false, s));
    if (marks) HIP_TRY(hipEventRecord(marks[4], s));
    // after the batch loop every generator has finished (n_yielded = n_t) at walk position
    // c0 + (its walk steps in all S batch steps) P: r + whole walks, i.e. c0 + r P (mod n_t)
    for (uint32_t t = 0; t < T; ++t) {
        auto& g = gens[t];
        const SrrGen& d = c->h_srr[t];
        if (g.n) g.c = (uint64_t)(((unsigned __int128)(d.r % g.n) * d.pt + g.c) % g.n);
        g.ny = g.n;
        g.fin = true;
    }
    c->srr_started = true;
    // (the pinned plan is read by the copies above; the next iteration drains the stream in its
    // state read before it rewrites the plan)
    return ALLL_OK;
}

int ensure_graph(alll_ctx* c, int variant, int j) {
    if (!c->use_graph || c->graph_exec[variant][j]) return ALLL_OK;
    hipError_t e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
        c->use_graph = false;
        c->graph_note = std::string("hipStreamBeginCapture: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        return ALLL_OK;
    }
    int rc = ALLL_OK;
    for (uint32_t i = 0; i < (1u << j) && rc == ALLL_OK; ++i) rc = enqueue_iteration(c, nullptr, variant);
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(c->stream, &g);
    if (rc != ALLL_OK || e != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        c->graph_note = rc != ALLL_OK ? "capture of the iteration failed: " + g_err
                                      : std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        c->use_graph = false;  // fall back to eager launches (alll_uses_graphs reports it)
        return ALLL_OK;
    }
    e = hipGraphInstantiate(&c->graph_exec[variant][j], g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        (void)hipGraphDestroy(g);
        c->graph_exec[variant][j] = nullptr;
        c->use_graph = false;
        c->graph_note = std::string("hipGraphInstantiate: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        return ALLL_OK;
    }
    c->graph[variant][j] = g;
    (void)hipGraphUpload(c->graph_exec[variant][j], c->stream);
    return ALLL_OK;
}

// n iterations: n / 8 replays of the 8-iteration graph, then one replay per set bit of n % 8
int launch_srr_iteration(alll_ctx* c, hipEvent_t* marks);

int launch_iterations(alll_ctx* c, uint64_t n) {
    if (c->b.srr_T) {
        int rc;
        for (uint64_t i = 0; i < n; ++i)
            if ((rc = launch_srr_iteration(c, nullptr))) return rc;
        return ALLL_OK;
    }
    if (c->b.rr_T && c->b.fp_ctl) {
        int rc;
        for (uint64_t i = 0; i < n; ++i)
            if ((rc = launch_rr_iteration(c, nullptr))) return rc;
        return ALLL_OK;
    }
    refresh_hint(c);
    const int variant = round0_variant(c);
    int rc;
    // every size is captured, instantiated and uploaded at the variant's first launch, so a
    // later batch never pays a capture
    for (int j = 0; j < GRAPH_SIZES; ++j)
        if ((rc = ensure_graph(c, variant, j))) return rc;
    if (!c->use_graph) {
        for (uint64_t i = 0; i < n; ++i)
            if ((rc = enqueue_iteration(c, nullptr, variant))) return rc;
        return post_state_copy(c);
    }
    for (; n >= GRAPH_UNROLL; n -= GRAPH_UNROLL)
        HIP_TRY(hipGraphLaunch(c->graph_exec[variant][GRAPH_SIZES - 1], c->stream));
    for (int j = GRAPH_SIZES - 2; j >= 0; --j)
        if ((n >> j) & 1u) HIP_TRY(hipGraphLaunch(c->graph_exec[variant][j], c->stream));
    return post_state_copy(c);
}

int fill_stats(alll_ctx* c, alll_stats* st) {
    int rc = read_state(c);
    if (rc) return rc;
    std::vector<unsigned long long> ts(2 * (size_t)c->b.n_tiles);
    if (!ts.empty())
        HIP_TRY(hipMemcpy(ts.data(), c->b.tile_stats, ts.size() * 8, hipMemcpyDeviceToHost));
    memset(st, 0, sizeof(*st));
    st->n_iterations = c->h_state->n_iter;
    for (uint32_t t = 0; t < c->b.n_tiles; ++t) {
        st->sum_mis_size += ts[2 * t];
        st->n_resamples += ts[2 * t + 1];
        const uint32_t r = c->tiles_per_rank ? t / c->tiles_per_rank : 0;
        if (r < ALLL_MAX_GPU_STATS) st->gpu_resamples[r] += ts[2 * t + 1];
    }
    if (c->opt.stream_batch && st->n_iterations) {
        // a stream iteration is evaluation + MIS + resample + the full check (SATInstance.h:
        // 91-147); the check is the next evaluation pass, so the stream iterations are the
        // resample rounds: every pass but a final non-resampling one (solved or capped), and
        // at least one (a start that is already satisfied)
        const uint64_t rounds = st->n_iterations - (c->h_state->done ? 1 : 0);
        st->n_iterations = rounds ? rounds : 1;
    }
    st->avg_mis_size = st->n_iterations ? st->sum_mis_size / st->n_iterations : 0;
    st->n_violated = c->h_state->u_total;
    st->solved = (c->h_state->done == 1) ? 1 : 0;
    st->n_gpus = c->world;
    st->lfmis_rounds_max = c->h_state->max_rounds;
    st->lfmis_tail_rounds = c->h_state->tail_rounds;
    return ALLL_OK;
}

bool is_gfx950(int dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

}  // namespace

extern "C" {

const char* alll_version(void) { return "alll-mi355x 0.1.0 (abi 1, gfx950)"; }
const char* alll_last_error(void) { return g_err.c_str(); }
void alll_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }

void alll_default_options(alll_options* o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->seed = 1;
    o->max_iters = 0;
    o->device = -1;
    o->n_threads = 1;
    o->rank = 0;
    o->world = 1;
    o->flags = 0;
    o->grid_rounds = 0;
}

int alll_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int alll_comm_unique_id(uint8_t out[128]) {
    if (!out) return fail(ALLL_ERR_INVALID_ARG, "null output");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    memcpy(out, &id, 128);
    return ALLL_OK;
}

int alll_create(const alll_problem* prob, const alll_options* opt_in, alll_ctx** out) {
    if (!prob || !out) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    alll_options opt;
    if (opt_in) opt = *opt_in; else alll_default_options(&opt);
    if (opt.world < 1 || opt.rank < 0 || opt.rank >= opt.world)
        return fail(ALLL_ERR_INVALID_ARG, "bad rank %d / world %d", opt.rank, opt.world);
    if (opt.world > ALLL_MAX_GPU_STATS) return fail(ALLL_ERR_UNSUPPORTED, "world > %d", ALLL_MAX_GPU_STATS);
    const uint64_t m = prob->n_clauses;
    if (m && (!prob->offsets)) return fail(ALLL_ERR_INVALID_ARG, "null offsets");
    if (m >= 0xFFFFFFFFull - TILE) return fail(ALLL_ERR_UNSUPPORTED, "more than 2^32-4097 clauses");
    // ---- validate the CSR on the host (the reference has UB here: Clause.h:40)
    const uint64_t L = m ? prob->offsets[m] : 0;
    if (m && prob->offsets[0] != 0) return fail(ALLL_ERR_BAD_INPUT, "offsets[0] != 0");
    if (L && !prob->literals) return fail(ALLL_ERR_INVALID_ARG, "null literals");
    if (L >= 0xFFFFFFFFull) return fail(ALLL_ERR_UNSUPPORTED, "more than 2^32-1 literals");
    // (host passes over the instance run on the process's threads: at 128M clauses / 384M
    // literals a serial pass costs ~0.5 s, and every rank of a sharded run makes them)
    const unsigned hnt = host_threads();
    int fixed_k = -1;
    if (m) {
        const uint64_t w0 = prob->offsets[1] - prob->offsets[0];
        std::vector<uint64_t> bad(hnt, ~0ull);
        std::vector<uint8_t> ragged(hnt, 0);
        parallel_chunks(m, hnt, [&](unsigned t, uint64_t c0, uint64_t c1) {
            for (uint64_t c = c0; c < c1; ++c) {
                if (prob->offsets[c + 1] < prob->offsets[c]) { bad[t] = c; return; }
                if (prob->offsets[c + 1] - prob->offsets[c] != w0) ragged[t] = 1;
            }
        });
        const uint64_t first_bad = *std::min_element(bad.begin(), bad.end());
        if (first_bad != ~0ull) return fail(ALLL_ERR_BAD_INPUT, "offsets decrease at %llu", (unsigned long long)first_bad);
        fixed_k = *std::max_element(ragged.begin(), ragged.end()) ? 0 : (int)std::min<uint64_t>(w0, 1 << 30);
    }
    // the streaming solve keeps the clause-order (CSR) layout: its window rule needs the first
    // violated clause index, read from a clause-order bitmask
    // the round-robin MIS of T > 1 chunks (the reference's n_threads > 1) walks clause-order
    // lists of violated clauses: fixed widths keep the hybrid evaluation, whose lists are turned
    // into clause-order flags (k_rr_mark); ragged widths the CSR evaluation
    const uint32_t rr_T = (opt.n_threads > 1 && !(opt.flags & ALLL_FLAG_LFMIS) && !opt.stream_batch)
                              ? (uint32_t)opt.n_threads : 0u;
    if (rr_T > RR_TMAX) return fail(ALLL_ERR_UNSUPPORTED, "n_threads %u > %u chunks", rr_T, RR_TMAX);
    // the streaming solve with n_threads > 1: T clause generators and the per-batch round robin
    // (SATInstance.h:70-153)
    const uint32_t srr_T = (opt.n_threads > 1 && !(opt.flags & ALLL_FLAG_LFMIS) && opt.stream_batch)
                               ? (uint32_t)opt.n_threads : 0u;
    if (srr_T) {
        if (srr_T > RR_TMAX) return fail(ALLL_ERR_UNSUPPORTED, "streaming solve: n_threads %u > %u", srr_T, RR_TMAX);
        if (opt.world > 1) return fail(ALLL_ERR_UNSUPPORTED, "streaming solve with n_threads > 1 runs on one GPU");
        // an empty clause is violated forever and, sharing no variable, joins the MIS at every batch
        // step; the reference never returns on it (as with one thread), and here its repeats past the
        // materialised steps would be miscounted: refused
        for (uint64_t c = 0; c < m; ++c)
            if (prob->offsets[c + 1] == prob->offsets[c])
                return fail(ALLL_ERR_UNSUPPORTED, "streaming solve with n_threads > 1: clause %llu is empty",
                            (unsigned long long)c);
    }
    // the reference's own random stream (ALLL_FLAG_REFERENCE_RNG, alll_refrng.hip): defined for the
    // one-thread loop on one GPU (the reference's T > 1 resample draws from T engines inside a
    // schedule(dynamic) loop, so its bits follow the thread timing)
    const bool refrng = (opt.flags & ALLL_FLAG_REFERENCE_RNG) != 0;
    if (refrng) {
        bool zid = true;
        for (int i = 0; i < 128; ++i) zid &= opt.comm_id[i] == 0;
        if (opt.n_threads > 1)
            return fail(ALLL_ERR_UNSUPPORTED, "reference-RNG mode: n_threads must be 1 (the reference's T > 1 "
                                              "resample draws from T engines in a schedule(dynamic) loop)");

        if (opt.world > 1 || !zid || (opt.flags & ALLL_FLAG_EXCHANGE_ALLREDUCE))
            return fail(ALLL_ERR_UNSUPPORTED, "reference-RNG mode runs on one GPU without the exchange path");
    }
    std::vector<uint32_t> rr_sets;
    if (rr_T) {
        rr_sets.resize(rr_T + 1);
        if (opt.set_starts) {
            if (opt.set_starts[0] != 0 || opt.set_starts[rr_T] != m)
                return fail(ALLL_ERR_INVALID_ARG, "set_starts must run from 0 to n_clauses");
            for (uint32_t q = 0; q <= rr_T; ++q) {
                if (q && opt.set_starts[q] < opt.set_starts[q - 1])
                    return fail(ALLL_ERR_INVALID_ARG, "set_starts decrease at %u", q);
                rr_sets[q] = (uint32_t)opt.set_starts[q];
            }
        } else {
            // example/main.cpp:149-178: chunk_size = ceil(m / T); clause c moves to the next
            // chunk when c > (t + 1) * chunk_size, so chunk q >= 1 starts at q * chunk_size + 1
            const uint64_t chunk = (m + rr_T - 1) / rr_T;
            rr_sets[0] = 0;
            for (uint32_t q = 1; q <= rr_T; ++q) rr_sets[q] = (uint32_t)std::min<uint64_t>(m, q * chunk + 1);
            rr_sets[rr_T] = (uint32_t)m;
        }
    }
    const int rr_width = fixed_k;  // common clause width (-1: no clauses, 0: ragged)
    if (fixed_k < 1 || fixed_k > MAX_FIXED_K || (opt.flags & ALLL_FLAG_GENERIC_CSR) || opt.stream_batch)
        fixed_k = 0;
    const uint64_t lim = 2ull * prob->n_vars;
    {
        std::vector<uint64_t> bad(hnt, ~0ull);
        parallel_chunks(L, hnt, [&](unsigned t, uint64_t j0, uint64_t j1) {
            for (uint64_t j = j0; j < j1; ++j)
                if (prob->literals[j] >= lim) { bad[t] = j; return; }
        });
        const uint64_t j = *std::min_element(bad.begin(), bad.end());
        if (j != ~0ull)
            return fail(ALLL_ERR_LITERAL_RANGE, "literal %u at position %llu exceeds n_vars %u",
                        prob->literals[j], (unsigned long long)j, prob->n_vars);
    }

    // ---- hot variables (skewed degree: power-law hubs): degree >= max(1024, 32 x mean degree),
    // at most HOT_MAX of the highest; flagged in bit 31 of every literal copy the device uses
    std::vector<uint8_t> is_hot;
    uint32_t n_hot = 0;
    if (L && prob->n_vars && prob->n_vars < (1u << 30)) {
        // degrees from per-thread 16-bit saturating histograms (4-5x faster than shared atomic
        // counters at 384M literals), exact recount for the rare saturated candidates
        const uint64_t thr = std::max<uint64_t>(HOT_THR_MIN, HOT_MEAN_X * (L / prob->n_vars + 1));
        const unsigned dnt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(hnt, (2ull << 30) / (2ull * prob->n_vars)));
        std::vector<std::vector<uint16_t>> hist(dnt);
        const unsigned used = parallel_chunks(L, dnt, [&](unsigned t, uint64_t j0, uint64_t j1) {
            std::vector<uint16_t>& h = hist[t];
            h.assign(prob->n_vars, 0);
            for (uint64_t j = j0; j < j1; ++j) {
                uint16_t& c = h[prob->literals[j] >> 1];
                c += c != 0xFFFF;
            }
        });
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> hot_t(hnt);
        std::vector<std::vector<uint32_t>> rec_t(hnt);
        parallel_chunks(prob->n_vars, hnt, [&](unsigned t, uint64_t v0, uint64_t v1) {
            for (uint64_t v = v0; v < v1; ++v) {
                uint64_t d = 0;
                bool sat = false;
                for (unsigned q = 0; q < used; ++q) { d += hist[q][v]; sat |= hist[q][v] == 0xFFFF; }
                // (a saturated count is a lower bound: such a variable is recounted exactly
                // whatever its sum, the threshold applies to exact sums only)
                if (sat) rec_t[t].push_back((uint32_t)v);
                else if (d >= thr) hot_t[t].push_back({(uint32_t)d, (uint32_t)v});
            }
        });
        hist.clear();
        std::vector<std::pair<uint32_t, uint32_t>> hot;
        std::vector<uint32_t> recount;  // (ascending: the chunks are in variable order)
        for (unsigned t = 0; t < hnt; ++t) {
            hot.insert(hot.end(), hot_t[t].begin(), hot_t[t].end());
            recount.insert(recount.end(), rec_t[t].begin(), rec_t[t].end());
        }
        if (!recount.empty()) {  // (a variable with >= 65535 literals in one thread's range)
            std::vector<uint64_t> d(recount.size(), 0);
            for (uint64_t j = 0; j < L; ++j) {
                const uint32_t v = prob->literals[j] >> 1;
                const auto it = std::lower_bound(recount.begin(), recount.end(), v);
                if (it != recount.end() && *it == v) ++d[it - recount.begin()];
            }
            for (size_t q = 0; q < recount.size(); ++q)
                if (d[q] >= thr) hot.push_back({(uint32_t)std::min<uint64_t>(d[q], 0xFFFFFFFFu), recount[q]});
        }
        if (!hot.empty()) {
            std::sort(hot.rbegin(), hot.rend());
            if (hot.size() > HOT_MAX) hot.resize(HOT_MAX);
            is_hot.assign(prob->n_vars, 0);
            for (auto& h : hot) is_hot[h.second] = 1;
            n_hot = (uint32_t)hot.size();
        }
    }

    // ---- device
    int ndev = alll_device_count();
    if (ndev <= 0) return fail(ALLL_ERR_NO_DEVICE, "no HIP device visible");
    int dev = opt.device;
    if (dev < 0) { if (hipGetDevice(&dev) != hipSuccess) dev = 0; }
    if (dev >= ndev) return fail(ALLL_ERR_NO_DEVICE, "device %d not visible (%d devices)", dev, ndev);
    if (!is_gfx950(dev)) return fail(ALLL_ERR_NO_DEVICE, "device %d is not gfx950 (MI355X)", dev);
    HIP_TRY(hipSetDevice(dev));

    alll_ctx* c = new (std::nothrow) alll_ctx();
    if (!c) return fail(ALLL_ERR_OOM, "host allocation failed");
    c->device = dev;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
            c->n_cu = prop.multiProcessorCount;
    }
    c->opt = opt;
    c->n_vars = prob->n_vars;
    c->m = m;
    c->n_lits = L;
    c->rank = opt.rank;
    c->world = opt.world;
    c->allreduce = (opt.flags & ALLL_FLAG_EXCHANGE_ALLREDUCE) != 0;
    c->use_graph = (opt.flags & ALLL_FLAG_NO_GRAPH) == 0;
    if (!c->use_graph) c->graph_note = "ALLL_FLAG_NO_GRAPH";
    c->grid_rounds = opt.grid_rounds ? opt.grid_rounds : DEFAULT_GRID_ROUNDS;
    c->small_u = SMALL_U_DEFAULT;
    if (const char* e = getenv("ALLL_SMALL_U")) c->small_u = strtoull(e, nullptr, 10);  // tuning, tests
    if (const char* e = getenv("ALLL_FUSE_SCATTER")) c->fuse_scatter = atoi(e) != 0;
    auto bail = [&](int rc) { alll_destroy(c); return rc; };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(ALLL_ERR_HIP, "hipStreamCreate failed"));
    for (auto& e : c->ev)
        if (hipEventCreate(&e) != hipSuccess) return bail(fail(ALLL_ERR_HIP, "hipEventCreate failed"));
    if (hipHostMalloc((void**)&c->h_state, sizeof(DevState), 0) != hipSuccess ||
        hipHostMalloc((void**)&c->h_async, sizeof(DevState), 0) != hipSuccess)
        return bail(fail(ALLL_ERR_OOM, "hipHostMalloc failed"));
    if (hipEventCreateWithFlags(&c->ev_async, hipEventDisableTiming) != hipSuccess)
        return bail(fail(ALLL_ERR_HIP, "hipEventCreate failed"));

    // ---- tiles and shards (contiguous clause ranges; concatenation = clause order)
    const uint32_t n_tiles = (uint32_t)((m + TILE - 1) / TILE);
    c->tiles_per_rank = (n_tiles + c->world - 1) / c->world;
    if (c->tiles_per_rank == 0) c->tiles_per_rank = 1;
    c->n_tiles_padded = c->tiles_per_rank * c->world;
    c->own_begin = std::min<uint32_t>(n_tiles, (uint32_t)c->rank * c->tiles_per_rank);
    c->own_end = std::min<uint32_t>(n_tiles, c->own_begin + c->tiles_per_rank);
    c->b.own_begin = c->own_begin;
    c->b.own_end = c->own_end;

    int rc;
    LoopBuffers& b = c->b;
    b.n_vars = c->n_vars;
    b.n_words = (c->n_vars + 31) / 32;
    b.win_words = LDS_WORDS;
    if (const char* e = getenv("ALLL_WIN_WORDS"))  // tests: small windows on small instances
        b.win_words = std::max<uint32_t>(16, std::min<uint32_t>(b.win_words, (uint32_t)std::max(0, atoi(e)))) / 8 * 8;
    b.n_cu = (uint32_t)c->n_cu;
    b.n_tiles = n_tiles;
    b.m = m;
    if (opt.stream_batch && m && !srr_T) {
        // key of the streaming solve: position in the generator sequence j*P mod m, so the
        // inverse of P mod m (P is prime, so it exists for every m < P)
        const uint64_t p = 9223372036854775783ull % m;
        int64_t r0 = (int64_t)m, r1 = (int64_t)p, t0 = 0, t1 = 1;
        while (r1) {
            const int64_t q = r0 / r1;
            int64_t x = r0 - q * r1; r0 = r1; r1 = x;
            x = t0 - q * t1; t0 = t1; t1 = x;
        }
        if (m > 1 && r0 != 1) return bail(fail(ALLL_ERR_UNSUPPORTED, "generator step not invertible mod %llu",
                                                (unsigned long long)m));
        b.stream_pinv = m > 1 ? (uint64_t)((t0 % (int64_t)m + (int64_t)m) % (int64_t)m) : 0;
        b.stream_batch = opt.stream_batch;
    }
    b.seed = opt.seed;
    if (rr_T) {
        uint32_t* d_sets = nullptr;
        if ((rc = dalloc(c, &b.rr_u, 12 * (size_t)m))) return bail(rc);  // scan entries (k_rr_entries)
        if (fixed_k > 0) {  // the hybrid evaluation's lists -> clause-order flags (k_rr_mark)
            if ((rc = dalloc(c, &b.rr_flag, (size_t)n_tiles * TILE))) return bail(rc);
            if ((rc = dalloc(c, &b.rr_tcnt, n_tiles))) return bail(rc);
        }
        if ((rc = dalloc(c, &d_sets, rr_T + 1))) return bail(rc);
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(d_sets, rr_sets.data(), (rr_T + 1) * 4ull, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(ALLL_ERR_HIP, "chunk upload failed"));
        b.rr_sets = d_sets;
        b.rr_T = rr_T;
        b.rr_k = (rr_width >= 1 && rr_width <= 8) ? (uint32_t)rr_width : 0u;
        // the batch kernel (fallback of the fixpoint): one workgroup per lane group, at most 64
        const uint32_t mw = std::min<uint32_t>(rr_T, 64);
        if ((rc = dalloc(c, &b.rr_ctl, RR_MW_CTL_WORDS))) return bail(rc);
        if ((rc = dalloc(c, &b.rr_gkey, RR_MW_GH))) return bail(rc);
        if ((rc = dalloc(c, &b.rr_gmin, RR_MW_GH, 0xFF))) return bail(rc);
        if ((rc = dalloc(c, &b.rr_ptr, rr_T))) return bail(rc);
        if ((rc = dalloc(c, &b.rr_end, rr_T))) return bail(rc);
        b.rr_mw = mw;
        // the fixpoint passes: keys {epoch | turn | entry} need >= 10 epoch
        // bits; ALLL_RR_FP=0 leaves every iteration to the batch kernels, ALLL_RR_FP_MAX sets the
        // passes per iteration (graph unroll)
        auto bits_of = [](uint64_t x) { uint32_t k = 1; while (k < 64 && (x >> k)) ++k; return k; };
        const uint32_t ib = bits_of(m), tb = bits_of(m + rr_T + 1);
        bool fp = rr_T <= FP_TMAX && ib + tb + 10 <= 64 && ib <= 28;  // (28: the claim pairs' slot tags)
        if (const char* e = getenv("ALLL_RR_FP")) fp = fp && atoi(e) != 0;
        if (fp) {
            const size_t nblk = m / FP_B + 2;
            if ((rc = dalloc(c, &b.fp_ctl, 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_in, m + FP_B))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_turn, m + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_v4, (rr_width >= 1 && rr_width <= 4) ? m + 1 : 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_sole, (size_t)m * ((rr_width >= 1 && rr_width <= 4) ? 4 : 8) + 16))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_list, 2 * (size_t)m + 2))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_tcnt, 2 * FP_G_MAX * ((size_t)m / 256 + 2)))) return bail(rc);  // (round tiles of 256)
            if ((rc = dalloc(c, &b.fp_owner, (size_t)prob->n_vars + 1, 0xFF))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_cov, (size_t)prob->n_vars + 16))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_own0, (size_t)prob->n_vars + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_vlist, (size_t)L + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_heavy, 4 * ((size_t)L / 64 + 2)))) return bail(rc);  // (segments of lists > 64 claims)
            if ((rc = dalloc(c, &b.fp_pairs, (size_t)L + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_blk, 2 * nblk + 2048))) return bail(rc);  // sums, offsets, changes, earliest changes
            if ((rc = dalloc(c, &b.fp_sf, rr_T + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_bnd, rr_T + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_pf, rr_T + 1))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_nseg, rr_T))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_seg, (size_t)rr_T * rr_T))) return bail(rc);
            if ((rc = dalloc(c, &b.fp_erase, rr_T))) return bail(rc);
            b.fp_ib = ib;
            b.fp_tb = tb;
            b.fp_hot = 0;  // (set with the hot-variable flags below)
            b.fp_max = FP_MAX_DEFAULT;
            if (const char* e = getenv("ALLL_RR_FP_MAX"))  // tests: iterations left to k_rr_mw mid-run
                b.fp_max = (uint32_t)std::max(1, std::min(250, atoi(e)));
            c->rr_p = std::min<uint32_t>(c->rr_p, b.fp_max);
            c->rr_pre.assign(b.fp_max + 1, nullptr);
            if (hipHostMalloc((void**)&c->h_fp, sizeof(RRFpCtl), 0) != hipSuccess)
                return bail(fail(ALLL_ERR_OOM, "hipHostMalloc failed"));
            // incremental passes on instances without hot variables
            // (ALLL_RR_INC=0: full passes only; tests, A/B)
            bool inc = n_hot == 0;
            if (const char* e = getenv("ALLL_RR_INC")) inc = inc && atoi(e) != 0;
            if (inc) {
                if ((rc = dalloc(c, &b.fp_blocker, m + 1, 0xFF)) || (rc = dalloc(c, &b.fp_covby, (size_t)prob->n_vars + 1)) ||
                    (rc = dalloc(c, &b.fp_sc, (size_t)prob->n_vars + 1)) || (rc = dalloc(c, &b.fp_dl, 3 * (size_t)m + 16 * std::min<size_t>(m, 1u << 16) + 64)) ||
                    (rc = dalloc(c, &b.fp_dmark, m + 1)) || (rc = dalloc(c, &b.fp_pbits, 2 * ((size_t)m / 8 + 80))) ||
                    (rc = dalloc(c, &b.fp_log, FP_LOG_WORDS)) ||
                    (rc = dalloc(c, &b.fp_lst, 2 * (size_t)m * ((rr_width >= 1 && rr_width <= 4) ? 4 : 8) + 16)))
                    return bail(rc);
                b.fp_inc = 1;
                b.fp_inc_after = 1;
                // the repair's limits (tests lower them to force the fallbacks: a pass that gives
                // up, wide rounds on small instances, barriers that time out)
                b.fp_rep_cap = FP_REP_CAP;
                b.fp_rw_min = FP_RW_MIN;
                b.fp_rw_timeout = FP_RW_TIMEOUT;
                if (const char* e = getenv("ALLL_RR_REP_CAP")) b.fp_rep_cap = (uint32_t)std::max(1, atoi(e));
                if (const char* e = getenv("ALLL_RR_RW_MIN")) b.fp_rw_min = (uint32_t)std::max(0, atoi(e));
                if (const char* e = getenv("ALLL_RR_RW_TIMEOUT")) b.fp_rw_timeout = strtoull(e, nullptr, 10);
                if (const char* e = getenv("ALLL_RR_INC_AFTER")) b.fp_inc_after = (uint32_t)std::max(1, atoi(e));
            }
        }
    }
    if (srr_T) {
        if ((rc = dalloc(c, &b.srr_gen, srr_T + 1)) || (rc = dalloc(c, &b.srr_plan, 1)) ||
            (rc = dalloc(c, &b.srr_first, srr_T)))
            return bail(rc);
        if (hipHostMalloc((void**)&c->h_srr, (srr_T + 1) * sizeof(SrrGen), 0) != hipSuccess ||
            hipHostMalloc((void**)&c->h_plan, sizeof(SrrPlan), 0) != hipSuccess ||
            hipHostMalloc((void**)&c->h_first, srr_T * 8ull, 0) != hipSuccess)
            return bail(fail(ALLL_ERR_OOM, "hipHostMalloc failed"));
        b.srr_T = srr_T;
        c->srr_batch = opt.stream_batch;
        // the generators of SATInstance.h:74-86 (T t_n_clauses = n_clauses / n_threads, the last
        // one takes the remainder), fresh
        c->sgen.resize(srr_T);
        const uint64_t tn = m / srr_T;
        for (uint32_t t = 0; t < srr_T; ++t) {
            c->sgen[t].base = (uint64_t)t * tn;
            c->sgen[t].n = t == srr_T - 1 ? m - c->sgen[t].base : tn;
        }
        c->use_graph = false;
        c->graph_note = "streaming solve with n_threads > 1: host-planned iterations (eager launches)";
    }
    if ((rc = dalloc(c, &b.A, b.n_words + 4))) return bail(rc);  // +4: 16-byte tail loads
    if ((rc = dalloc(c, &b.vmask, (size_t)c->n_tiles_padded * TILE_WORDS))) return bail(rc);
    if ((rc = dalloc(c, &b.tile_cnt, n_tiles))) return bail(rc);
    if ((rc = dalloc(c, &b.mis_cnt, n_tiles))) return bail(rc);
    const size_t ent_words = (fixed_k > 0 ? (size_t)fixed_k + 1 : 1);
    if ((rc = dalloc(c, &b.stage[0], (size_t)n_tiles * TILE * ent_words))) return bail(rc);
    if ((rc = dalloc(c, &b.stage[1], (size_t)n_tiles * TILE * ent_words))) return bail(rc);
    if ((rc = dalloc(c, &b.mis, (size_t)n_tiles * TILE))) return bail(rc);
    if ((rc = dalloc(c, &b.left, (size_t)n_tiles * TILE * ent_words))) return bail(rc);
    if ((rc = dalloc(c, &b.tmis, (size_t)n_tiles * TILE))) return bail(rc);
    if (refrng && m) {
        const uint64_t nmw = (m + 63) / 64, nblk = (nmw + 1023) / 1024;
        if ((rc = dalloc(c, &b.rrng_mask, (size_t)nmw)) || (rc = dalloc(c, &b.rrng_woff, (size_t)nmw)) ||
            (rc = dalloc(c, &b.rrng_bsum, (size_t)nblk + 1)))
            return bail(rc);
        b.rrng_cap = L / 63 + 2;  // a round draws ceil(bits / 63), bits <= every literal
        if ((rc = dalloc(c, &b.rrng_stream, (size_t)b.rrng_cap))) return bail(rc);
        // the parallel draws (alll_refrng.hip): engine positions for RRNG_POS_PER_DRAW per draw,
        // jump levels until 2^levels exceeds the most draws a round can take
        uint64_t nmax = std::min<uint64_t>(b.rrng_cap * RRNG_POS_PER_DRAW + 64, 0xFFFFFFF0ull);
        // (test knob: fewer positions, so that the parallel draws run past them and the
        // one-thread chain redoes the round)
        if (const char* e = getenv("ALLL_RRNG_NMAX"))
            if (*e) nmax = std::max<uint64_t>(8, std::min<uint64_t>(nmax, strtoull(e, nullptr, 10)));
        b.rrng_nmax = (uint32_t)nmax;
        b.rrng_levels = 1;
        while ((1ull << b.rrng_levels) <= b.rrng_cap) ++b.rrng_levels;
        if ((rc = dalloc(c, &b.rrng_jump, (size_t)b.rrng_levels * (nmax + 2))) ||
            (rc = dalloc(c, &b.rrng_val, (size_t)nmax + 2)))
            return bail(rc);
        if (opt.stream_batch && (rc = dalloc(c, &b.rrng_map, (size_t)m))) return bail(rc);
    } else if (refrng) {
        // (no clauses: the initial fill still draws; the mask pointer marks the mode)
        if ((rc = dalloc(c, &b.rrng_mask, 1))) return bail(rc);
    }
    // skewed instances (hot variables): owner slots and round-0 buckets by vmix (alll_internal.h)
    b.vmix_mul = 1u;
    b.vmix_mask = 0xFFFFFFFFu;
    uint64_t vrange = c->n_vars;  // owner slots / bucketed variable keys
    if (n_hot) {
        vrange = 1024;
        while (vrange < c->n_vars) vrange <<= 1;
        b.vmix_mul = 0x9E3779B1u;
        b.vmix_mask = (uint32_t)(vrange - 1);
    }
    if ((rc = dalloc(c, &b.owner, (size_t)vrange, 0xFF))) return bail(rc);
    {
        uint32_t inv = b.vmix_mul;  // Newton iteration for the inverse mod 2^32 (odd multiplier)
        for (int it = 0; it < 5; ++it) inv *= 2u - b.vmix_mul * inv;
        b.vmix_inv = inv;
    }
    if (b.fp_ctl) {
        // round robin: claimant lists by variable buckets (k_fp_bscatter / k_fp_bbuild): bucket =
        // vmix(v) / width, width a multiple of 64, one bucket per CU
        // when the width fits the LDS of k_fp_bbuild
        const uint64_t span = std::max<uint64_t>(vrange, 1);
        uint64_t width = (span + (uint64_t)c->n_cu - 1) / (uint64_t)c->n_cu;  // (two per CU: no faster)
        width = std::max<uint64_t>(1024, (width + 63) / 64 * 64);
        width = std::min<uint64_t>(width, 12288);
        uint64_t nb = (span + width - 1) / width;
        if (nb > BKT_MAX) {
            width = ((span + BKT_MAX - 1) / BKT_MAX + 63) / 64 * 64;
            nb = (span + width - 1) / width;
        }
        if (fp_bbuild_lds_bytes((uint32_t)width) > 160u * 1024 - 1024)
            return bail(fail(ALLL_ERR_UNSUPPORTED, "round robin: %u variables exceed the claimant buckets", c->n_vars));
        b.bkt_width = (uint32_t)width;
        b.bkt_magic = (uint32_t)((1ull << 32) / width);
        b.n_bkt = (uint32_t)nb;
        b.bkt_span = (uint32_t)span;
        std::vector<uint32_t> soff(c->n_vars + 1, 0u), breg(nb + 1, 0u);
        parallel_chunks(L, hnt, [&](unsigned, uint64_t j0, uint64_t j1) {
            for (uint64_t j = j0; j < j1; ++j) __atomic_fetch_add(&soff[prob->literals[j] >> 1], 1u, __ATOMIC_RELAXED);
        });
        uint32_t acc = 0;
        for (uint32_t v = 0; v < c->n_vars; ++v) {
            const uint32_t d = soff[v];
            soff[v] = acc;
            acc += d;
            breg[((uint64_t)((v * b.vmix_mul) & b.vmix_mask)) / width] += d;
        }
        soff[c->n_vars] = acc;
        acc = 0;
        for (uint64_t k = 0; k <= nb; ++k) { const uint32_t d = breg[k]; breg[k] = acc; acc += d; }
        uint32_t *d_soff = nullptr, *d_breg = nullptr;
        if ((rc = dalloc(c, &d_soff, soff.size())) || (rc = dalloc(c, &d_breg, breg.size())) ||
            (rc = dalloc(c, &b.fp_bfill, nb)) ||
            (rc = dalloc(c, &b.fp_sv, (size_t)nb * width)) || (rc = dalloc(c, &b.fp_sbcnt, nb)))
            return bail(rc);
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(d_soff, soff.data(), soff.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(d_breg, breg.data(), breg.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(ALLL_ERR_HIP, "claimant bucket upload failed"));
        b.fp_soff = d_soff;
        b.fp_breg = d_breg;
    }
    if ((rc = dalloc(c, &b.cover, (size_t)b.n_words * 32))) return bail(rc);  // whole words, zero-padded
    if ((rc = dalloc(c, &b.tile_stats, 2 * (size_t)n_tiles))) return bail(rc);
    if ((rc = dalloc(c, &b.delta, b.n_words))) return bail(rc);
    if ((rc = dalloc(c, &b.state, 1))) return bail(rc);
    if (opt.flags & ALLL_FLAG_KERNEL_TIMING) {
        if ((rc = dalloc(c, &b.ktime, (size_t)TIME_SLOTS * TIME_FIELDS))) return bail(rc);
        std::vector<unsigned long long> init((size_t)TIME_SLOTS * TIME_FIELDS, 0ull);
        for (uint32_t i = 0; i < TIME_SLOTS; ++i) init[(size_t)i * TIME_FIELDS] = ~0ull;
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(b.ktime, init.data(), init.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(ALLL_ERR_HIP, "timing buffer upload failed"));
    }
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) == hipSuccess && khz > 0)
            c->wall_khz = khz;
    }
    // ---- bucketed LFMIS round 0 (fixed width): one bucket per CU when a bucket's minima fit
    // in LDS (else ~300-1000 power-of-2 buckets), runs of up to 16 tiles
    if (fixed_k > 0 && !rr_T && !(opt.flags & ALLL_FLAG_ATOMIC_CLAIMS) && n_tiles > 0 && c->n_vars > 0) {
        uint32_t shift = BKT_SHIFT_MIN;
        while (shift < BKT_SHIFT_MAX && (vrange >> shift) > 384) ++shift;
        uint64_t width = (vrange + (uint64_t)c->n_cu - 1) / (uint64_t)c->n_cu;
        width = std::max<uint64_t>(width, 1u << BKT_SHIFT_MIN);
        if (width > (1u << BKT_SHIFT_MAX)) width = 1u << shift;
        const uint64_t nb = (vrange + width - 1) / width;
        // skewed pair load (a literal distribution whose hubs are not all flagged hot): the
        // fullest bucket's workgroup would serialise the round; such instances keep the atomic
        // claims.  Hot literals never become pairs (LDS hash + owner), and vmix spreads the
        // remaining high-degree variables of power-law instances over the buckets.
        bool skewed = false;
        if (nb <= BKT_MAX) {
            std::vector<std::vector<uint64_t>> lt(hnt, std::vector<uint64_t>(nb, 0));
            std::vector<uint64_t> lp(hnt, 0);
            const unsigned used = parallel_chunks(L, hnt, [&](unsigned t, uint64_t j0, uint64_t j1) {
                for (uint64_t j = j0; j < j1; ++j) {
                    const uint32_t v = prob->literals[j] >> 1;
                    if (n_hot && is_hot[v]) continue;
                    ++lt[t][((v * b.vmix_mul) & b.vmix_mask) / width];
                    ++lp[t];
                }
            });
            std::vector<uint64_t> load(nb, 0);
            uint64_t L_pairs = 0;
            for (unsigned t = 0; t < used; ++t) {
                for (uint64_t k = 0; k < nb; ++k) load[k] += lt[t][k];
                L_pairs += lp[t];
            }
            const uint64_t mx = *std::max_element(load.begin(), load.end());
            skewed = mx > 4 * (L_pairs / nb + 1);
        }
        // Runs: the tile range of every evaluation workgroup (min(n_tiles, CUs) of them, the
        // split of k_eval_hybrid) cut into rpw runs of at most RUN_TILES_MAX tiles, so that one
        // GPU's evaluation workgroups scatter their own runs (k_eval_hybrid `scatter`).
        const uint32_t nblk = std::min<uint32_t>(n_tiles, (uint32_t)c->n_cu);
        const uint32_t wmax = (n_tiles + nblk - 1) / nblk;
        const uint32_t rpw = (wmax + RUN_TILES_MAX - 1) / RUN_TILES_MAX;
        c->run_t0.assign((size_t)nblk * rpw + 1, 0u);
        uint32_t rt = 1;
        for (uint32_t w = 0; w < nblk; ++w) {
            const uint32_t t0 = (uint32_t)((uint64_t)n_tiles * w / nblk), t1 = (uint32_t)((uint64_t)n_tiles * (w + 1) / nblk);
            for (uint32_t j = 0; j < rpw; ++j) {
                const uint32_t a0 = t0 + (t1 - t0) * j / rpw, a1 = t0 + (t1 - t0) * (j + 1) / rpw;
                c->run_t0[(size_t)w * rpw + j] = a0;
                rt = std::max(rt, a1 - a0);
            }
        }
        c->run_t0.back() = n_tiles;
        const uint64_t area = (uint64_t)nblk * rpw * rt * TILE * fixed_k;  // pairs
        if (nb <= BKT_MAX && !skewed && area < (1ull << 32)) {  // pair positions are 32-bit in k_bresolve
            b.bkt_width = (uint32_t)width;
            b.bkt_magic = (uint32_t)((1ull << 32) / width);
            b.n_bkt = (uint32_t)nb;
            b.run_tiles = rt;
            b.n_runs = nblk * rpw;
            uint32_t* d_rt0 = nullptr;
            if ((rc = dalloc(c, &d_rt0, c->run_t0.size()))) return bail(rc);
            if (hipStreamSynchronize(c->stream) != hipSuccess ||
                hipMemcpy(d_rt0, c->run_t0.data(), c->run_t0.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
                return bail(fail(ALLL_ERR_HIP, "run table upload failed"));
            b.run_t0 = d_rt0;
            const size_t run_cap = (size_t)b.run_tiles * TILE * fixed_k;
            if ((rc = dalloc(c, &b.pairs, (size_t)b.n_runs * run_cap))) return bail(rc);
            if ((rc = dalloc(c, &b.runtab, (size_t)b.n_bkt * b.n_runs))) return bail(rc);
            if ((rc = dalloc(c, &b.run_pairs, b.n_runs))) return bail(rc);
            // below this many violated clauses the atomic round 0 is cheaper (fixed costs)
            c->bucket_min_u = std::max<uint64_t>(65536, m / 64);
            if (const char* e = getenv("ALLL_BUCKET_MIN_U")) c->bucket_min_u = strtoull(e, nullptr, 10);
        }
    }
    // ---- clause storage allocations, then drain the zero-fills before synchronous uploads
    ClauseView& cv = c->cv;
    cv.m = m;
    cv.k = (uint32_t)fixed_k;
    cv.lit_mask = 0x7FFFFFFFu;  // (bit 31: hot-variable flag)
    uint32_t *d_lits = nullptr, *d_t = nullptr, *d_o = nullptr;
    const uint64_t real_chunks = (m + CHUNK - 1) / CHUNK;
    if ((rc = dalloc(c, &d_lits, L))) return bail(rc);
    if (fixed_k > 0) {
        if ((rc = dalloc(c, &d_t, real_chunks * CHUNK * fixed_k))) return bail(rc);
    } else {
        if ((rc = dalloc(c, &d_o, m + 1))) return bail(rc);
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(fail(ALLL_ERR_HIP, "memset drain failed"));

    // ---- clauses: AoS literals (+ offsets or a chunk-transposed copy for fixed width k)
    // hot variables (chosen above) flagged in bit 31 of every literal copy the device uses
    std::vector<uint32_t> flagged;
    {
        if (n_hot) {
            flagged.assign(prob->literals, prob->literals + L);
            for (auto& l : flagged)
                if (is_hot[l >> 1]) l |= 0x80000000u;
            cv.n_hot = n_hot;
            if (b.fp_ctl) {
                b.fp_hot = 1;
                if ((rc = dalloc(c, &b.fp_hv, (size_t)prob->n_vars + 16))) return bail(rc);
            }
            // skewed instances need more rounds before the leftovers are few enough for
            // the single-workgroup tail (power-law 3-SAT at 10M clauses: 10 rounds)
            if (!opt.grid_rounds) c->grid_rounds = SKEWED_GRID_ROUNDS;
        }
        const uint32_t* src = flagged.empty() ? prob->literals : flagged.data();
        if (L && hipMemcpy(d_lits, src, L * 4, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(ALLL_ERR_HIP, "literal upload failed"));
    }
    cv.lits = d_lits;
    if (fixed_k > 0) {
        // Locality order for evaluation (results do not depend on it: the violated set is a
        // set and the LFMIS priorities are the original clause ids).  Inside every shard the
        // clauses are evaluated sorted by (largest, second largest) variable and each clause's
        // literals are stored by descending variable, so the gathers of slot 0 (and mostly
        // slot 1) of a wave hit a few cache lines.  perm[p] = original id of position p.
        //
        // Windows (instances with more than win_vars variables; ALLL_EVAL_WINDOWS=0/1 overrides):
        // the hybrid evaluation's LDS holds win_vars consecutive variables; clauses are first
        // grouped by the block of their smallest variable and each tile's LDS window starts at
        // its block, so the smallest variable (looked up by every clause) is an LDS hit.
        std::vector<uint32_t>& perm = c->perm;
        perm.resize(m);
        const uint64_t win_vars = (uint64_t)b.win_words * 32;
        bool windows = c->n_vars > win_vars;
        if (const char* e = getenv("ALLL_EVAL_WINDOWS")) windows = atoi(e) != 0;  // tuning, tests
        {
            const int K = fixed_k;
            struct Key { uint64_t k1; uint32_t k2, id; };
            auto key_of = [&](uint64_t cl) -> Key {
                uint32_t a = 0, b2 = 0, lo = ~0u;
                for (int j = 0; j < K; ++j) {
                    const uint32_t v = prob->literals[cl * K + j] >> 1;
                    if (v > a) { b2 = a; a = v; }
                    else if (v > b2) b2 = v;
                    lo = std::min(lo, v);
                }
                const uint64_t blk = windows ? lo / win_vars : 0;
                return {(blk << 32) | a, b2, (uint32_t)cl};
            };
            const unsigned nt = host_threads();
            auto sort_range = [&](uint64_t cb0, uint64_t ce0) {
                std::vector<Key> kv(ce0 - cb0);
                parallel_for(ce0 - cb0, nt, [&](uint64_t i) { kv[i] = key_of(cb0 + i); });
                parallel_sort(kv.data(), kv.size(), [](const Key& x, const Key& y) {
                    return x.k1 != y.k1 ? x.k1 < y.k1 : (x.k2 != y.k2 ? x.k2 < y.k2 : x.id < y.id);
                }, nt);
                parallel_for(kv.size(), nt, [&](uint64_t i) { perm[cb0 + i] = kv[i].id; });
            };
            // the own shard only: the other ranks' shards keep clause order (identity perm; their
            // violated lists come from the all-gathered clause-order mask and the AoS literals)
            parallel_for(m, nt, [&](uint64_t i) { perm[i] = (uint32_t)i; });
            const uint64_t cb0 = std::min<uint64_t>(m, (uint64_t)c->own_begin * TILE);
            const uint64_t ce0 = std::min<uint64_t>(m, (uint64_t)c->own_end * TILE);
            if (ce0 > cb0) sort_range(cb0, ce0);
        }
        // Packed clause ids: when the literals leave enough bits below the hot flag, slot j of
        // every clause also carries bits [j * id_bits, (j + 1) * id_bits) of its clause id, so
        // the evaluation emits clause ids and perm is never read on the device
        // (ALLL_PACKED_IDS=0 keeps positions + perm; tuning, tests).
        {
            const uint64_t max_lit = 2ull * std::max<uint64_t>(c->n_vars, 1) - 1;
            // (at least 6: the evaluation takes a variable's bit index from literal bits 1..5
            // without masking)
            const uint32_t lit_bits = std::max<uint32_t>(6, 64 - (uint32_t)__builtin_clzll(max_lit));
            const uint32_t spare = lit_bits < 31 ? 31 - lit_bits : 0;
            const uint32_t idb = m > 1 ? 64 - (uint32_t)__builtin_clzll(m - 1) : 1;
            const uint32_t per = (idb + fixed_k - 1) / fixed_k;
            bool pack = per <= spare;
            if (const char* e = getenv("ALLL_PACKED_IDS")) pack = pack && atoi(e) != 0;
            if (pack) {
                cv.id_shift = lit_bits;
                cv.id_bits = per;
                cv.lit_mask = (1u << lit_bits) - 1u;
            }
        }
        // (the own shard's chunks only: shards are tile-aligned, so they are whole chunks)
        const uint32_t id_mask = cv.id_bits ? (1u << cv.id_bits) - 1u : 0u;
        const uint64_t own_p0 = std::min<uint64_t>(m, (uint64_t)c->own_begin * TILE);
        const uint64_t own_p1 = std::min<uint64_t>(m, (uint64_t)c->own_end * TILE);
        const uint64_t g0 = own_p0 / CHUNK, g1 = (own_p1 + CHUNK - 1) / CHUNK;
        std::vector<uint32_t> t((g1 - g0) * CHUNK * fixed_k, 0u);
        parallel_for(own_p1 - own_p0, host_threads(), [&](uint64_t q) {
            const uint64_t p2 = own_p0 + q;
            uint32_t tmp[MAX_FIXED_K];
            const uint64_t cl = perm[p2];
            for (int j = 0; j < fixed_k; ++j)
                tmp[j] = flagged.empty() ? prob->literals[cl * fixed_k + j] : flagged[cl * fixed_k + j];
            // by descending variable (the hot flag, bit 31, is not part of it: slot K-1 must
            // hold the smallest variable, which the tile's window and bit 31 of win_base cover)
            std::sort(tmp, tmp + fixed_k, [](uint32_t x, uint32_t y) {
                return ((x & 0x7FFFFFFFu) >> 1) > ((y & 0x7FFFFFFFu) >> 1);
            });
            const uint64_t g = p2 / CHUNK - g0, r = p2 % CHUNK;
            for (int j = 0; j < fixed_k; ++j) {
                const uint32_t idp = cv.id_bits ? ((uint32_t)(cl >> (j * cv.id_bits)) & id_mask) << cv.id_shift : 0u;
                t[(g * fixed_k + j) * CHUNK + r] = tmp[j] | idp;
            }
        });
        if (!t.empty() && hipMemcpy(d_t + g0 * CHUNK * fixed_k, t.data(), t.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(ALLL_ERR_HIP, "transposed literal upload failed"));
        if (!cv.id_bits) {
            uint32_t* d_perm = nullptr;
            if ((rc = dalloc(c, &d_perm, m))) return bail(rc);
            if (hipStreamSynchronize(c->stream) != hipSuccess ||
                hipMemcpy(d_perm, perm.data(), m * 4, hipMemcpyHostToDevice) != hipSuccess)
                return bail(fail(ALLL_ERR_HIP, "permutation upload failed"));
            cv.perm = d_perm;
        }
        cv.lits_t = d_t;
        // a literal stream larger than the 256 MB Infinity Cache is read non-temporally (it
        // cannot stay cached between iterations and would evict the assignment words of the L2
        // lookups); ALLL_EVAL_NT=0/1 overrides (tuning, tests)
        cv.lits_nt = (uint64_t)real_chunks * CHUNK * fixed_k * 4 > (256ull << 20) ? 1u : 0u;
        if (const char* e = getenv("ALLL_EVAL_NT")) cv.lits_nt = atoi(e) != 0;
        cv.offs = nullptr;
        if (windows && m) {  // LDS window of every tile: the block of its first clause's smallest variable
            const uint32_t lds_words = std::min<uint32_t>(b.n_words, b.win_words);
            std::vector<uint32_t> wb(n_tiles, 0u);
            for (uint32_t tt = c->own_begin; tt < c->own_end; ++tt) {
                const uint64_t p = (uint64_t)tt * TILE;
                if (p >= m) break;
                const uint64_t cl = perm[p];
                uint32_t lo = ~0u;
                for (int j = 0; j < fixed_k; ++j) lo = std::min(lo, prob->literals[cl * fixed_k + j] >> 1);
                wb[tt] = std::min<uint64_t>((uint64_t)(lo / win_vars) * b.win_words, b.n_words - lds_words);
            }
            // bit 31: every clause of the tile has its smallest variable in the window (all but
            // the tiles at block boundaries), so k_eval_hybrid reads slot K-1 from LDS only
            parallel_for(c->own_end - c->own_begin, host_threads(), [&](uint64_t q) {
                const uint64_t tt = c->own_begin + q;
                bool all_in = true;
                for (uint64_t p = tt * TILE; p < std::min<uint64_t>(m, (tt + 1) * TILE) && all_in; ++p) {
                    const uint64_t cl = perm[p];
                    uint32_t lo = ~0u;
                    for (int j = 0; j < fixed_k; ++j) lo = std::min(lo, prob->literals[cl * fixed_k + j] >> 1);
                    all_in = (uint32_t)(lo / 32) - wb[tt] < lds_words;
                }
                if (all_in) wb[tt] |= 0x80000000u;
            });
            uint32_t* d_wb = nullptr;
            if ((rc = dalloc(c, &d_wb, n_tiles))) return bail(rc);
            if (hipStreamSynchronize(c->stream) != hipSuccess ||
                hipMemcpy(d_wb, wb.data(), n_tiles * 4ull, hipMemcpyHostToDevice) != hipSuccess)
                return bail(fail(ALLL_ERR_HIP, "window upload failed"));
            b.win_base = d_wb;
        }
    } else {
        std::vector<uint32_t> o32(m + 1);
        for (uint64_t i = 0; i <= m; ++i) o32[i] = m ? (uint32_t)prob->offsets[i] : 0u;
        if (hipMemcpy(d_o, o32.data(), (m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess)
            return bail(fail(ALLL_ERR_HIP, "offset upload failed"));
        cv.offs = d_o;
        // Ragged widths, T = 1, not streaming: chunk-transposed copy for k_eval_ragged (the
        // CSR arrays above stay: the LFMIS kernels read clauses by id).  ALLL_FLAG_GENERIC_CSR
        // keeps the clause-order CSR evaluation.
        // (the padding literal 64 * n_words must decode to an out-of-range word through the 25
        // word-index bits k_eval_ragged extracts, and leave bit 31 clear: n_words < 2^25;
        // ALLL_FLAG_NO_RANGED keeps the clause-order CSR evaluation like GENERIC_CSR)
        const bool ragged = m && !rr_T && !opt.stream_batch &&
                            !(opt.flags & (ALLL_FLAG_GENERIC_CSR | ALLL_FLAG_NO_RANGED)) &&
                            b.n_words < (1u << 25);
        if (ragged && (rc = build_ragged(c, prob))) return bail(rc);
    }

    // ---- state + initial assignment
    memset(c->h_state, 0, sizeof(DevState));
    c->h_state->limit_eval = ~0ull;
    c->h_state->limit_nores = ~0ull;
    c->h_state->round_next = 1;
    if (refrng) c->h_state->rd_state = opt.seed;  // (the random_device stand-in's state)
    if (hipMemcpyAsync(b.state, c->h_state, sizeof(DevState), hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return bail(fail(ALLL_ERR_HIP, "state upload failed"));
    if (launch_init_assignment(b, c->stream) != hipSuccess)
        return bail(fail(ALLL_ERR_HIP, "init kernel launch failed"));
    {  // kernel attributes (dynamic LDS), outside every stream capture
        const hipError_t e = prepare_kernels(cv, b);
        if (e != hipSuccess) return bail(fail(ALLL_ERR_HIP, "kernel attributes: %s", hipGetErrorString(e)));
    }
    if (b.fp_inc) {
        // the wide repair rounds synchronise their workgroups by a grid barrier: all of them must be
        // resident at once, else every incremental pass would wait for the barrier's timeout and
        // give up; without that guarantee the repair keeps to its one-workgroup rounds
        // (a failed query, or one that reports no resident workgroup at all -- seen in processes that
        // had imported torch, whose bundled HIP runtime answers it differently -- keeps the wide
        // rounds: their barriers time out safely, and are counted)
        int per_cu = 0;
        const uint32_t gw = std::min<uint32_t>(FP_RW_GRID, std::max(1, c->n_cu));
        (void)hipGetLastError();
        const hipError_t e = fp_repair_occupancy(cv, b, &per_cu);
        if (e == hipSuccess && per_cu > 0 && (uint64_t)per_cu * (uint64_t)c->n_cu < gw) b.fp_rw_min = ~0u;
        if (e != hipSuccess) (void)hipGetLastError();
        c->rw_occupancy = e == hipSuccess ? per_cu : -1;
        if (getenv("ALLL_DEBUG_OCCUPANCY"))  // (diagnostics)
            fprintf(stderr, "alll: k_fp_repair occupancy query %s, %d per CU, %d CUs, wide rounds %s\n",
                    hipGetErrorString(e), per_cu, c->n_cu, b.fp_rw_min == ~0u ? "off" : "on");
    }

    // ---- RCCL communicator (clause-sharded mode; world 1 with a comm id: a one-rank
    // communicator that runs the multi-GPU exchange path on one GPU)
    bool zero_id = true;
    for (int i = 0; i < 128; ++i) zero_id &= opt.comm_id[i] == 0;
    if ((c->world > 1 || !zero_id) && (cv.k > 0 || cv.rg_off)) {
        // the exchange's clause-order mask (this rank laid out its own shard only)
        if ((rc = dalloc(c, &b.cmask, (size_t)c->n_tiles_padded * TILE_WORDS))) return bail(rc);
        if ((rc = dalloc(c, &b.cflag, (size_t)c->tiles_per_rank * TILE + 64))) return bail(rc);
    }
    if (c->world > 1 && (rc = dalloc(c, &b.xcount, 4))) return bail(rc);
    if (c->world > 1 || !zero_id) {
        const bool zero = zero_id;
        if (!zero) {
            ncclUniqueId id;
            memcpy(&id, opt.comm_id, 128);
            ncclResult_t r = ncclCommInitRank(&c->comm, c->world, id, c->rank);
            if (r != ncclSuccess) return bail(fail(ALLL_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r)));
        } else {
            c->use_graph = false;  // host-staged exchange: eager launches
            c->graph_note = "host-staged exchange (eager launches)";
        }
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess)
        return bail(fail(ALLL_ERR_HIP, "create: stream sync failed: %s", hipGetErrorString(hipGetLastError())));
    c->hybrid = cv.k > 0 && !(opt.flags & ALLL_FLAG_NO_RANGED);
    char nm[64];
    if (cv.rg_off) snprintf(nm, sizeof nm, "k_eval_ragged");
    else if (c->hybrid) snprintf(nm, sizeof nm, "k_eval_hybrid<%u>", cv.k);
    else if (cv.k) snprintf(nm, sizeof nm, "k_eval_fixed<%u>", cv.k);
    else snprintf(nm, sizeof nm, "k_eval_csr");
    c->eval_name = nm;
    *out = c;
    return ALLL_OK;
}

int alll_destroy(alll_ctx* c) {
    if (!c) return ALLL_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (int v = 0; v < 3; ++v)
        for (int u = 0; u < GRAPH_SIZES; ++u) {
            if (c->graph_exec[v][u]) (void)hipGraphExecDestroy(c->graph_exec[v][u]);
            if (c->graph[v][u]) (void)hipGraphDestroy(c->graph[v][u]);
        }
    for (auto& g : c->rr_pre)
        if (g) (void)hipGraphExecDestroy(g);
    if (c->rr_more) (void)hipGraphExecDestroy(c->rr_more);
    if (c->rr_full) (void)hipGraphExecDestroy(c->rr_full);
    if (c->rr_post) (void)hipGraphExecDestroy(c->rr_post);
    for (auto g : c->rr_graph) (void)hipGraphDestroy(g);
    if (c->h_fp) (void)hipHostFree(c->h_fp);
    if (c->h_srr) (void)hipHostFree(c->h_srr);
    if (c->h_plan) (void)hipHostFree(c->h_plan);
    if (c->h_first) (void)hipHostFree(c->h_first);
    for (uint32_t* p : {c->b.srr_bcnt, c->b.srr_ent, c->b.srr_step})
        if (p) (void)hipFree(p);
    if (c->comm) ncclCommDestroy(c->comm);
    for (void* p : c->allocs) (void)hipFree(p);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->h_state) (void)hipHostFree(c->h_state);
    if (c->h_async) (void)hipHostFree(c->h_async);
    if (c->ev_async) (void)hipEventDestroy(c->ev_async);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return ALLL_OK;
}

int alll_set_host_exchange(alll_ctx* c, alll_exchange_fn fn, void* user) {
    if (!c) return fail(ALLL_ERR_INVALID_ARG, "null context");
    c->xfn = fn;
    c->xuser = user;
    c->use_graph = false;
    c->graph_note = "host-staged exchange (eager launches)";
    return ALLL_OK;
}

int alll_solve(alll_ctx* c, alll_stats* st) {
    if (!c) return fail(ALLL_ERR_INVALID_ARG, "null context");
    HIP_TRY(hipSetDevice(c->device));
    int rc = read_state(c);
    if (rc) return rc;
    // (streaming solve: max_iters counts stream iterations; the last one's check is one more
    // evaluation pass, which does not resample)
    const uint64_t cap = c->opt.max_iters ? c->opt.max_iters + (c->opt.stream_batch ? 1 : 0) : ~0ull;
    if (c->h_state->done != 1) {
        if ((rc = write_limits(c, cap, cap))) return rc;
        uint64_t batch = 1;
        for (;;) {
            if ((rc = launch_iterations(c, batch))) return rc;
            if ((rc = read_state(c))) return rc;
            if (c->h_state->done || c->h_state->n_iter >= cap) break;
            batch = std::min<uint64_t>(batch * 2, 64);
        }
    }
    alll_stats tmp;
    if ((rc = fill_stats(c, st ? st : &tmp))) return rc;
    if (c->h_state->done != 1)
        return fail(ALLL_ERR_MAX_ITERS, "not solved after %llu eval passes (%llu clauses violated)",
                    (unsigned long long)c->h_state->n_iter, (unsigned long long)c->h_state->u_total);
    return ALLL_OK;
}

int alll_run(alll_ctx* c, uint64_t n_iters, alll_stats* st) {
    if (!c) return fail(ALLL_ERR_INVALID_ARG, "null context");
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if (n_iters) {
        // no host round trip: the limit is set on the device (n_iter + n_iters), stream-ordered
        // before the iterations; after convergence every kernel is gated off
        HIP_TRY(launch_set_limits(c->b, n_iters, c->stream));
        if ((rc = launch_iterations(c, n_iters))) return rc;
    }
    if (st) return fill_stats(c, st);
    return ALLL_OK;
}

int alll_get_stats(alll_ctx* c, alll_stats* st) {
    if (!c || !st) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    return fill_stats(c, st);
}

int alll_synchronize(alll_ctx* c) {
    if (!c) return fail(ALLL_ERR_INVALID_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ALLL_OK;
}

int alll_verify(alll_ctx* c, int* valid, uint64_t* n_violated) {
    if (!c) return fail(ALLL_ERR_INVALID_ARG, "null context");
    HIP_TRY(hipSetDevice(c->device));
    // every rank evaluates its own shard (the only one laid out for its evaluation); the
    // counts are summed over the ranks
    HIP_TRY(eval_launch(c, c->own_begin, c->own_end, false));
    HIP_TRY(launch_reduce(c->b, 1, c->stream));
    uint64_t count = 0;
    if (c->world > 1) {
        // the mask alll_get_violated_mask returns on sharded runs (clause order: cmask, or the
        // CSR evaluation's own bitmask) refreshed from this evaluation: the own shard's piece,
        // then the other shards' pieces all-gathered
        const size_t words = (size_t)c->tiles_per_rank * TILE_WORDS;
        uint64_t* mask = c->b.cmask ? c->b.cmask : c->b.vmask;
        if (c->b.cmask) HIP_TRY(launch_cmark(c->cv, c->b, words, c->rank, false, c->stream));
        if (c->comm) {
            NCCL_TRY(ncclAllGather(mask + (size_t)c->rank * words, mask, words, ncclUint64, c->comm, c->stream));
        } else {
            int rc = host_exchange(c, ALLL_XCHG_ALLGATHER, mask, words * 8, (size_t)c->rank * words * 8);
            if (rc) return rc;
        }
    }
    if (c->world > 1) {
        if (c->comm) {
            NCCL_TRY(ncclAllReduce(c->b.xcount, c->b.xcount, 1, ncclUint32, ncclSum, c->comm, c->stream));
        } else {
            int rc = host_exchange(c, ALLL_XCHG_ALLREDUCE_SUM_U32, c->b.xcount, 4, 0);
            if (rc) return rc;
        }
        uint32_t x = 0;
        HIP_TRY(hipMemcpyAsync(&x, c->b.xcount, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        count = x;
    }
    int rc = read_state(c);
    if (rc) return rc;
    if (c->world == 1) count = c->h_state->count_out;
    if (valid) *valid = count == 0;
    if (n_violated) *n_violated = count;
    return ALLL_OK;
}

int alll_get_assignment_words(alll_ctx* c, uint32_t* out, uint64_t n_words) {
    if (!c || (!out && c->b.n_words)) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    if (n_words < c->b.n_words) return fail(ALLL_ERR_INVALID_ARG, "need %u words", c->b.n_words);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->b.n_words) HIP_TRY(hipMemcpy(out, c->b.A, c->b.n_words * 4ull, hipMemcpyDeviceToHost));
    return ALLL_OK;
}

int alll_set_assignment_words(alll_ctx* c, const uint32_t* in, uint64_t n_words) {
    if (!c || (!in && c->b.n_words)) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    if (n_words < c->b.n_words) return fail(ALLL_ERR_INVALID_ARG, "need %u words", c->b.n_words);
    HIP_TRY(hipSetDevice(c->device));
    std::vector<uint32_t> w(in, in + c->b.n_words);
    if (!w.empty() && (c->n_vars & 31)) w.back() &= (1u << (c->n_vars & 31)) - 1u;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->b.n_words) HIP_TRY(hipMemcpy(c->b.A, w.data(), c->b.n_words * 4ull, hipMemcpyHostToDevice));
    c->hint_u = ~0ull;  // the next pass's violated count is unknown: no small-set variant
    c->async_pending = false;
    return ALLL_OK;
}

int alll_get_assignment(alll_ctx* c, uint8_t* out, uint64_t n) {
    if (!c || (!out && c->n_vars)) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    if (n < c->n_vars) return fail(ALLL_ERR_INVALID_ARG, "need %u bytes", c->n_vars);
    std::vector<uint32_t> w(c->b.n_words);
    int rc = alll_get_assignment_words(c, w.data(), w.size());
    if (rc) return rc;
    for (uint32_t v = 0; v < c->n_vars; ++v) out[v] = (w[v >> 5] >> (v & 31)) & 1u;
    return ALLL_OK;
}

int alll_set_assignment(alll_ctx* c, const uint8_t* in, uint64_t n) {
    if (!c || (!in && c->n_vars)) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    if (n < c->n_vars) return fail(ALLL_ERR_INVALID_ARG, "need %u bytes", c->n_vars);
    std::vector<uint32_t> w(c->b.n_words, 0u);
    for (uint32_t v = 0; v < c->n_vars; ++v)
        if (in[v]) w[v >> 5] |= 1u << (v & 31);
    return alll_set_assignment_words(c, w.data(), w.size());
}

int alll_get_violated_mask(alll_ctx* c, uint64_t* out, uint64_t n_words) {
    if (!c) return fail(ALLL_ERR_INVALID_ARG, "null context");
    const uint64_t need = (c->m + 63) / 64;
    if (n_words < need || (!out && need)) return fail(ALLL_ERR_INVALID_ARG, "need %llu words", (unsigned long long)need);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->b.cmask && c->world > 1) {  // clause-sharded: the last all-gathered clause-order mask
        if (need) HIP_TRY(hipMemcpy(out, c->b.cmask, need * 8, hipMemcpyDeviceToHost));
        if (c->m & 63) out[need - 1] &= (1ull << (c->m & 63)) - 1ull;
    } else if (!c->perm.empty()) {  // fixed width: device bits are chunk ballots in evaluation order
        std::vector<uint64_t> ev((c->m + CHUNK - 1) / CHUNK * 4);
        HIP_TRY(hipMemcpy(ev.data(), c->b.vmask, ev.size() * 8, hipMemcpyDeviceToHost));
        std::fill(out, out + need, 0ull);
        for (uint64_t p = 0; p < c->m; ++p) {
            const uint64_t w = (p / CHUNK) * 4 + (p & 3), bit = (p % CHUNK) >> 2;
            if ((ev[w] >> bit) & 1ull) out[c->perm[p] >> 6] |= 1ull << (c->perm[p] & 63);
        }
    } else {
        if (need) HIP_TRY(hipMemcpy(out, c->b.vmask, need * 8, hipMemcpyDeviceToHost));
        if (c->m & 63) out[need - 1] &= (1ull << (c->m & 63)) - 1ull;
    }
    return ALLL_OK;
}

int alll_get_mis(alll_ctx* c, uint32_t* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    int rc = read_state(c);
    if (rc) return rc;
    const uint32_t nt = c->b.n_tiles;
    std::vector<uint32_t> cnt(nt);
    if (nt) HIP_TRY(hipMemcpy(cnt.data(), c->b.mis_cnt, nt * 4ull, hipMemcpyDeviceToHost));
    std::vector<uint32_t> all;
    std::vector<uint32_t> buf;
    for (uint32_t t = 0; t < nt; ++t) {
        if (!cnt[t]) continue;
        buf.resize(cnt[t]);
        HIP_TRY(hipMemcpy(buf.data(), c->b.mis + (size_t)t * TILE, cnt[t] * 4ull, hipMemcpyDeviceToHost));
        all.insert(all.end(), buf.begin(), buf.end());
    }
    if (c->h_state->tmis_cnt) {
        buf.resize(c->h_state->tmis_cnt);
        HIP_TRY(hipMemcpy(buf.data(), c->b.tmis, buf.size() * 4ull, hipMemcpyDeviceToHost));
        all.insert(all.end(), buf.begin(), buf.end());
    }
    std::sort(all.begin(), all.end());
    *n_out = all.size();
    if (out) {
        if (cap < all.size()) return fail(ALLL_ERR_INVALID_ARG, "need capacity %zu", all.size());
        std::copy(all.begin(), all.end(), out);
    }
    return ALLL_OK;
}

int alll_bench_eval(alll_ctx* c, int reps, double* avg_ms, uint64_t* n_violated) {
    if (!c || reps < 1) return fail(ALLL_ERR_INVALID_ARG, "bad argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(eval_launch(c, c->own_begin, c->own_end, false));  // warm
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    for (int i = 0; i < reps; ++i) HIP_TRY(eval_launch(c, c->own_begin, c->own_end, false));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    HIP_TRY(hipEventSynchronize(c->ev[1]));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    if (avg_ms) *avg_ms = ms / reps;
    if (n_violated) {
        int valid = 0;
        int rc = alll_verify(c, &valid, n_violated);
        if (rc) return rc;
    }
    return ALLL_OK;
}

int alll_profile(alll_ctx* c, uint64_t n_iters, alll_phase_times* out) {
    if (!c || !out) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    memset(out, 0, sizeof(*out));
    int rc = read_state(c);
    if (rc) return rc;
    if (c->h_state->done == 1) return ALLL_OK;
    if ((rc = write_limits(c, c->h_state->n_iter + n_iters, ~0ull))) return rc;
    double acc[4] = {0, 0, 0, 0};
    for (uint64_t i = 0; i < n_iters; ++i) {
        if (c->b.srr_T) rc = launch_srr_iteration(c, c->ev);
        else if (c->b.rr_T && c->b.fp_ctl) rc = launch_rr_iteration(c, c->ev);
        else rc = enqueue_iteration(c, c->ev, round0_variant(c));
        if (rc) return rc;
        HIP_TRY(hipEventSynchronize(c->ev[4]));
        float t;
        for (int p = 0; p < 4; ++p) {
            HIP_TRY(hipEventElapsedTime(&t, c->ev[p], c->ev[p + 1]));
            acc[p] += t;
        }
    }
    out->iterations = n_iters;
    out->eval_ms = acc[0] / n_iters;
    out->exchange_ms = acc[1] / n_iters;
    out->mis_ms = acc[2] / n_iters;
    out->resample_ms = acc[3] / n_iters;
    out->total_ms = (acc[0] + acc[1] + acc[2] + acc[3]) / n_iters;
    return ALLL_OK;
}

int alll_loop_times(alll_ctx* c, uint64_t first_iter, uint64_t n_iters, alll_phase_times* out) {
    if (!c || !out) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    memset(out, 0, sizeof(*out));
    if (!c->b.ktime) return fail(ALLL_ERR_INVALID_ARG, "created without ALLL_FLAG_KERNEL_TIMING");
    HIP_TRY(hipSetDevice(c->device));
    int rc = read_state(c);
    if (rc) return rc;
    const uint64_t done = c->h_state->n_iter;  // slots of iterations < done are complete
    if (first_iter + n_iters > done) n_iters = done > first_iter ? done - first_iter : 0;
    if (done > TIME_SLOTS && first_iter < done - TIME_SLOTS) {
        const uint64_t lo = done - TIME_SLOTS;
        n_iters = first_iter + n_iters > lo ? first_iter + n_iters - lo : 0;
        first_iter = lo;
    }
    if (n_iters == 0) return ALLL_OK;
    std::vector<unsigned long long> t((size_t)TIME_SLOTS * TIME_FIELDS);
    HIP_TRY(hipMemcpy(t.data(), c->b.ktime, t.size() * 8, hipMemcpyDeviceToHost));
    const double tick_ms = 1.0 / c->wall_khz;
    auto slot = [&](uint64_t i) { return &t[(size_t)(i % TIME_SLOTS) * TIME_FIELDS]; };
    double se = 0, sx = 0, sm = 0, sr = 0, st = 0;
    uint64_t ne = 0, nm = 0, nt = 0;
    for (uint64_t i = first_iter; i < first_iter + n_iters; ++i) {
        const unsigned long long* a = slot(i);
        if (a[0] == ~0ull || a[1] < a[0]) continue;  // not evaluated (converged / gated)
        se += (a[1] - a[0]) * tick_ms; ++ne;
        if (a[2] >= a[1]) sx += (a[2] - a[1]) * tick_ms;
        if (a[3] && a[3] >= a[2]) {
            sm += (a[3] - a[2]) * tick_ms; ++nm;
            // resample + launch gaps: LFMIS end to the next iteration's evaluation start
            const unsigned long long* z = slot(i + 1);
            if (i + 1 < done && z[0] != ~0ull && z[0] >= a[3]) {
                sr += (z[0] - a[3]) * tick_ms;
                st += (z[0] - a[0]) * tick_ms;
                ++nt;
            }
        }
    }
    out->iterations = ne;
    if (ne) { out->eval_ms = se / ne; out->exchange_ms = sx / ne; }
    if (nm) out->mis_ms = sm / nm;
    if (nt) { out->resample_ms = sr / nt; out->total_ms = st / nt; }
    return ALLL_OK;
}

int alll_shard_plan(uint64_t n_clauses, int world, int rank, uint64_t* clause_begin,
                    uint64_t* clause_end, uint64_t* mask_words_per_rank) {
    if (world < 1 || rank < 0 || rank >= world) return fail(ALLL_ERR_INVALID_ARG, "bad rank/world");
    const uint64_t n_tiles = (n_clauses + TILE - 1) / TILE;
    uint64_t tpr = (n_tiles + world - 1) / world;
    if (tpr == 0) tpr = 1;
    const uint64_t tb = std::min<uint64_t>(n_tiles, (uint64_t)rank * tpr);
    const uint64_t te = std::min<uint64_t>(n_tiles, tb + tpr);
    if (clause_begin) *clause_begin = std::min<uint64_t>(n_clauses, tb * TILE);
    if (clause_end) *clause_end = std::min<uint64_t>(n_clauses, te * TILE);
    if (mask_words_per_rank) *mask_words_per_rank = tpr * TILE_WORDS;
    return ALLL_OK;
}

int alll_plan_multi_gpu(uint64_t n_clauses, uint64_t n_literals, uint32_t n_vars, int world,
                        alll_multi_plan* out) {
    if (!out || world < 1) return fail(ALLL_ERR_INVALID_ARG, "bad arguments");
    memset(out, 0, sizeof(*out));
    const double m = (double)n_clauses, G = (double)world;
    const double k_avg = n_clauses ? (double)n_literals / m : 0.0;
    // evaluation: the literal stream + assignment + bitmask bytes (alll_eval_bytes) at the rate
    // the evaluation kernel reaches on one MI355X: 4.3 TB/s while the stream fits the 256 MB
    // Infinity Cache (M: 121.6 MB in 28 us), 3.3 TB/s beyond it (C4: 1,556 MB in 467 us)
    const double bytes = 4.0 * (double)n_literals + (double)n_vars / 8.0 + m / 8.0;
    const double eval_us = bytes / (bytes <= 200e6 ? 4.3e6 : 3.3e6);
    // violated clauses: a uniform assignment violates a k-clause with probability 2^-k
    const double u = m * std::pow(2.0, -k_avg);
    out->eval_us_1gpu = eval_us;
    out->eval_saved_us = eval_us * (1.0 - 1.0 / G);
    out->violated_est = u;
    if (world > 1) {
        // own shard's marking (k_cmark: 14.4 us for 0.75M violated clauses; k_cpack: 7.4 us per
        // 10M clauses), the in-graph all-gather (15 us latency + m/8 bytes at ~300 GB/s), the
        // other shards' violated clauses collected (4.5 us + a 64-byte line each at ~6 TB/s),
        // the round-0 scatter and reduce the exchange path runs unfused (2.6 + 4.6 us)
        const double mark = 14.4 * (u / G) / 0.75e6 + 7.4 * (m / G) / 10e6;
        const double gather = 15.0 + (m / 8.0) / 300e3;
        const double collect = 4.5 + u * (G - 1.0) / G * 64.0 / 6e6;
        out->exchange_us = mark + gather + collect + 2.6 + 4.6;
    }
    out->plan = world > 1 && out->eval_saved_us > out->exchange_us ? ALLL_PLAN_SHARD : ALLL_PLAN_REPLICATE;
    return ALLL_OK;
}

uint64_t alll_eval_bytes(alll_ctx* c) {
    // B_eval = 4 L + 4 (m+1) [CSR offsets only] + ceil(n/8) + ceil(m/8),
    // for this rank's clause shard.
    if (!c) return 0;
    const uint64_t cb = (uint64_t)c->own_begin * TILE;
    const uint64_t ce = std::min<uint64_t>(c->m, (uint64_t)c->own_end * TILE);
    const uint64_t ms = ce > cb ? ce - cb : 0;
    const uint64_t lits = c->cv.k ? ms * c->cv.k : (c->m ? (c->n_lits * ms) / c->m : 0);
    return 4 * lits + (c->cv.k ? 0 : 4 * (ms + 1)) + (c->n_vars + 7) / 8 + (ms + 7) / 8;
}

int alll_layout(alll_ctx* c) { return c ? (int)c->cv.k : -1; }

int alll_rr_pass_log(alll_ctx* c, uint32_t* out, uint32_t n_words) {
    if (!c || (!out && n_words)) return fail(ALLL_ERR_INVALID_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint32_t have = c->b.fp_log ? FP_LOG_WORDS : 0;
    const uint32_t nw = std::min(n_words, have);
    if (nw) HIP_TRY(hipMemcpy(out, c->b.fp_log, nw * 4ull, hipMemcpyDeviceToHost));
    for (uint32_t i = nw; i < n_words; ++i) out[i] = 0;
    return (int)nw;
}

int64_t alll_rr_barrier_timeouts(alll_ctx* c) {
    if (!c) return -1;
    if (!c->b.fp_ctl) return 0;
    if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    RRFpCtl ctl;
    if (hipMemcpy(&ctl, c->b.fp_ctl, sizeof ctl, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return ctl.rw_timeouts;
}

int alll_comm_size(alll_ctx* c) {
    if (!c) return -1;
    if (!c->comm) return c->world;
    int n = 0;
    if (ncclCommCount(c->comm, &n) != ncclSuccess) return -1;
    return n;
}

const char* alll_eval_kernel(alll_ctx* c) { return c ? c->eval_name.c_str() : ""; }

int alll_uses_graphs(alll_ctx* c, const char** why) {
    if (!c) return -1;
    if (why) *why = c->graph_note.c_str();
    return c->use_graph ? 1 : 0;
}

}  // extern "C"
