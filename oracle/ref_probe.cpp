// ref_probe.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A driver around the reference's OWN code, compiled from the sources where they lie
// under /root/reference (see oracle/Makefile; nothing is copied into this repo).  It
// produces the golden vectors that pin the oracle (tests/golden/) and times the
// reference's -p OpenMP path for bench.py's cpu_baseline leg.
//
//   trace <cnf> <T> <max_iters> <rd_seed> <out.bin>   per-iteration (A_i, U_i, M_i, dres)
//   solve <cnf> <T> <rd_seed>                          real SATInstance::solve, prints stats
//   bench <cnf> <T> <budget_s> <eval_reps>             eval-phase and full-iteration timing
//   bench-gen <n> <m> <k> <kind> <gen_seed> <T> <budget_s> <eval_reps>   same, generated instance
//   cnf   <cnf>                                        cnf_header_read/cnf_data_read output
//   stream <cnf> <batch> <rd_seed> <out.bin>           streaming solve (SATInstance.h:70-153), T=1:
//                                                      per-iteration (A_i, U_i in yield order, M_i in
//                                                      pick order, per-batch MIS sizes), final stats,
//                                                      and the real solve(getEnumeratedClause, ...)
//
// The load/encode/chunk sequence restates example/main.cpp:133-181 (main.cpp itself needs
// Boost.program_options, absent here).  std::random_device::_M_getval is interposed by a
// seeded LCG so VariablesArray init (VariablesArray.h:24) and every resample_clauses
// engine seed (SATInstance.h:346) are reproducible.
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>
#include <set>
#include <fstream>
#include <iostream>
#include <utility>
#include <omp.h>

static unsigned long long g_rd_state = 1;
unsigned int std::random_device::_M_getval() {
    g_rd_state = g_rd_state * 6364136223846793005ULL + 1442695040888963407ULL;
    return (unsigned int)(g_rd_state >> 33);
}

extern "C" {
#include "alll_oracle.h"
}

#define private public
#include "SATInstance.h"
#undef private
#include "cnf_io/cnf_io.h"

typedef uint32_t UINT_T;
typedef SATInstance<UINT_T>::ClauseArray ClauseArray;

struct Loaded {
    int v_num = 0, c_num = 0, l_num = 0;
    std::vector<ClauseArray*>* clauses = nullptr;
    std::vector<Clause<UINT_T>*> all;  // clause index -> Clause*
    std::unordered_map<const Clause<UINT_T>*, uint32_t> index;
};

// example/main.cpp:133-178
static Loaded load(const std::string& path, int n_threads) {
    Loaded L;
    if (cnf_header_read(path, &L.v_num, &L.c_num, &L.l_num)) {
        fprintf(stderr, "header read failed\n");
        exit(1);
    }
    int* l_c_num = new int[L.c_num + 1];
    int* l_val = new int[L.l_num + 1];
    cnf_data_read(path, L.v_num, L.c_num, L.l_num, l_c_num, l_val);
    int chunk_size = ceil(L.c_num / (double)n_threads);
    L.clauses = new std::vector<ClauseArray*>();
    for (int t = 0; t < n_threads; t++) L.clauses->push_back(new ClauseArray());
    int c, l, l_c;
    l = 0;
    unsigned short int t = 0;
    for (c = 0; c < L.c_num; c++) {
        auto literals = new std::vector<UINT_T>;
        for (l_c = 0; l_c < l_c_num[c]; l_c++) {
            literals->push_back((0 < l_val[l]) ? (2 * l_val[l]) - 2 : ((-2) * l_val[l]) - 1);
            l += 1;
        }
        if (c > (t + 1) * chunk_size) t += 1;
        auto cl = new Clause<UINT_T>(literals, t);
        L.clauses->at(t)->push_back(cl);
        L.all.push_back(cl);
        L.index[cl] = (uint32_t)c;
    }
    delete[] l_c_num;
    delete[] l_val;
    return L;
}

// Same chunking as load(), clauses from the oracle's generator (shared spec with the product).
static Loaded load_gen(uint32_t n, uint64_t m, uint32_t k, int kind, uint64_t seed, int n_threads) {
    Loaded L;
    L.v_num = (int)n;
    L.c_num = (int)m;
    L.l_num = (int)(m * k);
    std::vector<uint32_t> lits((size_t)m * k);
    orc_generate_ksat(seed, n, m, k, kind, 0, m, lits.data());
    int chunk_size = ceil(L.c_num / (double)n_threads);
    L.clauses = new std::vector<ClauseArray*>();
    for (int t = 0; t < n_threads; t++) L.clauses->push_back(new ClauseArray());
    unsigned short int t = 0;
    for (int c = 0; c < L.c_num; c++) {
        auto literals = new std::vector<UINT_T>(lits.begin() + (size_t)c * k, lits.begin() + (size_t)(c + 1) * k);
        if (c > (t + 1) * chunk_size) t += 1;
        L.clauses->at(t)->push_back(new Clause<UINT_T>(literals, t));
    }
    return L;
}

static void wr(FILE* f, const void* p, size_t n) { fwrite(p, 1, n, f); }
static void wr64(FILE* f, uint64_t x) { wr(f, &x, 8); }

// The P1 eval loop of parallel_solve (SATInstance.h:264-280), same pragma.
static std::vector<ClauseArray*>* eval_chunks(SATInstance<UINT_T>* S, std::vector<ClauseArray*>* clauses,
                                             int n_threads) {
    auto unsat_clauses = new std::vector<ClauseArray*>;
    for (int t = 0; t < n_threads; t++) unsat_clauses->push_back(new ClauseArray());
    auto var_arr = S->var_arr;
#pragma omp parallel for schedule(static, 1) default(none) shared(clauses, unsat_clauses, n_threads, var_arr)
    for (int t = 0; t < n_threads; t++) {
        for (auto clause = clauses->at(t)->begin(); clause != clauses->at(t)->end(); ++clause) {
            if ((*clause)->is_not_satisfied(var_arr->vars)) unsat_clauses->at(t)->push_back(*clause);
        }
    }
    return unsat_clauses;
}

static int cmd_trace(int argc, char** argv) {
    std::string path = argv[2];
    int T = atoi(argv[3]);
    uint64_t max_iters = strtoull(argv[4], 0, 10);
    g_rd_state = strtoull(argv[5], 0, 10);
    FILE* f = fopen(argv[6], "wb");
    Loaded L = load(path, T);
    auto S = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(L.v_num), T);
    for (auto c : *L.clauses) S->n_clauses += c->size();  // SATInstance.h:61-63
    omp_set_num_threads(T);
    wr(f, "ALRT", 4);
    uint32_t hdr[2] = {(uint32_t)L.v_num, (uint32_t)T};
    wr(f, hdr, 8);
    wr64(f, (uint64_t)L.c_num);
    // parallel_solve body (SATInstance.h:254-317) with the reference's own MIS / resample.
    auto statistics = new Statistics;
    for (int i = 0; i < T; i++) statistics->n_thread_resamples.push_back(0);
    auto mis = new ClauseArray();
    uint64_t it = 0;
    std::vector<uint8_t> A(L.v_num);
    while (true) {
        statistics->n_iterations += 1;
        for (int v = 0; v < L.v_num; ++v) A[v] = S->var_arr->vars[v] ? 1 : 0;
        auto unsat = eval_chunks(S, L.clauses, T);
        std::vector<uint32_t> U;
        for (auto s : *unsat)
            for (auto c : *s) U.push_back(L.index[c]);
        wr64(f, statistics->n_iterations);
        wr(f, A.data(), A.size());
        wr64(f, U.size());
        wr(f, U.data(), U.size() * 4);
        if (S->check_if_noUNSAT(unsat)) {
            wr64(f, 0);
            wr64(f, 0);
            break;
        }
        if (max_iters && statistics->n_iterations >= max_iters) {
            // capped: record the MIS the reference would pick, but do not resample
            S->populate_mis_parallel(unsat, mis, false);
            wr64(f, mis->size());
            for (auto c : *mis) { uint32_t x = L.index[c]; wr(f, &x, 4); }
            wr64(f, 0);
            mis->clear();
            break;
        }
        S->populate_mis_parallel(unsat, mis, false);
        statistics->avg_mis_size += mis->size();
        wr64(f, mis->size());
        for (auto c : *mis) { uint32_t x = L.index[c]; wr(f, &x, 4); }
        ull before = 0;
        for (auto x : statistics->n_thread_resamples) before += x;
        S->resample_clauses(mis, statistics);
        ull after = 0;
        for (auto x : statistics->n_thread_resamples) after += x;
        wr64(f, after - before);
        mis->clear();
        ++it;
    }
    for (int t = 0; t < T; t++) statistics->n_resamples += statistics->n_thread_resamples.at(t);
    statistics->avg_mis_size = (ull)(statistics->avg_mis_size / statistics->n_iterations);
    wr64(f, ~0ull);
    wr64(f, statistics->n_iterations);
    wr64(f, statistics->n_resamples);
    wr64(f, statistics->avg_mis_size);
    for (int v = 0; v < L.v_num; ++v) A[v] = S->var_arr->vars[v] ? 1 : 0;
    wr(f, A.data(), A.size());
    fclose(f);
    return 0;
}

static int cmd_solve(int argc, char** argv) {
    std::string path = argv[2];
    int T = atoi(argv[3]);
    g_rd_state = strtoull(argv[4], 0, 10);
    Loaded L = load(path, T);
    auto S = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(L.v_num), T);
    Statistics* st = S->solve(L.clauses);
    bool ok = S->verify_validity(L.clauses);
    printf("{\"n_iterations\": %llu, \"n_resamples\": %llu, \"avg_mis_size\": %llu, \"valid\": %d, \"assignment\": \"",
           st->n_iterations, st->n_resamples, st->avg_mis_size, ok ? 1 : 0);
    for (int v = 0; v < L.v_num; ++v) putchar(S->var_arr->vars[v] ? '1' : '0');
    printf("\"}\n");
    return 0;
}

static int cmd_cnf(int argc, char** argv) {
    std::string path = argv[2];
    int v = 0, c = 0, l = 0;
    if (cnf_header_read(path, &v, &c, &l)) { printf("{\"error\": 1}\n"); return 0; }
    std::vector<int> lc(c + 1, -1), lv(l + 1, 0);
    cnf_data_read(path, v, c, l, lc.data(), lv.data());
    printf("{\"v_num\": %d, \"c_num\": %d, \"l_num\": %d, \"l_c_num\": [", v, c, l);
    for (int i = 0; i < c; ++i) printf("%s%d", i ? ", " : "", lc[i]);
    printf("], \"l_val\": [");
    for (int i = 0; i < l; ++i) printf("%s%d", i ? ", " : "", lv[i]);
    printf("]}\n");
    return 0;
}

// CPU baseline: the reference's -p path (P1 eval with its OpenMP pragma, populate_mis_parallel,
// resample_clauses) on the node's host cores.
static int bench_loaded(Loaded& L, int T, double budget, int eval_reps, double load_s) {
    auto S = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(L.v_num), T);
    omp_set_num_threads(T);
    // (a) eval phase only, best of eval_reps
    double best = 0;
    for (int r = 0; r < eval_reps; ++r) {
        auto a = std::chrono::steady_clock::now();
        auto u = eval_chunks(S, L.clauses, T);
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
        if (r == 0 || dt < best) best = dt;
        for (auto s : *u) delete s;
        delete u;
    }
    // (b) full iterations within the wall budget
    auto statistics = new Statistics;
    for (int i = 0; i < T; i++) statistics->n_thread_resamples.push_back(0);
    auto mis = new ClauseArray();
    uint64_t iters = 0;
    bool solved = false;
    auto b0 = std::chrono::steady_clock::now();
    double el = 0;
    while (el < budget) {
        statistics->n_iterations += 1;
        auto unsat = eval_chunks(S, L.clauses, T);
        if (S->check_if_noUNSAT(unsat)) { solved = true; break; }
        S->populate_mis_parallel(unsat, mis, false);
        statistics->avg_mis_size += mis->size();
        S->resample_clauses(mis, statistics);
        mis->clear();
        ++iters;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count();
    }
    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count();
    printf("{\"threads\": %d, \"n_vars\": %d, \"n_clauses\": %d, \"load_s\": %.6f, \"eval_best_s\": %.6f, "
           "\"eval_clause_evals_per_s\": %.6e, \"iters\": %llu, \"iters_s\": %.6f, \"solved\": %d}\n",
           T, L.v_num, L.c_num, load_s, best, best > 0 ? L.c_num / best : 0.0, (unsigned long long)iters, el,
           solved ? 1 : 0);
    return 0;
}

// CPU baseline: the reference's -p path (P1 eval with its OpenMP pragma, populate_mis_parallel,
// resample_clauses) on the node's host cores.
static int cmd_bench(int argc, char** argv) {
    std::string path = argv[2];
    int T = atoi(argv[3]);
    g_rd_state = 12345;
    auto t0 = std::chrono::steady_clock::now();
    Loaded L = load(path, T);
    double load_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return bench_loaded(L, T, atof(argv[4]), atoi(argv[5]), load_s);
}

//   bench-gen <n> <m> <k> <kind> <gen_seed> <T> <budget_s> <eval_reps>
static int cmd_bench_gen(int argc, char** argv) {
    uint32_t n = (uint32_t)strtoul(argv[2], 0, 10);
    uint64_t m = strtoull(argv[3], 0, 10);
    uint32_t k = (uint32_t)strtoul(argv[4], 0, 10);
    int kind = atoi(argv[5]);
    uint64_t seed = strtoull(argv[6], 0, 10);
    int T = atoi(argv[7]);
    g_rd_state = 12345;
    auto t0 = std::chrono::steady_clock::now();
    Loaded L = load_gen(n, m, k, kind, seed, T);
    double load_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return bench_loaded(L, T, atof(argv[8]), atoi(argv[9]), load_s);
}

// ---- streaming solve (SATInstance.h:70-153) with T = 1 -------------------------------------
// The clause callback returns a fresh copy of clause idx (the solver deletes what it yields);
// every copy is registered so yielded clauses can be mapped back to their index.
static Loaded* g_stream = nullptr;
static std::unordered_map<const Clause<UINT_T>*, uint32_t> g_copy_index;
static Clause<UINT_T>* stream_clause(UINT_T idx, unsigned short t_id) {
    if (!g_stream || idx >= (UINT_T)g_stream->all.size()) return nullptr;
    auto cl = new Clause<UINT_T>(new std::vector<UINT_T>(*g_stream->all[idx]->literals), t_id);
    g_copy_index[cl] = (uint32_t)idx;
    return cl;
}

static int cmd_stream(int argc, char** argv) {
    std::string path = argv[2];
    const UINT_T batch = (UINT_T)strtoul(argv[3], 0, 10);
    const unsigned long long rd_seed = strtoull(argv[4], 0, 10);
    FILE* f = fopen(argv[5], "wb");
    Loaded L = load(path, 1);
    g_stream = &L;
    const UINT_T n_clauses = (UINT_T)L.c_num;
    wr(f, "ALRS", 4);
    uint32_t hdr[2] = {(uint32_t)L.v_num, (uint32_t)batch};
    wr(f, hdr, 8);
    wr64(f, (uint64_t)L.c_num);
    // (1) the loop of SATInstance::solve(getEnumeratedClause, n_clauses, batch_size) with T = 1,
    //     the reference's own ClauseGenerator, populate_mis_parallel and resample_clauses,
    //     recording each iteration
    g_rd_state = rd_seed;
    auto S = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(L.v_num), 1);
    omp_set_num_threads(1);
    auto statistics = new Statistics;
    statistics->n_thread_resamples.push_back(0);
    S->n_clauses = n_clauses;
    auto gen = new ClauseGenerator<UINT_T>(stream_clause, 0, n_clauses, 0, batch);
    std::vector<uint8_t> A(L.v_num);
    bool solved = false;
    while (!solved) {
        solved = true;
        statistics->n_iterations += 1;
        for (int v = 0; v < L.v_num; ++v) A[v] = S->var_arr->vars[v] ? 1 : 0;
        auto mis = new ClauseArray();
        std::vector<uint32_t> U, M, cum;
        bool finished = false;
        ull dres = 0;
        while (!finished) {
            auto clauses = new std::vector<ClauseArray*>;
            clauses->push_back(gen->yieldRandomUNSATClauseBatch(S->var_arr->vars));
            for (auto c : *clauses->at(0)) U.push_back(g_copy_index[c]);
            finished = gen->has_finished_yielding();
            // parallel_solve(clauses, mis, stream = true, resample = finished), SATInstance.h:217-320
            auto result = new Statistics;
            result->n_thread_resamples.push_back(0);
            result->n_iterations = 1;
            S->populate_mis_parallel(clauses, mis, true);
            result->avg_mis_size += mis->size();
            cum.push_back((uint32_t)mis->size());
            if (finished) {
                for (auto c : *mis) M.push_back(g_copy_index[c]);
                S->resample_clauses(mis, result);
                mis->clear();  // (the reference also frees the clauses; ids recorded above)
            }
            result->n_resamples += result->n_thread_resamples.at(0);
            statistics->avg_mis_size += result->avg_mis_size;
            statistics->n_resamples += result->n_resamples;
            statistics->n_thread_resamples.at(0) += result->n_thread_resamples.at(0);
            dres += result->n_resamples;
            delete result;
        }
        delete mis;
        for (UINT_T k = 0; k < n_clauses; k++) {  // SATInstance.h:130-147
            if (!solved) continue;
            auto c = gen->yieldNextClause();
            if (c->is_not_satisfied(S->var_arr->vars)) solved = false;
            delete c->literals;
            delete c;
        }
        wr64(f, statistics->n_iterations);
        wr(f, A.data(), A.size());
        wr64(f, U.size());
        wr(f, U.data(), U.size() * 4);
        wr64(f, M.size());
        wr(f, M.data(), M.size() * 4);
        wr64(f, cum.size());
        wr(f, cum.data(), cum.size() * 4);
        wr64(f, dres);
        if (statistics->n_iterations >= 100000) break;  // (probe safety cap)
    }
    statistics->avg_mis_size /= statistics->n_iterations;
    wr64(f, ~0ull);
    wr64(f, statistics->n_iterations);
    wr64(f, statistics->n_resamples);
    wr64(f, statistics->avg_mis_size);
    for (int v = 0; v < L.v_num; ++v) A[v] = S->var_arr->vars[v] ? 1 : 0;
    wr(f, A.data(), A.size());
    // (2) the real SATInstance::solve(getEnumeratedClause, ...) with the same interposed RNG
    g_rd_state = rd_seed;
    auto S2 = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(L.v_num), 1);
    std::streambuf* saved = std::cout.rdbuf();
    std::ofstream devnull("/dev/null");
    std::cout.rdbuf(devnull.rdbuf());  // it prints "New solve iteration..." every iteration
    Statistics* st = S2->solve(stream_clause, (ull)n_clauses, batch);
    std::cout.rdbuf(saved);
    wr64(f, st->n_iterations);
    wr64(f, st->n_resamples);
    wr64(f, st->avg_mis_size);
    for (int v = 0; v < L.v_num; ++v) A[v] = S2->var_arr->vars[v] ? 1 : 0;
    wr(f, A.data(), A.size());
    fclose(f);
    return 0;
}

// ---- streaming solve (SATInstance.h:70-153) with T > 1 threads ------------------------------
// The loop of SATInstance::solve(getEnumeratedClause, n_clauses, batch_size) with the reference's
// own ClauseGenerators (:74-86), populate_mis_parallel and resample_clauses, recording per
// iteration A, every generator's state {n_yielded, finished, c}, per batch step the violated list
// of every generator (yield order) and the MIS size after the step, then the MIS (pick order).
// Two parts are restated: (1) the batches are requested generator by generator on this thread
// (the reference asks all generators at once, :105-108; they are independent, so the lists are
// the same, and the callback's index map needs no lock); (2) the end-of-iteration check
// (:129-147) shares one `solved` flag between T threads, so where each thread stops is a race in
// the reference: it is run here in lock step (step k yields clause k of every generator with
// k < n_t; the steps stop after the first that finds a violated clause), the schedule
// oracle/alll_oracle.c restates.  The real solve() is not run for T > 1: its check is racy.
//   stream-rr <cnf> <batch> <T> <rd_seed> <out.bin>
static int cmd_stream_rr(int argc, char** argv) {
    std::string path = argv[2];
    const UINT_T batch = (UINT_T)strtoul(argv[3], 0, 10);
    const int T = atoi(argv[4]);
    const unsigned long long rd_seed = strtoull(argv[5], 0, 10);
    FILE* f = fopen(argv[6], "wb");
    Loaded L = load(path, 1);
    g_stream = &L;
    const UINT_T n_clauses = (UINT_T)L.c_num;
    wr(f, "ALRQ", 4);
    uint32_t hdr[4] = {(uint32_t)L.v_num, (uint32_t)batch, (uint32_t)T, 0u};
    wr(f, hdr, 16);
    wr64(f, (uint64_t)L.c_num);
    g_rd_state = rd_seed;
    auto S = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(L.v_num), T);
    omp_set_num_threads(T);
    auto statistics = new Statistics;
    for (int t = 0; t < T; t++) statistics->n_thread_resamples.push_back(0);
    S->n_clauses = n_clauses;
    // SATInstance.h:74-86
    UINT_T t_n_clauses = (UINT_T)n_clauses / T;
    std::vector<ClauseGenerator<UINT_T>*> gens;
    for (int t = 0; t < T; t++) {
        UINT_T offset = (UINT_T)t * t_n_clauses;
        if (t == T - 1) t_n_clauses = n_clauses - offset;
        gens.push_back(new ClauseGenerator<UINT_T>(stream_clause, (unsigned short)t, t_n_clauses, offset, batch));
    }
    auto wr_gens = [&]() {
        for (auto g : gens) {
            wr64(f, (uint64_t)g->n_yielded_clauses);
            wr64(f, g->finished_yielding ? 1ull : 0ull);
            wr64(f, (uint64_t)g->c);
        }
    };
    std::vector<uint8_t> A(L.v_num);
    bool solved = false;
    while (!solved) {
        solved = true;
        statistics->n_iterations += 1;
        for (int v = 0; v < L.v_num; ++v) A[v] = S->var_arr->vars[v] ? 1 : 0;
        wr64(f, statistics->n_iterations);
        wr(f, A.data(), A.size());
        wr_gens();
        auto mis = new ClauseArray();
        std::vector<uint32_t> M;
        std::vector<std::vector<uint32_t>> step_lists;  // T lists per step
        std::vector<uint64_t> cum;
        bool finished = false;
        ull dres = 0;
        while (!finished) {
            auto clauses = new std::vector<ClauseArray*>;
            for (int t = 0; t < T; t++) clauses->push_back(gens[t]->yieldRandomUNSATClauseBatch(S->var_arr->vars));
            for (int t = 0; t < T; t++) {
                std::vector<uint32_t> u;
                for (auto c : *clauses->at(t)) u.push_back(g_copy_index[c]);
                step_lists.push_back(u);
            }
            finished = true;
            for (int t = 0; t < T; t++)
                if (!gens[t]->has_finished_yielding()) { finished = false; break; }
            // parallel_solve(clauses, mis, stream = true, resample = finished), SATInstance.h:217-320
            auto result = new Statistics;
            for (int t = 0; t < T; t++) result->n_thread_resamples.push_back(0);
            result->n_iterations = 1;
            S->populate_mis_parallel(clauses, mis, true);
            result->avg_mis_size += mis->size();
            cum.push_back(mis->size());
            if (finished) {
                for (auto c : *mis) M.push_back(g_copy_index[c]);
                S->resample_clauses(mis, result);
                mis->clear();  // (the reference also frees the clauses; ids recorded above)
            }
            for (int t = 0; t < T; t++) result->n_resamples += result->n_thread_resamples.at(t);
            statistics->avg_mis_size += result->avg_mis_size;
            statistics->n_resamples += result->n_resamples;
            dres += result->n_resamples;
            delete result;
            if (step_lists.size() > 4000000) { fprintf(stderr, "probe step cap\n"); return 1; }
        }
        delete mis;
        wr64(f, cum.size());
        for (size_t s = 0; s < cum.size(); ++s) {
            for (int t = 0; t < T; t++) {
                const auto& u = step_lists[s * T + t];
                wr64(f, u.size());
                wr(f, u.data(), u.size() * 4);
            }
            wr64(f, cum[s]);
        }
        wr64(f, M.size());
        wr(f, M.data(), M.size() * 4);
        wr64(f, dres);
        // check (SATInstance.h:129-147) in lock step
        uint64_t maxn = 0;
        for (auto g : gens) maxn = std::max<uint64_t>(maxn, g->n_clauses);
        for (uint64_t k = 0; k < maxn && solved; ++k) {
            bool found = false;
            for (int t = 0; t < T; t++) {
                if (k >= (uint64_t)gens[t]->n_clauses) continue;
                auto c = gens[t]->yieldNextClause();
                if (c->is_not_satisfied(S->var_arr->vars)) found = true;
                delete c->literals;
                delete c;
            }
            if (found) solved = false;
        }
        wr64(f, solved ? 1ull : 0ull);
        if (statistics->n_iterations >= 2000) break;  // (probe safety cap)
    }
    statistics->avg_mis_size /= statistics->n_iterations;
    wr64(f, ~0ull);
    wr64(f, statistics->n_iterations);
    wr64(f, statistics->n_resamples);
    wr64(f, statistics->avg_mis_size);
    for (int v = 0; v < L.v_num; ++v) A[v] = S->var_arr->vars[v] ? 1 : 0;
    wr(f, A.data(), A.size());
    wr_gens();
    fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ref_probe trace|solve|bench|cnf ...\n");
        return 2;
    }
    std::string cmd = argv[1];
    if (cmd == "trace" && argc >= 7) return cmd_trace(argc, argv);
    if (cmd == "solve" && argc >= 5) return cmd_solve(argc, argv);
    if (cmd == "bench" && argc >= 6) return cmd_bench(argc, argv);
    if (cmd == "bench-gen" && argc >= 10) return cmd_bench_gen(argc, argv);
    if (cmd == "cnf") return cmd_cnf(argc, argv);
    if (cmd == "stream" && argc >= 6) return cmd_stream(argc, argv);
    if (cmd == "stream-rr" && argc >= 7) return cmd_stream_rr(argc, argv);
    fprintf(stderr, "bad arguments\n");
    return 2;
}
