// SATInstance.h -- compatibility header: the reference's public API
// (library/include/SATInstance.h:25-203: both solve overloads, verify_validity, writeDIMACS)
// over the MI355X solver's C-ABI
// (include/alll.h).  Existing call sites (example/main.cpp) compile unchanged; the device,
// seed and iteration cap are additive settings (env ALLL_DEVICE, ALLL_SEED, ALLL_MAX_ITERS).
#ifndef ALLL_COMPAT_SATINSTANCE_H
#define ALLL_COMPAT_SATINSTANCE_H

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include <omp.h>  // main.cpp calls omp_get_num_procs() through this header

#include "Clause.h"
#include "RandomBoolGenerator.h"
#include "VariablesArray.h"
#include "alll.h"

using namespace std;

typedef struct Statistics {
    ull n_iterations = 0;
    ull n_resamples = 0;
    ull avg_mis_size = 0;
    vector<ull> n_thread_resamples;
} Statistics;

template <typename T>
class SATInstance {
   public:
    using ClauseArray = typename Clause<T>::ClauseArray;

    T n_vars;
    ull n_clauses = 0;
    VariablesArray<T>* var_arr;

    SATInstance(VariablesArray<T>* va, int n_threads) : var_arr(va), n_threads_(n_threads) {
        n_vars = va->n_vars;
    }

    // Moser-Tardos resample loop on the GPU; starts from var_arr->vars and writes the final
    // assignment back into it.  Throws std::runtime_error on device / input errors; a cap
    // from ALLL_MAX_ITERS that is reached returns the statistics (verify_validity is false).
    Statistics* solve(vector<ClauseArray*>* clauses) {
        for (auto c : *clauses) n_clauses += c->size();
        vector<uint64_t> offs(1, 0);
        vector<uint32_t> lits;
        for (auto chunk : *clauses)
            for (auto cl : *chunk) {
                for (auto l : *cl->literals) lits.push_back((uint32_t)l);
                offs.push_back(lits.size());
            }
        // n_threads > 1: the MIS is the reference's round robin over these chunks
        // (SATInstance.h:270-276, 414-447), one chunk per thread
        vector<uint64_t> starts;
        if (n_threads_ > 1) {
            if (clauses->size() != (size_t)n_threads_)
                throw std::runtime_error("alll: n_threads clause chunks expected");
            starts.push_back(0);
            for (auto chunk : *clauses) starts.push_back(starts.back() + chunk->size());
        }
        return run_solver(offs, lits, 0, starts.empty() ? nullptr : starts.data());
    }

    // Streaming solve (reference SATInstance.h:70-153): clauses come from a callback by index.
    // With 288 GB of HBM the instance is materialised once (each index with the t_id of the
    // generator whose range holds it, SATInstance.h:74-86) and the GPU runs the streaming
    // semantics of n_threads generators (alll_options.stream_batch): one thread's MIS follows the
    // generator's yield order, T > 1 threads' MIS is the per-batch round robin over the T
    // generators.  A batch size of 0 is taken as 1 (the reference's generators never finish).
    // T > 1 throws std::runtime_error where the reference would not return (alll.h).
    Statistics* solve(Clause<T>* (*getEnumeratedClause)(T, unsigned short int), ull n_clauses, T batch_size) {
        this->n_clauses = n_clauses;
        vector<uint64_t> offs(1, 0);
        vector<uint32_t> lits;
        const int nt = n_threads_ > 0 ? n_threads_ : 1;
        const ull per = n_clauses / (ull)nt;  // (T t_n_clauses, SATInstance.h:74; the last takes the rest)
        for (ull i = 0; i < n_clauses; ++i) {
            const unsigned short t = (unsigned short)(per ? std::min<ull>(i / per, (ull)nt - 1) : (ull)nt - 1);
            Clause<T>* cl = getEnumeratedClause((T)i, t);
            if (!cl) throw std::runtime_error("alll: clause generator returned nullptr");
            for (auto l : *cl->literals) lits.push_back((uint32_t)l);
            offs.push_back(lits.size());
            delete cl->literals;
            delete cl;
        }
        return run_solver(offs, lits, batch_size > 0 ? (uint64_t)batch_size : 1);
    }

    // DIMACS export of a generated instance (reference SATInstance.h:175-203, same layout).
    void writeDIMACS(Clause<T>* (*getEnumeratedClause)(T, unsigned short int), ull n_clauses, ofstream* out_f) {
        this->n_clauses = n_clauses;
        *out_f << "p cnf " << n_vars << " " << n_clauses << endl;
        for (ull i = 0; i < n_clauses; i++) {
            Clause<T>* clause = getEnumeratedClause((T)i, 0);
            if (!clause) throw std::runtime_error("alll: clause generator returned nullptr");
            for (auto& l : *(clause->literals)) {
                if (l & 1) *out_f << " " << to_string(-((intmax_t)(l >> 1)) - 1);
                else *out_f << " " << to_string((l >> 1) + 1);
            }
            *out_f << " 0" << endl;
            delete clause->literals;
            delete clause;
            if (i % 1000 == 0) out_f->flush();
        }
        out_f->flush();
    }

    // Host check over var_arr->vars, like the reference.
    bool verify_validity(vector<ClauseArray*>* clauses) const {
        for (auto chunk : *clauses)
            for (auto cl : *chunk)
                if (cl->is_not_satisfied(var_arr->vars)) return false;
        return true;
    }

   private:
    int n_threads_{};

    Statistics* run_solver(const vector<uint64_t>& offs, const vector<uint32_t>& lits, uint64_t stream_batch,
                           const uint64_t* set_starts = nullptr) {
        alll_problem p{(uint32_t)n_vars, 0, offs.size() - 1, offs.data(), lits.data()};
        alll_options o;
        alll_default_options(&o);
        o.seed = alll_compat::env_u64("ALLL_SEED", 1);
        o.max_iters = alll_compat::env_u64("ALLL_MAX_ITERS", 0);
        o.device = (int32_t)alll_compat::env_u64("ALLL_DEVICE", (uint64_t)-1);
        o.n_threads = n_threads_ > 0 ? n_threads_ : 1;
        o.stream_batch = stream_batch;
        o.set_starts = set_starts;
        // ALLL_MIS=lfmis: keep the one-set MIS for n_threads > 1 (faster, a different valid MIS)
        if (const char* e = std::getenv("ALLL_MIS"))
            if (std::string(e) == "lfmis") o.flags |= ALLL_FLAG_LFMIS;
        // ALLL_REFERENCE_RNG=<state>: the reference's own random stream; the
        // context's fill draws the same first value as VariablesArray did, so the resample rounds
        // take the stand-in's next values, as the reference's do (one VariablesArray and one solve
        // per process, as in example/main.cpp)
        if (const char* e = std::getenv("ALLL_REFERENCE_RNG"))
            if (*e) {
                o.flags |= ALLL_FLAG_REFERENCE_RNG;
                o.seed = alll_compat::env_u64("ALLL_REFERENCE_RNG", 0);
            }
        alll_ctx* ctx = nullptr;
        check(alll_create(&p, &o, &ctx));
        vector<uint8_t> a(n_vars > 0 ? n_vars : 1);
        for (T i = 0; i < n_vars; ++i) a[i] = var_arr->vars[i] ? 1 : 0;
        int rc = alll_set_assignment(ctx, a.data(), a.size());
        alll_stats st;
        if (rc == ALLL_OK) rc = alll_solve(ctx, &st);
        if (rc == ALLL_OK || rc == ALLL_ERR_MAX_ITERS) {
            const int r2 = alll_get_assignment(ctx, a.data(), a.size());
            if (r2 != ALLL_OK) rc = r2;
        }
        alll_destroy(ctx);
        if (rc != ALLL_OK && rc != ALLL_ERR_MAX_ITERS) check(rc);
        for (T i = 0; i < n_vars; ++i) var_arr->vars[i] = a[i] != 0;
        auto s = new Statistics;
        s->n_iterations = st.n_iterations;
        s->n_resamples = st.n_resamples;
        s->avg_mis_size = st.avg_mis_size;
        const int nt = n_threads_ > st.n_gpus ? n_threads_ : st.n_gpus;
        s->n_thread_resamples.assign(nt > 0 ? nt : 1, 0);
        for (int g = 0; g < st.n_gpus && g < ALLL_MAX_GPU_STATS; ++g) s->n_thread_resamples[g] = st.gpu_resamples[g];
        return s;
    }

    static void check(int rc) {
        if (rc != ALLL_OK) throw std::runtime_error(std::string("alll: ") + alll_last_error());
    }
};

#endif
