// SATInstance.h -- compatibility header: the reference's public API
// (library/include/SATInstance.h:25-66, 156-173) over the MI355X solver's C-ABI
// (include/alll.h).  Existing call sites (example/main.cpp) compile unchanged; the device,
// seed and iteration cap are additive settings (env ALLL_DEVICE, ALLL_SEED, ALLL_MAX_ITERS).
#ifndef ALLL_COMPAT_SATINSTANCE_H
#define ALLL_COMPAT_SATINSTANCE_H

#include <cstdint>
#include <cstdio>
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
        alll_problem p{(uint32_t)n_vars, 0, offs.size() - 1, offs.data(), lits.data()};
        alll_options o;
        alll_default_options(&o);
        o.seed = alll_compat::env_u64("ALLL_SEED", 1);
        o.max_iters = alll_compat::env_u64("ALLL_MAX_ITERS", 0);
        o.device = (int32_t)alll_compat::env_u64("ALLL_DEVICE", (uint64_t)-1);
        o.n_threads = n_threads_ > 0 ? n_threads_ : 1;
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

    // Host check over var_arr->vars, like the reference.
    bool verify_validity(vector<ClauseArray*>* clauses) const {
        for (auto chunk : *clauses)
            for (auto cl : *chunk)
                if (cl->is_not_satisfied(var_arr->vars)) return false;
        return true;
    }

   private:
    int n_threads_{};

    static void check(int rc) {
        if (rc != ALLL_OK) throw std::runtime_error(std::string("alll: ") + alll_last_error());
    }
};

#endif
