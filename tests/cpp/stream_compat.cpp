// Test driver (not product code): the compatibility SATInstance API's streaming solve and
// writeDIMACS, compiled against include/alll_compat exactly like a reference consumer.
//   stream_compat <cnf-in> <batch> <dimacs-out> [n_threads]
//   stream_compat order <m> <batch>   yield order of ClauseGenerator over m always-violated clauses
// loads a DIMACS file (one clause per line) into a table served by the clause callback, runs
// solve(getEnumeratedClause, n_clauses, batch), prints the statistics and the assignment as
// JSON, and writes the instance back with writeDIMACS.
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "ClauseGenerator.h"
#include "SATInstance.h"

typedef uint32_t UINT_T;
static std::vector<std::vector<UINT_T>> g_clauses;

static Clause<UINT_T>* enumerated(UINT_T idx, unsigned short t_id) {
    if (idx >= g_clauses.size()) return nullptr;
    return new Clause<UINT_T>(new std::vector<UINT_T>(g_clauses[idx]), t_id);
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    if (std::string(argv[1]) == "order") {
        const UINT_T m = (UINT_T)atol(argv[2]);
        for (UINT_T i = 0; i < m; ++i) g_clauses.push_back({2 * i});  // x_i: violated when all false
        std::vector<char> vars(m + 1, 0);
        ClauseGenerator<UINT_T> gen(enumerated, 0, m, 0, (UINT_T)atol(argv[3]));
        printf("[");
        bool first = true;
        for (int pass = 0; pass < 2; ++pass) {  // two full walks: the step state carries over
            do {
                auto batch = gen.yieldRandomUNSATClauseBatch(reinterpret_cast<const bool*>(vars.data()));
                for (auto c : *batch) {
                    printf("%s%u", first ? "" : ", ", (*c->literals)[0] / 2);
                    first = false;
                    delete c->literals;
                    delete c;
                }
                delete batch;
            } while (!gen.has_finished_yielding());
        }
        printf("]\n");
        return 0;
    }
    std::ifstream in(argv[1]);
    std::string line;
    long n_vars = 0;
    while (std::getline(in, line)) {
        if (line.empty() || line[0] == 'c') continue;
        std::istringstream ss(line);
        if (line[0] == 'p') {
            std::string p, cnf;
            long m;
            ss >> p >> cnf >> n_vars >> m;
            continue;
        }
        std::vector<UINT_T> cl;
        long x;
        while (ss >> x && x != 0) cl.push_back(x > 0 ? 2 * (x - 1) : 2 * (-x - 1) + 1);
        g_clauses.push_back(cl);
    }
    auto var_arr = new VariablesArray<UINT_T>((UINT_T)n_vars);
    SATInstance<UINT_T> S(var_arr, argc > 4 ? atoi(argv[4]) : 1);
    Statistics* st = nullptr;
    try {
        st = S.solve(enumerated, (ull)g_clauses.size(), (UINT_T)atol(argv[2]));
    } catch (const std::exception& e) {
        printf("{\"error\": \"%s\"}\n", e.what());
        return 3;
    }
    printf("{\"n_iterations\": %llu, \"n_resamples\": %llu, \"avg_mis_size\": %llu, \"threads\": %zu, \"assignment\": \"",
           st->n_iterations, st->n_resamples, st->avg_mis_size, st->n_thread_resamples.size());
    for (long v = 0; v < n_vars; ++v) putchar(var_arr->vars[v] ? '1' : '0');
    printf("\"}\n");
    std::ofstream out(argv[3]);
    S.writeDIMACS(enumerated, (ull)g_clauses.size(), &out);
    return 0;
}
