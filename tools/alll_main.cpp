// alll_main.cpp -- command-line driver with the flags and output of the reference's
// example/main.cpp (-h, -o, -p N, --sat PATH; main.cpp:48-93) without Boost, over the
// compatibility SATInstance API (include/alll_compat) and the MI355X solver.
// Additive flags: --seed S, --max-iters K, --device D, --reference-rng STATE.
//
// Output parity with main.cpp: the INFORMATION block (n_clauses printed before solve, so 0:
// main.cpp:192-194), STATISTICS with one line per thread (:236-247), SATISFIABLE / ERROR
// and exit code from verify_validity (:268-295); -o writes <path minus 4 chars>.out / .csv
// (:102-107, 196-200, 228-230, 248-250, 272-276).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "SATInstance.h"

typedef uint32_t UINT_T;
typedef SATInstance<UINT_T>::ClauseArray ClauseArray;

static void output(const string& str, ofstream* out_f, bool dump) {
    cout << str;
    if (dump) *out_f << str;
}

static string now_str() {
    auto t = chrono::system_clock::to_time_t(chrono::system_clock::now());
    string s = ctime(&t);
    s.pop_back();
    return s;
}

static void usage() {
    cout << "Options:\n"
            "  -h [ --help ]             Help\n"
            "  -o [ --output ]           Output meta-data and statistics to separate files\n"
            "  -p [ --parallel ] arg (=0) Use parallel solver\n"
            "  --sat arg                 Path to SAT instance in DIMACS-CNF format\n"
            "  --seed arg (=1)           Philox seed (MI355X solver)\n"
            "  --reference-rng arg       the reference's own random stream, random_device stand-in state (MI355X solver)\n"
            "  --max-iters arg (=0)      Cap on eval passes, 0 = unlimited (MI355X solver)\n"
            "  --device arg (=-1)        HIP device (MI355X solver)\n";
}

int main(int argc, char* argv[]) {
    int n_threads = 1;
    bool dump = false;
    string cnf_fpath;
    const int procs = omp_get_num_procs();  // main.cpp:77
    for (int i = 1; i < argc; ++i) {
        string a = argv[i];
        auto need = [&](const char* what) -> string {
            if (i + 1 >= argc) {
                cerr << "the required argument for option '" << what << "' is missing" << endl;
                exit(1);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (a == "-o" || a == "--output") dump = true;
        else if (a == "-p" || a == "--parallel") {
            int p = atoi(need("--parallel").c_str());
            if (p < 0 || p > procs) n_threads = procs;  // main.cpp:77-83
            else if (p > 0) n_threads = p;
            else n_threads = 1;
        } else if (a == "--sat") cnf_fpath = need("--sat");
        else if (a == "--seed") setenv("ALLL_SEED", need("--seed").c_str(), 1);
        else if (a == "--reference-rng") setenv("ALLL_REFERENCE_RNG", need("--reference-rng").c_str(), 1);
        else if (a == "--max-iters") setenv("ALLL_MAX_ITERS", need("--max-iters").c_str(), 1);
        else if (a == "--device") setenv("ALLL_DEVICE", need("--device").c_str(), 1);
        else { cerr << "unrecognised option '" << a << "'" << endl; return 1; }
    }
    if (cnf_fpath.empty()) {
        cerr << "the option '--sat' is required but missing" << endl;
        return 1;
    }
    ofstream* out_f = nullptr;
    ofstream* stat_f = nullptr;
    if (dump) {
        string o = cnf_fpath, s = cnf_fpath;
        o.replace(o.size() - 4, 4, ".out");
        s.replace(s.size() - 4, 4, ".csv");
        out_f = new ofstream(o);
        stat_f = new ofstream(s);
    }
    output("Log " + now_str() + ": Reading CNF file\n", out_f, dump);
    auto start = chrono::high_resolution_clock::now();

    uint32_t v_num = 0;
    uint64_t c_num = 0, l_num = 0;
    if (alll_dimacs_read(cnf_fpath.c_str(), &v_num, &c_num, nullptr, nullptr, &l_num) == ALLL_ERR_BAD_INPUT ||
        c_num == 0 && v_num == 0) {
        cout << "The header information could not be read. Exiting..." << endl;
        exit(1);
    }
    vector<uint64_t> offs(c_num + 1);
    vector<uint32_t> lits(l_num + 1);
    int rc = alll_dimacs_read(cnf_fpath.c_str(), &v_num, &c_num, offs.data(), lits.data(), &l_num);
    if (rc != ALLL_OK) {
        cout << "ERROR: " << alll_last_error() << endl;
        exit(1);
    }
    // chunking of main.cpp:149-178 (chunk 0 receives chunk_size + 1 clauses)
    int chunk_size = (int)ceil(c_num / (double)n_threads);
    auto clauses = new vector<ClauseArray*>();
    for (int t = 0; t < n_threads; t++) clauses->push_back(new ClauseArray());
    unsigned short int t = 0;
    for (uint64_t c = 0; c < c_num; c++) {
        auto literals = new vector<UINT_T>(lits.begin() + offs[c], lits.begin() + offs[c + 1]);
        if ((long long)c > (long long)(t + 1) * chunk_size) t += 1;
        clauses->at(t)->push_back(new Clause<UINT_T>(literals, t));
    }
    auto satInstance = new SATInstance<UINT_T>(new VariablesArray<UINT_T>(v_num), n_threads);

    auto stop = chrono::high_resolution_clock::now();
    auto read_duration = chrono::duration_cast<chrono::milliseconds>(stop - start);
    output("Log " + now_str() + ": Read complete; Duration: " + to_string(read_duration.count() / 1000.0) + "s\n\n",
           out_f, dump);
    output("------------ INFORMATION ------------\n\t\t\t# Variables\t= " + to_string(satInstance->n_vars) +
               "\n\t\t\t# Clauses\t= " + to_string(satInstance->n_clauses) +
               "\n-------------------------------------\n\n",
           out_f, dump);
    if (dump) {
        *stat_f << to_string(read_duration.count() / 1000.0) + ",";
        *stat_f << to_string(satInstance->n_vars) + ",";
        *stat_f << to_string(satInstance->n_clauses) + ",";
    }
    string solve_info = "Starting parallel solve (# Threads = " + to_string(n_threads) + ")";
    output("Log " + now_str() + ": " + solve_info + "\n", out_f, dump);
    start = chrono::high_resolution_clock::now();
    Statistics* statistics = nullptr;
    try {
        statistics = satInstance->solve(clauses);
    } catch (const std::exception& e) {
        cout << "ERROR: " << e.what() << endl;
        return 2;
    }
    stop = chrono::high_resolution_clock::now();
    auto solve_duration = chrono::duration_cast<chrono::milliseconds>(stop - start);
    output("Log " + now_str() + ": Completed solve; Duration: " + to_string(solve_duration.count() / 1000.0) +
               "s\n\n",
           out_f, dump);
    if (dump) *stat_f << to_string(solve_duration.count()) + ",";
    output("------------ STATISTICS -------------\n# Iterations\t= " + to_string(statistics->n_iterations) +
               "\n# Resamples\t= " + to_string(statistics->n_resamples),
           out_f, dump);
    for (int q = 0; q < n_threads; q++)
        output("\n\tThread " + to_string(q + 1) + ": " + to_string(statistics->n_thread_resamples.at(q)), out_f, dump);
    output("\n\nAvg. UNSAT MIS Size = " + to_string(statistics->avg_mis_size) +
               "\n-------------------------------------\n\n",
           out_f, dump);
    if (dump) {
        *stat_f << to_string(n_threads) + ",";
        *stat_f << to_string(statistics->n_iterations) + "\n";
    }
    if (satInstance->verify_validity(clauses)) {
        output("SATISFIABLE\n", out_f, dump);
        if (dump) {
            for (ull i = 0; i < satInstance->n_vars; i++)
                *out_f << "\nVariable " + to_string(i + 1) + " = " + to_string((satInstance->var_arr->vars)[i]);
            stat_f->close();
            out_f->close();
        }
        return 0;
    }
    output("ERROR: Solver converged to an invalid solution!\n", out_f, dump);
    if (dump) {
        stat_f->close();
        out_f->close();
    }
    return 1;
}
