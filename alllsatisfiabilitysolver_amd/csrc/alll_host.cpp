// alll_host.cpp -- host-only helpers of the C-ABI: the DIMACS loader and the synthetic
// k-SAT generator.  No GPU needed.
//
// DIMACS clause semantics follow example/cnf_io/cnf_io.cpp (cnf_header_read :487-705,
// cnf_data_read :126-328) as used by example/main.cpp:133-178, including its quirks:
//   * a last line without '\n' is not read (getline sets eof, the loop breaks: :277-281);
//   * lines starting with 'c'/'C' and lines of blanks only are skipped;
//   * words are split on ' ' only (s_word_extract_first :1419-1486);
//   * a word is read like s_to_i4 (:1305-1416): optional sign, digits, stop at the first
//     non-digit; a word that starts with anything else ends that line;
//   * 0 closes a clause, clauses may span lines and share lines.
// Where the reference is undefined (fewer clauses than the header, literal outside
// [1, V], counts beyond int) this loader reports an error instead.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "alll.h"

extern "C" void alll_internal_set_error(const char* msg);

namespace {

// error text shared with alll_last_error() (alll_runtime.cpp)
struct ErrSink {
    void operator=(const std::string& m) { alll_internal_set_error(m.c_str()); }
} g_host_err;

inline bool ws6(char ch) {
    return ch == ' ' || ch == '\f' || ch == '\n' || ch == '\r' || ch == '\t' || ch == '\v';
}

// Result of reading one word: kind 0 = number (value), 1 = not a number (ends the line).
struct Word {
    int kind;
    long long value;
};

inline Word read_word(const char* p, const char* e) {
    long long sign = 1, v = 0;
    const char* q = p;
    if (q < e && (*q == '-' || *q == '+')) {
        sign = (*q == '-') ? -1 : 1;
        ++q;
        if (q >= e || *q < '0' || *q > '9') return {1, 0};
    } else if (q >= e || *q < '0' || *q > '9') {
        return {1, 0};
    }
    while (q < e && *q >= '0' && *q <= '9') {
        v = v * 10 + (*q - '0');
        if (v > (1ll << 40)) v = 1ll << 40;  // clamp; flagged as out of range by the caller
        ++q;
    }
    return {0, sign * v};
}

struct Parsed {
    long long V = 0, C = 0;
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lits;
    uint64_t closed = 0;
    int rc = ALLL_OK;
};

bool parse_header(const char* ls, const char* le, long long& V, long long& C) {
    if (le - ls < 2 || !(ls[0] == 'p' || ls[0] == 'P') || !ws6(ls[1])) return false;
    const char* p = ls + 2;
    while (p < le && (*p == ' ' || *p == '\t')) ++p;  // s_adjustl skips blanks and tabs
    if (le - p < 4) return false;
    if ((p[0] | 32) != 'c' || (p[1] | 32) != 'n' || (p[2] | 32) != 'f' || !ws6(p[3])) return false;
    p += 4;
    while (p < le && (*p == ' ' || *p == '\t')) ++p;
    long long vals[2];
    for (int i = 0; i < 2; ++i) {
        while (p < le && *p == ' ') ++p;
        const char* we = p;
        while (we < le && *we != ' ') ++we;
        if (we == p) return false;
        Word w = read_word(p, we);
        if (w.kind) return false;
        vals[i] = w.value;
        p = we;
    }
    V = vals[0];
    C = vals[1];
    return V >= 0 && C >= 0 && V <= 0x7FFFFFFFll && C <= 0x7FFFFFFFll;
}

int parse(const char* buf, uint64_t len, Parsed& P) {
    const char* p = buf;
    const char* end = buf + len;
    bool header = false;
    uint64_t nl = 0;
    while (p < end) {
        const char* le = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (!le) break;  // unterminated last line is dropped
        const char* ls = p;
        p = le + 1;
        if (le > ls && (ls[0] == 'c' || ls[0] == 'C')) continue;
        const char* t = le;
        while (t > ls && t[-1] == ' ') --t;
        if (t == ls) continue;
        if (!header) {
            if (!parse_header(ls, le, P.V, P.C)) {
                g_host_err = "DIMACS: first non-comment line is not a valid 'p cnf V C' header";
                return ALLL_ERR_BAD_INPUT;
            }
            header = true;
            P.offs.reserve((size_t)P.C + 1);
            P.offs.push_back(0);
            continue;
        }
        const char* q = ls;
        while (true) {
            while (q < le && *q == ' ') ++q;
            const char* we = q;
            while (we < le && *we != ' ') ++we;
            if (we == q) break;
            Word w = read_word(q, we);
            if (w.kind) break;
            q = we;
            if (P.closed >= (uint64_t)P.C) continue;  // clauses beyond the header are ignored
            if (w.value != 0) {
                const long long x = w.value;
                if (x > P.V || -x > P.V) {
                    if (P.rc == ALLL_OK) {
                        P.rc = ALLL_ERR_LITERAL_RANGE;
                        g_host_err = "DIMACS: literal outside [1, V] in clause " + std::to_string(P.closed);
                    }
                    continue;
                }
                P.lits.push_back(x > 0 ? (uint32_t)(2 * x - 2) : (uint32_t)(-2 * x - 1));
                ++nl;
            } else {
                P.offs.push_back(nl);
                ++P.closed;
            }
        }
    }
    if (!header) {
        g_host_err = "DIMACS: no 'p cnf' header";
        return ALLL_ERR_BAD_INPUT;
    }
    if (P.closed < (uint64_t)P.C) {
        g_host_err = "DIMACS: header announces " + std::to_string(P.C) + " clauses, found " +
                     std::to_string(P.closed);
        return ALLL_ERR_BAD_INPUT;
    }
    return P.rc;
}

// ---- parallel loader (large inputs) ------------------------------------------------------
// Same semantics as parse(): the header is found serially; the data lines after it (up to the
// last '\n': an unterminated last line is dropped) are cut at line starts into one chunk per
// thread.  Every line's words are independent of other lines, so pass 1 counts the numbers
// per chunk (literals, clause-closing zeros), a prefix over the chunks gives each chunk its
// first clause index and literal position, and pass 2 writes literals and clause ends in
// place.  Clauses beyond the header's count are ignored as in parse().

// Calls f(value) for every number word of the data lines in [b, e); e[-1] is a '\n', which
// serves as the sentinel of every scan.  One pass per byte, fusing the line, word and number
// rules of parse()/read_word().
inline bool is_digit(char ch) { return (unsigned)(ch - '0') <= 9u; }

template <typename F>
inline void for_each_number(const char* b, const char* e, F&& f) {
    const char* p = b;
    while (p < e) {
        if (*p == 'c' || *p == 'C') {  // comment line
            p = static_cast<const char*>(memchr(p, '\n', (size_t)(e - p))) + 1;
            continue;
        }
        for (;;) {
            while (*p == ' ') ++p;
            const char ch = *p;
            if (ch == '\n') {
                ++p;
                break;
            }
            const char* q = p;
            long long sign = 1;
            if (ch == '-' || ch == '+') {
                sign = (ch == '-') ? -1 : 1;
                ++q;
            }
            if (!is_digit(*q)) {  // not a number: the rest of the line is ignored
                p = static_cast<const char*>(memchr(p, '\n', (size_t)(e - p))) + 1;
                break;
            }
            long long v = 0;
            do {
                v = v * 10 + (*q - '0');
                if (v > (1ll << 40)) v = 1ll << 40;
                ++q;
            } while (is_digit(*q));
            while (*q != ' ' && *q != '\n') ++q;  // trailing non-digits of the word
            p = q;
            if (!f(sign * v)) return;
        }
    }
}

struct ChunkCount {
    const char* b;
    const char* e;
    uint64_t lits = 0, zeros = 0;
    uint64_t tail = 0;     // literals after the chunk's last zero
    uint64_t bad = ~0ull;  // clause (counted within the chunk) of the first out-of-range literal
};

// returns ALLL_OK / ALLL_ERR_BAD_INPUT / ALLL_ERR_LITERAL_RANGE; offsets/literals may be null
int parse_parallel(const char* buf, uint64_t len, unsigned nt, uint32_t* n_vars, uint64_t* n_clauses,
                   uint64_t* offsets, uint32_t* literals, uint64_t* n_literals) {
    // header: first line that is neither a comment nor blank
    const char* end = buf + len;
    const char* p = buf;
    long long V = 0, C = 0;
    bool header = false;
    while (p < end) {
        const char* le = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (!le) break;
        const char* ls = p;
        p = le + 1;
        if (le > ls && (ls[0] == 'c' || ls[0] == 'C')) continue;
        const char* t = le;
        while (t > ls && t[-1] == ' ') --t;
        if (t == ls) continue;
        if (!parse_header(ls, le, V, C)) {
            g_host_err = "DIMACS: first non-comment line is not a valid 'p cnf V C' header";
            return ALLL_ERR_BAD_INPUT;
        }
        header = true;
        break;
    }
    if (!header) {
        g_host_err = "DIMACS: no 'p cnf' header";
        return ALLL_ERR_BAD_INPUT;
    }
    // data: [p, data_end), data_end just after the last '\n'
    const char* data_end = p;
    for (const char* q = end; q > p; --q)
        if (q[-1] == '\n') { data_end = q; break; }
    std::vector<ChunkCount> ch;
    const uint64_t span = (uint64_t)(data_end - p);
    const char* cb = p;
    for (unsigned i = 1; i <= nt && cb < data_end; ++i) {
        const char* ce = (i == nt) ? data_end : p + span * i / nt;
        if (ce < cb) ce = cb;
        if (ce < data_end) {
            const char* nl = static_cast<const char*>(memchr(ce, '\n', (size_t)(data_end - ce)));
            ce = nl ? nl + 1 : data_end;
        }
        ch.push_back({cb, ce});
        cb = ce;
    }
    auto run = [&](auto&& body) {
        std::vector<std::thread> th;
        for (size_t i = 0; i < ch.size(); ++i) th.emplace_back(body, i);
        for (auto& t : th) t.join();
    };
    run([&](size_t i) {
        ChunkCount& c = ch[i];
        for_each_number(c.b, c.e, [&](long long v) {
            if (v == 0) {
                ++c.zeros;
                c.tail = 0;
            } else if (v <= V && -v <= V) {  // out-of-range literals are skipped, as in parse()
                ++c.lits;
                ++c.tail;
            } else if (c.bad == ~0ull) {
                c.bad = c.zeros;
            }
            return true;
        });
    });
    std::vector<uint64_t> cl_base(ch.size() + 1, 0), lit_base(ch.size() + 1, 0);
    for (size_t i = 0; i < ch.size(); ++i) {
        cl_base[i + 1] = cl_base[i] + ch[i].zeros;
        lit_base[i + 1] = lit_base[i] + ch[i].lits;
    }
    if (cl_base[ch.size()] < (uint64_t)C) {
        g_host_err = "DIMACS: header announces " + std::to_string(C) + " clauses, found " +
                     std::to_string(cl_base[ch.size()]);
        return ALLL_ERR_BAD_INPUT;
    }
    // literals of the first C clauses: up to the C-th zero
    uint64_t nlits = 0;
    if (C > 0 && cl_base[ch.size()] == (uint64_t)C) {  // all literals but those after the last zero
        nlits = lit_base[ch.size()];
        for (size_t i = ch.size(); i-- > 0;) {
            nlits -= ch[i].tail;
            if (ch[i].zeros) break;
        }
    } else if (C > 0) {  // clauses past the header's count: find where the C-th ends
        size_t t = 0;
        while (cl_base[t + 1] < (uint64_t)C) ++t;
        uint64_t cl = cl_base[t], lp = lit_base[t];
        for_each_number(ch[t].b, ch[t].e, [&](long long v) {
            if (v) {
                lp += (v <= V && -v <= V);
                return true;
            }
            return ++cl < (uint64_t)C;
        });
        nlits = lp;
    }
    // pass 2: literals and clause ends in place
    if (offsets || literals) {
        if (offsets) offsets[0] = 0;
        run([&](size_t i) {
            uint64_t cl = cl_base[i], lp = lit_base[i];
            if (cl >= (uint64_t)C) return;
            for_each_number(ch[i].b, ch[i].e, [&](long long x) {
                if (x != 0) {
                    if (x <= V && -x <= V) {
                        if (literals) literals[lp] = x > 0 ? (uint32_t)(2 * x - 2) : (uint32_t)(-2 * x - 1);
                        ++lp;
                    }
                    return true;
                }
                if (offsets) offsets[cl + 1] = lp;
                return ++cl < (uint64_t)C;
            });
        });
    }
    if (n_vars) *n_vars = (uint32_t)V;
    if (n_clauses) *n_clauses = (uint64_t)C;
    if (n_literals) *n_literals = nlits;
    uint64_t first_bad = ~0ull;  // the first out-of-range literal among the first C clauses
    for (size_t i = 0; i < ch.size() && first_bad == ~0ull; ++i)
        if (ch[i].bad != ~0ull && cl_base[i] + ch[i].bad < (uint64_t)C) first_bad = cl_base[i] + ch[i].bad;
    if (first_bad != ~0ull) {
        g_host_err = "DIMACS: literal outside [1, V] in clause " + std::to_string(first_bad);
        return ALLL_ERR_LITERAL_RANGE;
    }
    return ALLL_OK;
}

unsigned loader_threads(uint64_t len) {
    uint64_t min_parallel = 8ull << 20;  // below this the serial parse is as fast
    if (const char* e = getenv("ALLL_DIMACS_MIN_PARALLEL")) min_parallel = strtoull(e, nullptr, 10);
    if (len < min_parallel) return 1;
    unsigned nt = std::min(32u, std::thread::hardware_concurrency());
    if (const char* e = getenv("ALLL_DIMACS_THREADS")) nt = (unsigned)std::max(1l, std::min(256l, strtol(e, nullptr, 10)));
    return std::max(2u, nt);
}

int deliver(const Parsed& P, uint32_t* n_vars, uint64_t* n_clauses, uint64_t* offsets,
            uint32_t* literals, uint64_t* n_literals) {
    if (n_vars) *n_vars = (uint32_t)P.V;
    if (n_clauses) *n_clauses = (uint64_t)P.C;
    if (n_literals) *n_literals = P.lits.size();
    if (offsets) std::copy(P.offs.begin(), P.offs.end(), offsets);
    if (literals) std::copy(P.lits.begin(), P.lits.end(), literals);
    return ALLL_OK;
}

// --- generator (same specification as the oracle's; checked equal in tests) -----------
inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline uint32_t draw(uint64_t r, uint32_t n, int kind) {
    uint64_t u = r >> 32;
    if (kind == 1) {  // v = floor(n u^5): density ~ v^-0.8
        const uint64_t u1 = u;
        u = (u * u1) >> 32;
        u = (u * u1) >> 32;
        u = (u * u1) >> 32;
        u = (u * u1) >> 32;
    }
    return (uint32_t)((u * (uint64_t)n) >> 32);
}

void gen_range(uint64_t seed, uint32_t n, uint32_t k, int kind, uint64_t cb, uint64_t ce,
               uint64_t base, uint32_t* out) {
    for (uint64_t c = cb; c < ce; ++c) {
        uint64_t s = mix64(seed ^ mix64(c + 0x632BE59BD9B4E019ull));
        uint32_t* o = out + (c - base) * k;
        for (uint32_t j = 0; j < k; ++j) {
            for (;;) {
                s += 0x9E3779B97F4A7C15ull;
                const uint64_t r = mix64(s);
                const uint32_t v = draw(r, n, kind);
                bool dup = false;
                for (uint32_t q = 0; q < j; ++q) dup |= (o[q] >> 1) == v;
                if (!dup) {
                    o[j] = 2u * v + (uint32_t)(r & 1u);
                    break;
                }
            }
        }
    }
}

uint32_t philox_x_host(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0;
        c1 = (uint32_t)p1;
        c2 = n2;
        c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c0;
}

// The reference's VariablesArray fill (VariablesArray.h:23-34) in the reference-RNG mode: the
// same stream as k_rrng_init (alll_refrng.hip) -- the random_device stand-in's
// next value seeds minstd_rand0, libstdc++'s uniform_int_distribution<unsigned long long> upscales
// its values to 64 bits, RBG serves 63 bits of each, lowest first.
struct RefRbg {
    static constexpr uint64_t M = 2147483647ull, MIN = 1ull, RANGE = M - 1ull - MIN, UR = RANGE + 1ull;
    static constexpr uint64_t Q1 = ~0ull / UR, Q2 = Q1 / UR, UE = Q2 + 1ull, SC = RANGE / UE, PAST = UE * SC;
    uint64_t x;
    uint64_t next() {
        x = (x * 16807ull) % M;
        return x;
    }
    uint64_t inner() {
        uint64_t r;
        do r = next() - MIN;
        while (r >= PAST);
        return r / SC;
    }
    uint64_t middle() {
        uint64_t ret, tmp;
        do {
            tmp = UR * inner();
            ret = tmp + (next() - MIN);
        } while (ret > Q1 || ret < tmp);
        return ret;
    }
    uint64_t draw() {
        uint64_t ret, tmp;
        do {
            tmp = UR * middle();
            ret = tmp + (next() - MIN);
        } while (ret < tmp);
        return ret;
    }
};

}  // namespace

extern "C" {

int alll_reference_initial_assignment(uint64_t rd_state, uint32_t n_vars, uint8_t* out) {
    if (!out && n_vars) return ALLL_ERR_INVALID_ARG;
    rd_state = rd_state * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t seed = (uint32_t)(rd_state >> 33);
    RefRbg g{(uint64_t)seed % RefRbg::M};
    if (!g.x) g.x = 1;
    uint64_t m = 1;
    for (uint32_t v = 0; v < n_vars; ++v) {
        if (m == 1) m = g.draw() | (1ull << 63);
        out[v] = (uint8_t)(m & 1u);
        m >>= 1;
    }
    return ALLL_OK;
}

int alll_initial_assignment(uint64_t seed, uint32_t n_vars, uint8_t* out) {
    if (!out && n_vars) return ALLL_ERR_INVALID_ARG;
    for (uint32_t w = 0; w < (n_vars + 31) / 32; ++w) {
        const uint32_t x = philox_x_host(w, 0u, 0xFFFFFFFFu, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
        for (uint32_t b = 0; b < 32 && 32 * w + b < n_vars; ++b) out[32 * w + b] = (x >> b) & 1u;
    }
    return ALLL_OK;
}

int alll_dimacs_parse(const char* buf, uint64_t len, uint32_t* n_vars, uint64_t* n_clauses,
                      uint64_t* offsets, uint32_t* literals, uint64_t* n_literals) {
    if (!buf && len) return ALLL_ERR_INVALID_ARG;
    const unsigned nt = loader_threads(len);
    if (nt > 1) return parse_parallel(buf, len, nt, n_vars, n_clauses, offsets, literals, n_literals);
    Parsed P;
    int rc = parse(buf, len, P);
    if (rc == ALLL_ERR_BAD_INPUT) return rc;
    int rc2 = deliver(P, n_vars, n_clauses, offsets, literals, n_literals);
    return rc ? rc : rc2;
}

int alll_dimacs_read(const char* path, uint32_t* n_vars, uint64_t* n_clauses, uint64_t* offsets,
                     uint32_t* literals, uint64_t* n_literals) {
    if (!path) return ALLL_ERR_INVALID_ARG;
    int fd = open(path, O_RDONLY);
    if (fd < 0) {
        g_host_err = std::string("cannot open ") + path;
        return ALLL_ERR_IO;
    }
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
        close(fd);
        return ALLL_ERR_IO;
    }
    const uint64_t len = (uint64_t)sb.st_size;
    const char* buf = "";
    void* mp = nullptr;
    if (len) {
        mp = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
        if (mp == MAP_FAILED) {
            close(fd);
            return ALLL_ERR_IO;
        }
        madvise(mp, len, MADV_SEQUENTIAL);
        buf = static_cast<const char*>(mp);
    }
    int rc = alll_dimacs_parse(buf, len, n_vars, n_clauses, offsets, literals, n_literals);
    if (mp) munmap(mp, len);
    close(fd);
    return rc;
}

int alll_generate_ksat(uint64_t gen_seed, uint32_t n_vars, uint64_t n_clauses, uint32_t k,
                       int kind, uint64_t c_begin, uint64_t c_end, uint32_t* literals) {
    if (k == 0 || k > 64 || n_vars < k || c_end > n_clauses || c_begin > c_end || !literals ||
        (kind != 0 && kind != 1))
        return ALLL_ERR_INVALID_ARG;
    const uint64_t n = c_end - c_begin;
    unsigned nt = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    if (n < (1u << 20)) nt = 1;
    if (nt == 1) {
        gen_range(gen_seed, n_vars, k, kind, c_begin, c_end, c_begin, literals);
        return ALLL_OK;
    }
    std::vector<std::thread> th;
    for (unsigned i = 0; i < nt; ++i) {
        const uint64_t a = c_begin + n * i / nt, b = c_begin + n * (i + 1) / nt;
        th.emplace_back(gen_range, gen_seed, n_vars, k, kind, a, b, c_begin, literals);
    }
    for (auto& t : th) t.join();
    return ALLL_OK;
}

}  // extern "C"
