// CPU model of the round robin's fixpoint passes on a random 3-SAT instance
// of the bench's shape: per iteration, the passes P <- LFMIS(turns(P)) from a first guess until
// they repeat, with per-pass statistics (picks changed, the earliest turn whose decision changed,
// entries whose turn changed).  A study tool for the pass count; not part of the product.
//   g++ -O2 -std=c++17 -fopenmp -o build/rr_sim tools/microbench/rr_sim.cpp
//   build/rr_sim [n] [m] [T] [iterations] [guess: 0 density, 1 per-set density, 2 previous picks' levels]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

struct Rec { uint32_t l0, step, L, o; };

static std::vector<std::vector<Rec>> schedule(const std::vector<uint32_t>& n, std::vector<uint32_t>* erase) {
    const uint32_t T = (uint32_t)n.size();
    std::vector<uint32_t> live(T), done(T, 0);
    std::iota(live.begin(), live.end(), 0u);
    std::vector<std::vector<Rec>> segs(T);
    uint64_t t = 0, step = 0;
    if (erase) erase->clear();
    while (!live.empty()) {
        const uint64_t L = live.size();
        uint64_t best = ~0ull, istar = 0;
        std::vector<uint64_t> offs(L);
        for (uint64_t i = 0; i < L; ++i) {
            offs[i] = (i + L - (t % L) - 1) % L;
            const uint64_t key = (uint64_t)(n[live[i]] - done[live[i]]) * L + offs[i];
            if (key < best) { best = key; istar = i; }
        }
        const uint64_t E = step + best;
        for (uint64_t i = 0; i < L; ++i) {
            const uint32_t s = live[i];
            segs[s].push_back({done[s], (uint32_t)step, (uint32_t)L, (uint32_t)offs[i]});
            if (i == istar) done[s] = n[s];
            else {
                const int64_t q = (int64_t)E - (int64_t)step - (int64_t)offs[i];
                done[s] += q > 0 ? (uint32_t)((q + L - 1) / L) : 0u;
            }
        }
        if (erase) erase->push_back((uint32_t)E);
        live.erase(live.begin() + istar);
        t = istar;
        step = E + 1;
    }
    return segs;
}

static uint32_t turn_of(const std::vector<Rec>& r, uint32_t lev) {
    size_t k = 0;
    while (k + 1 < r.size() && r[k + 1].l0 <= lev) ++k;
    return r[k].step + (lev - r[k].l0) * r[k].L + r[k].o;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 2500000, m = argc > 2 ? atoi(argv[2]) : 10000000;
    const uint32_t T = argc > 3 ? atoi(argv[3]) : 16, iters = argc > 4 ? atoi(argv[4]) : 12;
    const int guess_mode = argc > 5 ? atoi(argv[5]) : 0;
    // > 0: windowed passes (block Gauss-Seidel over the turn timeline): a pass adopts the new
    // decisions of entries whose turn lies below the window end only; the window moves on once
    // such a pass changes nothing below its end (that prefix is then exact)
    const double win = argc > 6 ? atof(argv[6]) : 0.0;
    // 1: passes after the first are incremental: the entries whose lower-neighbour set changed
    // (an order flip in a shared variable's claimant list) are re-decided by Jacobi rounds over
    // the dirty entries (a changed decision dirties its upper neighbours); checked against the
    // full LFMIS of the same turns
    const int incr = argc > 7 ? atoi(argv[7]) : 0;
    // > 0: near pairs of claimants (|turn difference| < margin after pass 1) and the drift of
    // every entry's level since pass 1; checks that every order flip of a later pass is a near pair
    const uint32_t margin = argc > 8 ? atoi(argv[8]) : 0;
    const int near_pass = argc > 9 ? atoi(argv[9]) : 2;  // the pass whose turns define the near pairs
    std::mt19937_64 rng(12345);
    std::vector<uint32_t> lit((size_t)m * 3);
    for (uint32_t c = 0; c < m; ++c) {
        uint32_t v[3];
        for (int j = 0; j < 3; ++j) {
            bool dup;
            do {
                v[j] = (uint32_t)(rng() % n);
                dup = false;
                for (int q = 0; q < j; ++q) dup |= v[q] == v[j];
            } while (dup);
            lit[(size_t)c * 3 + j] = v[j] * 2 + (uint32_t)(rng() & 1);
        }
    }
    std::vector<uint8_t> A(n);
    for (auto& a : A) a = rng() & 1;
    // chunk starts (example/main.cpp rule)
    std::vector<uint32_t> cs(T + 1);
    const uint64_t chunk = (m + T - 1) / T;
    cs[0] = 0;
    for (uint32_t q = 1; q <= T; ++q) cs[q] = (uint32_t)std::min<uint64_t>(m, q * chunk + 1);
    cs[T] = m;
    std::vector<uint32_t> stamp(n, 0);
    uint32_t st = 0;
    double dens = 0.5;
    std::vector<double> set_dens(T, 0.5);
    long tot_passes = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        std::vector<uint32_t> U;
        for (uint32_t c = 0; c < m; ++c) {
            bool sat = false;
            for (int j = 0; j < 3; ++j) { const uint32_t l = lit[(size_t)c * 3 + j]; sat |= (A[l >> 1] ^ (l & 1)) != 0; }
            if (!sat) U.push_back(c);
        }
        const uint32_t u = (uint32_t)U.size();
        std::vector<uint32_t> setof(u), sf(T + 1);
        for (uint32_t s = 0, i = 0; s < T; ++s) {
            sf[s] = i;
            while (i < u && U[i] < cs[s + 1]) setof[i++] = s;
        }
        sf[T] = u;
        // claimant lists per variable (entries), for the incremental passes
        std::vector<uint32_t> voff(n + 1, 0), vl((size_t)u * 3);
        for (uint32_t i = 0; i < u; ++i) for (int j = 0; j < 3; ++j) ++voff[(lit[(size_t)U[i] * 3 + j] >> 1) + 1];
        for (uint32_t v = 0; v < n; ++v) voff[v + 1] += voff[v];
        {
            std::vector<uint32_t> fill(voff.begin(), voff.end() - 1);
            for (uint32_t i = 0; i < u; ++i) for (int j = 0; j < 3; ++j) vl[fill[lit[(size_t)U[i] * 3 + j] >> 1]++] = i;
        }
        std::vector<uint8_t> P(u), Pn(u);
        for (uint32_t i = 0; i < u; ++i) {
            const uint32_t s = setof[i];
            const uint64_t pos = i - sf[s];
            const double d = guess_mode == 1 ? set_dens[s] : dens;
            P[i] = (uint64_t)((pos + 1) * d) > (uint64_t)(pos * d);
        }
        std::vector<uint32_t> turn(u), prev_turn(u, 0), order(u), blocker(u, ~0u), covby(n, 0);
        std::vector<uint64_t> key(u);
        std::vector<uint32_t> lev1, turn1;
        std::vector<uint8_t> late;
        uint64_t n_near = 0;
        uint32_t e0_1 = 0;
        int passes = 0;
        uint64_t work = 0;        // entries processed by the passes (those with turn >= the exact prefix)
        uint32_t we = 0, ws = 0;  // window [ws, we) of turns (windowed mode)
        printf("iter %u: |U| = %u\n", it, u);
        for (;;) {
            std::vector<uint32_t> cnt(T, 0), lev(u);
            for (uint32_t i = 0; i < u; ++i) { lev[i] = cnt[setof[i]]; cnt[setof[i]] += P[i]; }
            std::vector<uint32_t> er;
            auto segs = schedule(cnt, &er);
            uint32_t tch = 0;
            for (uint32_t i = 0; i < u; ++i) {
                turn[i] = turn_of(segs[setof[i]], lev[i]);
                tch += passes > 0 && turn[i] != prev_turn[i];
                key[i] = ((uint64_t)turn[i] << 32) | i;
            }
            std::iota(order.begin(), order.end(), 0u);
            std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
            ++st;
            std::vector<uint32_t> fblocker(u, ~0u);
            for (uint32_t q = 0; q < u; ++q) {
                const uint32_t i = order[q], c = U[i];
                bool free_ = true;
                for (int j = 0; j < 3; ++j) {
                    const uint32_t v = lit[(size_t)c * 3 + j] >> 1;
                    if (stamp[v] == st) { if (free_) fblocker[i] = covby[v]; free_ = false; }
                }
                Pn[i] = free_;
                if (free_) for (int j = 0; j < 3; ++j) { stamp[lit[(size_t)c * 3 + j] >> 1] = st; covby[lit[(size_t)c * 3 + j] >> 1] = i; }
            }
            ++passes;
            if (margin && passes == near_pass) {
                lev1 = lev;
                turn1 = turn;
                e0_1 = er.empty() ? 0 : er[0];
                n_near = 0;
                uint64_t pairs = 0;
                for (uint32_t v = 0; v < n; ++v)
                    for (uint32_t a = voff[v]; a < voff[v + 1]; ++a)
                        for (uint32_t b2 = a + 1; b2 < voff[v + 1]; ++b2) {
                            const uint32_t x = vl[a], y = vl[b2];
                            ++pairs;
                            const uint32_t d = turn[x] > turn[y] ? turn[x] - turn[y] : turn[y] - turn[x];
                            const bool lt = turn[x] + margin >= e0_1 || turn[y] + margin >= e0_1;
                            if (d < margin || lt) ++n_near;
                        }
                printf("    near pairs (margin %u): %llu of %llu claimant pairs, first erasure %u\n", margin,
                       (unsigned long long)n_near, (unsigned long long)pairs, e0_1);
            } else if (margin && passes > near_pass) {
                int32_t dmax = 0;
                for (uint32_t i = 0; i < u; ++i) dmax = std::max<int32_t>(dmax, std::abs((int32_t)lev[i] - (int32_t)lev1[i]));
                uint64_t flips = 0, missed = 0;
                for (uint32_t v = 0; v < n; ++v)
                    for (uint32_t a = voff[v]; a < voff[v + 1]; ++a)
                        for (uint32_t b2 = a + 1; b2 < voff[v + 1]; ++b2) {
                            const uint32_t x = vl[a], y = vl[b2];
                            const bool o1 = ((uint64_t)prev_turn[x] << 32 | x) < ((uint64_t)prev_turn[y] << 32 | y);
                            const bool o2 = key[x] < key[y];
                            if (o1 == o2) continue;
                            ++flips;
                            const uint32_t d = turn1[x] > turn1[y] ? turn1[x] - turn1[y] : turn1[y] - turn1[x];
                            const bool lt = turn1[x] + margin >= e0_1 || turn1[y] + margin >= e0_1;
                            missed += !(d < margin || lt);
                        }
                printf("    drift: max |lev - lev1| %d (x T = %d), first erasure %u (pass 1: %u); flips %llu, not near %llu\n",
                       dmax, dmax * (int)T, er.empty() ? 0 : er[0], e0_1, (unsigned long long)flips,
                       (unsigned long long)missed);
            }
            if (incr == 2 && passes > 1) {
                // blocker-based: every entry out of P (the last pass's picks, LFMIS of the last
                // turns) keeps the P-neighbour below it that blocked it; under the new turns it is
                // dirty iff that blocker is no longer below it.  Jacobi rounds then re-decide the
                // dirty entries (a changed decision dirties the neighbours above it)
                auto knew = [&](uint32_t i) { return key[i]; };
                std::vector<uint8_t> Q(P), dirty(u, 0);
                std::vector<uint32_t> dl;
                for (uint32_t y = 0; y < u; ++y)
                    if (!P[y] && knew(blocker[y]) > knew(y)) { dirty[y] = 1; dl.push_back(y); }
                const uint32_t nd0 = (uint32_t)dl.size();
                {  // list slots (with the entry itself) of the dirty entries' variables
                    uint32_t hist[8] = {0};
                    for (uint32_t x : dl) {
                        uint32_t tot = 0;
                        for (int j = 0; j < 3; ++j) { const uint32_t v = lit[(size_t)U[x] * 3 + j] >> 1; const uint32_t c = voff[v + 1] - voff[v]; if (c > 1) tot += c; }
                        hist[std::min<uint32_t>(tot / 4, 7)]++;
                    }
                    printf("    dirty list slots /4: %u %u %u %u %u %u %u %u\n", hist[0], hist[1], hist[2], hist[3], hist[4], hist[5], hist[6], hist[7]);
                }
                uint64_t dwork = 0;
                int rounds = 0;
                std::vector<uint32_t> nblk(u);
                while (!dl.empty()) {
                    ++rounds;
                    dwork += dl.size();
                    std::vector<std::pair<uint32_t, uint8_t>> chg;
                    for (uint32_t x : dl) {
                        uint32_t bk = ~0u;
                        for (int j = 0; j < 3 && bk == ~0u; ++j) {
                            const uint32_t v = lit[(size_t)U[x] * 3 + j] >> 1;
                            for (uint32_t a = voff[v]; a < voff[v + 1]; ++a) {
                                const uint32_t y = vl[a];
                                if (y != x && Q[y] && knew(y) < knew(x)) { bk = y; break; }
                            }
                        }
                        const uint8_t in = bk == ~0u;
                        if (!in) nblk[x] = bk;
                        if (in != Q[x]) chg.push_back({x, in});
                    }
                    for (uint32_t x : dl) dirty[x] = 0;
                    for (uint32_t x : dl) if (!Q[x] || true) blocker[x] = nblk[x];
                    std::vector<uint32_t> nd;
                    for (auto& c : chg) {
                        Q[c.first] = c.second;
                        const uint32_t x = c.first;
                        for (int j = 0; j < 3; ++j) {
                            const uint32_t v = lit[(size_t)U[x] * 3 + j] >> 1;
                            for (uint32_t a = voff[v]; a < voff[v + 1]; ++a) {
                                const uint32_t y = vl[a];
                                if (y != x && knew(y) > knew(x) && !dirty[y]) { dirty[y] = 1; nd.push_back(y); }
                            }
                        }
                    }
                    dl.swap(nd);
                }
                uint32_t bad = 0, nch = 0;
                for (uint32_t i = 0; i < u; ++i) { bad += Q[i] != Pn[i]; nch += Q[i] != P[i]; }
                printf("    blocker-incremental: dirty %u, Jacobi rounds %d, work %llu, changes %u, mismatches vs full %u\n",
                       nd0, rounds, (unsigned long long)dwork, nch, bad);
            }
            if (incr == 1 && passes > 1) {
                // keys of the last pass (prev_turn) and of this one (turn)
                auto kold = [&](uint32_t i) { return ((uint64_t)prev_turn[i] << 32) | i; };
                auto knew = [&](uint32_t i) { return key[i]; };
                std::vector<uint8_t> dirty(u, 0);
                uint32_t c0 = 0;
                for (uint32_t v = 0; v < n; ++v) {
                    for (uint32_t a = voff[v]; a < voff[v + 1]; ++a)
                        for (uint32_t b2 = a + 1; b2 < voff[v + 1]; ++b2) {
                            const uint32_t x = vl[a], y = vl[b2];
                            if ((kold(x) < kold(y)) != (knew(x) < knew(y))) {
                                c0 += !dirty[x] + !dirty[y];
                                dirty[x] = dirty[y] = 1;
                            }
                        }
                }
                std::vector<uint8_t> Q(P);  // decisions being repaired (start: the last pass's)
                std::vector<uint32_t> dl;
                for (uint32_t i = 0; i < u; ++i) if (dirty[i]) dl.push_back(i);
                uint64_t dwork = 0;
                int rounds = 0;
                while (!dl.empty()) {
                    ++rounds;
                    dwork += dl.size();
                    std::vector<std::pair<uint32_t, uint8_t>> chg;
                    for (uint32_t x : dl) {
                        bool in = true;
                        for (int j = 0; j < 3; ++j) {
                            const uint32_t v = lit[(size_t)U[x] * 3 + j] >> 1;
                            for (uint32_t a = voff[v]; a < voff[v + 1]; ++a) {
                                const uint32_t y = vl[a];
                                if (y != x && knew(y) < knew(x) && Q[y]) in = false;
                            }
                        }
                        if ((uint8_t)in != Q[x]) chg.push_back({x, (uint8_t)in});
                    }
                    for (auto& c : chg) dirty[c.first] = 0;
                    for (uint32_t x : dl) dirty[x] = 0;
                    std::vector<uint32_t> nd;
                    for (auto& c : chg) {
                        Q[c.first] = c.second;
                        const uint32_t x = c.first;
                        for (int j = 0; j < 3; ++j) {
                            const uint32_t v = lit[(size_t)U[x] * 3 + j] >> 1;
                            for (uint32_t a = voff[v]; a < voff[v + 1]; ++a) {
                                const uint32_t y = vl[a];
                                if (y != x && knew(y) > knew(x) && !dirty[y]) { dirty[y] = 1; nd.push_back(y); }
                            }
                        }
                    }
                    dl.swap(nd);
                }
                uint32_t bad = 0;
                for (uint32_t i = 0; i < u; ++i) bad += Q[i] != Pn[i];
                printf("    incremental: flips dirty %u, Jacobi rounds %d, dirty work %llu, mismatches vs full %u\n",
                       c0, rounds, (unsigned long long)dwork, bad);
            }
            const uint32_t nsteps = er.empty() ? 0 : er.back() + 1;
            if (win > 0 && passes == 1) we = (uint32_t)(win * nsteps) + 1;
            const bool last_window = win <= 0 || we >= nsteps;
            uint32_t ch = 0, tmin = ~0u, picks = 0, chw = 0;
            for (uint32_t i = 0; i < u; ++i) {
                if (turn[i] >= ws && (last_window || turn[i] < we)) ++work;
                if (!last_window && turn[i] >= we) Pn[i] = P[i];  // beyond the window: kept
                picks += Pn[i];
                if (Pn[i] != P[i]) { ++ch; tmin = std::min(tmin, turn[i]); }
            }
            (void)chw;
            printf("  pass %2d: picks %7u changed %6u earliest change at turn %8d of %8u (%.3f), first erasure %u, "
                   "turns changed %u\n", passes, picks, ch, (int)(tmin == ~0u ? -1 : (int)tmin), nsteps,
                   tmin == ~0u ? 1.0 : (double)tmin / nsteps, er.empty() ? 0 : er[0], tch);
            blocker = fblocker;
            prev_turn = turn;
            if (ch == 0 && !last_window) {  // the window's prefix is exact: the next window
                ws = we;
                we = (uint32_t)std::min<uint64_t>((uint64_t)we + (uint64_t)(win * nsteps) + 1, nsteps);
                continue;
            }
            if (ch == 0) break;
            if (win > 0 && tmin > ws) ws = tmin;  // (decisions below the earliest change are exact)
            P.swap(Pn);
            if (passes > 200) { printf("no fixpoint\n"); return 1; }
        }
        tot_passes += passes;
        uint32_t picks = 0;
        std::vector<uint32_t> cnt(T, 0);
        for (uint32_t i = 0; i < u; ++i) { picks += P[i]; cnt[setof[i]] += P[i]; }
        dens = (double)picks / u;
        for (uint32_t s = 0; s < T; ++s) set_dens[s] = sf[s + 1] > sf[s] ? (double)cnt[s] / (sf[s + 1] - sf[s]) : 0.5;
        printf("iter %u: |M| = %u, passes %d, entry work %.2f full passes\n", it, picks, passes, (double)work / u);
        // resample the MIS clauses' variables
        for (uint32_t i = 0; i < u; ++i)
            if (P[i]) for (int j = 0; j < 3; ++j) A[lit[(size_t)U[i] * 3 + j] >> 1] = rng() & 1;
    }
    printf("mean passes %.2f\n", (double)tot_passes / iters);
}
