/* alll_oracle.h -- TEST INFRASTRUCTURE ONLY (see alll_oracle.c header). */
#ifndef ALLL_ORACLE_H
#define ALLL_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_stats {
    uint64_t n_iterations;
    uint64_t n_resamples;
    uint64_t avg_mis_size;
    uint64_t sum_mis_size;
    uint64_t last_violated;
    int32_t solved;
    int32_t pad;
} orc_stats;

typedef void (*orc_iter_cb)(void* user, uint64_t n_iter, uint64_t n_violated, uint64_t n_mis,
                            uint64_t d_resamples, const uint32_t* A);

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void orc_init_assignment(uint64_t seed, uint32_t n_vars, uint32_t* A);
uint32_t orc_resample_bit(uint64_t seed, uint64_t iter, uint32_t v);
int orc_generate_ksat(uint64_t gen_seed, uint32_t n_vars, uint64_t n_clauses, uint32_t k, int kind,
                      uint64_t c_begin, uint64_t c_end, uint32_t* lits);
int orc_clause_violated(const uint64_t* offs, const uint32_t* lits, const uint32_t* A, uint64_t c);
uint64_t orc_eval(uint64_t m, const uint64_t* offs, const uint32_t* lits, const uint32_t* A,
                  uint64_t* vmask);
uint64_t orc_mask_to_list(uint64_t m, const uint64_t* vmask, uint32_t* U);
uint64_t orc_lfmis(uint32_t n_vars, const uint64_t* offs, const uint32_t* lits, const uint32_t* U,
                   uint64_t nu, uint32_t* M, uint8_t* scratch_used);
void orc_chunk_bounds(uint64_t m, uint32_t T, uint64_t* starts);
uint64_t orc_rr_mis(uint32_t n_vars, const uint64_t* offs, const uint32_t* lits, const uint32_t* U,
                    uint64_t nu, uint32_t T, const uint64_t* chunk_starts, uint32_t* M,
                    uint8_t* scratch_used);
/* the reference's own RNG (reference-RNG mode): random_device stand-in, RBG<minstd_rand0> */
typedef struct { uint64_t x, m; } orc_rbg;
uint32_t orc_refrng_rd_next(uint64_t* state);
void orc_rbg_seed(orc_rbg* g, uint32_t seed);
uint32_t orc_rbg_sample(orc_rbg* g);
void orc_refrng_init(uint64_t* rd_state, uint32_t n_vars, uint32_t* A);
int orc_solve_refrng(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
                     uint64_t rd_seed, uint64_t max_iters, uint32_t* A, orc_stats* st,
                     orc_iter_cb cb, void* cb_user);
int orc_solve_stream_refrng(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits,
                            uint64_t rd_seed, uint64_t max_iters, uint64_t batch, uint32_t* A, orc_stats* st,
                            orc_iter_cb cb, void* cb_user);
int orc_solve(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
              uint64_t max_iters, uint32_t* A, orc_stats* st, orc_iter_cb cb, void* cb_user);
int orc_solve_rr(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
                 uint64_t max_iters, uint32_t T, const uint64_t* chunk_starts, uint32_t* A, orc_stats* st,
                 orc_iter_cb cb, void* cb_user);
void orc_stream_order(uint64_t m, uint32_t* order);
int orc_solve_stream(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
                     uint64_t max_iters, uint64_t batch, uint32_t* A, orc_stats* st, orc_iter_cb cb,
                     void* cb_user);
int orc_solve_stream_rr(uint32_t n_vars, uint64_t m, const uint64_t* offs, const uint32_t* lits, uint64_t seed,
                        uint64_t max_iters, uint64_t batch, uint32_t T, uint64_t step_cap, uint32_t* A,
                        orc_stats* st, orc_iter_cb cb, void* cb_user);
int orc_dimacs_parse(const char* buf, uint64_t len, uint32_t* v_num, uint64_t* c_num, uint64_t* offs,
                     uint32_t* lits, uint64_t* l_num);

#ifdef __cplusplus
}
#endif
#endif
