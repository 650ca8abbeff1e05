/* TEST INFRASTRUCTURE ONLY -- CPU restatement of minimap2 (index + asm10 mapping without
 * base-level alignment), the checker for libhymet_gpu's mapping path.  See mm_oracle.c. */
#ifndef MM_ORACLE_H
#define MM_ORACLE_H
#include <stdint.h>

typedef struct { uint64_t x, y; } mmo128_t;

typedef struct {
    int32_t mid_occ;          /* set from the index (mm_idx_cal_max_occ + clamps) when <= 0 */
    float mid_occ_frac;       /* 2e-4 */
    int32_t min_mid_occ, max_mid_occ;  /* asm: 50, 500 */
    float q_occ_frac;         /* 0.01 */
    int32_t max_max_occ, occ_dist;     /* 4095, 500 */
    int32_t min_cnt, min_chain_score;  /* 3, 40 */
    int32_t bw, bw_long, max_gap, max_chain_skip;  /* 1000, 100000, 10000, 25 */
    int32_t rmq_inner_dist, rmq_size_cap, rmq_rescue_size;  /* 1000, 100000, 1000 */
    float rmq_rescue_ratio;   /* 0.1 */
    float chain_gap_scale, chain_skip_scale;  /* 0.8, 0.0 */
    float mask_level, pri_ratio, alt_drop;    /* 0.5, 0.8, 0.15 */
    int32_t mask_len, best_n, a, b, seed;     /* INT_MAX, 50, 1, 9, 11 */
} mmo_opt_t;

typedef struct {
    int32_t qs, qe, rs, re, rid, rev;
    int32_t mlen, blen, mapq, cnt, score, subsc, parent, id, n_sub, strand_retained;
    float div;
    int32_t as;   /* first anchor (internal) */
    uint32_t hash;
    int32_t pad;
} mmo_reg_t;

#endif
