/* TEST INFRASTRUCTURE ONLY -- CPU oracle for the align stage.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this (through
 * oracle/build/liboracle.so); the product library never links it.
 *
 * What it restates: minimap2 as the reference drives it --
 *   scripts/minimap2.sh:12  `minimap2 -I2g -d reference.mmi combined_genomes.fasta`
 *                           (default indexing: k=15, w=10, no HPC, parts of <= 2e9 bases)
 *   scripts/minimap2.sh:23  `minimap2 -x asm10 reference.mmi input/ *.fna > resultados.paf`
 *                           (asm10 mapping options, PAF without base-level alignment)
 * minimap2 is third-party (C, MIT), unpinned in environment.yml:10 and absent from the
 * container.  This file restates the published algorithm of minimap2 2.28
 * (sketch.c mm_sketch; index.c mm_idx_add/mm_idx_post/mm_idx_cal_max_occ; seed.c
 * mm_seed_mz_flt/mm_seed_collect_all/mm_seed_select/mm_collect_matches; map.c
 * collect_seed_hits/mm_map_frag/mm_est_err; lchain.c mg_lchain_rmq/mg_chain_backtrack/
 * compact_a; hit.c mm_gen_regs/mm_set_parent/mm_select_sub/mm_set_mapq/
 * mm_filter_strand_retained; format.c write_tags).
 *
 * PARITY: PINNED at set level against the real minimap2 PAF the reference ships
 * (case/truth/zymo_mc/zymo_mc_vs_refs.paf, with its 25 genomes committed under
 * tests/golden/zymo): on the 322 contigs re-cut from their primary hits this restatement
 * gives 318/322 first primaries on the same (target, strand), mapq 60 on all 278 of the
 * fixture's mapq-60 primaries, secondaries recall 71/92 and precision 76/81
 * (tests/test_zymo_real.py).  Line-level fields (s1, cm, dv, coordinates)
 * stay unpinned: minimap2 itself is absent and the fixture's query FASTA is not shipped,
 * so the re-cut queries differ from the real contigs.  The PAF tag layout and mapq formula
 * are pinned by the same fixture (tests/test_mm_oracle.py).
 * Where minimap2's result depends on the internal permutation of its unstable in-place MSD
 * radix sort or on the shape of its AVL RMQ tree, this restatement fixes a canonical order
 * (documented in DESIGN.md §Align, "canonical tie-breaks"):
 *   T1 anchors sorted by the full 128-bit (x, y) key            (radix_sort_128x on x only)
 *   T2 RMQ ties on equal priority -> the larger anchor index     (krmq_rmq, tree-shape dependent)
 *   T3 backtrack order by (f, anchor index) descending           (radix_sort_128x on f only)
 *   T4 region order by the full (score<<32|cnt^hash, as<<32|cnt) key, descending
 * The chaining itself is computed per (strand, target) group, which is exactly equivalent
 * (mg_lchain_rmq drains both trees whenever x>>32 changes).
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mm_oracle.h"

typedef mmo128_t m128;

/* ------------------------------------------------------------------ helpers */
/* minimap2 seq_nt4_table: A/C/G/T(U) in either case, everything else ambiguous */
static int nt4_code(unsigned char c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': case 'U': case 'u': return 3;
    default: return 4;
    }
}

static inline uint64_t hash64m(uint64_t key, uint64_t mask) { /* sketch.c hash64 */
    key = (~key + (key << 21)) & mask;
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8)) & mask;
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4)) & mask;
    key = key ^ key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}
static inline uint64_t hash64(uint64_t key) { /* hit.c hash64 (Thomas Wang) */
    key = (~key + (key << 21));
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8));
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4));
    key = key ^ key >> 28;
    key = (key + (key << 31));
    return key;
}
static inline uint32_t wang32(uint32_t key) { /* khash __ac_Wang_hash */
    key += ~(key << 15);
    key ^= (key >> 10);
    key += (key << 3);
    key ^= (key >> 6);
    key += ~(key << 11);
    key ^= (key >> 16);
    return key;
}
static inline uint32_t x31_hash(const char *s) { /* khash __ac_X31_hash_string */
    uint32_t h = (uint32_t)(signed char)*s;
    if (h)
        for (++s; *s; ++s) h = (h << 5) - h + (uint32_t)(signed char)*s;
    return h;
}

static int cmp128(const void *pa, const void *pb) {
    const m128 *a = (const m128 *)pa, *b = (const m128 *)pb;
    if (a->x != b->x) return a->x < b->x ? -1 : 1;
    if (a->y != b->y) return a->y < b->y ? -1 : 1;
    return 0;
}
static int cmpu64(const void *pa, const void *pb) {
    uint64_t a = *(const uint64_t *)pa, b = *(const uint64_t *)pb;
    return a < b ? -1 : a > b;
}
static int cmpu32(const void *pa, const void *pb) {
    uint32_t a = *(const uint32_t *)pa, b = *(const uint32_t *)pb;
    return a < b ? -1 : a > b;
}

typedef struct { m128 *a; int64_t n, m; } v128;
static void v128_push(v128 *v, m128 e) {
    if (v->n == v->m) { v->m = v->m ? v->m * 2 : 256; v->a = (m128 *)realloc(v->a, sizeof(m128) * (size_t)v->m); }
    v->a[v->n++] = e;
}

/* ---------------------------------------------------------- sketch.c mm_sketch */
void mmo_sketch(const char *str, int len, int w, int k, uint32_t rid, v128 *p) {
    uint64_t shift1 = 2 * (k - 1), mask = (1ULL << 2 * k) - 1, kmer[2] = {0, 0};
    int i, j, l, buf_pos, min_pos, kmer_span = 0;
    m128 buf[256], min = {UINT64_MAX, UINT64_MAX};
    memset(buf, 0xff, w * 16);
    for (i = l = buf_pos = min_pos = 0; i < len; ++i) {
        int c = nt4_code((unsigned char)str[i]);
        m128 info = {UINT64_MAX, UINT64_MAX};
        if (c < 4) {
            int z;
            kmer_span = l + 1 < k ? l + 1 : k;
            kmer[0] = (kmer[0] << 2 | c) & mask;
            kmer[1] = (kmer[1] >> 2) | (3ULL ^ c) << shift1;
            if (kmer[0] == kmer[1]) continue; /* skip symmetric k-mers */
            z = kmer[0] < kmer[1] ? 0 : 1;
            ++l;
            if (l >= k && kmer_span < 256) {
                info.x = hash64m(kmer[z], mask) << 8 | kmer_span;
                info.y = (uint64_t)rid << 32 | (uint32_t)i << 1 | z;
            }
        } else
            l = 0, kmer_span = 0;
        buf[buf_pos] = info;
        if (l == w + k - 1 && min.x != UINT64_MAX) { /* first window: identical k-mers */
            for (j = buf_pos + 1; j < w; ++j)
                if (min.x == buf[j].x && buf[j].y != min.y) v128_push(p, buf[j]);
            for (j = 0; j < buf_pos; ++j)
                if (min.x == buf[j].x && buf[j].y != min.y) v128_push(p, buf[j]);
        }
        if (info.x <= min.x) {
            if (l >= w + k && min.x != UINT64_MAX) v128_push(p, min);
            min = info, min_pos = buf_pos;
        } else if (buf_pos == min_pos) {
            if (l >= w + k - 1 && min.x != UINT64_MAX) v128_push(p, min);
            for (j = buf_pos + 1, min.x = UINT64_MAX; j < w; ++j)
                if (min.x >= buf[j].x) min = buf[j], min_pos = j;
            for (j = 0; j <= buf_pos; ++j)
                if (min.x >= buf[j].x) min = buf[j], min_pos = j;
            if (l >= w + k - 1 && min.x != UINT64_MAX) {
                for (j = buf_pos + 1; j < w; ++j)
                    if (min.x == buf[j].x && min.y != buf[j].y) v128_push(p, buf[j]);
                for (j = 0; j <= buf_pos; ++j)
                    if (min.x == buf[j].x && min.y != buf[j].y) v128_push(p, buf[j]);
            }
        }
        if (++buf_pos == w) buf_pos = 0;
    }
    if (min.x != UINT64_MAX) v128_push(p, min);
}

/* exported for tests: minimizers of one sequence */
int64_t mmo_sketch_seq(const char *s, int len, int w, int k, uint32_t rid, m128 *out, int64_t cap) {
    v128 v = {0, 0, 0};
    mmo_sketch(s, len, w, k, rid, &v);
    int64_t n = v.n;
    if (n <= cap) memcpy(out, v.a, sizeof(m128) * (size_t)n);
    free(v.a);
    return n <= cap ? n : -n;
}

/* ------------------------------------------------------------------- index */
typedef struct {
    int w, k, n_seq;
    int64_t *len;        /* per sequence */
    int64_t n_keys;
    uint64_t *keys;      /* sorted distinct minimizer hashes (x>>8) */
    int64_t *koff;       /* n_keys+1 offsets into pos */
    uint64_t *pos;       /* y values, sorted per key (rid<<32 | pos<<1 | strand) */
} mmo_idx_t;

/* index.c: mm_idx_add pushes every minimizer; mm_idx_post sorts by x, groups by x>>8 and
 * sorts each position list by y (radix_sort_64) -- the final content is order-free. */
mmo_idx_t *mmo_idx_build(const char *buf, const int64_t *starts, const int64_t *lens, int n_seq, int w, int k) {
    mmo_idx_t *mi = (mmo_idx_t *)calloc(1, sizeof(mmo_idx_t));
    mi->w = w, mi->k = k, mi->n_seq = n_seq;
    mi->len = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_seq + 1));
    v128 v = {0, 0, 0};
    for (int i = 0; i < n_seq; i++) {
        mi->len[i] = lens[i];
        if (lens[i] > 0) mmo_sketch(buf + starts[i], (int)lens[i], w, k, (uint32_t)i, &v);
    }
    for (int64_t i = 0; i < v.n; i++) v.a[i].x >>= 8; /* key = hash (span dropped) */
    qsort(v.a, (size_t)v.n, sizeof(m128), cmp128);
    int64_t nk = 0;
    for (int64_t i = 0; i < v.n; i++)
        if (i == 0 || v.a[i].x != v.a[i - 1].x) nk++;
    mi->n_keys = nk;
    mi->keys = (uint64_t *)malloc(8 * (size_t)(nk + 1));
    mi->koff = (int64_t *)malloc(8 * (size_t)(nk + 1));
    mi->pos = (uint64_t *)malloc(8 * (size_t)(v.n + 1));
    int64_t j = 0;
    for (int64_t i = 0; i < v.n; i++) {
        if (i == 0 || v.a[i].x != v.a[i - 1].x) { mi->keys[j] = v.a[i].x; mi->koff[j] = i; j++; }
        mi->pos[i] = v.a[i].y;
    }
    mi->koff[nk] = v.n;
    free(v.a);
    return mi;
}

/* an index from already sorted (key, positions) arrays -- e.g. exported by the device
 * index after tests/test_mm_index_gpu.py proved the two identical -- so that a CPU
 * baseline need not re-sketch gigabases of references single-threaded */
mmo_idx_t *mmo_idx_from_arrays(const uint64_t *keys, const int64_t *koff, int64_t n_keys, const uint64_t *pos,
                               const int64_t *lens, int n_seq, int w, int k) {
    mmo_idx_t *mi = (mmo_idx_t *)calloc(1, sizeof(mmo_idx_t));
    mi->w = w, mi->k = k, mi->n_seq = n_seq, mi->n_keys = n_keys;
    mi->len = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_seq + 1));
    memcpy(mi->len, lens, sizeof(int64_t) * (size_t)n_seq);
    mi->keys = (uint64_t *)malloc(8 * (size_t)(n_keys + 1));
    mi->koff = (int64_t *)malloc(8 * (size_t)(n_keys + 1));
    mi->pos = (uint64_t *)malloc(8 * (size_t)(koff[n_keys] + 1));
    memcpy(mi->keys, keys, 8 * (size_t)n_keys);
    memcpy(mi->koff, koff, 8 * (size_t)(n_keys + 1));
    memcpy(mi->pos, pos, 8 * (size_t)koff[n_keys]);
    return mi;
}

void mmo_idx_destroy(mmo_idx_t *mi) {
    if (!mi) return;
    free(mi->len); free(mi->keys); free(mi->koff); free(mi->pos); free(mi);
}

int64_t mmo_idx_n_keys(const mmo_idx_t *mi) { return mi->n_keys; }
int64_t mmo_idx_n_pos(const mmo_idx_t *mi) { return mi->koff[mi->n_keys]; }
void mmo_idx_export(const mmo_idx_t *mi, uint64_t *keys, int64_t *koff, uint64_t *pos) {
    memcpy(keys, mi->keys, 8 * (size_t)mi->n_keys);
    memcpy(koff, mi->koff, 8 * (size_t)(mi->n_keys + 1));
    memcpy(pos, mi->pos, 8 * (size_t)mi->koff[mi->n_keys]);
}

static const uint64_t *idx_get(const mmo_idx_t *mi, uint64_t key, int *n) {
    int64_t lo = 0, hi = mi->n_keys - 1;
    *n = 0;
    while (lo <= hi) {
        int64_t m = (lo + hi) >> 1;
        if (mi->keys[m] < key) lo = m + 1;
        else if (mi->keys[m] > key) hi = m - 1;
        else { *n = (int)(mi->koff[m + 1] - mi->koff[m]); return mi->pos + mi->koff[m]; }
    }
    return 0;
}

/* index.c mm_idx_cal_max_occ: (ks_ksmall of per-key counts at (1-f)*n) + 1 */
int32_t mmo_idx_cal_max_occ(const mmo_idx_t *mi, float f) {
    if (f <= 0.) return INT32_MAX;
    size_t n = (size_t)mi->n_keys;
    if (n == 0) return INT32_MAX;
    uint32_t *a = (uint32_t *)malloc(4 * n);
    for (size_t i = 0; i < n; i++) a[i] = (uint32_t)(mi->koff[i + 1] - mi->koff[i]);
    qsort(a, n, 4, cmpu32);
    size_t kk = (size_t)(uint32_t)((1. - f) * n);
    if (kk >= n) kk = n - 1;
    uint32_t t = a[kk] + 1;
    free(a);
    return (int32_t)t;
}

/* options.c mm_mapopt_init + mm_set_opt("asm10") + mm_mapopt_update */
void mmo_opt_asm10(mmo_opt_t *o) {
    memset(o, 0, sizeof(*o));
    o->mid_occ = 0;
    o->mid_occ_frac = 2e-4f;
    o->min_mid_occ = 50, o->max_mid_occ = 500;
    o->q_occ_frac = 0.01f;
    o->max_max_occ = 4095, o->occ_dist = 500;
    o->min_cnt = 3, o->min_chain_score = 40;
    o->bw = 1000, o->bw_long = 100000;
    o->max_gap = 10000, o->max_chain_skip = 25;
    o->rmq_inner_dist = 1000, o->rmq_size_cap = 100000, o->rmq_rescue_size = 1000;
    o->rmq_rescue_ratio = 0.1f;
    o->chain_gap_scale = 0.8f, o->chain_skip_scale = 0.0f;
    o->mask_level = 0.5f, o->pri_ratio = 0.8f, o->alt_drop = 0.15f;
    o->mask_len = INT_MAX, o->best_n = 50, o->a = 1, o->b = 9, o->seed = 11;
}

int32_t mmo_opt_update_mid_occ(mmo_opt_t *o, const mmo_idx_t *mi) {
    if (o->mid_occ <= 0) {
        o->mid_occ = mmo_idx_cal_max_occ(mi, o->mid_occ_frac);
        if (o->mid_occ < o->min_mid_occ) o->mid_occ = o->min_mid_occ;
        if (o->max_mid_occ > o->min_mid_occ && o->mid_occ > o->max_mid_occ) o->mid_occ = o->max_mid_occ;
    }
    if (o->bw_long < o->bw) o->bw_long = o->bw;
    return o->mid_occ;
}

/* ------------------------------------------------------------------- seeds */
typedef struct {
    uint32_t n, q_pos, q_span, flt, seg_id, is_tandem;
    const uint64_t *cr;
} seed_t;

/* seed.c mm_seed_mz_flt: drop query minimizers over-represented in the query itself */
static void seed_mz_flt(v128 *mv, int32_t q_occ_max, float q_occ_frac) {
    if (mv->n <= q_occ_max || q_occ_frac <= 0.0f || q_occ_max <= 0) return;
    m128 *a = (m128 *)malloc(sizeof(m128) * (size_t)mv->n);
    for (int64_t i = 0; i < mv->n; i++) a[i].x = mv->a[i].x, a[i].y = (uint64_t)i;
    qsort(a, (size_t)mv->n, sizeof(m128), cmp128);
    for (int64_t st = 0, i = 1; i <= mv->n; ++i) {
        if (i == mv->n || a[i].x != a[st].x) {
            int32_t cnt = (int32_t)(i - st);
            if (cnt > q_occ_max && cnt > mv->n * q_occ_frac)
                for (int64_t j = st; j < i; ++j) mv->a[a[j].y].x = 0;
            st = i;
        }
    }
    free(a);
    int64_t j = 0;
    for (int64_t i = 0; i < mv->n; ++i)
        if (mv->a[i].x != 0) mv->a[j++] = mv->a[i];
    mv->n = j;
}

/* seed.c mm_seed_select: in each streak of high-occurrence seeds keep the
 * max_high_occ least frequent ones (ties: earlier index) */
static void seed_select(int32_t n, seed_t *a, int len, int max_occ, int max_max_occ, int dist) {
    int32_t i, last0, m;
    if (n == 0 || n == 1) return;
    for (i = m = 0; i < n; ++i)
        if ((int)a[i].n > max_occ) ++m;
    if (m == 0) return;
    for (i = 0, last0 = -1; i <= n; ++i) {
        if (i == n || (int)a[i].n <= max_occ) {
            if (i - last0 > 1) {
                int32_t ps = last0 < 0 ? 0 : (int32_t)(a[last0].q_pos >> 1);
                int32_t pe = i == n ? len : (int32_t)(a[i].q_pos >> 1);
                int32_t st = last0 + 1, en = i, j, k;
                int32_t max_high_occ = (int32_t)((double)(pe - ps) / dist + .499);
                if (max_high_occ > 0) {
                    if (max_high_occ > 128) max_high_occ = 128;
                    /* choose the max_high_occ smallest (n, j) -- what the binary heap keeps */
                    int32_t cnt = en - st;
                    uint64_t *b = (uint64_t *)malloc(8 * (size_t)cnt);
                    for (j = st, k = 0; j < en; ++j, ++k) b[k] = (uint64_t)a[j].n << 32 | (uint32_t)j;
                    qsort(b, (size_t)cnt, 8, cmpu64);
                    int32_t keep = cnt < max_high_occ ? cnt : max_high_occ;
                    for (k = 0; k < keep; ++k) a[(uint32_t)b[k]].flt = 1;
                    free(b);
                }
                for (j = st; j < en; ++j) a[j].flt ^= 1;
                for (j = st; j < en; ++j)
                    if ((int)a[j].n > max_max_occ) a[j].flt = 1;
            }
            last0 = i;
        }
    }
}

/* seed.c mm_collect_matches + map.c collect_seed_hits (anchors sorted, T1) */
static m128 *collect_anchors(const mmo_opt_t *opt, int max_occ, const mmo_idx_t *mi, const v128 *mv, int qlen,
                             int64_t *n_a, int *rep_len, int *n_mini_pos, uint64_t **mini_pos) {
    seed_t *m = (seed_t *)calloc((size_t)(mv->n + 1), sizeof(seed_t));
    int32_t n_m0 = 0, n_m = 0;
    *mini_pos = (uint64_t *)malloc(8 * (size_t)(mv->n + 1));
    *n_mini_pos = 0;
    for (int64_t i = 0; i < mv->n; ++i) {
        const m128 *p = &mv->a[i];
        int t;
        const uint64_t *cr = idx_get(mi, p->x >> 8, &t);
        if (t == 0) continue;
        seed_t *q = &m[n_m0++];
        q->q_pos = (uint32_t)p->y, q->q_span = p->x & 0xff, q->cr = cr, q->n = (uint32_t)t, q->seg_id = (uint32_t)(p->y >> 32);
        q->is_tandem = q->flt = 0;
        if (i > 0 && p->x >> 8 == mv->a[i - 1].x >> 8) q->is_tandem = 1;
        if (i < mv->n - 1 && p->x >> 8 == mv->a[i + 1].x >> 8) q->is_tandem = 1;
    }
    if (opt->occ_dist > 0 && opt->max_max_occ > max_occ)
        seed_select(n_m0, m, qlen, max_occ, opt->max_max_occ, opt->occ_dist);
    else
        for (int32_t i = 0; i < n_m0; ++i)
            if ((int)m[i].n > max_occ) m[i].flt = 1;
    int rep_st = 0, rep_en = 0;
    *rep_len = 0, *n_a = 0;
    for (int32_t i = 0; i < n_m0; ++i) {
        seed_t *q = &m[i];
        if (q->flt) {
            int en = (q->q_pos >> 1) + 1, st = en - q->q_span;
            if (st > rep_en) { *rep_len += rep_en - rep_st; rep_st = st, rep_en = en; }
            else rep_en = en;
        } else {
            *n_a += q->n;
            (*mini_pos)[(*n_mini_pos)++] = (uint64_t)q->q_span << 32 | q->q_pos >> 1;
            m[n_m++] = *q;
        }
    }
    *rep_len += rep_en - rep_st;
    m128 *a = (m128 *)malloc(sizeof(m128) * (size_t)(*n_a + 1));
    int64_t k = 0;
    for (int32_t i = 0; i < n_m; ++i) {
        seed_t *q = &m[i];
        for (uint32_t j = 0; j < q->n; ++j) {
            uint64_t r = q->cr[j];
            int32_t rpos = (uint32_t)r >> 1;
            m128 *p = &a[k++];
            if ((r & 1) == (q->q_pos & 1)) {
                p->x = (r & 0xffffffff00000000ULL) | (uint32_t)rpos;
                p->y = (uint64_t)q->q_span << 32 | q->q_pos >> 1;
            } else {
                p->x = 1ULL << 63 | (r & 0xffffffff00000000ULL) | (uint32_t)rpos;
                p->y = (uint64_t)q->q_span << 32 | (uint32_t)(qlen - ((q->q_pos >> 1) + 1 - q->q_span) - 1);
            }
        }
    }
    free(m);
    qsort(a, (size_t)*n_a, sizeof(m128), cmp128);
    return a;
}

/* ------------------------------------------------------------ lchain.c RMQ chaining */
static inline float mg_log2(float x) {
    union { float f; uint32_t i; } z = {x};
    float log_2 = ((z.i >> 23) & (int)(0xff)) - 128;
    z.i &= ~(255 << 23);
    z.i += 127 << 23;
    log_2 += (-0.34484843f * z.f + 2.02466578f) * z.f - 0.67487759f;
    return log_2;
}

static inline int32_t comput_sc_simple(const m128 *ai, const m128 *aj, float chn_pen_gap, float chn_pen_skip,
                                       int32_t *exact, int32_t *width) {
    int32_t dq = (int32_t)ai->y - (int32_t)aj->y, dr, dd, dg, q_span, sc;
    dr = (int32_t)(ai->x - aj->x);
    *width = dd = dr > dq ? dr - dq : dq - dr;
    dg = dr < dq ? dr : dq;
    q_span = aj->y >> 32 & 0xff;
    sc = q_span < dg ? q_span : dg;
    if (exact) *exact = (dd == 0 && dg <= q_span);
    if (dd || dq > q_span) {
        float lin_pen, log_pen;
        lin_pen = chn_pen_gap * (float)dd + chn_pen_skip * (float)dg;
        log_pen = dd >= 1 ? mg_log2(dd + 1) : 0.0f;
        sc -= (int)(lin_pen + .5f * log_pen);
    }
    return sc;
}

typedef struct { double pri; int64_t i; } rmq_node;
static inline int rmq_better(rmq_node a, rmq_node b) { /* T2: min pri, ties -> larger index */
    if (a.i < 0) return 0;
    if (b.i < 0) return 1;
    if (a.pri != b.pri) return a.pri < b.pri;
    return a.i > b.i;
}

typedef struct { int32_t y; int64_t i; } yi_t;
static int cmp_yi(const void *pa, const void *pb) {
    const yi_t *a = (const yi_t *)pa, *b = (const yi_t *)pb;
    if (a->y != b->y) return a->y < b->y ? -1 : 1;
    return (a->i > b->i) - (a->i < b->i);
}
/* number of elements e in sorted[0..n) with (e.y, e.i) <= (y, i) */
static int64_t count_le(const yi_t *s, int64_t n, int32_t y, int64_t i) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t m = (lo + hi) >> 1;
        if (s[m].y < y || (s[m].y == y && s[m].i <= i)) lo = m + 1;
        else hi = m;
    }
    return lo;
}

/* mg_lchain_rmq over one (strand, target) group [g0, g1) of the x-sorted anchors */
static void chain_group(int64_t g0, int64_t g1, const m128 *a, int max_dist, int max_dist_inner, int bw, int max_chn_skip,
                        int cap_rmq_size, float chn_pen_gap, float chn_pen_skip, int32_t *f, int64_t *p, int32_t *v,
                        int32_t *t) {
    int64_t n = g1 - g0, P = 1;
    while (P < n) P <<= 1;
    yi_t *srt = (yi_t *)malloc(sizeof(yi_t) * (size_t)n);
    int64_t *rank = (int64_t *)malloc(8 * (size_t)n);
    for (int64_t j = 0; j < n; j++) srt[j].y = (int32_t)a[g0 + j].y, srt[j].i = g0 + j;
    qsort(srt, (size_t)n, sizeof(yi_t), cmp_yi);
    for (int64_t r = 0; r < n; r++) rank[srt[r].i - g0] = r;
    rmq_node *tr = (rmq_node *)malloc(sizeof(rmq_node) * (size_t)(2 * P));
    for (int64_t j = 0; j < 2 * P; j++) tr[j].i = -1, tr[j].pri = 0;
    char *in_inner = (char *)calloc((size_t)n, 1);
    int64_t size_outer = 0, size_inner = 0;
    int64_t i0 = g0, st = g0, st_inner = g0;
    for (int64_t i = g0; i < g1; ++i) {
        int64_t max_j = -1;
        int32_t q_span = a[i].y >> 32 & 0xff, max_f = q_span;
        if (i0 < i && a[i0].x != a[i].x) {
            for (int64_t j = i0; j < i; ++j) {
                int64_t leaf = P + rank[j - g0];
                tr[leaf].i = j;
                tr[leaf].pri = -(f[j] + 0.5 * chn_pen_gap * ((int32_t)a[j].x + (int32_t)a[j].y));
                for (int64_t u = leaf >> 1; u >= 1; u >>= 1) tr[u] = rmq_better(tr[2 * u], tr[2 * u + 1]) ? tr[2 * u] : tr[2 * u + 1];
                size_outer++;
                if (max_dist_inner > 0) in_inner[j - g0] = 1, size_inner++;
            }
            i0 = i;
        }
        while (st < i && (a[i].x > a[st].x + max_dist || size_outer > cap_rmq_size)) {
            if (st < i0) {
                int64_t leaf = P + rank[st - g0];
                tr[leaf].i = -1;
                for (int64_t u = leaf >> 1; u >= 1; u >>= 1) tr[u] = rmq_better(tr[2 * u], tr[2 * u + 1]) ? tr[2 * u] : tr[2 * u + 1];
                size_outer--;
            }
            ++st;
        }
        if (max_dist_inner > 0) {
            while (st_inner < i && (a[i].x > a[st_inner].x + max_dist_inner || size_inner > cap_rmq_size)) {
                if (st_inner < i0) in_inner[st_inner - g0] = 0, size_inner--;
                ++st_inner;
            }
        }
        /* RMQ over (y_i - max_dist, INT32_MAX) .. (y_i, 0) in (y, i) order */
        int32_t yi = (int32_t)a[i].y;
        int64_t lo = count_le(srt, n, yi - max_dist, INT32_MAX);
        int64_t hi = count_le(srt, n, yi, 0) - 1;
        rmq_node best = {0, -1};
        if (lo <= hi && size_outer > 0) {
            int64_t l = lo + P, r = hi + P + 1;
            while (l < r) {
                if (l & 1) { if (rmq_better(tr[l], best)) best = tr[l]; l++; }
                if (r & 1) { --r; if (rmq_better(tr[r], best)) best = tr[r]; }
                l >>= 1, r >>= 1;
            }
        }
        if (best.i >= 0) {
            int32_t sc, exact, width, n_skip = 0;
            int64_t j = best.i;
            sc = f[j] + comput_sc_simple(&a[i], &a[j], chn_pen_gap, chn_pen_skip, &exact, &width);
            if (width <= bw && sc > max_f) max_f = sc, max_j = j;
            if (!exact && size_inner > 0 && yi > 0) {
                int64_t r = count_le(srt, n, yi - 1, INT64_MAX) - 1;
                for (; r >= 0; --r) {
                    if (srt[r].y < yi - max_dist_inner) break;
                    int64_t jj = srt[r].i;
                    if (!in_inner[jj - g0]) continue;
                    int32_t w2;
                    sc = f[jj] + comput_sc_simple(&a[i], &a[jj], chn_pen_gap, chn_pen_skip, 0, &w2);
                    if (w2 <= bw) {
                        if (sc > max_f) {
                            max_f = sc, max_j = jj;
                            if (n_skip > 0) --n_skip;
                        } else if (t[jj] == (int32_t)i) {
                            if (++n_skip > max_chn_skip) break;
                        }
                        if (p[jj] >= 0) t[p[jj]] = (int32_t)i;
                    }
                }
            }
        }
        f[i] = max_f, p[i] = max_j;
        v[i] = max_j >= 0 && v[max_j] > max_f ? v[max_j] : max_f;
    }
    free(srt); free(rank); free(tr); free(in_inner);
}

/* lchain.c mg_chain_bk_end */
static int64_t chain_bk_end(int32_t max_drop, const m128 *z, const int32_t *f, const int64_t *p, int32_t *t, int64_t k) {
    int64_t i = z[k].y, end_i = -1, max_i = i;
    int32_t max_s = 0;
    if (i < 0 || t[i] != 0) return i;
    do {
        int32_t s;
        t[i] = 2;
        end_i = i = p[i];
        s = i < 0 ? (int32_t)z[k].x : (int32_t)z[k].x - f[i];
        if (s > max_s) max_s = s, max_i = i;
        else if (max_s - s > max_drop) break;
    } while (i >= 0 && t[i] == 0);
    for (i = z[k].y; i >= 0 && i != end_i; i = p[i]) t[i] = 0;
    return max_i;
}

typedef struct { uint64_t u; int64_t first; int64_t *ids; } chain_t;  /* ids: anchor indices start->end */

/* lchain.c mg_chain_backtrack restricted to one group (chains never cross groups); T3 order */
static void backtrack_group(int64_t g0, int64_t g1, const int32_t *f, const int64_t *p, int32_t *t, int min_cnt, int min_sc,
                            int max_drop, chain_t **chains, int64_t *n_ch, int64_t *m_ch) {
    int64_t n_z = 0;
    for (int64_t i = g0; i < g1; ++i)
        if (f[i] >= min_sc) ++n_z;
    if (n_z == 0) return;
    m128 *z = (m128 *)malloc(sizeof(m128) * (size_t)n_z);
    int64_t k = 0;
    for (int64_t i = g0; i < g1; ++i)
        if (f[i] >= min_sc) z[k].x = (uint64_t)f[i], z[k++].y = (uint64_t)i;
    qsort(z, (size_t)n_z, sizeof(m128), cmp128);
    for (int64_t i = g0; i < g1; ++i) t[i] = 0;
    int64_t *tmp = (int64_t *)malloc(8 * (size_t)(g1 - g0 + 1));
    for (k = n_z - 1; k >= 0; --k) {
        if (t[z[k].y] == 0) {
            int64_t end_i = chain_bk_end(max_drop, z, f, p, t, k), i, nv = 0;
            for (i = (int64_t)z[k].y; i != end_i; i = p[i]) tmp[nv++] = i, t[i] = 1;
            int32_t sc = i < 0 ? (int32_t)z[k].x : (int32_t)z[k].x - f[i];
            if (sc >= min_sc && nv > 0 && nv >= min_cnt) {
                if (*n_ch == *m_ch) { *m_ch = *m_ch ? *m_ch * 2 : 64; *chains = (chain_t *)realloc(*chains, sizeof(chain_t) * (size_t)*m_ch); }
                chain_t *c = &(*chains)[(*n_ch)++];
                c->u = (uint64_t)sc << 32 | (uint32_t)nv;
                c->ids = (int64_t *)malloc(8 * (size_t)nv);
                for (int64_t q = 0; q < nv; q++) c->ids[q] = tmp[nv - 1 - q];
                c->first = c->ids[0];
            }
            /* else: rejected, the t[] marks stay set exactly as in minimap2 (n_v rolled back) */
        }
    }
    free(tmp); free(z);
}

static __thread const m128 *g_sort_a;  /* qsort context; thread-local so bench.py can map from threads */
static int cmp_chain_first(const void *pa, const void *pb) {
    const chain_t *a = (const chain_t *)pa, *b = (const chain_t *)pb;
    return cmp128(&g_sort_a[a->first], &g_sort_a[b->first]);  /* compact_a: first-anchor x (ties: y) */
}

/* full mg_lchain_rmq + backtrack + compact_a on the x-sorted anchors.  Returns the new
 * anchor array (chains concatenated, chains sorted by first-anchor x) and u[] */
static m128 *lchain_rmq(int max_dist, int max_dist_inner, int bw, int max_chn_skip, int cap_rmq_size, int min_cnt,
                        int min_sc, float chn_pen_gap, float chn_pen_skip, int64_t n, m128 *a, int *n_u_, uint64_t **u_) {
    *n_u_ = 0, *u_ = 0;
    if (n == 0 || a == 0) { free(a); return 0; }
    if (max_dist < bw) max_dist = bw;
    if (max_dist_inner <= 0 || max_dist_inner >= max_dist) max_dist_inner = 0;
    int32_t *f = (int32_t *)malloc(4 * (size_t)n), *v = (int32_t *)malloc(4 * (size_t)n), *t = (int32_t *)calloc((size_t)n, 4);
    int64_t *p = (int64_t *)malloc(8 * (size_t)n);
    chain_t *ch = 0;
    int64_t n_ch = 0, m_ch = 0;
    for (int64_t g0 = 0; g0 < n;) {
        int64_t g1 = g0 + 1;
        while (g1 < n && a[g1].x >> 32 == a[g0].x >> 32) g1++;
        chain_group(g0, g1, a, max_dist, max_dist_inner, bw, max_chn_skip, cap_rmq_size, chn_pen_gap, chn_pen_skip, f, p, v, t);
        backtrack_group(g0, g1, f, p, t, min_cnt, min_sc, bw, &ch, &n_ch, &m_ch);
        g0 = g1;
    }
    free(f); free(v); free(t); free(p);
    if (n_ch == 0) { free(a); free(ch); return 0; }
    g_sort_a = a;
    qsort(ch, (size_t)n_ch, sizeof(chain_t), cmp_chain_first);
    int64_t tot = 0;
    for (int64_t c = 0; c < n_ch; c++) tot += (int32_t)ch[c].u;
    m128 *b = (m128 *)malloc(sizeof(m128) * (size_t)tot);
    uint64_t *u = (uint64_t *)malloc(8 * (size_t)n_ch);
    int64_t k = 0;
    for (int64_t c = 0; c < n_ch; c++) {
        u[c] = ch[c].u;
        for (int64_t q = 0; q < (int32_t)ch[c].u; q++) b[k++] = a[ch[c].ids[q]];
        free(ch[c].ids);
    }
    free(ch); free(a);
    *n_u_ = (int)n_ch, *u_ = u;
    return b;
}

/* ---------------------------------------------------------------- hit.c regions */
static void reg_set_coor(mmo_reg_t *r, int32_t qlen, const m128 *a) {
    int32_t k = r->as, q_span = (int32_t)(a[k].y >> 32 & 0xff);
    r->rev = a[k].x >> 63;
    r->rid = a[k].x << 1 >> 33;
    r->rs = (int32_t)a[k].x + 1 > q_span ? (int32_t)a[k].x + 1 - q_span : 0;
    r->re = (int32_t)a[k + r->cnt - 1].x + 1;
    if (!r->rev) {
        r->qs = (int32_t)a[k].y + 1 - q_span;
        r->qe = (int32_t)a[k + r->cnt - 1].y + 1;
    } else {
        r->qs = qlen - ((int32_t)a[k + r->cnt - 1].y + 1);
        r->qe = qlen - ((int32_t)a[k].y + 1 - q_span);
    }
    /* mm_cal_fuzzy_len */
    r->mlen = r->blen = a[r->as].y >> 32 & 0xff;
    for (int i = r->as + 1; i < r->as + r->cnt; ++i) {
        int span = a[i].y >> 32 & 0xff;
        int tl = (int32_t)a[i].x - (int32_t)a[i - 1].x;
        int ql = (int32_t)a[i].y - (int32_t)a[i - 1].y;
        r->blen += tl > ql ? tl : ql;
        r->mlen += tl > span && ql > span ? span : tl < ql ? tl : ql;
    }
}

static mmo_reg_t *gen_regs(uint32_t hash, int qlen, int n_u, const uint64_t *u, const m128 *a) {
    if (n_u == 0) return 0;
    m128 *z = (m128 *)malloc(sizeof(m128) * (size_t)n_u);
    for (int i = 0, k = 0; i < n_u; ++i) {
        uint32_t h = (uint32_t)hash64((hash64(a[k].x) + hash64(a[k].y)) ^ hash);
        z[i].x = u[i] ^ h;
        z[i].y = (uint64_t)k << 32 | (int32_t)u[i];
        k += (int32_t)u[i];
    }
    qsort(z, (size_t)n_u, sizeof(m128), cmp128); /* T4 */
    for (int i = 0; i < n_u >> 1; ++i) { m128 tmp = z[i]; z[i] = z[n_u - 1 - i]; z[n_u - 1 - i] = tmp; }
    mmo_reg_t *r = (mmo_reg_t *)calloc((size_t)n_u, sizeof(mmo_reg_t));
    for (int i = 0; i < n_u; ++i) {
        mmo_reg_t *ri = &r[i];
        ri->id = i;
        ri->parent = -1;
        ri->score = (int32_t)(z[i].x >> 32);
        ri->hash = (uint32_t)z[i].x;
        ri->cnt = (int32_t)z[i].y;
        ri->as = (int32_t)(z[i].y >> 32);
        ri->div = -1.0f;
        reg_set_coor(ri, qlen, a);
    }
    free(z);
    return r;
}

static void set_parent(float mask_level, int mask_len, int n, mmo_reg_t *r, int sub_diff, float alt_diff_frac) {
    (void)sub_diff; (void)alt_diff_frac;
    if (n <= 0) return;
    for (int i = 0; i < n; ++i) r[i].id = i;
    uint64_t *cov = (uint64_t *)malloc(8 * (size_t)n);
    int *w = (int *)malloc(sizeof(int) * (size_t)n);
    int i, j, k;
    w[0] = 0, r[0].parent = 0;
    for (i = 1, k = 1; i < n; ++i) {
        mmo_reg_t *ri = &r[i];
        int si = ri->qs, ei = ri->qe, n_cov = 0, uncov_len = 0;
        for (j = 0; j < k; ++j) {
            mmo_reg_t *rp = &r[w[j]];
            int sj = rp->qs, ej = rp->qe;
            if (ej <= si || sj >= ei) continue;
            if (sj < si) sj = si;
            if (ej > ei) ej = ei;
            cov[n_cov++] = (uint64_t)sj << 32 | (uint32_t)ej;
        }
        if (n_cov == 0) goto set_parent_test;
        else {
            int x = si;
            qsort(cov, (size_t)n_cov, 8, cmpu64);
            for (int jj = 0; jj < n_cov; ++jj) {
                if ((int)(cov[jj] >> 32) > x) uncov_len += (int)(cov[jj] >> 32) - x;
                x = (int32_t)cov[jj] > x ? (int32_t)cov[jj] : x;
            }
            if (ei > x) uncov_len += ei - x;
        }
        for (j = 0; j < k; ++j) {
            mmo_reg_t *rp = &r[w[j]];
            int sj = rp->qs, ej = rp->qe, min, max, ol;
            if (ej <= si || sj >= ei) continue;
            min = ej - sj < ei - si ? ej - sj : ei - si;
            max = ej - sj > ei - si ? ej - sj : ei - si;
            ol = si < sj ? (ei < sj ? 0 : ei < ej ? ei - sj : ej - sj) : (ej < si ? 0 : ej < ei ? ej - si : ei - si);
            if ((float)ol / min - (float)uncov_len / max > mask_level && uncov_len <= mask_len) {
                int cnt_sub = 0, sci = ri->score;
                ri->parent = rp->parent;
                rp->subsc = rp->subsc > sci ? rp->subsc : sci;
                if (ri->cnt >= rp->cnt) cnt_sub = 1;
                if (cnt_sub) ++rp->n_sub;
                break;
            }
        }
    set_parent_test:
        if (j == k) w[k++] = i, ri->parent = i, ri->n_sub = 0;
    }
    free(cov); free(w);
}

static void sync_regs(int n_regs, mmo_reg_t *regs) {
    int max_id = -1;
    if (n_regs <= 0) return;
    for (int i = 0; i < n_regs; ++i) max_id = max_id > regs[i].id ? max_id : regs[i].id;
    int n_tmp = max_id + 1;
    int *tmp = (int *)malloc(sizeof(int) * (size_t)n_tmp);
    for (int i = 0; i < n_tmp; ++i) tmp[i] = -1;
    for (int i = 0; i < n_regs; ++i)
        if (regs[i].id >= 0) tmp[regs[i].id] = i;
    for (int i = 0; i < n_regs; ++i) {
        mmo_reg_t *r = &regs[i];
        r->id = i;
        if (r->parent >= 0 && tmp[r->parent] >= 0) r->parent = tmp[r->parent];
        else r->parent = -1;
    }
    free(tmp);
}

static void select_sub(float pri_ratio, int min_diff, int best_n, int check_strand, int min_strand_sc, int *n_, mmo_reg_t *r) {
    if (pri_ratio > 0.0f && *n_ > 0) {
        int i, k, n = *n_, n_2nd = 0;
        for (i = k = 0; i < n; ++i) {
            int p = r[i].parent;
            if (p == i) {
                r[k++] = r[i];
            } else if ((r[i].score >= r[p].score * pri_ratio || r[i].score + min_diff >= r[p].score) && n_2nd < best_n) {
                if (!(r[i].qs == r[p].qs && r[i].qe == r[p].qe && r[i].rid == r[p].rid && r[i].rs == r[p].rs && r[i].re == r[p].re))
                    r[k++] = r[i], ++n_2nd;
            } else if (check_strand && n_2nd < best_n && r[i].score > min_strand_sc && r[i].rev != r[p].rev) {
                r[i].strand_retained = 1;
                r[k++] = r[i], ++n_2nd;
            }
        }
        if (k != n) sync_regs(k, r);
        *n_ = k;
    }
}

static int get_mini_idx(int qlen, const m128 *a, int32_t n, const uint64_t *mini_pos) {
    int32_t x, L = 0, R = n - 1;
    x = (int32_t)a->y;
    if (a->x >> 63) x = qlen - 1 - (int32_t)a->y + (int32_t)(a->y >> 32 & 0xff) - 1;
    while (L <= R) {
        int32_t m = (int32_t)(((uint64_t)L + R) >> 1);
        int32_t y = (int32_t)mini_pos[m];
        if (y < x) L = m + 1;
        else if (y > x) R = m - 1;
        else return m;
    }
    return -1;
}

static void est_err(const int64_t *ref_len, int qlen, int n_regs, mmo_reg_t *regs, const m128 *a, int32_t n, const uint64_t *mini_pos) {
    uint64_t sum_k = 0;
    if (n == 0) return;
    for (int i = 0; i < n; ++i) sum_k += mini_pos[i] >> 32 & 0xff;
    float avg_k = (float)sum_k / n;
    for (int i = 0; i < n_regs; ++i) {
        mmo_reg_t *r = &regs[i];
        int32_t st, en, j, k, n_match, n_tot, l_ref;
        r->div = -1.0f;
        if (r->cnt == 0) continue;
        st = en = get_mini_idx(qlen, r->rev ? &a[r->as + r->cnt - 1] : &a[r->as], n, mini_pos);
        if (st < 0) continue;
        l_ref = (int32_t)ref_len[r->rid];
        for (k = 1, j = st + 1, n_match = 1; j < n && k < r->cnt; ++j) {
            int32_t x = get_mini_idx(qlen, r->rev ? &a[r->as + r->cnt - 1 - k] : &a[r->as + k], n, mini_pos);
            if (x == j) ++k, ++n_match;
            en = j;
        }
        n_tot = en - st + 1;
        if (r->qs > avg_k && r->rs > avg_k) ++n_tot;
        if (qlen - r->qe > avg_k && l_ref - r->re > avg_k) ++n_tot;
        r->div = n_match >= n_tot ? 0.0f : (float)(1.0 - pow((double)n_match / n_tot, 1.0 / avg_k));
    }
}

static int filter_strand_retained(int n_regs, mmo_reg_t *r) {
    int i, k;
    for (i = k = 0; i < n_regs; ++i) {
        int p = r[i].parent;
        if (!r[i].strand_retained || r[i].div < r[p].div * 5.0f || r[i].div < 0.01f) {
            if (k < i) r[k++] = r[i];
            else ++k;
        }
    }
    return k;
}

static void set_mapq(int n_regs, mmo_reg_t *regs, int min_chain_sc, int rep_len) {
    static const float q_coef = 40.0f;
    int64_t sum_sc = 0;
    if (n_regs == 0) return;
    for (int i = 0; i < n_regs; ++i)
        if (regs[i].parent == regs[i].id) sum_sc += regs[i].score;
    float uniq_ratio = (float)sum_sc / (sum_sc + rep_len);
    for (int i = 0; i < n_regs; ++i) {
        mmo_reg_t *r = &regs[i];
        if (r->parent == r->id) {
            int mapq, subsc;
            float pen_s1 = (r->score > 100 ? 1.0f : 0.01f * r->score) * uniq_ratio;
            float pen_cm = r->cnt > 10 ? 1.0f : 0.1f * r->cnt;
            pen_cm = pen_s1 < pen_cm ? pen_s1 : pen_cm;
            subsc = r->subsc > min_chain_sc ? r->subsc : min_chain_sc;
            float x = (float)subsc / r->score;
            mapq = (int)(pen_cm * q_coef * (1.0f - x) * logf(r->score));
            mapq -= (int)(4.343f * logf(r->n_sub + 1) + .499f);
            mapq = mapq > 0 ? mapq : 0;
            r->mapq = mapq < 60 ? mapq : 60;
        } else
            r->mapq = 0;
    }
}

/* map.c mm_map_frag for one single-segment query against one index part.
 * Writes up to cap regions to out[]; returns the region count (negative if cap too small). */
int mmo_map(const mmo_idx_t *mi, const mmo_opt_t *opt, const char *qseq, int qlen, const char *qname,
            mmo_reg_t *out, int cap, int *rep_len_out) {
    int rep_len = 0, n_mini_pos = 0, n_regs0 = 0;
    uint64_t *mini_pos = 0, *u = 0;
    int64_t n_a = 0;
    *rep_len_out = 0;
    if (qlen == 0) return 0;
    uint32_t hash = qname ? x31_hash(qname) : 0;
    hash ^= wang32((uint32_t)qlen) + wang32((uint32_t)opt->seed);
    hash = wang32(hash);
    v128 mv = {0, 0, 0};
    mmo_sketch(qseq, qlen, mi->w, mi->k, 0, &mv);
    if (opt->q_occ_frac > 0.0f) seed_mz_flt(&mv, opt->mid_occ, opt->q_occ_frac);
    m128 *a = collect_anchors(opt, opt->mid_occ, mi, &mv, qlen, &n_a, &rep_len, &n_mini_pos, &mini_pos);
    free(mv.a);
    float chn_pen_gap = opt->chain_gap_scale * 0.01 * mi->k;
    float chn_pen_skip = opt->chain_skip_scale * 0.01 * mi->k;
    a = lchain_rmq(opt->max_gap, opt->rmq_inner_dist, opt->bw, opt->max_chain_skip, opt->rmq_size_cap, opt->min_cnt,
                   opt->min_chain_score, chn_pen_gap, chn_pen_skip, n_a, a, &n_regs0, &u);
    if (opt->bw_long > opt->bw && n_regs0 > 1) { /* re-chain / long-join */
        int32_t st = (int32_t)a[0].y, en = (int32_t)a[(int32_t)u[0] - 1].y;
        if (qlen - (en - st) > opt->rmq_rescue_size || en - st > qlen * opt->rmq_rescue_ratio) {
            n_a = 0;
            for (int i = 0; i < n_regs0; ++i) n_a += (int32_t)u[i];
            free(u);
            qsort(a, (size_t)n_a, sizeof(m128), cmp128);
            a = lchain_rmq(opt->max_gap, opt->rmq_inner_dist, opt->bw_long, opt->max_chain_skip, opt->rmq_size_cap,
                           opt->min_cnt, opt->min_chain_score, chn_pen_gap, chn_pen_skip, n_a, a, &n_regs0, &u);
        }
    }
    mmo_reg_t *regs = gen_regs(hash, qlen, n_regs0, u, a);
    set_parent(opt->mask_level, opt->mask_len, n_regs0, regs, opt->a * 2 + opt->b, opt->alt_drop);
    select_sub(opt->pri_ratio, mi->k * 2, opt->best_n, 1, (int)(opt->max_gap * 0.8), &n_regs0, regs);
    est_err(mi->len, qlen, n_regs0, regs, a, n_mini_pos, mini_pos);
    n_regs0 = filter_strand_retained(n_regs0, regs);
    set_mapq(n_regs0, regs, opt->min_chain_score, rep_len);
    *rep_len_out = rep_len;
    int ret = n_regs0 <= cap ? n_regs0 : -n_regs0;
    if (n_regs0 <= cap && n_regs0 > 0) memcpy(out, regs, sizeof(mmo_reg_t) * (size_t)n_regs0);
    free(regs); free(a); free(u); free(mini_pos);
    return ret;
}

/* exported for tests: the anchors + chaining arrays of one query (first pass) */
int64_t mmo_debug_anchors(const mmo_idx_t *mi, const mmo_opt_t *opt, const char *qseq, int qlen, m128 *out, int64_t cap,
                          int *rep_len) {
    int n_mini_pos = 0;
    uint64_t *mini_pos = 0;
    int64_t n_a = 0;
    v128 mv = {0, 0, 0};
    mmo_sketch(qseq, qlen, mi->w, mi->k, 0, &mv);
    if (opt->q_occ_frac > 0.0f) seed_mz_flt(&mv, opt->mid_occ, opt->q_occ_frac);
    m128 *a = collect_anchors(opt, opt->mid_occ, mi, &mv, qlen, &n_a, rep_len, &n_mini_pos, &mini_pos);
    free(mv.a);
    free(mini_pos);
    if (n_a <= cap) memcpy(out, a, sizeof(m128) * (size_t)n_a);
    free(a);
    return n_a <= cap ? n_a : -n_a;
}

/* exported for tests: first-pass chaining scores f[] and predecessors p[] */
int64_t mmo_debug_chain(const m128 *a_in, int64_t n, int max_dist, int max_dist_inner, int bw, int max_chn_skip,
                        int cap_rmq_size, float chn_pen_gap, float chn_pen_skip, int32_t *f, int64_t *p) {
    int32_t *v = (int32_t *)malloc(4 * (size_t)(n + 1)), *t = (int32_t *)calloc((size_t)(n + 1), 4);
    if (max_dist < bw) max_dist = bw;
    if (max_dist_inner <= 0 || max_dist_inner >= max_dist) max_dist_inner = 0;
    for (int64_t g0 = 0; g0 < n;) {
        int64_t g1 = g0 + 1;
        while (g1 < n && a_in[g1].x >> 32 == a_in[g0].x >> 32) g1++;
        chain_group(g0, g1, a_in, max_dist, max_dist_inner, bw, max_chn_skip, cap_rmq_size, chn_pen_gap, chn_pen_skip, f, p, v, t);
        g0 = g1;
    }
    free(v); free(t);
    return n;
}

/* exported for tests: mm_set_mapq for one primary region (hit.c), given the query's
 * sum of primary scores and rep_len */
int mmo_mapq_one(int score, int subsc, int cnt, int n_sub, int64_t sum_sc, int rep_len, int min_chain_sc) {
    mmo_reg_t r;
    memset(&r, 0, sizeof(r));
    r.score = score, r.subsc = subsc, r.cnt = cnt, r.n_sub = n_sub, r.parent = 0, r.id = 0;
    mmo_reg_t pad;
    memset(&pad, 0, sizeof(pad));
    /* emulate sum_sc with a second primary holding the remainder */
    pad.parent = 1, pad.id = 1, pad.score = (int)(sum_sc - score);
    mmo_reg_t two[2] = {r, pad};
    set_mapq(sum_sc - score > 0 ? 2 : 1, two, min_chain_sc, rep_len);
    return two[0].mapq;
}
