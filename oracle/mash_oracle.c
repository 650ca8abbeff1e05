/* TEST INFRASTRUCTURE ONLY -- CPU oracle for the Mash screen stage.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * (as oracle/build/liboracle.so); the product library never links it.
 *
 * Restates, from the public Mash 2.3 algorithm (third-party, unpinned: environment.yml:9;
 * called by scripts/mash.sh:14 as `mash screen -p 8 -v 0.9 DB input/ *.fna`):
 *   - MurmurHash3_x64_128 (Austin Appleby, public domain), word 0 kept (k > 16 => 64-bit);
 *     MurmurHash3_x86_32 for k <= 16 (Mash's 32-bit sketches, hashes32), widened to uint64
 *   - CommandScreen hashSequence: uppercase unless preserveCase; a k-mer is skipped if any
 *     base is outside the alphabet (ACGT); canonical = forward unless memcmp(rc, fwd) < 0;
 *     every occurrence of a table hash increments its count; every k-mer is offered to
 *     the pool bottom-s heap (distinct hashes)
 *   - per-reference shared / median depth (sorted depths[shared/2])
 *   - MinHashHeap::estimateSetSize = 2^64 (2^32 for 32-bit hashes) * |heap| / max(heap)
 *     (truncated to uint64)
 * Parity with Mash itself is UNPINNED (no mash binary or .msh fixture in the container,
 * SURVEY.md §8c); the hash function is pinned by tests/golden/murmur3_kat.json, produced
 * from scikit-learn's vendored MurmurHash3.cpp (tests/golden/make_murmur_kat.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33; return k;
}

uint64_t oracle_murmur3_x64_128_h0(const uint8_t *data, int len, uint32_t seed) {
    const int nblocks = len / 16;
    uint64_t h1 = seed, h2 = seed;
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    for (int i = 0; i < nblocks; i++) {
        uint64_t k1, k2;
        memcpy(&k1, data + 16 * i, 8);
        memcpy(&k2, data + 16 * i + 8, 8);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *tail = data + nblocks * 16;
    uint64_t k1 = 0, k2 = 0;
    switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)tail[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)tail[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)tail[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)tail[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)tail[9] << 8;   /* fallthrough */
    case 9:  k2 ^= (uint64_t)tail[8];
             k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; /* fallthrough */
    case 8:  k1 ^= (uint64_t)tail[7] << 56; /* fallthrough */
    case 7:  k1 ^= (uint64_t)tail[6] << 48; /* fallthrough */
    case 6:  k1 ^= (uint64_t)tail[5] << 40; /* fallthrough */
    case 5:  k1 ^= (uint64_t)tail[4] << 32; /* fallthrough */
    case 4:  k1 ^= (uint64_t)tail[3] << 24; /* fallthrough */
    case 3:  k1 ^= (uint64_t)tail[2] << 16; /* fallthrough */
    case 2:  k1 ^= (uint64_t)tail[1] << 8;  /* fallthrough */
    case 1:  k1 ^= (uint64_t)tail[0];
             k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
}

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t oracle_murmur3_x86_32(const uint8_t *data, int len, uint32_t seed) {
    const int nblocks = len / 4;
    uint32_t h1 = seed;
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    for (int i = 0; i < nblocks; i++) {
        uint32_t k1;
        memcpy(&k1, data + 4 * i, 4);
        k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
        h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
    }
    const uint8_t *tail = data + 4 * nblocks;
    uint32_t k1 = 0;
    switch (len & 3) {
    case 3: k1 ^= (uint32_t)tail[2] << 16; /* fallthrough */
    case 2: k1 ^= (uint32_t)tail[1] << 8;  /* fallthrough */
    case 1: k1 ^= tail[0];
            k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16; h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}

/* Mash's k-mer hash: 64-bit word 0 of x64_128 for k > 16, x86_32 for k <= 16 */
static inline uint64_t mash_hash(const uint8_t *km, int k, uint32_t seed) {
    return k > 16 ? oracle_murmur3_x64_128_h0(km, k, seed) : (uint64_t)oracle_murmur3_x86_32(km, k, seed);
}

/* ---- simple open-addressing set/map over uint64 keys ---- */
typedef struct { uint64_t *key; uint32_t *val; uint8_t *used; uint64_t mask; } omap_t;

static void omap_init(omap_t *m, uint64_t n) {
    uint64_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    m->key = (uint64_t *)calloc(cap, 8);
    m->val = (uint32_t *)calloc(cap, 4);
    m->used = (uint8_t *)calloc(cap, 1);
    m->mask = cap - 1;
}
static void omap_free(omap_t *m) { free(m->key); free(m->val); free(m->used); }
static inline uint64_t omap_slot(const omap_t *m, uint64_t k) {
    uint64_t s = (k * 0x9E3779B97F4A7C15ULL) >> 17 & m->mask;
    while (m->used[s] && m->key[s] != k) s = (s + 1) & m->mask;
    return s;
}

int cmp64(const void *a, const void *b);
static int cmpu32o(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

/* bottom-s distinct set: a buffer of candidates below the current cut, compacted
 * (sort + unique + truncate to s) whenever it fills. */
typedef struct { uint64_t *b; int64_t n, cap, s; int full; uint64_t cut; } bottom_t;
static void bottom_compact(bottom_t *bt) {
    qsort(bt->b, (size_t)bt->n, 8, cmp64);
    int64_t m = 0;
    for (int64_t i = 0; i < bt->n; i++)
        if (m == 0 || bt->b[i] != bt->b[m - 1]) bt->b[m++] = bt->b[i];
    if (m >= bt->s) { m = bt->s; bt->full = 1; bt->cut = bt->b[m - 1]; }
    bt->n = m;
}
static inline void bottom_offer(bottom_t *bt, uint64_t h) {
    if (bt->full && h >= bt->cut) return;
    bt->b[bt->n++] = h;
    if (bt->n == bt->cap) bottom_compact(bt);
}

static const char *ORACLE_ACGT = "ACGT";

/* Screen the pooled query sequences against one sketch DB.
 *   seq/seq_off/nseq : concatenated ASCII query sequences (pool of all input files)
 *   ref_hashes/ref_off/nrefs : each reference's sorted hash list (CSR)
 * Outputs per reference: shared[i], median[i]; *set_size = pool set-size estimate.
 * oracle_screen_prepare builds the hash -> count table once (Mash builds it per run);
 * oracle_screen_run hashes a pool against it.  Returns 0, or -1 for unsupported k. */
typedef struct { omap_t tab; const uint64_t *ref_hashes; const int64_t *ref_off; int64_t nrefs; } oscreen_t;

void *oracle_screen_prepare(const uint64_t *ref_hashes, const int64_t *ref_off, int64_t nrefs) {
    oscreen_t *o = (oscreen_t *)calloc(1, sizeof(oscreen_t));
    int64_t H = ref_off[nrefs];
    omap_init(&o->tab, (uint64_t)H);
    for (int64_t i = 0; i < H; i++) {
        uint64_t s = omap_slot(&o->tab, ref_hashes[i]);
        o->tab.used[s] = 1; o->tab.key[s] = ref_hashes[i]; o->tab.val[s] = 0;
    }
    o->ref_hashes = ref_hashes; o->ref_off = ref_off; o->nrefs = nrefs;
    return o;
}

void oracle_screen_free(void *h) {
    oscreen_t *o = (oscreen_t *)h;
    if (!o) return;
    omap_free(&o->tab);
    free(o);
}

int oracle_screen_run(void *h, const char *seq, const int64_t *seq_off, int64_t nseq, int k, uint32_t seed,
                      int preserve_case, int64_t sketch_size, uint32_t *shared, uint32_t *median, uint64_t *set_size,
                      uint64_t *n_kmers) {
    oscreen_t *o = (oscreen_t *)h;
    if (k < 1 || k > 32) return -1;
    omap_t *tab = &o->tab;
    for (uint64_t i = 0; i <= tab->mask; i++) tab->val[i] = 0;
    bottom_t bt;
    bt.s = sketch_size; bt.cap = 8 * sketch_size + 64; bt.n = 0; bt.full = 0; bt.cut = 0;
    bt.b = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)bt.cap);
    uint64_t nk = 0;
    char *up = NULL, *rc = NULL;
    int64_t upcap = 0;
    for (int64_t q = 0; q < nseq; q++) {
        int64_t L = seq_off[q + 1] - seq_off[q];
        if (L < k) continue;
        if (L > upcap) { upcap = L; up = (char *)realloc(up, L); rc = (char *)realloc(rc, L); }
        const char *s0 = seq + seq_off[q];
        for (int64_t i = 0; i < L; i++) {
            char c = s0[i];
            if (!preserve_case && c > 96 && c < 123) c -= 32;
            up[i] = c;
        }
        for (int64_t i = 0; i < L; i++) {
            char c = up[L - 1 - i];
            rc[i] = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
        }
        for (int64_t j = 0; j + k <= L; j++) {
            int good = 1;
            for (int t = 0; t < k; t++) {
                char c = up[j + t];
                if (c != 'A' && c != 'C' && c != 'G' && c != 'T') { good = 0; break; }
            }
            if (!good) continue;
            const char *fw = up + j, *rv = rc + (L - j - k);
            const char *km = memcmp(rv, fw, (size_t)k) < 0 ? rv : fw;
            uint64_t hh = mash_hash((const uint8_t *)km, k, seed);
            nk++;
            bottom_offer(&bt, hh);
            uint64_t s = omap_slot(tab, hh);
            if (tab->used[s]) tab->val[s]++;
        }
    }
    free(up); free(rc);
    bottom_compact(&bt);
    *n_kmers = nk;
    if (bt.n == 0) *set_size = 0;
    else *set_size = (uint64_t)((k > 16 ? 18446744073709551616.0 : 4294967296.0) * (double)bt.n / (double)bt.b[bt.n - 1]);
    uint32_t *dep = NULL;
    int64_t depcap = 0;
    for (int64_t r = 0; r < o->nrefs; r++) {
        int64_t n = o->ref_off[r + 1] - o->ref_off[r];
        if (n > depcap) { depcap = n; dep = (uint32_t *)realloc(dep, 4 * n); }
        int64_t m = 0;
        for (int64_t i = 0; i < n; i++) {
            uint32_t c = tab->val[omap_slot(tab, o->ref_hashes[o->ref_off[r] + i])];
            if (c > 0) dep[m++] = c;
        }
        qsort(dep, (size_t)m, 4, cmpu32o);
        shared[r] = (uint32_t)m;
        median[r] = m > 0 ? dep[m / 2] : 0;
    }
    free(dep);
    free(bt.b);
    return 0;
}

int oracle_screen(const char *seq, const int64_t *seq_off, int64_t nseq, int k, uint32_t seed,
                  int preserve_case, int64_t sketch_size,
                  const uint64_t *ref_hashes, const int64_t *ref_off, int64_t nrefs,
                  uint32_t *shared, uint32_t *median, uint64_t *set_size, uint64_t *n_kmers) {
    if (k < 1 || k > 32) return -1;
    void *h = oracle_screen_prepare(ref_hashes, ref_off, nrefs);
    int rc = oracle_screen_run(h, seq, seq_off, nseq, k, seed, preserve_case, sketch_size, shared, median, set_size, n_kmers);
    oracle_screen_free(h);
    return rc;
}

/* Mash `sketch` restatement (used to build synthetic .msh DBs in tests/bench): the
 * bottom-s distinct hashes of one sequence set (canonical k-mers), sorted ascending. */
int64_t oracle_sketch(const char *seq, const int64_t *seq_off, int64_t nseq, int k, uint32_t seed,
                      int64_t s, uint64_t *out) {
    int64_t dummy_off[2] = {0, 0};
    uint32_t sh, md; uint64_t ss, nk;
    (void)dummy_off; (void)sh; (void)md; (void)ss; (void)nk;
    /* gather every canonical hash then select: simple and adequate for test sizes */
    int64_t total = 0;
    for (int64_t q = 0; q < nseq; q++) { int64_t L = seq_off[q + 1] - seq_off[q]; if (L >= k) total += L - k + 1; }
    uint64_t *all = (uint64_t *)malloc(8 * (size_t)(total + 1));
    int64_t n = 0;
    char *up = NULL, *rc = NULL; int64_t cap = 0;
    for (int64_t q = 0; q < nseq; q++) {
        int64_t L = seq_off[q + 1] - seq_off[q];
        if (L < k) continue;
        if (L > cap) { cap = L; up = (char *)realloc(up, L); rc = (char *)realloc(rc, L); }
        const char *s0 = seq + seq_off[q];
        for (int64_t i = 0; i < L; i++) { char c = s0[i]; if (c > 96 && c < 123) c -= 32; up[i] = c; }
        for (int64_t i = 0; i < L; i++) { char c = up[L - 1 - i]; rc[i] = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N'; }
        for (int64_t j = 0; j + k <= L; j++) {
            int good = 1;
            for (int t = 0; t < k; t++) { char c = up[j + t]; if (c != 'A' && c != 'C' && c != 'G' && c != 'T') { good = 0; break; } }
            if (!good) continue;
            const char *fw = up + j, *rv = rc + (L - j - k);
            all[n++] = mash_hash((const uint8_t *)(memcmp(rv, fw, (size_t)k) < 0 ? rv : fw), k, seed);
        }
    }
    free(up); free(rc);
    /* sort all (test sizes only) */
    qsort(all, (size_t)n, 8, cmp64);
    int64_t m = 0;
    for (int64_t i = 0; i < n && m < s; i++)
        if (i == 0 || all[i] != all[i - 1]) out[m++] = all[i];
    free(all);
    (void)ORACLE_ACGT;
    return m;
}

int cmp64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}
