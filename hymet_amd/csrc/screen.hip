// Mash `screen` on MI355X (replaces scripts/mash.sh:14).
//
// Kernels
//   table_insert   : distinct sketch hashes -> open-addressing table in HBM (linear probing
//                    from a multiplicative-hash home slot), one atomicCAS per hash.  An 8-byte
//                    slot holds the key's high 32 bits and the smallest DB index holding the key
//                    (its canonical index); a probe that matches the high word checks the full key
//                    against the DB's hash array at that index.  Device-scope atomics are done
//                    past the L2 on this part, so any second store per insert (a canonical-index
//                    word beside the key) is another random line write: +4.3 ms on 1e8 hashes
//                    (tools/insert_bench.hip); here the CAS writes both at once.  Hit counts are kept per canonical index, in the
//                    DB's own order: the same on every rank whatever slots the parallel insertion
//                    gave the keys, so the ranks' counts add up as they are (one all-reduce).
//   canon_of       : per DB hash, the canonical index of its key (duplicates across references
//                    share one counter): written by the insert, fixed up for duplicates (a key
//                    held by several references: rare, listed by the insert).
//   screen_count<K>: one thread = one 64-position tile of the pooled, packed query bases.
//                    Rolling 2-bit forward / reverse-complement words decide the canonical
//                    strand by integer compare (== Mash's memcmp on ASCII, since A<C<G<T);
//                    rolling ASCII byte windows feed MurmurHash3_x64_128 (seeded, word 0; or
//                    MurmurHash3_x86_32 for k <= 16, Mash's 32-bit sketches, widened to 64 bits)
//                    without re-expanding the k-mer; each hash probes up to 4 DB tables and
//                    bumps a uint32 count; hashes under a threshold are appended as bottom-s
//                    candidates for the pool set-size estimate (MinHashHeap::estimateSetSize).
//   screen_stats   : one 256-thread block per reference: gather its counts through the
//                    canonical map, shared = #>0, median = k-th smallest positive count by a
//                    bisection over the value range with block reductions (no sort).
// Roofline: HBM/latency bound (random 8-B key probes); algorithmic bytes per k-mer are
// 0.375 (packed read) + 8 per DB probe (+4 per hit), DESIGN.md §Screen.
#include "common.hpp"

namespace {

constexpr uint64_t kEmpty = ~0ull;

// A slot's key word: the key's high 32 bits for 64-bit sketches (a match is then checked against
// the full key in the DB's hash array), the whole key for Mash's 32-bit sketches (k <= 16: the
// hashes are MurmurHash3_x86_32 values, so the word is the key and no check is needed)
__device__ __forceinline__ uint32_t key_word(uint64_t h, bool lo) { return lo ? (uint32_t)h : (uint32_t)(h >> 32); }

// Home slot of a hash: multiplicative (Fibonacci) hashing of the full 64 bits.  The top bits
// alone would crowd every real sketch into the bottom of the table: a bottom-s MinHash sketch
// holds the s SMALLEST hashes of its genome, so their top bits are all zero.
__device__ __forceinline__ uint64_t home_slot(uint64_t h, int shift) { return (h * 0x9E3779B97F4A7C15ull) >> shift; }
#ifndef HYMET_SCREEN_TILE
#define HYMET_SCREEN_TILE 64
#endif
constexpr int kTile = HYMET_SCREEN_TILE;  // k-mer start positions per thread (multiple of 32: lanes stay in phase)
constexpr int kMaxDb = 4;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// MurmurHash3_x64_128 word 0 of a K-byte key held little-endian in w[0..3].
template <int K>
__device__ __forceinline__ uint64_t murmur3_h0(const uint64_t (&w)[4], uint32_t seed) {
    constexpr uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    constexpr int NB = K / 16, TAIL = K & 15;
    uint64_t h1 = seed, h2 = seed;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint64_t k1 = w[2 * b], k2 = w[2 * b + 1];
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    if constexpr (TAIL > 8) {
        uint64_t k2 = w[2 * NB + 1];
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    if constexpr (TAIL > 0) {
        uint64_t k1 = w[2 * NB];
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)K;
    h2 ^= (uint64_t)K;
    h1 += h2;
    h2 += h1;
    h1 = fmix64(h1);
    h2 = fmix64(h2);
    return h1 + h2;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// MurmurHash3_x86_32 of a K-byte key (K <= 16) held little-endian in w[0..1], bytes past K zero.
template <int K>
__device__ __forceinline__ uint32_t murmur3_x86_32(const uint64_t (&w)[4], uint32_t seed) {
    constexpr uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    constexpr int NB = K / 4, TAIL = K & 3;
    uint32_t h1 = seed;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t k1 = (uint32_t)(w[b >> 1] >> (32 * (b & 1)));
        k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
        h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
    }
    if constexpr (TAIL > 0) {
        uint32_t k1 = (uint32_t)(w[NB >> 1] >> (32 * (NB & 1)));  // the K & 3 tail bytes, zero above
        k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)K;
    h1 ^= h1 >> 16; h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}

template <int K>
__device__ __forceinline__ uint64_t mash_hash(const uint64_t (&w)[4], uint32_t seed) {
    if constexpr (K <= 16) return (uint64_t)murmur3_x86_32<K>(w, seed);
    else return murmur3_h0<K>(w, seed);
}

struct CountParams {
    const uint32_t *w2b;
    const uint32_t *wm;
    int64_t n_bases, pos_begin, pos_end;
    uint32_t seed;
    int ndb;
    const uint64_t *tab[kMaxDb];   // slots: key's high 32 bits, canonical index
    const uint64_t *hashes[kMaxDb];  // the DB's hashes (full-key check of a high-word match)
    uint64_t mask[kMaxDb];
    int shift[kMaxDb];
    uint32_t *counts[kMaxDb];      // per canonical index, + [nhash] for the all-ones hash
    uint64_t nhash[kMaxDb];
    uint64_t cand_thr;
    uint64_t *cand;
    int64_t cand_cap;
    unsigned long long *cand_n;
    unsigned long long *nkmers;
};

__device__ __forceinline__ uint32_t ascii_of(uint32_t c) { return (0x54474341u >> (8 * c)) & 0xFFu; }

template <int K>
__global__ __launch_bounds__(256) void screen_count_kernel(CountParams P) {
    constexpr bool LO = K <= 16;  // 32-bit sketches: tables built with key_bits 32
    constexpr int NW = (K + 7) / 8;
    constexpr int TOPB = K - 8 * (NW - 1);
    constexpr uint64_t TOPMASK = TOPB == 8 ? ~0ull : ((1ull << (8 * TOPB)) - 1);
    constexpr uint64_t KMASK = K == 32 ? ~0ull : ((1ull << (2 * K)) - 1);
    const int64_t n_pos = P.pos_end - P.pos_begin;
    const int64_t n_tiles = (n_pos + kTile - 1) / kTile;
    uint64_t nk = 0;
    for (int64_t tile = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; tile < n_tiles;
         tile += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p0 = P.pos_begin + tile * kTile;                 // first k-mer start
        const int64_t p1 = min(p0 + kTile, P.pos_end);                 // one past last start
        const int64_t iend = min(p1 + K - 1, P.n_bases);                // bases to read: [p0, iend)
        uint64_t fwd = 0, rc = 0;
        uint64_t F[4] = {0, 0, 0, 0}, R[4] = {0, 0, 0, 0};
        int run = 0;
        uint32_t cw = 0, mw = 0;
        for (int64_t i = p0; i < iend; i++) {
            if (((i & 15) == 0) || i == p0) cw = P.w2b[i >> 4];
            if (((i & 31) == 0) || i == p0) mw = P.wm[i >> 5];
            const uint32_t c = (cw >> (2 * (i & 15))) & 3u;
            const uint32_t bad = (mw >> (i & 31)) & 1u;
            run = bad ? 0 : run + 1;
            fwd = ((fwd << 2) | c) & KMASK;
            rc = (rc >> 2) | ((uint64_t)(3u - c) << (2 * (K - 1)));
#pragma unroll
            for (int j = 0; j < NW - 1; j++) F[j] = (F[j] >> 8) | (F[j + 1] << 56);
            F[NW - 1] = (F[NW - 1] >> 8) | ((uint64_t)ascii_of(c) << (8 * (TOPB - 1)));
#pragma unroll
            for (int j = NW - 1; j > 0; j--) R[j] = (R[j] << 8) | (R[j - 1] >> 56);
            R[0] = (R[0] << 8) | ascii_of(3u - c);
            R[NW - 1] &= TOPMASK;
            if (run < K) continue;                                       // invalid base inside the k-mer
            const int64_t p = i - (K - 1);
            if (p < p0) continue;                                        // warm-up only
            const uint64_t h = (rc < fwd) ? mash_hash<K>(R, P.seed) : mash_hash<K>(F, P.seed);
            nk++;
            if (h < P.cand_thr) {
                unsigned long long idx = atomicAdd(P.cand_n, 1ull);
                if ((int64_t)idx < P.cand_cap) P.cand[idx] = h;
            }
#pragma unroll
            for (int d = 0; d < kMaxDb; d++) {
                if (d >= P.ndb) break;
                if (h == kEmpty) {
                    atomicAdd(&P.counts[d][P.nhash[d]], 1u);
                    continue;
                }
                const uint64_t *tab = P.tab[d];
                uint64_t s = home_slot(h, P.shift[d]);
                for (;;) {
                    const uint64_t w = tab[s];
                    if (w == kEmpty) break;
                    if ((uint32_t)(w >> 32) == key_word(h, LO) && (LO || P.hashes[d][(uint32_t)w] == h)) {
                        atomicAdd(&P.counts[d][(uint32_t)w], 1u);
                        break;
                    }
                    s = (s + 1) & P.mask[d];
                }
            }
        }
    }
    // wave reduction of the k-mer count, one atomic per wave
    unsigned long long v = nk;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(P.nkmers, v);
}

// insert: one CAS of (key's high word, own index) into the first slot that is empty or holds
// the key.  Finding the key already there (a hash shared by references: the high word matches
// and the full key at the holder's index), the thread lowers the slot's index to its own if
// smaller (a 64-bit atomicMin: the high words are equal) and lists itself with the index it
// saw; canon_of[i] = i is written for every hash and fixed for the listed ones after.
__global__ __launch_bounds__(256) void table_insert_kernel(const uint64_t *__restrict__ hashes, int64_t n,
                                                           unsigned long long *tab, uint64_t mask, int shift,
                                                           int64_t *dups, int32_t *canon_of, bool lo) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = hashes[i];
    canon_of[i] = h == kEmpty ? (int32_t)n : (int32_t)i;
    if (h == kEmpty) return;
    const unsigned long long want = (uint64_t)key_word(h, lo) << 32 | (uint32_t)i;
    uint64_t s = home_slot(h, shift);
    for (;;) {
        const unsigned long long prev = atomicCAS(&tab[s], (unsigned long long)kEmpty, want);
        if (prev == kEmpty) return;  // claimed
        if ((uint32_t)(prev >> 32) == key_word(h, lo) && (lo || hashes[(uint32_t)prev] == h)) {  // the key is there already
            atomicMin(&tab[s], want);
            const unsigned long long k = atomicAdd(reinterpret_cast<unsigned long long *>(dups), 1ull);
            dups[1 + k] = (int64_t)((uint64_t)i << 32 | (uint32_t)prev);
            return;
        }
        s = (s + 1) & mask;
    }
}

// listed duplicates (after every insert and atomicMin): each, and the index it found holding
// the key (the owner is found by the first duplicate to arrive), take the slot's final index
__global__ __launch_bounds__(256) void dup_fix_kernel(const uint64_t *__restrict__ hashes, const int64_t *dups,
                                                      const unsigned long long *tab, uint64_t mask, int shift,
                                                      int32_t *canon_of, bool lo) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= dups[0]) return;
    const uint64_t e = (uint64_t)dups[1 + k];
    const uint32_t j = (uint32_t)(e >> 32), p = (uint32_t)e;
    const uint64_t h = hashes[j];
    uint64_t s = home_slot(h, shift);
    unsigned long long w;
    for (;;) {  // the key's slot (it is in the table: j's CAS found it)
        w = tab[s];
        if ((uint32_t)(w >> 32) == key_word(h, lo) && (lo || hashes[(uint32_t)w] == h)) break;
        s = (s + 1) & mask;
    }
    canon_of[j] = (int32_t)(uint32_t)w;
    canon_of[p] = (int32_t)(uint32_t)w;
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    T s = 0;
    for (int j = 0; j < (int)(blockDim.x >> 6); j++) s += red[j];
    return s;
}

__device__ __forceinline__ uint32_t block_max(uint32_t v, uint32_t *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_down(v, o, 64));
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    uint32_t s = 0;
    for (int j = 0; j < (int)(blockDim.x >> 6); j++) s = max(s, red[j]);
    return s;
}

constexpr int kStatsLds = 4096;

__global__ __launch_bounds__(256) void screen_stats_kernel(const int64_t *__restrict__ ref_off,
                                                           const int32_t *__restrict__ canon_of,
                                                           const uint32_t *__restrict__ counts, uint32_t *shared,
                                                           uint32_t *median) {
    __shared__ uint32_t vals[kStatsLds];
    __shared__ uint32_t red[8];
    const int64_t r = blockIdx.x;
    const int64_t b = ref_off[r], n = ref_off[r + 1] - b;
    const bool in_lds = n <= kStatsLds;
    uint32_t pos = 0, mx = 0;
    for (int64_t j = threadIdx.x; j < n; j += blockDim.x) {
        const uint32_t c = counts[canon_of[b + j]];
        if (in_lds) vals[j] = c;
        pos += c > 0;
        mx = max(mx, c);
    }
    const uint32_t sh = block_sum<uint32_t>(pos, red);
    const uint32_t vmax = block_max(mx, red);
    uint32_t med = 0;
    if (sh > 0) {
        const uint32_t kk = sh / 2;  // Mash: depths sorted ascending, element shared/2
        uint32_t lo = 1, hi = vmax;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            uint32_t cnt = 0;
            for (int64_t j = threadIdx.x; j < n; j += blockDim.x) {
                const uint32_t c = in_lds ? vals[j] : counts[canon_of[b + j]];
                cnt += (c > 0 && c <= mid);
            }
            cnt = block_sum<uint32_t>(cnt, red);
            if (cnt > kk) hi = mid;
            else lo = mid + 1;
        }
        med = lo;
    }
    if (threadIdx.x == 0) {
        shared[r] = sh;
        median[r] = med;
    }
}

template <int K>
int launch_count(hymet_ctx *ctx, const CountParams &P, int64_t n_tiles) {
    int64_t blocks = hymet::cdiv(n_tiles, 256);
    const int64_t cap = (int64_t)ctx->n_cu * 16;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    hymet::ProfScope _ps(ctx, "screen_count", (double)(P.pos_end - P.pos_begin) * (0.375 + 8.0 * P.ndb));
    hipLaunchKernelGGL(screen_count_kernel<K>, dim3((unsigned)blocks), dim3(256), 0, ctx->stream, P);
    HY_CHECK_LAUNCH("screen_count_kernel");
    return HYMET_OK;
}

int log2_exact(int64_t v) {
    int l = 0;
    while ((1ll << l) < v) l++;
    return l;
}

}  // namespace

extern "C" {

int64_t hymet_screen_table_slots(int64_t n_hashes) {
    int64_t s = 1024;
    while (s < 2 * n_hashes) s <<= 1;
    return s;
}

int hymet_screen_table_build(hymet_ctx *ctx, const uint64_t *d_hashes, int64_t n, uint64_t *d_table, int64_t n_slots,
                             int64_t *d_scratch, int32_t *d_canon_of, int key_bits) {
    HY_ARG(ctx && d_table && d_scratch && d_canon_of, "hymet_screen_table_build: null argument");
    HY_ARG(key_bits == 32 || key_bits == 64, "hymet_screen_table_build: key_bits must be 32 or 64");
    const bool lo = key_bits == 32;
    HY_ARG(n_slots >= 1024 && (n_slots & (n_slots - 1)) == 0, "hymet_screen_table_build: n_slots must be a power of two >= 1024");
    HY_ARG(n_slots >= 2 * n, "hymet_screen_table_build: n_slots must be >= 2*n_hashes");
    HY_ARG(n < (1ll << 31) - 1, "hymet_screen_table_build: more than 2^31 - 2 hashes");
    HY_HIP(hipSetDevice(ctx->device));
    HY_HIP(hipMemsetAsync(d_table, 0xFF, (size_t)n_slots * 8, ctx->stream));  // empty: all ones (no index is 2^32 - 1)
    if (n <= 0) return HYMET_OK;
    HY_HIP(hipMemsetAsync(d_scratch, 0, 8, ctx->stream));                    // the duplicate count
    const int lg = log2_exact(n_slots);
    hymet::ProfScope _ps(ctx, "screen_table_build");
    const dim3 grid((unsigned)hymet::cdiv(n, 256));
    hipLaunchKernelGGL(table_insert_kernel, grid, dim3(256), 0, ctx->stream, d_hashes, n, (unsigned long long *)d_table,
                       (uint64_t)(n_slots - 1), 64 - lg, d_scratch, d_canon_of, lo);
    HY_CHECK_LAUNCH("table_insert_kernel");
    hipLaunchKernelGGL(dup_fix_kernel, grid, dim3(256), 0, ctx->stream, d_hashes, (const int64_t *)d_scratch,
                       (const unsigned long long *)d_table, (uint64_t)(n_slots - 1), 64 - lg, d_canon_of, lo);
    HY_CHECK_LAUNCH("dup_fix_kernel");
    return HYMET_OK;
}

int hymet_screen_count(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, int64_t n_bases, int64_t pos_begin,
                       int64_t pos_end, int k, uint32_t seed, int ndb, const uint64_t *const *h_d_tables,
                       const int64_t *h_n_slots, const uint64_t *const *h_d_hashes, const int64_t *h_n_hashes,
                       uint32_t *const *h_d_counts, uint64_t cand_thr, uint64_t *d_cand,
                       int64_t cand_cap, unsigned long long *d_cand_n, unsigned long long *d_nkmers) {
    HY_ARG(ctx && d_2b && d_mask && d_cand_n && d_nkmers, "hymet_screen_count: null argument");
    HY_ARG(k >= 1 && k <= 32, "hymet_screen_count: k must be in 1..32");
    HY_ARG(ndb >= 0 && ndb <= kMaxDb, "hymet_screen_count: ndb must be 0..4");
    HY_ARG(cand_cap == 0 || d_cand, "hymet_screen_count: d_cand is null");
    if (pos_end > n_bases - k + 1) pos_end = n_bases - k + 1;
    if (pos_begin < 0) pos_begin = 0;
    if (pos_end <= pos_begin) return HYMET_OK;
    CountParams P{};
    P.w2b = d_2b;
    P.wm = d_mask;
    P.n_bases = n_bases;
    P.pos_begin = pos_begin;
    P.pos_end = pos_end;
    P.seed = seed;
    P.ndb = ndb;
    for (int d = 0; d < ndb; d++) {
        const int64_t ns = h_n_slots[d];
        HY_ARG(ns >= 1024 && (ns & (ns - 1)) == 0, "hymet_screen_count: table size must be a power of two");
        HY_ARG(h_d_tables[d] && h_d_hashes[d] && h_d_counts[d] && h_n_hashes[d] >= 0, "hymet_screen_count: null table");
        P.tab[d] = h_d_tables[d];
        P.hashes[d] = h_d_hashes[d];
        P.mask[d] = (uint64_t)(ns - 1);
        P.shift[d] = 64 - log2_exact(ns);
        P.counts[d] = h_d_counts[d];
        P.nhash[d] = (uint64_t)h_n_hashes[d];
    }
    P.cand_thr = cand_thr;
    P.cand = d_cand;
    P.cand_cap = cand_cap;
    P.cand_n = d_cand_n;
    P.nkmers = d_nkmers;
    HY_HIP(hipSetDevice(ctx->device));
    const int64_t n_tiles = hymet::cdiv(pos_end - pos_begin, kTile);
    switch (k) {
#define HY_K(KK) \
    case KK: return launch_count<KK>(ctx, P, n_tiles);
        HY_K(1) HY_K(2) HY_K(3) HY_K(4) HY_K(5) HY_K(6) HY_K(7) HY_K(8)
        HY_K(9) HY_K(10) HY_K(11) HY_K(12) HY_K(13) HY_K(14) HY_K(15) HY_K(16)
        HY_K(17) HY_K(18) HY_K(19) HY_K(20) HY_K(21) HY_K(22) HY_K(23) HY_K(24)
        HY_K(25) HY_K(26) HY_K(27) HY_K(28) HY_K(29) HY_K(30) HY_K(31) HY_K(32)
#undef HY_K
    }
    return hymet::fail(HYMET_E_ARG, "unreachable k");
}

int hymet_screen_stats(hymet_ctx *ctx, const int64_t *d_ref_off, int64_t n_refs, const int32_t *d_canon_of,
                       const uint32_t *d_counts, uint32_t *d_shared, uint32_t *d_median) {
    HY_ARG(ctx && d_ref_off && d_canon_of && d_counts && d_shared && d_median, "hymet_screen_stats: null argument");
    if (n_refs <= 0) return HYMET_OK;
    HY_ARG(n_refs < (1ll << 31), "hymet_screen_stats: too many references");
    HY_HIP(hipSetDevice(ctx->device));
    hymet::ProfScope _ps(ctx, "screen_stats");  // O(H) gather, bytes not modelled
    hipLaunchKernelGGL(screen_stats_kernel, dim3((unsigned)n_refs), dim3(256), 0, ctx->stream, d_ref_off, d_canon_of,
                       d_counts, d_shared, d_median);
    HY_CHECK_LAUNCH("screen_stats_kernel");
    return HYMET_OK;
}

}  // extern "C"
