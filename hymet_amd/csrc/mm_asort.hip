// Grouped anchor sort: the anchor keys of a mapping batch (q | rev | rid | rpos, value y;
// write_anchor_keys_kernel / rechain_keys_kernel) into (key, y) order -- minimap2's radix
// sort of a query's anchors by x (map.c collect_seed_hits -> radix_sort_128x), with the
// canonical full (x, y) tie order T1 -- written out directly as the anchor
// set (x, y), so no unpack pass follows.
//
// The keys arrive query-major (one query's anchors are contiguous), so the global LSD sort
// over ~47 key bits (six 8-bit passes over 12 B per anchor) is replaced by work local to a
// query:
//   * a query of <= 4096 anchors is sorted whole in one block;
//   * a larger query is cut into tiles of 4096 anchors; every tile counts its anchors per
//     bin = (rev, rid) in LDS; a per-query scan turns the counts into each (tile, bin) run's
//     position and lists the non-empty bins -- the (query, strand, target) groups; the tiles
//     scatter their anchors to their runs; every group of <= 4096 anchors is then sorted by
//     (rpos, y) in one block, and the larger groups (a query against its own genome) by one
//     device radix sort over all of them together (key = group rank | key bits below the bin).
// A block sort packs (the key's bits below q or below rid, y) into one 64-bit word, sorts it
// in registers (bitonic, ITEMS per thread) and merges the runs in LDS: merge path splits,
// then each thread's outputs by a bitonic half-cleaner over two windows of ITEMS words
// (independent LDS loads instead of a serial merge).  Segments of <= 64 anchors take a wave
// bitonic sort on (key, y), those of <= 8 a register network in one thread; class lists
// are filled with one global atomic per class and block.  Equal keys after the device radix
// sort (one target position hit by several query minimizers) are put in y order on write.
// Index parts of more than 2047 targets use coarse bins of 2^cs consecutive targets (the
// bin histogram always fits LDS), sorted inside by (low target bits, rpos, y).  The caller
// falls back to the device sort of the whole batch (return 1) when the packed words would
// not fit 64 bits.
#include "mm_common.hpp"
#include "sort.hpp"

namespace hymet {
namespace mm {
namespace {

constexpr int kTile = 4096;     // largest query (or group) sorted whole in one block
// anchors per tile of a large query: the (tile, bin) count matrix is mostly zeros (a tile's
// anchors crowd into a few bins), so fewer, larger tiles cut its traffic (4096 -> 16384:
// query_scan / tile_hist touch a quarter of the rows)
constexpr int kPart = 16384;
constexpr int kMaxBins = 4096;  // (rev, rid) bins held in LDS

struct Seg {
    int64_t s;  // first anchor
    int32_t n;  // anchors
    int32_t q;  // query
};

// segment classes: thread (<= 8), wave (<= 64), blocks of 256 / 512 / 1024 / 2048 / 4096 and,
// for (query, strand, target) groups, 8192 / 16384 (a 1024-thread block sorting 16384 words in
// 136 KB of LDS), large
enum { kThread = 0, kWave, kB256, kB512, kB1K, kB2K, kB4K, kB8K, kB16K, kLarge, kClasses };

// queries: up to kTile sorted whole, larger ones tiled
__device__ __forceinline__ int seg_class(int64_t n) {
    return n <= 8 ? kThread : n <= 64 ? kWave : n <= 256 ? kB256 : n <= 512 ? kB512 : n <= 1024 ? kB1K : n <= 2048 ? kB2K
         : n <= kTile ? kB4K : kLarge;
}
// groups of a tiled query: whole up to 16384 (the device radix sort only above)
__device__ __forceinline__ int seg_class_group(int64_t n) {
    return n <= kTile ? seg_class(n) : n <= 8192 ? kB8K : n <= 16384 ? kB16K : kLarge;
}

// the anchor set written for sorted position i: x, y (the sorted key itself is not written),
// and the set's chaining-group heads: bit i of hb is set where the key above rpos -- (query,
// strand, target) -- differs from position i-1's, so chain_set numbers the groups from this
// bitmap instead of re-reading x (hb zeroed by grouped_anchor_sort; a word may straddle two
// writers' segments, hence the atomic)
struct AnchorOut {
    uint64_t *ax, *ay;
    int rb, pb;
    uint64_t yhi;
    uint32_t *hb;
    uint32_t *ax32;  // x's low word (rpos) alone: the chaining kernels' reads, 4 B per anchor instead of 8
    __device__ __forceinline__ void put(int64_t i, uint64_t k, uint32_t y) const {
        const uint64_t rev = k >> (rb + pb) & 1, rid = k >> pb & ((1ull << rb) - 1), rpos = k & ((1ull << pb) - 1);
        ax[i] = rev << 63 | rid << 32 | rpos;
        ay[i] = yhi << 32 | y;
        ax32[i] = (uint32_t)rpos;
    }
    // k written at i, kp at i - 1 (first: i starts a writer's segment -- a query or a bin, a
    // head either way)
    __device__ __forceinline__ void head(int64_t i, uint64_t k, uint64_t kp, bool first) const {
        if (first || (k >> pb) != (kp >> pb)) atomicOr(hb + (i >> 5), 1u << (i & 31));
    }
};

// one slot per lane with `pred` in list cnt's range: one atomic per wave (every lane calls)
__device__ __forceinline__ int wave_append(int32_t *cnt, bool pred) {
    const uint64_t m = __ballot(pred);
    if (m == 0) return -1;
    const int lane = threadIdx.x & 63, leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(cnt, __popcll(m));
    base = __shfl(base, leader, 64);
    return pred ? base + __popcll(m & ((1ull << lane) - 1)) : -1;
}

// Append the block's segments to their class lists: LDS counts per class, then one global
// atomic per class and block (a global atomic per item serialises on the 8 counters).
// ITEMS segments per thread; cls < 0: none.
template <int ITEMS>
__device__ __forceinline__ void block_append(const Seg (&sg)[ITEMS], const int (&cls)[ITEMS], Seg *lists, int64_t cap,
                                             int32_t *cnt) {
    __shared__ int32_t lc[kClasses], gb[kClasses];
    if (threadIdx.x < kClasses) lc[threadIdx.x] = 0;
    __syncthreads();
    int slot[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        slot[j] = -1;
        for (int k = 0; k < kClasses; k++) {
            const int sl = wave_append(&lc[k], cls[j] == k);
            if (sl >= 0) slot[j] = sl;
        }
    }
    __syncthreads();
    if (threadIdx.x < kClasses) gb[threadIdx.x] = lc[threadIdx.x] ? atomicAdd(&cnt[threadIdx.x], lc[threadIdx.x]) : 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        // the counters persist across calls (cleared by each kernel's last block): a stale
        // count must never write past a list; the host checks the totals against cap
        const int64_t at = cls[j] >= 0 ? (int64_t)gb[cls[j]] + slot[j] : cap;
        if (at < cap) lists[cls[j] * cap + at] = sg[j];
    }
}

// queries by size class (large: tiles counted)
__global__ __launch_bounds__(256) void query_class_kernel(const int64_t *qoff, int n_q, Seg *lists, int64_t cap, int32_t *cnt,
                                                          uint32_t *nt, int64_t *mail) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = q < n_q;
    const int64_t s = ok ? qoff[q] : 0, n = ok ? qoff[q + 1] - s : 0;
    if (ok) nt[q] = n > kTile ? (uint32_t)((n + kPart - 1) / kPart) : 0;
    const Seg sg[1] = {Seg{s, (int32_t)n, q}};
    const int cls[1] = {n > 0 ? seg_class(n) : -1};
    block_append<1>(sg, cls, lists, cap, cnt);
    publish_counters(cnt, kClasses, mail);
}

// LDS atomicAdd(&h[bin], 1) for the active lanes, returning the old values: the lanes of up
// to two bins shared by many lanes (a query's anchors crowd into its genome's bins) take one
// atomic per bin, the rest one each
__device__ __forceinline__ uint32_t lds_rank(uint32_t *h, int bin, bool active) {
    const int lane = threadIdx.x & 63;
    uint64_t pending = __ballot(active);
    uint32_t r = 0;
    for (int it = 0; it < 2 && pending; it++) {
        const int leader = __ffsll((unsigned long long)pending) - 1;
        const int lb = __shfl(bin, leader, 64);
        const uint64_t m = __ballot(active && bin == lb) & pending;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&h[lb], (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, leader, 64);
        if (m >> lane & 1) r = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
        pending &= ~m;
    }
    if (pending >> lane & 1) r = atomicAdd(&h[bin], 1u);
    return r;
}

__global__ void tile_map_kernel(const Seg *large, int n_large, const int64_t *tpos, int64_t *tile_a0, int32_t *tile_q,
                                int32_t *tile_n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_large) return;
    const Seg S = large[i];
    int64_t t = tpos[S.q];
    for (int64_t a = 0; a < S.n; a += kPart, t++) {
        tile_a0[t] = S.s + a;
        tile_q[t] = S.q;
        tile_n[t] = (int32_t)min((int64_t)kPart, (int64_t)S.n - a);
    }
}

__global__ __launch_bounds__(256) void tile_hist_kernel(const uint64_t *__restrict__ key, const int64_t *__restrict__ tile_a0,
                                                        const int32_t *__restrict__ tile_n, int pb, int nbins,
                                                        uint32_t *__restrict__ H) {
    __shared__ uint32_t h[kMaxBins];
    const int64_t a0 = tile_a0[blockIdx.x];
    const int n = tile_n[blockIdx.x];
    for (int b = threadIdx.x; b < nbins; b += 256) h[b] = 0;
    __syncthreads();
    // every lane runs the loop (wave-level ballots inside); eight rows of keys loaded at a time,
    // at clamped positions (straight-line loads: the waits are counted, not vmcnt(0) per row)
    for (int e0 = 0; e0 < n; e0 += 256 * 8) {
        uint64_t kv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) kv[u] = key[a0 + min(e0 + 256 * u + (int)threadIdx.x, n - 1)];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const bool act = e0 + 256 * u + (int)threadIdx.x < n;
            (void)lds_rank(h, act ? (int)((kv[u] >> pb) & (nbins - 1)) : 0, act);
        }
    }
    __syncthreads();
    uint32_t *row = H + (int64_t)blockIdx.x * nbins;
    for (int b = threadIdx.x; b < nbins; b += 256) row[b] = h[b];
}

// one block per large query: H[t][b] <- offset (within the query) of tile t's bin-b run;
// every non-empty bin appended to the group list.  A thread per bin (rows of 1024 bins) walks
// the bin down the query's tiles: a long contig has hundreds of tiles, and its block is the
// launch's tail (256 threads walking four rows of bins one after the other took 1.3 ms per
// launch on C4)
__global__ __launch_bounds__(1024) void query_scan_kernel(const Seg *large, const int64_t *tpos, int nbins,
                                                          uint32_t *__restrict__ H, Seg *groups, int64_t cap,
                                                          int32_t *n_groups, int64_t *mail) {
    __shared__ uint32_t wsum[16], wgrp[16];
    __shared__ int32_t gbase;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const Seg S = large[blockIdx.x];
    const int64_t t0 = tpos[S.q], t1 = t0 + (S.n + kPart - 1) / kPart;
    uint32_t carry = 0;  // anchors in the bins of earlier rows (block-uniform)
    for (int r = 0; r < nbins; r += 1024) {  // bins r + tid, in bin order across rows
        const int b = r + tid;
        uint32_t run = 0;
        if (b < nbins)
            for (int64_t t = t0; t < t1; t += 32) {  // 32 loads in flight (clamped rows: straight-line)
                uint32_t v[32];
#pragma unroll
                for (int j = 0; j < 32; j++) v[j] = H[min(t + j, t1 - 1) * nbins + b];
#pragma unroll
                for (int j = 0; j < 32; j++)
                    if (t + j < t1) {
                        H[(t + j) * nbins + b] = run;  // exclusive within the bin, across tiles
                        run += v[j];
                    }
            }
        uint32_t inc = run;  // inclusive scan over the row's bins: waves, then the wave sums
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += o;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t wex = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t x = wsum[k];
            wex += k < w ? x : 0u;
            tot += x;
        }
        const uint32_t base = carry + wex + inc - run;
        carry += tot;
        if (b < nbins && run > 0)
            for (int64_t t = t0; t < t1; t += 32) {
                uint32_t v[32];
#pragma unroll
                for (int j = 0; j < 32; j++) v[j] = H[min(t + j, t1 - 1) * nbins + b];
#pragma unroll
                for (int j = 0; j < 32; j++)
                    if (t + j < t1) H[(t + j) * nbins + b] = v[j] + base;
            }
        // the row's non-empty bins appended with one global atomic per block (one per wave
        // serialised ~40k returning atomics per launch on the single counter)
        const bool ne = b < nbins && run > 0;
        const uint64_t nm = __ballot(ne);
        if (lane == 0) wgrp[w] = (uint32_t)__popcll(nm);
        __syncthreads();
        uint32_t gex = 0, gtot = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t x = wgrp[k];
            gex += k < w ? x : 0u;
            gtot += x;
        }
        if (tid == 0) gbase = gtot ? atomicAdd(n_groups, (int32_t)gtot) : 0;
        __syncthreads();
        if (ne) {
            const int64_t slot = (int64_t)gbase + gex + __popcll(nm & ((1ull << lane) - 1));
            if (slot < cap) groups[slot] = Seg{S.s + base, (int32_t)run, S.q};  // host checks the total
        }
        __syncthreads();  // wsum / wgrp / gbase are rewritten by the next row
    }
    publish_counters(n_groups, 1, mail);
}

// The scatter of a large query's tile to its (tile, bin) runs.  Consecutive anchors of a tile
// fall into many bins (one minimizer hits every strain of the taxon), so writing each anchor
// straight to its run position scattered 12-byte writes over as many cache lines; instead each
// round of kSub anchors is ranked by bin in LDS (wave-aggregated atomics), its bin counts are
// scanned, the round is laid out bin by bin in LDS, and written run by run (consecutive lanes,
// consecutive addresses).
// LDS per block: 12 B per round anchor + 8 B per bin (sized to the part's bins at launch:
// 1024 bins and 2048 anchors = 32 KB, five blocks per CU; measured on C4: 3072 anchors in a
// static 68 KB was 323 ms/step of mm_anchor_gsort, 44 KB dynamic 300, 2048 anchors 288)
#ifndef HYMET_SCATTER_SUB
#define HYMET_SCATTER_SUB 2048
#endif
constexpr int kSub = HYMET_SCATTER_SUB;

__global__ __launch_bounds__(256) void tile_scatter_kernel(const uint64_t *__restrict__ key, const uint32_t *__restrict__ val,
                                                           const int64_t *__restrict__ tile_a0, const int32_t *__restrict__ tile_q,
                                                           const int32_t *__restrict__ tile_n, const int64_t *__restrict__ qoff,
                                                           int pb, int nbins, const uint32_t *__restrict__ H,
                                                           uint64_t *__restrict__ okey, uint32_t *__restrict__ oval) {
    extern __shared__ uint64_t smem[];
    uint64_t *sk = smem;                                   // [kSub]
    uint32_t *sv = reinterpret_cast<uint32_t *>(sk + kSub);  // [kSub]
    uint32_t *c = sv + kSub;                               // [nbins] run position of every bin for the next round
    uint32_t *lo = c + nbins;                              // [nbins] round: bin counts, then their exclusive offsets
    __shared__ uint32_t wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t a0 = tile_a0[blockIdx.x];
    const int n = tile_n[blockIdx.x];
    const uint32_t *row = H + (int64_t)blockIdx.x * nbins;
    for (int b = tid; b < nbins; b += 256) c[b] = row[b];
    const int64_t base = qoff[tile_q[blockIdx.x]];
    const int per = (nbins + 255) / 256, b0 = min(tid * per, nbins), b1 = min(b0 + per, nbins);
    for (int r0 = 0; r0 < n; r0 += kSub) {
        const int m = min(kSub, n - r0);
        for (int b = tid; b < nbins; b += 256) lo[b] = 0;
        __syncthreads();
        uint64_t kk[kSub / 256];
        uint32_t vv[kSub / 256], rk[kSub / 256];
        int bn[kSub / 256];
#pragma unroll
        for (int j = 0; j < kSub / 256; j++) {  // the round's loads first, at clamped positions
            const int e = min(j * 256 + tid, m - 1);
            kk[j] = key[a0 + r0 + e];
            vv[j] = val[a0 + r0 + e];
        }
#pragma unroll
        for (int j = 0; j < kSub / 256; j++) {  // every lane runs the loop (wave-level ballots inside)
            const bool act = j * 256 + tid < m;
            bn[j] = (int)((kk[j] >> pb) & (uint64_t)(nbins - 1));
            rk[j] = lds_rank(lo, bn[j], act);
        }
        __syncthreads();
        {  // exclusive scan of the bin counts: per-thread spans, then a block scan of span sums
            uint32_t sum = 0;
            for (int b = b0; b < b1; b++) sum += lo[b];
            uint32_t inc = sum;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
                if (lane >= d) inc += o;
            }
            if (lane == 63) wsum[w] = inc;
            __syncthreads();
            uint32_t ex = inc - sum;
            for (int k = 0; k < w; k++) ex += wsum[k];
            for (int b = b0; b < b1; b++) {
                const uint32_t t = lo[b];
                lo[b] = ex;
                ex += t;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kSub / 256; j++)
            if (j * 256 + tid < m) {
                const uint32_t slot = lo[bn[j]] + rk[j];
                sk[slot] = kk[j];
                sv[slot] = vv[j];
            }
        __syncthreads();
        for (int s = tid; s < m; s += 256) {
            const uint64_t k = sk[s];
            const int b = (int)((k >> pb) & (uint64_t)(nbins - 1));
            const int64_t pos = base + c[b] + (s - lo[b]);
            okey[pos] = k;
            oval[pos] = sv[s];
        }
        __syncthreads();
        for (int b = tid; b < nbins; b += 256) c[b] += (b + 1 < nbins ? lo[b + 1] : (uint32_t)m) - lo[b];
        __syncthreads();
    }
}

// groups by size class, 4 per thread; a single-anchor group is final where the scatter put it
__global__ __launch_bounds__(256) void group_class_kernel(const Seg *groups, int64_t G, Seg *lists, int64_t cap, int32_t *cnt,
                                                          const uint64_t *key, const uint32_t *val, AnchorOut out,
                                                          int64_t *mail) {
    Seg sg[4];
    int cls[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int64_t g = (int64_t)blockIdx.x * 1024 + j * 256 + threadIdx.x;
        sg[j] = g < G ? groups[g] : Seg{0, 0, 0};
        if (sg[j].n == 1) {
            const uint64_t k = key[sg[j].s];
            out.put(sg[j].s, k, val[sg[j].s]);
            out.head(sg[j].s, k, k, true);
        }
        cls[j] = sg[j].n > 1 ? seg_class_group(sg[j].n) : -1;
    }
    block_append<4>(sg, cls, lists, cap, cnt);
    publish_counters(cnt, kClasses, mail);
}

// one thread per segment of <= 8 anchors: sorting network on (key, y) in registers
__global__ __launch_bounds__(256) void thread_seg_sort_kernel(const Seg *list, int n_seg, const uint64_t *key,
                                                              const uint32_t *val, AnchorOut out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_seg) return;
    const Seg S = list[i];
    uint64_t k[8];
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        k[j] = j < S.n ? key[S.s + j] : ~0ull;
        v[j] = j < S.n ? val[S.s + j] : ~0u;
    }
#pragma unroll
    for (int w = 2; w <= 8; w <<= 1)
#pragma unroll
        for (int d = w >> 1; d > 0; d >>= 1)
#pragma unroll
            for (int a = 0; a < 8; a++) {
                const int b = a ^ d;
                if (b > a) {
                    const bool up = (a & w) == 0;
                    const bool gt = k[a] > k[b] || (k[a] == k[b] && v[a] > v[b]);
                    if (gt == up) {
                        const uint64_t tk = k[a];
                        k[a] = k[b];
                        k[b] = tk;
                        const uint32_t tv = v[a];
                        v[a] = v[b];
                        v[b] = tv;
                    }
                }
            }
#pragma unroll
    for (int j = 0; j < 8; j++)
        if (j < S.n) {
            out.put(S.s + j, k[j], v[j]);
            out.head(S.s + j, k[j], k[j > 0 ? j - 1 : 0], j == 0);
        }
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return (uint64_t)(uint32_t)hi << 32 | (uint32_t)lo;
}

// one wave per segment of <= 64 anchors: bitonic sort on (key, y) in registers
__global__ __launch_bounds__(64) void wave_seg_sort_kernel(const Seg *list, const uint64_t *key, const uint32_t *val,
                                                           AnchorOut out) {
    const Seg S = list[blockIdx.x];
    const int lane = threadIdx.x;
    uint64_t k = ~0ull;
    uint32_t v = ~0u;
    if (lane < S.n) {
        k = key[S.s + lane];
        v = val[S.s + lane];
    }
    for (int w = 2; w <= 64; w <<= 1)
        for (int j = w >> 1; j > 0; j >>= 1) {
            const uint64_t ok = shfl_xor64(k, j);
            const uint32_t ov = (uint32_t)__shfl_xor((int)v, j, 64);
            const bool up = (lane & w) == 0, lower = (lane & j) == 0;
            const bool other_less = ok < k || (ok == k && ov < v);
            if ((lower == up) == other_less) {  // the lower lane of an ascending pair keeps the min
                k = ok;
                v = ov;
            }
        }
    const uint64_t kp = (uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(k >> 32), 1, 64) << 32 |
                        (uint32_t)__shfl_up((int)(uint32_t)k, 1, 64);  // lane - 1's word
    if (lane < S.n) {
        out.put(S.s + lane, k, v);
        out.head(S.s + lane, k, kp, lane == 0);
    }
}

__device__ __forceinline__ int lds_ix(int e) { return e + (e >> 4); }  // one pad word per 16: blocked access without bank conflicts

// ascending bitonic network over a thread's N words (unrolled: registers only)
template <int N>
__device__ __forceinline__ void reg_sort(uint64_t (&k)[N]) {
#pragma unroll
    for (int w = 2; w <= N; w <<= 1)
#pragma unroll
        for (int j = w >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < N; i++) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t a = k[i], b = k[l];
                    const bool up = (i & w) == 0;
                    k[i] = up ? min(a, b) : max(a, b);
                    k[l] = up ? max(a, b) : min(a, b);
                }
            }
}

// one block of BLOCK threads per segment of <= BLOCK * ITEMS anchors: packed words
// w = (key bits [0, nbits)) << ybits | y sorted by register networks + LDS merge path
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void block_seg_sort_kernel(const Seg *list, const uint64_t *key, const uint32_t *val,
                                                               int nbits, int ybits, AnchorOut out) {
    constexpr int CAP = BLOCK * ITEMS;
    __shared__ uint64_t sm[CAP + CAP / 16];
    const Seg S = list[blockIdx.x];
    const int tid = threadIdx.x;
    const uint64_t lm = (1ull << nbits) - 1, ym = (1ull << ybits) - 1;
    const uint64_t hi_bits = key[S.s] & ~lm;
    {  // coalesced load, striped: every row's loads issued before any is used (clamped positions)
        uint64_t kr[ITEMS];
        uint32_t vr[ITEMS];
#pragma unroll
        for (int u = 0; u < ITEMS; u++) {
            const int e = min(u * BLOCK + tid, S.n - 1);
            kr[u] = key[S.s + e];
            vr[u] = val[S.s + e];
        }
#pragma unroll
        for (int u = 0; u < ITEMS; u++) {
            const int e = u * BLOCK + tid;
            sm[lds_ix(e)] = e < S.n ? ((kr[u] & lm) << ybits | vr[u]) : ~0ull;
        }
    }
    __syncthreads();
    uint64_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) k[j] = sm[lds_ix(tid * ITEMS + j)];
    reg_sort<ITEMS>(k);
    for (int run = ITEMS; run < CAP; run <<= 1) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; j++) sm[lds_ix(tid * ITEMS + j)] = k[j];
        __syncthreads();
        const int o = tid * ITEMS, base = o & ~(2 * run - 1), diag = o - base;
        const int a0 = base, b0 = base + run;
        int lo = max(0, diag - run), hi = min(diag, run);
        while (lo < hi) {  // merge path: first lo with A[lo] > B[diag - 1 - lo]
            const int mid = (lo + hi) >> 1;
            if (sm[lds_ix(a0 + mid)] <= sm[lds_ix(b0 + diag - 1 - mid)]) lo = mid + 1;
            else hi = mid;
        }
        // the thread's ITEMS outputs are the ITEMS smallest of A[ai..] and B[bi..]: min(A[ai + j],
        // B[bi + ITEMS-1-j]) holds exactly those as a bitonic sequence -- independent LDS
        // loads and a half-cleaner network instead of a serial merge
        const int ai = a0 + lo, bi = b0 + diag - lo;
        const int ae = a0 + run, be = b0 + run;
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const int ia = ai + j, ib = bi + ITEMS - 1 - j;
            const uint64_t va = ia < ae ? sm[lds_ix(ia)] : ~0ull, vb = ib < be ? sm[lds_ix(ib)] : ~0ull;
            k[j] = min(va, vb);
        }
#pragma unroll
        for (int d = ITEMS >> 1; d > 0; d >>= 1)
#pragma unroll
            for (int i = 0; i < ITEMS; i++)
                if ((i & d) == 0) {
                    const uint64_t x = k[i], y = k[i + d];
                    k[i] = min(x, y);
                    k[i + d] = max(x, y);
                }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; j++) sm[lds_ix(tid * ITEMS + j)] = k[j];
    __syncthreads();
    for (int e = tid; e < S.n; e += BLOCK) {  // coalesced write
        const uint64_t w = sm[lds_ix(e)], wp = sm[lds_ix(e > 0 ? e - 1 : 0)];
        out.put(S.s + e, hi_bits | w >> ybits, (uint32_t)(w & ym));
        out.head(S.s + e, hi_bits | w >> ybits, hi_bits | wp >> ybits, e == 0);
    }
}

// groups above 4096 anchors: gathered as (rank << pb | rpos, y), sorted together, put back
__global__ __launch_bounds__(256) void big_gather_kernel(const Seg *list, const int64_t *dst, int pb, const uint64_t *key,
                                                         const uint32_t *val, uint64_t *tk, uint32_t *tv) {
    const Seg S = list[blockIdx.x];
    const int64_t d = dst[blockIdx.x];
    const uint64_t pm = (1ull << pb) - 1;
    for (int e = threadIdx.x; e < S.n; e += 256) {
        tk[d + e] = (uint64_t)blockIdx.x << pb | (key[S.s + e] & pm);
        tv[d + e] = val[S.s + e];
    }
}

// sorted big groups back into place; runs of equal key take their y values in order
// (insertion sort by the run's first lane; such runs are short and rare)
__global__ __launch_bounds__(256) void big_put_kernel(const Seg *list, const int64_t *dst, int pb, const uint64_t *key,
                                                      const uint64_t *tk, const uint32_t *tv, AnchorOut out) {
    const Seg S = list[blockIdx.x];
    const int64_t d = dst[blockIdx.x];
    const uint64_t pm = (1ull << pb) - 1;
    const uint64_t hi_bits = key[S.s] & ~pm;
    for (int e = threadIdx.x; e < S.n; e += 256) {
        const uint64_t k = tk[d + e];
        const bool prev_eq = e > 0 && tk[d + e - 1] == k;
        if (prev_eq) continue;
        out.head(S.s + e, hi_bits | (k & pm), hi_bits | (tk[d + (e > 0 ? e - 1 : 0)] & pm), e == 0);
        int f = e;
        while (f + 1 < S.n && tk[d + f + 1] == k) f++;
        if (f == e) {
            out.put(S.s + e, hi_bits | (k & pm), tv[d + e]);
            continue;
        }
        uint32_t ys[64];
        const int m = min(f - e + 1, 64);
        for (int a = 0; a < m; a++) {
            const uint32_t v = tv[d + e + a];
            int b = a;
            while (b > 0 && ys[b - 1] > v) {
                ys[b] = ys[b - 1];
                b--;
            }
            ys[b] = v;
        }
        for (int a = 0; a < m; a++) out.put(S.s + e + a, hi_bits | (k & pm), ys[a]);
        for (int a = m; a <= f - e; a++) out.put(S.s + e + a, hi_bits | (k & pm), tv[d + e + a]);  // > 64 equal keys: input order
    }
}

__global__ void seg_len_kernel(const Seg *list, int n, uint32_t *len) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) len[i] = (uint32_t)list[i].n;
}

int bits_of(int64_t v) {
    int b = 1;
    while ((1ll << b) <= v) b++;
    return b;
}

// sort the segments of `lists` (class-major, capacity cap; counts hc), all but the large class
int sort_segments(hymet_ctx *ctx, const Seg *lists, int64_t cap, const int32_t *hc, const uint64_t *key,
                  const uint32_t *val, int nbits, int ybits, const AnchorOut &out) {
    hipStream_t st = ctx->stream;
#define HY_SEG_LAUNCH(cls, kern, block)                                                                                     \
    if (hc[cls] > 0) {                                                                                                      \
        hipLaunchKernelGGL(kern, dim3((unsigned)hc[cls]), dim3(block), 0, st, lists + cls * cap, key, val, nbits, ybits, out); \
        HY_CHECK_LAUNCH(#kern);                                                                                             \
    }
    if (hc[kThread] > 0) {
        hipLaunchKernelGGL(thread_seg_sort_kernel, dim3((unsigned)cdiv(hc[kThread], 256)), dim3(256), 0, st, lists + kThread * cap,
                           hc[kThread], key, val, out);
        HY_CHECK_LAUNCH("thread_seg_sort_kernel");
    }
    if (hc[kWave] > 0) {
        hipLaunchKernelGGL(wave_seg_sort_kernel, dim3((unsigned)hc[kWave]), dim3(64), 0, st, lists + kWave * cap, key, val, out);
        HY_CHECK_LAUNCH("wave_seg_sort_kernel");
    }
    HY_SEG_LAUNCH(kB256, (block_seg_sort_kernel<64, 4>), 64)
    HY_SEG_LAUNCH(kB512, (block_seg_sort_kernel<64, 8>), 64)
    // (A/B knobs: threads per block of the 1K / 2K / 4K / 8K classes; items = class size / threads)
#ifndef HYMET_SORT_T1K
#define HYMET_SORT_T1K 64
#endif
#ifndef HYMET_SORT_T2K
#define HYMET_SORT_T2K 128
#endif
#ifndef HYMET_SORT_T4K
#define HYMET_SORT_T4K 256
#endif
#ifndef HYMET_SORT_T8K
#define HYMET_SORT_T8K 512
#endif
    HY_SEG_LAUNCH(kB1K, (block_seg_sort_kernel<HYMET_SORT_T1K, 1024 / HYMET_SORT_T1K>), HYMET_SORT_T1K)
    HY_SEG_LAUNCH(kB2K, (block_seg_sort_kernel<HYMET_SORT_T2K, 2048 / HYMET_SORT_T2K>), HYMET_SORT_T2K)
    HY_SEG_LAUNCH(kB4K, (block_seg_sort_kernel<HYMET_SORT_T4K, 4096 / HYMET_SORT_T4K>), HYMET_SORT_T4K)
    HY_SEG_LAUNCH(kB8K, (block_seg_sort_kernel<HYMET_SORT_T8K, 8192 / HYMET_SORT_T8K>), HYMET_SORT_T8K)
    HY_SEG_LAUNCH(kB16K, (block_seg_sort_kernel<1024, 16>), 1024)
#undef HY_SEG_LAUNCH
    return HYMET_OK;
}

}  // namespace

int grouped_anchor_sort(hymet_ctx *ctx, const uint64_t *key, const uint32_t *val, int64_t n, const int64_t *d_qoff, int n_q,
                        int rb, int pb, uint64_t yhi, int64_t max_qlen, uint64_t *okey, uint32_t *oval, uint64_t *ax,
                        uint64_t *ay, uint32_t *hb, uint32_t *ax32) {
    // bins = (strand, target) -- or, for parts of more than 2047 targets, (strand, target >> cs):
    // coarse bins of 2^cs consecutive targets, sorted inside by (low target bits, rpos, y)
    const int cs = std::max(0, 1 + rb - 12);
    const int nbins = 1 << (1 + rb - cs);
    const int gb = pb + cs;  // key bits below the bin
    const int ybits = bits_of(max_qlen);
    if (n <= 0 || n_q <= 0 || 1 + rb + pb + ybits > 63) return 1;
    hipStream_t st = ctx->stream;
    const AnchorOut out{ax, ay, rb, pb, yhi, hb, ax32};
    HY_HIP(hipMemsetAsync(hb, 0, head_bits_bytes(n), st));
    // 1 queries by size
    DevBuf qlists, nt;
    HY_HIP(qlists.alloc(sizeof(Seg) * kClasses * (size_t)n_q, st));
    HY_HIP(nt.alloc(4 * (size_t)(n_q + 1), st));
    hipLaunchKernelGGL(query_class_kernel, dim3((unsigned)cdiv(n_q, 256)), dim3(256), 0, st, d_qoff, n_q, qlists.as<Seg>(),
                       (int64_t)n_q, ctx->dctr + kCtrQClass, nt.as<uint32_t>(), mb_dev(ctx, kMbQClass));
    HY_CHECK_LAUNCH("query_class_kernel");
    HY_HIP(hipStreamSynchronize(st));
    int32_t hq[kClasses] = {};
    for (int c = 0; c < kClasses; c++) {
        hq[c] = (int32_t)mb_read(ctx, kMbQClass + c);
        if (hq[c] < 0 || hq[c] > n_q) return hymet::fail(HYMET_E_INTERNAL, "grouped_anchor_sort: query class count > cap");
    }
    ProfScope _ps(ctx, "mm_anchor_gsort", 52.0 * (double)n);  // key+y read, scatter write, sort read, x+y write
    // 2 small queries: sorted whole
    int rc = sort_segments(ctx, qlists.as<Seg>(), n_q, hq, key, val, 1 + rb + pb, ybits, out);
    if (rc || hq[kLarge] == 0) return rc;
    // 3 large queries: tiles, bin histograms, per-query scan, scatter
    const int nl = hq[kLarge];
    const Seg *large = qlists.as<Seg>() + kLarge * (size_t)n_q;
    DevBuf tpos;
    HY_HIP(tpos.alloc(8 * (size_t)(n_q + 1), st));
    int64_t NT = 0;
    rc = exclusive_scan_u32_i64(ctx, nt.as<uint32_t>(), tpos.as<int64_t>(), n_q, &NT);
    if (rc) return rc;
    DevBuf ta0, tq, tn, H;
    HY_HIP(ta0.alloc(8 * (size_t)NT, st));
    HY_HIP(tq.alloc(4 * (size_t)NT, st));
    HY_HIP(tn.alloc(4 * (size_t)NT, st));
    HY_HIP(H.alloc(4 * (size_t)NT * nbins, st));
    hipLaunchKernelGGL(tile_map_kernel, dim3((unsigned)cdiv(nl, 256)), dim3(256), 0, st, large, nl, tpos.as<int64_t>(),
                       ta0.as<int64_t>(), tq.as<int32_t>(), tn.as<int32_t>());
    HY_CHECK_LAUNCH("tile_map_kernel");
    hipLaunchKernelGGL(tile_hist_kernel, dim3((unsigned)NT), dim3(256), 0, st, key, ta0.as<int64_t>(), tn.as<int32_t>(), gb,
                       nbins, H.as<uint32_t>());
    HY_CHECK_LAUNCH("tile_hist_kernel");
    const int64_t gcap = std::min<int64_t>(n, NT * (int64_t)nbins);  // a group holds >= 1 anchor
    HY_ARG(gcap < INT32_MAX, "grouped_anchor_sort: too many groups in one batch");
    DevBuf groups;
    HY_HIP(groups.alloc(sizeof(Seg) * (size_t)(gcap + 1), st));
    hipLaunchKernelGGL(query_scan_kernel, dim3((unsigned)nl), dim3(1024), 0, st, large, tpos.as<int64_t>(), nbins,
                       H.as<uint32_t>(), groups.as<Seg>(), gcap, ctx->dctr + kCtrGroups, mb_dev(ctx, kMbGroups));
    HY_CHECK_LAUNCH("query_scan_kernel");
    HY_ARG(nbins >= 1 && nbins <= kMaxBins, "grouped_anchor_sort: bin count out of range");
    hipLaunchKernelGGL(tile_scatter_kernel, dim3((unsigned)NT), dim3(256), (size_t)kSub * 12 + (size_t)nbins * 8, st, key, val, ta0.as<int64_t>(), tq.as<int32_t>(),
                       tn.as<int32_t>(), d_qoff, gb, nbins, H.as<uint32_t>(), okey, oval);
    HY_CHECK_LAUNCH("tile_scatter_kernel");
    // 4 groups of the large queries, sorted in place by (rpos, y)
    HY_HIP(hipStreamSynchronize(st));
    const int32_t G = (int32_t)mb_read(ctx, kMbGroups);
    if (G == 0) return HYMET_OK;
    if (G < 0 || G > gcap) return hymet::fail(HYMET_E_INTERNAL, "grouped_anchor_sort: group count > cap");
    DevBuf glists;
    HY_HIP(glists.alloc(sizeof(Seg) * kClasses * (size_t)G, st));
    hipLaunchKernelGGL(group_class_kernel, dim3((unsigned)cdiv(G, 1024)), dim3(256), 0, st, groups.as<Seg>(), (int64_t)G,
                       glists.as<Seg>(), (int64_t)G, ctx->dctr + kCtrGClass, okey, oval, out, mb_dev(ctx, kMbGClass));
    HY_CHECK_LAUNCH("group_class_kernel");
    HY_HIP(hipStreamSynchronize(st));
    int32_t hg[kClasses] = {};
    for (int c = 0; c < kClasses; c++) {
        hg[c] = (int32_t)mb_read(ctx, kMbGClass + c);
        if (hg[c] < 0 || hg[c] > G) return hymet::fail(HYMET_E_INTERNAL, "grouped_anchor_sort: group class count > cap");
    }
    rc = sort_segments(ctx, glists.as<Seg>(), (int64_t)G, hg, okey, oval, gb, ybits, out);
    if (rc) return rc;
    if (hg[kLarge] > 0) {
        const int nbig = hg[kLarge];
        const Seg *big = glists.as<Seg>() + kLarge * (size_t)G;
        DevBuf blen, bdst, tk, tk2, tv, tv2;
        HY_HIP(blen.alloc(4 * (size_t)(nbig + 1), st));
        HY_HIP(bdst.alloc(8 * (size_t)(nbig + 1), st));
        hipLaunchKernelGGL(seg_len_kernel, dim3((unsigned)cdiv(nbig, 256)), dim3(256), 0, st, big, nbig, blen.as<uint32_t>());
        HY_CHECK_LAUNCH("seg_len_kernel");
        int64_t NB = 0;
        rc = exclusive_scan_u32_i64(ctx, blen.as<uint32_t>(), bdst.as<int64_t>(), nbig, &NB);
        if (rc) return rc;
        HY_HIP(tk.alloc(8 * (size_t)NB, st));
        HY_HIP(tk2.alloc(8 * (size_t)NB, st));
        HY_HIP(tv.alloc(4 * (size_t)NB, st));
        HY_HIP(tv2.alloc(4 * (size_t)NB, st));
        hipLaunchKernelGGL(big_gather_kernel, dim3((unsigned)nbig), dim3(256), 0, st, big, bdst.as<int64_t>(), gb, okey, oval,
                           tk.as<uint64_t>(), tv.as<uint32_t>());
        HY_CHECK_LAUNCH("big_gather_kernel");
        const int end_bit = gb + bits_of(nbig);
        HY_ARG(end_bit <= 64, "grouped_anchor_sort: group rank and key bits exceed 64");
        uint64_t *kk = tk.as<uint64_t>(), *kka = tk2.as<uint64_t>();
        uint32_t *vv = tv.as<uint32_t>(), *vva = tv2.as<uint32_t>();
        rc = radix_sort_pairs(ctx, kk, kka, vv, vva, NB, 0, end_bit);
        if (rc) return rc;
        hipLaunchKernelGGL(big_put_kernel, dim3((unsigned)nbig), dim3(256), 0, st, big, bdst.as<int64_t>(), gb, okey,
                           kk, vv, out);
        HY_CHECK_LAUNCH("big_put_kernel");
    }
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet
