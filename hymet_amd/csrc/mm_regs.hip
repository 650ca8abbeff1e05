// Per-query region selection (minimap2 hit.c / map.c after chaining):
// mm_gen_regs (score + hash order), mm_reg_set_coor / mm_cal_fuzzy_len, mm_set_parent,
// mm_select_sub (+ mm_sync_regs), mm_est_err, mm_filter_strand_retained, mm_set_mapq.
// Everything that walks a chain's anchors is anchor-parallel and runs first:
//   chain_stats_flat_kernel two chained anchors per thread: mlen/blen terms (mm_reg_set_coor),
//                           its minimizer index (mm_est_err's get_mini_idx, by table lookup)
//                           and the first anchor, in est_err's walking order, whose index does
//                           not increase -- est_err's sequential two-pointer walk matches
//                           exactly the prefix before it; segmented per chain;
//   query_sumk_kernel       one wave per query: sum of minimizer spans (avg_k).
// regions_kernel then runs one thread per query: a query has few chains (tens) and every step
// left is an O(n^2)-at-most scan over them.  Scratch lives in global memory at the query's
// chain range.  Float/double arithmetic is written in the order of hit.c (-ffp-contract=off).
#include "mm_common.hpp"

#include <cstdio>
#include <cstdlib>

namespace hymet {
namespace mm {
namespace {

__device__ __forceinline__ uint32_t wang32(uint32_t key) {
    key += ~(key << 15);
    key ^= (key >> 10);
    key += (key << 3);
    key ^= (key >> 6);
    key += ~(key << 11);
    key ^= (key >> 16);
    return key;
}

struct U128 {
    uint64_t x, y;
};
__device__ __forceinline__ bool lt128(const U128 &a, const U128 &b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }

template <typename T, typename Less>
__device__ void heap_sort(T *a, int64_t n, Less less) {
    auto sift = [&](int64_t i, int64_t m) {
        for (;;) {
            int64_t l = 2 * i + 1, r = l + 1, b = i;
            if (l < m && less(a[b], a[l])) b = l;
            if (r < m && less(a[b], a[r])) b = r;
            if (b == i) return;
            T t = a[b];
            a[b] = a[i];
            a[i] = t;
            i = b;
        }
    };
    for (int64_t i = n / 2 - 1; i >= 0; --i) sift(i, n);
    for (int64_t e = n - 1; e > 0; --e) {
        T t = a[0];
        a[0] = a[e];
        a[e] = t;
        sift(0, e);
    }
}

__device__ __forceinline__ int64_t upper_idx(const int64_t *off, int64_t n, int64_t v) {  // last s with off[s] <= v
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (off[mid] <= v) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

struct RegParams {
    const uint64_t *ax, *ay;       // the chained anchor set
    const int64_t *ids, *cfirst;   // backtrack output (chains end -> start) and each chain's first slot in it
    const uint64_t *cu;            // score<<32 | count per chain
    const int64_t *cboff;          // chain -> offset of its anchors in chain order (region `as`)
    const int64_t *qc;             // n_q + 1 chain offsets
    const int64_t *qb;             // n_q + 1 anchor offsets
    const uint64_t *mini_pos;
    const int64_t *mp_off;         // n_q + 1
    const int64_t *qlen;
    const uint32_t *name_hash;
    const int32_t *rep_len;
    const int64_t *ref_len;
    int n_q;
    int seed, k;
    float mask_level, pri_ratio;
    int mask_len, best_n, max_gap, min_chain_score;
    U128 *z;
    hymet_mm_reg *regs;
    int32_t *w;
    uint64_t *cov;
    int32_t *tmp;
    int32_t *n_regs;
    // per-chain anchor statistics (chain_stats_flat_kernel)
    const int32_t *c_mlen, *c_blen, *c_st, *c_last, *c_fv;
    const uint64_t *q_sumk;
    const uint32_t *skip_q;        // queries whose regions come from the long join (nullable)
    int wave_min;                  // queries of more chains than this take regions_wave_kernel
    int lds_max;                   // ... and hold their regions in LDS up to this many (kRegSmall)
    unsigned long long *prof;      // HYMET_REG_PROF: wave-kernel cycles per step (nullptr = off)
    int prim_regs;                 // set_parent primaries held in registers (64; HYMET_REG_PRIM in tests)
};

// (x0, y0): the chain's first anchor, (x1, y1): its last
__device__ void set_coor(hymet_mm_reg *r, int32_t qlen, uint64_t x0, uint64_t y0, uint64_t x1, uint64_t y1, int32_t mlen,
                         int32_t blen) {
    const int32_t q_span = (int32_t)(y0 >> 32 & 0xff);
    r->rev = (int32_t)(x0 >> 63);
    r->rid = (int32_t)(x0 << 1 >> 33);
    r->rs = (int32_t)x0 + 1 > q_span ? (int32_t)x0 + 1 - q_span : 0;
    r->re = (int32_t)x1 + 1;
    if (!r->rev) {
        r->qs = (int32_t)y0 + 1 - q_span;
        r->qe = (int32_t)y1 + 1;
    } else {
        r->qs = qlen - ((int32_t)y1 + 1);
        r->qe = qlen - ((int32_t)y0 + 1 - q_span);
    }
    r->mlen = mlen;  // span(first) + sum over consecutive anchors (chain_stats_flat_kernel)
    r->blen = blen;
}

struct AnchorStatParams {
    const uint64_t *ax, *ay, *cu;
    const int64_t *ids, *cfirst;  // backtrack output (chains end -> start), each chain's first slot in it
    const int64_t *cboff, *qb, *qlen, *mp_off;
    const uint64_t *mini_pos;
    int64_t NB, NC;
    int n_q;
    const uint32_t *cq;      // query of each chain
    int32_t *c_mlen, *c_blen, *c_st, *c_last;
    const MiniWord *mtab;    // query base -> minimizer index (or -1): word (qbase[q] + position) >> 6
    const int64_t *qbase;
    const uint32_t *skip_q;  // queries whose chains are superseded by the long join (nullable)
};

// Per-chain anchor statistics, flat over the chained anchors in chain order (position b of
// chain c: b - cboff[c] from its start), read in place from the backtrack output and the
// anchor set -- no copy of the chained anchors is made (a copy cost 48 B per anchor written
// and read back).  mm_reg_set_coor's mlen/blen sums, and for mm_est_err the walk-order
// first/last minimizer index and the first anchor whose index does not increase (est_err's
// loop `for (k=1, j=st+1; j<nm && k<cnt; ++j) if (idx(k) == j) ++k, ++n_match;` matches
// anchor k iff idx(1..k) strictly increase from st; the first that does not, or has no
// minimizer, stalls it to the end).  The minimizer index (get_mini_idx) is one 16-byte load
// from a position -> index table (MiniWord: start bits and a base index per 64 query bases,
// -1 where no seeded minimizer starts; built by mini_bits/base_kernel in hymet_mm_map).  Each block finds its
// lanes' chains by a search over the next 256 chain offsets staged in LDS; neighbours in
// chain order come from the adjacent lanes (a load only at a wave edge); then a segmented
// wave reduction by chain and one atomic per chain piece in the wave.  c_mlen / c_blen
// start at 0, c_fv at INT32_MAX (every anchor offers cnt).
__device__ __forceinline__ int32_t mini_idx_at(const AnchorStatParams &P, int64_t q, int qlen, uint64_t ax, uint64_t ay) {
    int32_t x = (int32_t)ay;
    if (ax >> 63) x = qlen - 1 - (int32_t)ay + (int32_t)(ay >> 32 & 0xff) - 1;
    return (x >= 0 && x < qlen) ? mini_word_idx(P.mtab[(P.qbase[q] + x) >> 6], x) : -1;
}

// chain_stats_flat_kernel: kStatItems chain-order positions per thread (rows of 256 in a
// block), their loads issued row after row before any is used -- one position per thread
// left every thread waiting on a chain of ~6 dependent loads (chain, query, chain slot,
// anchor, minimizer index) with nothing else in flight.  Two per thread: C4 one-stream
// 108.6 ms per step at four, 86.6 at two, 196.5 at eight (the register-held rows cost
// occupancy; profiles/r05_chain_stats/)
#ifndef HYMET_STAT_ITEMS
#define HYMET_STAT_ITEMS 2
#endif
constexpr int kStatItems = HYMET_STAT_ITEMS;
constexpr int kStatSpan = 256 * kStatItems;  // chain-order positions per block

// the chain holding chain-order position kStatSpan b, for every block b of
// chain_stats_flat_kernel (one thread per chain writes the block starts inside it: no
// per-block binary search, whose ~log2(NC) dependent loads held the whole block)
__global__ void block_chain_kernel(const int64_t *cboff, int64_t NC, int64_t NB, int32_t *blk_c0) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= NC) return;
    const int64_t s = cboff[c], e = c + 1 < NC ? cboff[c + 1] : NB;
    for (int64_t b = (s + kStatSpan - 1) / kStatSpan; b * kStatSpan < e; ++b) blk_c0[b] = (int32_t)c;
}

__global__ __launch_bounds__(256) void chain_stats_flat_kernel(AnchorStatParams P, const int32_t *blk_c0, int32_t *c_fv) {
    constexpr int K = kStatItems;
    __shared__ int32_t s_st[kStatSpan + 1];  // block-relative starts of chains c0 .. c0 + kStatSpan (clamped)
    const int64_t b0 = (int64_t)blockIdx.x * kStatSpan;
    const int64_t cb0 = blk_c0[blockIdx.x];  // last c with cboff[c] <= b0
    for (int i = threadIdx.x; i <= kStatSpan; i += blockDim.x) {
        const int64_t cc = cb0 + i;
        s_st[i] = cc < P.NC ? (int32_t)min(P.cboff[cc] - b0, (int64_t)kStatSpan) : kStatSpan;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int64_t c[K], q[K], f0[K];  // chain, query, slot of chain-order position 0 in ids
    bool act[K];
    int32_t cnt[K], j[K], qlen[K], cur[K];
    uint64_t x[K], y[K];
    // a block inside one chain (long chains: most blocks) skips the searches and sums its
    // statistics over the block
    const bool one_chain = s_st[1] >= kStatSpan;
    int32_t t_dm = 0, t_db = 0, t_fv = INT32_MAX;
    int64_t qb[K];
    if (one_chain) {
        // the block's one chain: its values are block-uniform (scalar loads), every position's
        // anchor one slot further down the chain
        const int64_t qq = (int64_t)P.cq[cb0];
        const int32_t cn = (int32_t)P.cu[cb0];
        const int64_t cbs = P.cboff[cb0], f00 = P.cfirst[cb0] + cn - 1;
        const int ql = (int)P.qlen[qq];
        const int64_t qbb = P.qbase[qq];
        const bool sk = P.skip_q && P.skip_q[qq];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int64_t b = b0 + 256 * k + threadIdx.x;
            c[k] = b < P.NB ? cb0 : -1;
            q[k] = qq, cnt[k] = cn, f0[k] = f00, qlen[k] = ql, qb[k] = qbb;
            act[k] = b < P.NB && !sk;
            j[k] = act[k] ? (int32_t)(b - cbs) : 0;
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int r = 256 * k + (int)threadIdx.x;  // block-relative position
            const int64_t b = b0 + r;
            c[k] = -1;
            if (b < P.NB) {
                int lo = 0, hi = kStatSpan;  // last i with s_st[i] <= r (s_st[0] <= 0, nondecreasing)
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_st[mid] <= r) lo = mid;
                    else hi = mid - 1;
                }
                c[k] = cb0 + lo;
                if (lo == kStatSpan) {  // beyond the staged chains (chains with no anchors in the range)
                    int64_t l2 = c[k], h2 = P.NC - 1;
                    while (l2 < h2) {
                        const int64_t mid = (l2 + h2 + 1) >> 1;
                        if (P.cboff[mid] <= b) l2 = mid;
                        else h2 = mid - 1;
                    }
                    c[k] = l2;
                }
            }
        }
        // (every load below is unconditional, at a valid index for inactive positions -- chain 0,
        // its first slot -- so the rows' loads stay straight-line code and are all in flight
        // before the first is used)
#pragma unroll
        for (int k = 0; k < K; k++) q[k] = (int64_t)P.cq[c[k] >= 0 ? c[k] : 0];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int64_t cc = c[k] >= 0 ? c[k] : 0;
            cnt[k] = (int32_t)P.cu[cc];
            const int64_t cb = P.cboff[cc];
            f0[k] = P.cfirst[cc] + cnt[k] - 1;
            j[k] = (int32_t)(b0 + 256 * k + threadIdx.x - cb);
            qlen[k] = (int)P.qlen[q[k]];
            qb[k] = P.qbase[q[k]];
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            act[k] = c[k] >= 0;
            if (P.skip_q) act[k] = act[k] && !P.skip_q[q[k]];
            if (!act[k]) j[k] = 0;
        }
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        const int64_t a = P.ids[f0[k] - j[k]];
        x[k] = P.ax[a], y[k] = P.ay[a];
    }
#pragma unroll
    for (int k = 0; k < K; k++) {  // mini_idx_at, its table read unconditional
        int32_t xq = (int32_t)y[k];
        if (x[k] >> 63) xq = qlen[k] - 1 - (int32_t)y[k] + (int32_t)(y[k] >> 32 & 0xff) - 1;
        const bool inq = xq >= 0 && xq < qlen[k];
        const int32_t xc = inq ? xq : 0;
        const int32_t v = mini_word_idx(P.mtab[(qb[k] + xc) >> 6], xc);
        cur[k] = act[k] && inq ? v : -1;
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
        // chain-order neighbours (anchor and minimizer index) from the adjacent lanes (same
        // chain), else loaded
        const int32_t ci = (int32_t)c[k];
        const int32_t cprev = __shfl_up(ci, 1, 64), cnext = __shfl_down(ci, 1, 64);
        uint64_t xp = __shfl_up(x[k], 1, 64), yp = __shfl_up(y[k], 1, 64);
        uint64_t xn = __shfl_down(x[k], 1, 64), yn = __shfl_down(y[k], 1, 64);
        const int32_t cur_p = __shfl_up(cur[k], 1, 64), cur_n = __shfl_down(cur[k], 1, 64);
        int dm = 0, db = 0, fv = INT32_MAX;
        if (act[k]) {
            const bool rev = x[k] >> 63;
            const bool own_p = lane > 0 && cprev == ci, own_n = lane < 63 && cnext == ci;
            if (j[k] > 0 && !own_p) {
                const int64_t a = P.ids[f0[k] - j[k] + 1];
                xp = P.ax[a], yp = P.ay[a];
            }
            if (rev && j[k] + 1 < cnt[k] && !own_n) {
                const int64_t a = P.ids[f0[k] - j[k] - 1];
                xn = P.ax[a], yn = P.ay[a];
            }
            const int32_t span = (int32_t)(y[k] >> 32 & 0xff);
            if (j[k] == 0) {
                dm = db = span;
            } else {  // hit.c mm_reg_set_coor
                const int32_t tl = (int32_t)x[k] - (int32_t)xp;
                const int32_t ql = (int32_t)y[k] - (int32_t)yp;
                db = tl > ql ? tl : ql;
                dm = tl > span && ql > span ? span : tl < ql ? tl : ql;
            }
            const int32_t kk = rev ? cnt[k] - 1 - j[k] : j[k];  // est_err walking order
            fv = cnt[k];
            if (kk >= 1) {
                const int32_t prev = rev ? (own_n ? cur_n : mini_idx_at(P, q[k], qlen[k], xn, yn))
                                         : (own_p ? cur_p : mini_idx_at(P, q[k], qlen[k], xp, yp));
                if (cur[k] < 0 || cur[k] <= prev) fv = kk;
            }
            if (kk == 0) P.c_st[c[k]] = cur[k];
            if (kk == cnt[k] - 1) P.c_last[c[k]] = cur[k];
        }
        if (one_chain) {  // summed over the block below: one atomic per block and counter
            t_dm += dm, t_db += db, t_fv = min(t_fv, fv);
            continue;
        }
        const int32_t cr = act[k] ? ci : -1;
        // segmented inclusive reduction over lanes of the same chain (contiguous in the wave)
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t co = __shfl_up(cr, d, 64);
            const int dmo = __shfl_up(dm, d, 64), dbo = __shfl_up(db, d, 64), fvo = __shfl_up(fv, d, 64);
            if (lane >= d && co == cr) dm += dmo, db += dbo, fv = min(fv, fvo);
        }
        const int32_t cn = __shfl_down(cr, 1, 64);
        if (act[k] && (lane == 63 || cn != cr)) {  // last lane of its chain piece in this wave
            atomicAdd(P.c_mlen + c[k], dm);
            atomicAdd(P.c_blen + c[k], db);
            atomicMin(c_fv + c[k], fv);
        }
    }
    if (one_chain) {
        // device-scope atomics go through the fabric, not an XCD's L2: a long chain's rows
        // each adding to the same three counters (~10^7 per launch) were the kernel's bound
        __shared__ int32_t r_dm[4], r_db[4], r_fv[4];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            t_dm += __shfl_xor(t_dm, o, 64);
            t_db += __shfl_xor(t_db, o, 64);
            t_fv = min(t_fv, __shfl_xor(t_fv, o, 64));
        }
        const int w = threadIdx.x >> 6;
        if (lane == 0) r_dm[w] = t_dm, r_db[w] = t_db, r_fv[w] = t_fv;
        __syncthreads();
        if (threadIdx.x == 0 && act[0]) {  // (a skipped query's chain: no update, as per lane)
            atomicAdd(P.c_mlen + cb0, r_dm[0] + r_dm[1] + r_dm[2] + r_dm[3]);
            atomicAdd(P.c_blen + cb0, r_db[0] + r_db[1] + r_db[2] + r_db[3]);
            atomicMin(c_fv + cb0, min(min(r_fv[0], r_fv[1]), min(r_fv[2], r_fv[3])));
        }
    }
}

// one wave per query: sum of minimizer spans (avg_k)
__global__ __launch_bounds__(64) void query_sumk_kernel(const uint64_t *mini_pos, const int64_t *mp_off, int n_q,
                                                        unsigned long long *sumk) {
    for (int q = blockIdx.x; q < n_q; q += gridDim.x) {
        unsigned long long sk = 0;
        const int64_t m1 = mp_off[q + 1];
        for (int64_t m = mp_off[q] + threadIdx.x; m < m1; m += 256) {  // 4 loads in flight per lane
            uint64_t v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = m + 64 * j < m1 ? mini_pos[m + 64 * j] : 0;
#pragma unroll
            for (int j = 0; j < 4; j++) sk += v[j] >> 32 & 0xff;
        }
        for (int o = 32; o > 0; o >>= 1) sk += __shfl_xor(sk, o, 64);
        if (threadIdx.x == 0) sumk[q] = sk;
    }
}

// Queries of more than kRegWave chains take regions_wave_kernel (one wave each); the thread
// kernel leaves them.  Real genomes make such queries common: a contig that carries a
// repeat (an IS element, an rRNA operon) hits every copy in every strain, hundreds to
// thousands of chains, and one thread walking them through global memory took ~0.9 s per
// step on the Zymo-backbone workload.  From 17 chains on: at C5 (5,000 candidates, ~350 PAF
// lines per contig) the thread kernel's divergent 17-48-chain queries held the regions scope
// at 1.52 s per step, 0.40 s with them on the wave kernel; C4 unchanged (1,258 vs 1,255 ms)
// (profiles/r05_chain_stats/, profiles/r05_c5_pmc/).
constexpr int kRegWave = 16;
constexpr int kRegSmall = 256;  // the wave kernel holds a query's regions in LDS up to this many
constexpr int kRegEntryBytes = 16 + 16 + 4 * 3 + 8;  // slot, aux, wl, psub, pns, covb per entry
// global scratch of the wave kernel per chain: a query of n > kRegSmall chains takes m < 2n
// entries at qc[q] * kRegScrStride -- 112 = 2 x 56 B keeps every query's base 16-byte aligned
// for the int4 / U128 accesses (104 B per chain left odd qc[q] 8-byte aligned)
constexpr int kRegScrStride = 2 * ((kRegEntryBytes + 15) & ~15) - 16;
static_assert(kRegScrStride % 16 == 0 && kRegScrStride >= 2 * kRegEntryBytes, "regions scratch stride");

__device__ __forceinline__ bool wave_query(const RegParams &P, int q, int n, int32_t qlen) {
    return n > P.wave_min && qlen != 0 && !(P.skip_q && P.skip_q[q]);
}

// the per-query steps, sequential: one thread per query (and the wave kernel's fallback for
// queries of more than kRegLds chains)
__device__ void regions_seq(const RegParams &P, int q) {
    const int64_t c0 = P.qc[q], c1 = P.qc[q + 1];
    int n = (int)(c1 - c0);
    const int32_t qlen = (int32_t)P.qlen[q];
    if (n == 0 || qlen == 0 || (P.skip_q && P.skip_q[q])) {
        P.n_regs[q] = 0;
        return;
    }
    const int64_t b0 = P.qb[q];
    U128 *z = P.z + c0;
    hymet_mm_reg *r = P.regs + c0;
    uint32_t hash = P.name_hash[q];
    hash ^= wang32((uint32_t)qlen) + wang32((uint32_t)P.seed);
    hash = wang32(hash);
    // ---- mm_gen_regs
    for (int i = 0; i < n; ++i) {
        const int64_t k = P.cboff[c0 + i] - b0;
        const uint64_t u = P.cu[c0 + i];
        const int64_t a = P.ids[P.cfirst[c0 + i] + (int32_t)u - 1];  // the chain's first anchor
        const uint32_t h = (uint32_t)hash64((hash64(P.ax[a]) + hash64(P.ay[a])) ^ hash);
        z[i].x = u ^ h;
        z[i].y = (uint64_t)k << 32 | (uint32_t)i;  // (mm_gen_regs: count; k is unique per chain, so
                                                   // the low word never orders -- the chain index instead)
    }
    heap_sort(z, n, [](const U128 &a, const U128 &b) { return lt128(a, b); });
    for (int i = 0; i < n >> 1; ++i) {
        U128 t = z[i];
        z[i] = z[n - 1 - i];
        z[n - 1 - i] = t;
    }
    for (int i = 0; i < n; ++i) {
        hymet_mm_reg *ri = &r[i];
        ri->id = i;
        ri->parent = -1;
        ri->score = (int32_t)(z[i].x >> 32);
        ri->hash = (uint32_t)z[i].x;
        const int64_t c = c0 + (uint32_t)z[i].y;
        ri->cnt = (int32_t)P.cu[c];
        ri->as = (int32_t)(z[i].y >> 32);
        ri->div = -1.0f;
        ri->subsc = 0;
        ri->n_sub = 0;
        ri->strand_retained = 0;
        ri->mapq = 0;
        ri->pad = (int32_t)(c - c0);  // the region's chain, until mm_est_err (cleared in mm_set_mapq)
        const int64_t a0 = P.ids[P.cfirst[c] + ri->cnt - 1], a1 = P.ids[P.cfirst[c]];  // first, last anchor
        set_coor(ri, qlen, P.ax[a0], P.ay[a0], P.ax[a1], P.ay[a1], P.c_mlen[c], P.c_blen[c]);
    }
    // ---- mm_set_parent (mask_level, mask_len; no alignment: no dp_max branch)
    {
        int32_t *w = P.w + c0;
        uint64_t *cov = P.cov + c0;
        for (int i = 0; i < n; ++i) r[i].id = i;
        int i, j, k;
        w[0] = 0, r[0].parent = 0;
        for (i = 1, k = 1; i < n; ++i) {
            hymet_mm_reg *ri = &r[i];
            const int si = ri->qs, ei = ri->qe;
            int n_cov = 0, uncov_len = 0;
            for (j = 0; j < k; ++j) {
                const hymet_mm_reg *rp = &r[w[j]];
                int sj = rp->qs, ej = rp->qe;
                if (ej <= si || sj >= ei) continue;
                if (sj < si) sj = si;
                if (ej > ei) ej = ei;
                cov[n_cov++] = (uint64_t)(uint32_t)sj << 32 | (uint32_t)ej;
            }
            if (n_cov == 0) goto set_parent_test;
            {
                int x = si;
                heap_sort(cov, n_cov, [](uint64_t a, uint64_t b) { return a < b; });
                for (int jj = 0; jj < n_cov; ++jj) {
                    if ((int)(cov[jj] >> 32) > x) uncov_len += (int)(cov[jj] >> 32) - x;
                    x = (int32_t)cov[jj] > x ? (int32_t)cov[jj] : x;
                }
                if (ei > x) uncov_len += ei - x;
            }
            for (j = 0; j < k; ++j) {
                hymet_mm_reg *rp = &r[w[j]];
                const int sj = rp->qs, ej = rp->qe;
                if (ej <= si || sj >= ei) continue;
                const int mn = ej - sj < ei - si ? ej - sj : ei - si;
                const int mx = ej - sj > ei - si ? ej - sj : ei - si;
                const int ol = si < sj ? (ei < sj ? 0 : ei < ej ? ei - sj : ej - sj) : (ej < si ? 0 : ej < ei ? ej - si : ei - si);
                if (__fsub_rn(__fdiv_rn((float)ol, (float)mn), __fdiv_rn((float)uncov_len, (float)mx)) > P.mask_level &&
                    uncov_len <= P.mask_len) {
                    const int sci = ri->score;
                    ri->parent = rp->parent;
                    rp->subsc = rp->subsc > sci ? rp->subsc : sci;
                    if (ri->cnt >= rp->cnt) ++rp->n_sub;
                    break;
                }
            }
        set_parent_test:
            if (j == k) w[k++] = i, ri->parent = i, ri->n_sub = 0;
        }
    }
    // ---- mm_select_sub (check_strand = 1) + mm_sync_regs
    {
        const int min_diff = P.k * 2;
        const int min_strand_sc = (int)(P.max_gap * 0.8);
        int i, k, n_2nd = 0;
        for (i = k = 0; i < n; ++i) {
            const int p = r[i].parent;
            if (p == i) {
                r[k++] = r[i];
            } else if (((float)r[i].score >= __fmul_rn((float)r[p].score, P.pri_ratio) || r[i].score + min_diff >= r[p].score) &&
                       n_2nd < P.best_n) {
                if (!(r[i].qs == r[p].qs && r[i].qe == r[p].qe && r[i].rid == r[p].rid && r[i].rs == r[p].rs && r[i].re == r[p].re))
                    r[k++] = r[i], ++n_2nd;
            } else if (n_2nd < P.best_n && r[i].score > min_strand_sc && r[i].rev != r[p].rev) {
                r[i].strand_retained = 1;
                r[k++] = r[i], ++n_2nd;
            }
        }
        if (k != n) {
            int32_t *tmp = P.tmp + c0;
            int max_id = -1;
            for (i = 0; i < k; ++i) max_id = max_id > r[i].id ? max_id : r[i].id;
            for (i = 0; i <= max_id; ++i) tmp[i] = -1;
            for (i = 0; i < k; ++i)
                if (r[i].id >= 0) tmp[r[i].id] = i;
            for (i = 0; i < k; ++i) {
                r[i].id = i;
                if (r[i].parent >= 0 && tmp[r[i].parent] >= 0) r[i].parent = tmp[r[i].parent];
                else r[i].parent = -1;
            }
        }
        n = k;
    }
    // ---- mm_est_err (the per-anchor walk was done by chain_stats_flat_kernel)
    {
        const int64_t m0 = P.mp_off[q];
        const int32_t nm = (int32_t)(P.mp_off[q + 1] - m0);
        if (nm > 0) {
            const uint64_t sum_k = P.q_sumk[q];
            const float avg_k = __fdiv_rn((float)sum_k, (float)nm);
            for (int i = 0; i < n; ++i) {
                hymet_mm_reg *ri = &r[i];
                ri->div = -1.0f;
                if (ri->cnt == 0) continue;
                const int64_t c = c0 + ri->pad;
                const int32_t st = P.c_st[c];
                if (st < 0) continue;
                const int32_t fv = P.c_fv[c] < ri->cnt ? P.c_fv[c] : ri->cnt;
                const int32_t n_match = fv;
                const int32_t en = fv == ri->cnt ? P.c_last[c] : nm - 1;
                const int32_t l_ref = (int32_t)P.ref_len[ri->rid];
                int32_t n_tot = en - st + 1;
                if ((float)ri->qs > avg_k && (float)ri->rs > avg_k) ++n_tot;
                if ((float)(qlen - ri->qe) > avg_k && (float)(l_ref - ri->re) > avg_k) ++n_tot;
                ri->div = n_match >= n_tot ? 0.0f : (float)(1.0 - pow((double)n_match / n_tot, 1.0 / (double)avg_k));
            }
        }
    }
    // ---- mm_filter_strand_retained
    {
        int i, k;
        for (i = k = 0; i < n; ++i) {
            const int p = r[i].parent;
            if (!r[i].strand_retained || r[i].div < __fmul_rn(r[p].div, 5.0f) || r[i].div < 0.01f) {
                if (k < i) r[k++] = r[i];
                else ++k;
            }
        }
        n = k;
    }
    // ---- mm_set_mapq (no alignment)
    {
        const float q_coef = 40.0f;
        int64_t sum_sc = 0;
        for (int i = 0; i < n; ++i)
            if (r[i].parent == r[i].id) sum_sc += r[i].score;
        const float uniq_ratio = __fdiv_rn((float)sum_sc, (float)(sum_sc + P.rep_len[q]));
        for (int i = 0; i < n; ++i) {
            hymet_mm_reg *ri = &r[i];
            ri->pad = 0;
            if (ri->parent == ri->id) {
                const float pen_s1 = __fmul_rn(ri->score > 100 ? 1.0f : __fmul_rn(0.01f, (float)ri->score), uniq_ratio);
                float pen_cm = ri->cnt > 10 ? 1.0f : __fmul_rn(0.1f, (float)ri->cnt);
                pen_cm = pen_s1 < pen_cm ? pen_s1 : pen_cm;
                const int subsc = ri->subsc > P.min_chain_score ? ri->subsc : P.min_chain_score;
                const float x = __fdiv_rn((float)subsc, (float)ri->score);
                int mapq = (int)__fmul_rn(__fmul_rn(__fmul_rn(pen_cm, q_coef), __fsub_rn(1.0f, x)), logf((float)ri->score));
                mapq -= (int)__fadd_rn(__fmul_rn(4.343f, logf((float)(ri->n_sub + 1))), .499f);
                mapq = mapq > 0 ? mapq : 0;
                ri->mapq = mapq < 60 ? mapq : 60;
            } else
                ri->mapq = 0;
        }
    }
    P.n_regs[q] = n;
}

__device__ __forceinline__ void list_append(bool pred, int q, int32_t *list, int32_t *cnt) {  // one atomic per wave
    const uint64_t m = __ballot(pred);
    if (!m) return;
    const int lane = threadIdx.x & 63, leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(cnt, __popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) list[base + __popcll(m & ((1ull << lane) - 1))] = q;
}

// one thread per query; the queries of many chains are listed for regions_wave_kernel
__global__ __launch_bounds__(64) void regions_kernel(RegParams P, int32_t *big, int32_t *n_big) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = q < P.n_q ? (int)(P.qc[q + 1] - P.qc[q]) : 0;
    const bool wq = q < P.n_q && wave_query(P, q, n, (int32_t)P.qlen[q]);
    list_append(wq, q, big, n_big);
    if (q >= P.n_q || wq) return;
    regions_seq(P, q);
}

// ---- one wave per query of many chains: the same steps, lane-parallel where the sequential
// code's decisions allow it, sequential (but on LDS-resident data) where they do not.
__device__ __forceinline__ void wsync() { __syncthreads(); }  // one-wave blocks: LDS order + convergence

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return (uint64_t)(uint32_t)hi << 32 | (uint32_t)lo;
}
// ascending sort of one value per lane across the wave (bitonic network)
__device__ __forceinline__ uint64_t wave_sort_u64(uint64_t v) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int s = 2; s <= 64; s <<= 1)
#pragma unroll
        for (int d = s >> 1; d > 0; d >>= 1) {
            const uint64_t o = shfl_xor64(v, d);
            const bool up = (lane & s) == 0, low = (lane & d) == 0;
            v = (low == up) ? (o < v ? o : v) : (o > v ? o : v);
        }
    return v;
}
__device__ __forceinline__ int wave_excl_max(int v, int init) {  // max over lanes < l (init before lane 0)
    const int lane = threadIdx.x;
    int x = __shfl_up(v, 1, 64);
    if (lane == 0) x = init;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(x, d, 64);
        if (lane >= d) x = max(x, o);
    }
    return x;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
__device__ __forceinline__ int64_t wave_sum_l(int64_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
// descending bitonic sort of m (a power of two) 128-bit keys in LDS, or in the global scratch
// of a query beyond the LDS capacity.  A pass's pairs are disjoint, so kSortU of each lane's
// pairs are loaded before any is compared and stored: in global memory one round trip per
// kSortU pairs instead of per pair (a 5,000-chain query's sort was one wave's serial walk of
// ~6,000 round trips, the launch's tail).
constexpr int kSortU = 4;
__device__ __forceinline__ int bitonic_lo(int t, int d) { return (t / d) * 2 * d + (t % d); }
__device__ void lds_sort_desc(U128 *a, int m) {
    const int half = m >> 1;
    for (int s = 2; s <= m; s <<= 1)
        for (int d = s >> 1; d > 0; d >>= 1) {
            for (int t0 = threadIdx.x; t0 < half; t0 += 64 * kSortU) {
                U128 x[kSortU], y[kSortU];
#pragma unroll
                for (int u = 0; u < kSortU; u++) {
                    const int t = t0 + 64 * u, i = bitonic_lo(t < half ? t : 0, d);
                    x[u] = a[i], y[u] = a[i + d];
                }
#pragma unroll
                for (int u = 0; u < kSortU; u++) {
                    const int t = t0 + 64 * u, i = bitonic_lo(t < half ? t : 0, d);
                    if (t < half && (((i & s) == 0) ? lt128(x[u], y[u]) : lt128(y[u], x[u]))) a[i] = y[u], a[i + d] = x[u];
                }
            }
            wsync();
        }
}
__device__ void lds_sort_asc_u64(uint64_t *a, int m) {
    const int half = m >> 1;
    for (int s = 2; s <= m; s <<= 1)
        for (int d = s >> 1; d > 0; d >>= 1) {
            for (int t0 = threadIdx.x; t0 < half; t0 += 64 * kSortU) {
                uint64_t x[kSortU], y[kSortU];
#pragma unroll
                for (int u = 0; u < kSortU; u++) {
                    const int t = t0 + 64 * u, i = bitonic_lo(t < half ? t : 0, d);
                    x[u] = a[i], y[u] = a[i + d];
                }
#pragma unroll
                for (int u = 0; u < kSortU; u++) {
                    const int t = t0 + 64 * u, i = bitonic_lo(t < half ? t : 0, d);
                    if (t < half && (((i & s) == 0) ? y[u] < x[u] : x[u] < y[u])) a[i] = y[u], a[i + d] = x[u];
                }
            }
            wsync();
        }
}

// the per-query work of one wave on a scratch area of cap entries (LDS, or global memory for
// the queries beyond the LDS capacity; a separate large-LDS launch could not be placed while
// the other mapping stream's chaining grid held the CUs' LDS)
__device__ __forceinline__ void regions_wave(const RegParams &P, int q, unsigned char *rsm, int cap);

// a persistent grid over the listed queries; the last block clears the list counter
__global__ __launch_bounds__(64) void regions_wave_kernel(RegParams P, const int32_t *big, int32_t *n_big, int64_t *mail,
                                                          unsigned char *gscratch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    const int nb = __builtin_amdgcn_readfirstlane(*n_big);
    for (int w = blockIdx.x; w < nb; w += gridDim.x) {
        const int q = __builtin_amdgcn_readfirstlane(big[w]);
        const int n = (int)(P.qc[q + 1] - P.qc[q]);
        if (n <= P.lds_max) {
            regions_wave(P, q, rsm, kRegSmall);
        } else {
            int m = 64;
            while (m < n) m <<= 1;  // < 2n: the query's share of gscratch (kRegScrStride per chain) holds it
            regions_wave(P, q, gscratch + (size_t)P.qc[q] * kRegScrStride, m);
        }
        __threadfence_block();
        wsync();
    }
    publish_counters(n_big, 1, mail);
}

__device__ __forceinline__ void regions_wave(const RegParams &P, int q, unsigned char *rsm, const int CAP) {
    const int lane = threadIdx.x;
    // profiling: section k's cycles added to prof[k - 1] (prof[6]: queries, prof[7]: chains)
    uint64_t rp_t = P.prof ? clock64() : 0;
#define RPROF(k)                                                                       \
    if (P.prof) {                                                                      \
        const uint64_t rp_n = clock64();                                               \
        if ((k) > 0) atomicAdd(P.prof + (k) - 1, lane == 0 ? (unsigned long long)(rp_n - rp_t) : 0ull); \
        rp_t = rp_n;                                                                   \
    }
    const int64_t c0 = P.qc[q], c1 = P.qc[q + 1];
    int n = (int)(c1 - c0);
    const int32_t qlen = (int32_t)P.qlen[q];
    // LDS: slot[i] = (qs, qe, score, cnt) of region i (first the sort keys, in place), aux[i] =
    // (rid | rev << 31, rs, re, -), then per-step arrays
    U128 *zs = reinterpret_cast<U128 *>(rsm);
    int4 *slot = reinterpret_cast<int4 *>(rsm);
    int4 *aux = reinterpret_cast<int4 *>(rsm + 16 * CAP);
    int32_t *wl = reinterpret_cast<int32_t *>(rsm + 32 * CAP);  // primaries (set_parent), kept list (select_sub)
    int32_t *psub = wl + CAP, *pns = psub + CAP;                 // per primary: subsc, n_sub (set_parent)
    uint64_t *covb = reinterpret_cast<uint64_t *>(pns + CAP);    // overlapping intervals (set_parent)
    const int64_t b0 = P.qb[q];
    hymet_mm_reg *r = P.regs + c0;
    uint32_t hash = P.name_hash[q];
    hash ^= wang32((uint32_t)qlen) + wang32((uint32_t)P.seed);
    hash = wang32(hash);
    RPROF(0);
    // ---- mm_gen_regs: keys (score<<32 | cnt) ^ hash, sorted descending (keys are distinct:
    // y holds the chain's anchor offset), padded to a power of two with (0, 0)
    int m = 64;
    while (m < n) m <<= 1;
    for (int i = lane; i < m; i += 64) {
        U128 zz{0, 0};
        if (i < n) {
            const int64_t k = P.cboff[c0 + i] - b0;
            const uint64_t u = P.cu[c0 + i];
            const int64_t a = P.ids[P.cfirst[c0 + i] + (int32_t)u - 1];
            const uint32_t h = (uint32_t)hash64((hash64(P.ax[a]) + hash64(P.ay[a])) ^ hash);
            zz.x = u ^ h;
            zz.y = (uint64_t)k << 32 | (uint32_t)i;  // the chain index, not its count (as regions_seq)
        }
        zs[i] = zz;
    }
    wsync();
    RPROF(1);
    lds_sort_desc(zs, m);
    for (int i = lane; i < n; i += 64) {
        const U128 zi = zs[i];
        hymet_mm_reg ri;
        ri.id = i;
        ri.parent = -1;
        ri.score = (int32_t)(zi.x >> 32);
        ri.hash = (uint32_t)zi.x;
        const int64_t c = c0 + (uint32_t)zi.y;
        ri.cnt = (int32_t)P.cu[c];
        ri.as = (int32_t)(zi.y >> 32);
        ri.div = -1.0f;
        ri.subsc = 0;
        ri.n_sub = 0;
        ri.strand_retained = 0;
        ri.mapq = 0;
        ri.pad = (int32_t)(c - c0);  // the region's chain, until mm_est_err (cleared in mm_set_mapq)
        const int64_t a0 = P.ids[P.cfirst[c] + ri.cnt - 1], a1 = P.ids[P.cfirst[c]];
        set_coor(&ri, qlen, P.ax[a0], P.ay[a0], P.ax[a1], P.ay[a1], P.c_mlen[c], P.c_blen[c]);
        r[i] = ri;
        slot[i] = make_int4(ri.qs, ri.qe, ri.score, ri.cnt);  // this lane's own sort slot
        aux[i] = make_int4(ri.rid | ri.rev << 31, ri.rs, ri.re, 0);
    }
    wsync();
    RPROF(2);
    // ---- mm_set_parent: sequential over regions; each region is tested against all primaries
    // so far lane-parallel (the sequential loop's first match = the lowest matching lane).
    // Primaries 0..63 live in registers (lane j: primary j's qs, qe, cnt, region index and
    // its subsc / n_sub so far) and the regions' (qs, qe, score, cnt) come 64 at a time from
    // LDS, so a query of up to 64 primaries runs its walk without an LDS round trip or barrier
    // per region; primaries from the 65th on keep the LDS lists (wl / psub / pns).
    // (P.prim_regs < 64, tests: fewer primaries in registers, the rest through the lists.)
    {
        const int R = P.prim_regs;
        int ps = 0, pe = 0, pc = 0, pw = 0, psb = 0, pnb = 0;  // lane j: primary j (j < 64)
        if (lane == 0) {
            const int4 s0 = slot[0];
            ps = s0.x, pe = s0.y, pc = s0.w;
            r[0].parent = 0;
            if (R == 0) wl[0] = 0, psub[0] = 0, pns[0] = 0;
        }
        if (R == 0) wsync();
        int k = 1;
        int4 my = make_int4(0, 0, 0, 0);  // lane l: region (i & ~63) + l
        for (int i = 1; i < n; ++i) {
            if (i == 1 || (i & 63) == 0) my = slot[min((i & ~63) + lane, n - 1)];
            const int li = i & 63;
            const int si = __builtin_amdgcn_readlane(my.x, li), ei = __builtin_amdgcn_readlane(my.y, li);
            const int sci = __builtin_amdgcn_readlane(my.z, li), cnti = __builtin_amdgcn_readlane(my.w, li);
            int jfound = -1;
            if (k <= R) {
                const bool ov = lane < k && !(pe <= si || ps >= ei);
                const uint64_t mov = __ballot(ov);
                if (mov) {
                    // uncovered length of [si, ei]: the sorted sweep x = running max of ends
                    const uint64_t kvl = ov ? (uint64_t)(uint32_t)max(ps, si) << 32 | (uint32_t)min(pe, ei) : ~0ull;
                    const int ncov = __popcll(mov);
                    int uncov = 0, carry = si;
                    if (ncov == 1) {  // one overlapping primary: its clipped interval is the union
                        const int l1 = __ffsll((unsigned long long)mov) - 1;
                        const int s_ = (int)__builtin_amdgcn_readlane((int)(kvl >> 32), l1);
                        const int e_ = (int)__builtin_amdgcn_readlane((int)(uint32_t)kvl, l1);
                        uncov = s_ > si ? s_ - si : 0;
                        carry = max(si, e_);
                    } else {
                        const uint64_t kv = wave_sort_u64(kvl);
                        const int s_ = (int)(kv >> 32), e_ = lane < ncov ? (int)(uint32_t)kv : INT32_MIN;
                        const int x = wave_excl_max(e_, si);
                        uncov = wave_sum_i(lane < ncov && s_ > x ? s_ - x : 0);
                        carry = max(si, wave_max_i(e_));
                    }
                    if (ei > carry) uncov += ei - carry;
                    bool hit = false;
                    if (ov) {
                        const int sj = ps, ej = pe;
                        const int mn = ej - sj < ei - si ? ej - sj : ei - si;
                        const int mx = ej - sj > ei - si ? ej - sj : ei - si;
                        const int ol = si < sj ? (ei < sj ? 0 : ei < ej ? ei - sj : ej - sj)
                                               : (ej < si ? 0 : ej < ei ? ej - si : ei - si);
                        hit = __fsub_rn(__fdiv_rn((float)ol, (float)mn), __fdiv_rn((float)uncov, (float)mx)) > P.mask_level &&
                              uncov <= P.mask_len;
                    }
                    const uint64_t mh = __ballot(hit);
                    if (mh) jfound = __ffsll((unsigned long long)mh) - 1;
                }
            } else {
                // overlapping primaries, clipped, gathered in primary order (chunk 0 from registers)
                int ncov = 0;
                for (int jb = 0; jb < k; jb += 64) {
                    const int j = jb + lane;
                    int sj = ps, ej = pe;
                    if (j >= R) {
                        sj = 0, ej = 0;
                        if (j < k) {
                            const int4 o = slot[wl[j]];
                            sj = o.x, ej = o.y;
                        }
                    }
                    const bool ov = j < k && !(ej <= si || sj >= ei);
                    const uint64_t mov = __ballot(ov);
                    if (ov) covb[ncov + __popcll(mov & ((1ull << lane) - 1))] = (uint64_t)(uint32_t)max(sj, si) << 32 | (uint32_t)min(ej, ei);
                    ncov += __popcll(mov);
                }
                wsync();
                if (ncov > 0) {
                    int uncov = 0, carry = si;
                    if (ncov == 1) {
                        const uint64_t kv = covb[0];
                        const int s_ = (int)(kv >> 32), e_ = (int)(uint32_t)kv;
                        uncov = s_ > si ? s_ - si : 0;
                        carry = max(si, e_);
                    } else if (ncov <= 64) {
                        const uint64_t kv = wave_sort_u64(lane < ncov ? covb[lane] : ~0ull);
                        const int s_ = (int)(kv >> 32), e_ = lane < ncov ? (int)(uint32_t)kv : INT32_MIN;
                        const int x = wave_excl_max(e_, si);
                        uncov = wave_sum_i(lane < ncov && s_ > x ? s_ - x : 0);
                        carry = max(si, wave_max_i(e_));
                    } else {
                        int mm = 64;
                        while (mm < ncov) mm <<= 1;
                        for (int t = ncov + lane; t < mm; t += 64) covb[t] = ~0ull;
                        wsync();
                        lds_sort_asc_u64(covb, mm);
                        for (int tb = 0; tb < ncov; tb += 64) {
                            const int t = tb + lane;
                            const uint64_t kv = t < ncov ? covb[t] : ~0ull;
                            const int s_ = (int)(kv >> 32), e_ = t < ncov ? (int)(uint32_t)kv : INT32_MIN;
                            const int x = wave_excl_max(e_, carry);
                            uncov += wave_sum_i(t < ncov && s_ > x ? s_ - x : 0);
                            carry = max(carry, wave_max_i(e_));
                        }
                    }
                    if (ei > carry) uncov += ei - carry;
                    // the first primary (in order) that region i is a secondary of
                    for (int jb = 0; jb < k && jfound < 0; jb += 64) {
                        const int j = jb + lane;
                        bool hit = false;
                        int sj = ps, ej = pe;
                        bool in = true;
                        if (j >= R) {
                            in = j < k;
                            if (in) {
                                const int4 o = slot[wl[j]];
                                sj = o.x, ej = o.y;
                            }
                        }
                        if (in && !(ej <= si || sj >= ei)) {
                            const int mn = ej - sj < ei - si ? ej - sj : ei - si;
                            const int mx = ej - sj > ei - si ? ej - sj : ei - si;
                            const int ol = si < sj ? (ei < sj ? 0 : ei < ej ? ei - sj : ej - sj)
                                                   : (ej < si ? 0 : ej < ei ? ej - si : ei - si);
                            hit = __fsub_rn(__fdiv_rn((float)ol, (float)mn), __fdiv_rn((float)uncov, (float)mx)) > P.mask_level &&
                                  uncov <= P.mask_len;
                        }
                        const uint64_t mh = __ballot(hit);
                        if (mh) jfound = jb + __ffsll((unsigned long long)mh) - 1;
                    }
                }
            }
            if (jfound >= 0) {
                if (jfound < R) {
                    const int p = __builtin_amdgcn_readlane(pw, jfound);
                    if (lane == 0) r[i].parent = p;
                    if (lane == jfound) {
                        psb = psb > sci ? psb : sci;
                        if (cnti >= pc) ++pnb;
                    }
                } else {
                    const int p = wl[jfound];
                    if (lane == 0) {
                        r[i].parent = p;
                        psub[jfound] = psub[jfound] > sci ? psub[jfound] : sci;
                        if (cnti >= slot[p].w) ++pns[jfound];
                    }
                    wsync();
                }
            } else {
                if (k < R) {
                    if (lane == k) ps = si, pe = ei, pc = cnti, pw = i, psb = 0, pnb = 0;
                } else {
                    if (lane == 0) wl[k] = i, psub[k] = 0, pns[k] = 0;
                }
                if (lane == 0) r[i].parent = i;
                ++k;
                if (k > R) wsync();
            }
        }
        if (lane < k && lane < R) {
            r[pw].subsc = psb;
            r[pw].n_sub = pnb;
        }
        for (int j = R + lane; j < k; j += 64) {
            r[wl[j]].subsc = psub[j];
            r[wl[j]].n_sub = pns[j];
        }
    }
    __threadfence_block();
    wsync();
    RPROF(3);
    // ---- mm_select_sub (check_strand = 1) + mm_sync_regs.  The sequential loop compacts in
    // place and reads r[p] afterwards, so a parent position already overwritten by a kept
    // region holds THAT region: position p holds the p-th kept region once more than p are
    // kept.  Decisions run in order (lane by lane inside each 64-region chunk), on the
    // original records held in LDS; the compaction is applied afterwards.
    int nk = 0;
    {
        const int min_diff = P.k * 2;
        const int min_strand_sc = (int)(P.max_gap * 0.8);
        int n_2nd = 0;
        int32_t *kept = wl;                 // kept[o] = original index of output position o
        uint64_t *sflag = covb;             // strand_retained, one bit per original index
        for (int t = lane; t < (n + 63) / 64; t += 64) sflag[t] = 0;
        wsync();
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            const int pl = i < n ? r[i].parent : 0;
            uint64_t keepm = 0, strm = 0;
            const int cnt_chunk = min(64, n - base);
            for (int l = 0; l < cnt_chunk; ++l) {
                const int ii = base + l, p = __builtin_amdgcn_readlane(pl, l);
                bool keep = false, str = false;
                if (p == ii) {
                    keep = true;
                } else {
                    const int src = nk > p ? kept[p] : p;  // what position p holds by now
                    const int4 mi = slot[ii], xi = aux[ii], mp = slot[src], xp = aux[src];
                    if (((float)mi.z >= __fmul_rn((float)mp.z, P.pri_ratio) || mi.z + min_diff >= mp.z) && n_2nd < P.best_n) {
                        if (!(mi.x == mp.x && mi.y == mp.y && (xi.x & 0x7fffffff) == (xp.x & 0x7fffffff) && xi.y == xp.y &&
                              xi.z == xp.z))
                            keep = true, ++n_2nd;
                    } else if (n_2nd < P.best_n && mi.z > min_strand_sc && ((uint32_t)xi.x >> 31) != ((uint32_t)xp.x >> 31)) {
                        keep = str = true, ++n_2nd;
                    }
                }
                if (keep) {
                    if (lane == 0) kept[nk] = ii;
                    keepm |= 1ull << l;
                    ++nk;
                }
                if (str) strm |= 1ull << l;
                wsync();
            }
            if (lane == 0) sflag[base >> 6] = strm;
            wsync();
        }
        // compaction (output chunks in order: every source index is >= its output position)
        if (nk != n) {
            for (int ob = 0; ob < nk; ob += 64) {
                const int o = ob + lane;
                hymet_mm_reg v;
                if (o < nk) {
                    const int src = kept[o];
                    v = r[src];
                    if (sflag[src >> 6] >> (src & 63) & 1) v.strand_retained = 1;
                }
                __threadfence_block();
                wsync();
                if (o < nk) r[o] = v;
                __threadfence_block();
                wsync();
            }
            // mm_sync_regs: ids are the original indices; new index of original j = its position
            int32_t *pos_of = psub;  // n entries
            for (int j = lane; j < n; j += 64) pos_of[j] = -1;
            wsync();
            for (int o = lane; o < nk; o += 64) pos_of[kept[o]] = o;
            wsync();
            for (int o = lane; o < nk; o += 64) {
                const int par = r[o].parent;
                r[o].id = o;
                r[o].parent = par >= 0 && pos_of[par] >= 0 ? pos_of[par] : -1;
            }
        } else {
            for (int o = lane; o < n; o += 64)
                if (sflag[o >> 6] >> (o & 63) & 1) r[o].strand_retained = 1;
        }
        n = nk;
    }
    __threadfence_block();
    wsync();
    RPROF(4);
    // ---- mm_est_err (per region)
    {
        const int64_t m0 = P.mp_off[q];
        const int32_t nm = (int32_t)(P.mp_off[q + 1] - m0);
        if (nm > 0) {
            const uint64_t sum_k = P.q_sumk[q];
            const float avg_k = __fdiv_rn((float)sum_k, (float)nm);
            for (int i = lane; i < n; i += 64) {
                hymet_mm_reg *ri = &r[i];
                float div = -1.0f;
                if (ri->cnt != 0) {
                    const int64_t c = c0 + ri->pad;
                    const int32_t st = P.c_st[c];
                    if (st >= 0) {
                        const int32_t fv = P.c_fv[c] < ri->cnt ? P.c_fv[c] : ri->cnt;
                        const int32_t n_match = fv;
                        const int32_t en = fv == ri->cnt ? P.c_last[c] : nm - 1;
                        const int32_t l_ref = (int32_t)P.ref_len[ri->rid];
                        int32_t n_tot = en - st + 1;
                        if ((float)ri->qs > avg_k && (float)ri->rs > avg_k) ++n_tot;
                        if ((float)(qlen - ri->qe) > avg_k && (float)(l_ref - ri->re) > avg_k) ++n_tot;
                        div = n_match >= n_tot ? 0.0f : (float)(1.0 - pow((double)n_match / n_tot, 1.0 / (double)avg_k));
                    }
                }
                ri->div = div;
            }
        }
    }
    __threadfence_block();
    wsync();
    RPROF(5);
    // ---- mm_filter_strand_retained: exact in parallel up to the first dropped region (no
    // position has moved before it); from there the sequential loop (drops are rare)
    {
        int first_drop = n;
        for (int base = 0; base < n && first_drop == n; base += 64) {
            const int i = base + lane;
            bool drop = false;
            if (i < n && r[i].strand_retained) {
                const int p = r[i].parent;
                drop = !(r[i].div < __fmul_rn(r[p].div, 5.0f) || r[i].div < 0.01f);
            }
            const uint64_t md = __ballot(drop);
            if (md) first_drop = base + __ffsll((unsigned long long)md) - 1;
        }
        if (first_drop < n) {
            if (lane == 0) {
                int i, k = first_drop;
                for (i = first_drop + 1; i < n; ++i) {
                    const int p = r[i].parent;
                    if (!r[i].strand_retained || r[i].div < __fmul_rn(r[p].div, 5.0f) || r[i].div < 0.01f) r[k++] = r[i];
                }
                psub[0] = k;
            }
            __threadfence_block();
            wsync();
            n = psub[0];
        }
    }
    __threadfence_block();
    wsync();
    // ---- mm_set_mapq (no alignment)
    {
        const float q_coef = 40.0f;
        int64_t sum_sc = 0;
        for (int i = lane; i < n; i += 64)
            if (r[i].parent == r[i].id) sum_sc += r[i].score;
        sum_sc = wave_sum_l(sum_sc);
        const float uniq_ratio = __fdiv_rn((float)sum_sc, (float)(sum_sc + P.rep_len[q]));
        for (int i = lane; i < n; i += 64) {
            hymet_mm_reg *ri = &r[i];
            ri->pad = 0;
            if (ri->parent == ri->id) {
                const float pen_s1 = __fmul_rn(ri->score > 100 ? 1.0f : __fmul_rn(0.01f, (float)ri->score), uniq_ratio);
                float pen_cm = ri->cnt > 10 ? 1.0f : __fmul_rn(0.1f, (float)ri->cnt);
                pen_cm = pen_s1 < pen_cm ? pen_s1 : pen_cm;
                const int subsc = ri->subsc > P.min_chain_score ? ri->subsc : P.min_chain_score;
                const float x = __fdiv_rn((float)subsc, (float)ri->score);
                int mapq = (int)__fmul_rn(__fmul_rn(__fmul_rn(pen_cm, q_coef), __fsub_rn(1.0f, x)), logf((float)ri->score));
                mapq -= (int)__fadd_rn(__fmul_rn(4.343f, logf((float)(ri->n_sub + 1))), .499f);
                mapq = mapq > 0 ? mapq : 0;
                ri->mapq = mapq < 60 ? mapq : 60;
            } else
                ri->mapq = 0;
        }
    }
    RPROF(6);
    if (P.prof) {
        atomicAdd(P.prof + 6, lane == 0 ? 1ull : 0ull);
        atomicAdd(P.prof + 7, lane == 0 ? (unsigned long long)(c1 - c0) : 0ull);
    }
#undef RPROF
    if (lane == 0) P.n_regs[q] = n;
}

// per-chain stats accumulators: mlen = blen = 0, first-anchor minimum = 0x7f7f7f7f
__global__ void chain_stats_init_kernel(int32_t *c_mlen, int32_t *c_blen, int32_t *c_fv, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c_mlen[i] = 0, c_blen[i] = 0, c_fv[i] = 0x7f7f7f7f;
}

}  // namespace

int launch_regions(hymet_ctx *ctx, const uint64_t *ax, const uint64_t *ay, const int64_t *ids, const int64_t *cfirst,
                   const uint64_t *cu, const int64_t *cboff,
                   const int64_t *qc, const int64_t *qb, const uint64_t *mini_pos, const int64_t *mp_off, const int64_t *qlen,
                   const uint32_t *name_hash, const int32_t *rep_len, const int64_t *ref_len, int n_q, const hymet_mm_opt *o,
                   int k, void *z, hymet_mm_reg *regs, int32_t *w, uint64_t *cov, int32_t *tmp, int32_t *n_regs,
                   int64_t NB, int64_t NC, int64_t NM, const uint32_t *cq,
                   const MiniWord *mtab, const int64_t *qbase, const uint32_t *skip_q, uint64_t *sumk, bool sumk_done) {
    if (n_q <= 0) return HYMET_OK;
    hipStream_t st = ctx->stream;
    DevBuf cst, blk;
    HY_HIP(cst.alloc(4 * 5 * (size_t)(NC + 1), st));
    int32_t *c_mlen = cst.as<int32_t>(), *c_blen = c_mlen + (NC + 1), *c_st = c_blen + (NC + 1), *c_last = c_st + (NC + 1),
            *c_fv = c_last + (NC + 1);
    {
        // chain slot (8) + anchor x, y (16) + its minimizer-table read (4: 16 B per 64 bases) per chained anchor
        ProfScope _ps(ctx, "mm_chain_stats", (double)NB * (8.0 + 16.0 + 4.0) + (double)NM * 8.0);
        AnchorStatParams A{ax, ay, cu, ids, cfirst, cboff, qb, qlen, mp_off, mini_pos, NB, NC, n_q, cq,
                           c_mlen, c_blen, c_st, c_last, mtab, qbase, skip_q};
        if (NB > 0) {
            hipLaunchKernelGGL(chain_stats_init_kernel, dim3((unsigned)cdiv(NC + 1, 256)), dim3(256), 0, st, c_mlen, c_blen,
                               c_fv, NC + 1);
            HY_CHECK_LAUNCH("chain_stats_init_kernel");
            HY_HIP(blk.alloc(4 * (size_t)(cdiv(NB, kStatSpan) + 1), st));
            hipLaunchKernelGGL(block_chain_kernel, dim3((unsigned)cdiv(NC, 256)), dim3(256), 0, st, cboff, NC, NB,
                               blk.as<int32_t>());
            HY_CHECK_LAUNCH("block_chain_kernel");
            hipLaunchKernelGGL(chain_stats_flat_kernel, dim3((unsigned)cdiv(NB, kStatSpan)), dim3(256), 0, st, A,
                               (const int32_t *)blk.as<int32_t>(), c_fv);
            HY_CHECK_LAUNCH("chain_stats_flat_kernel");
        }
        if (!sumk_done) {  // per query, shared by the batch's two chain sets
            const int nqb = n_q < ctx->n_cu * 64 ? n_q : ctx->n_cu * 64;
            hipLaunchKernelGGL(query_sumk_kernel, dim3((unsigned)nqb), dim3(64), 0, st, mini_pos, mp_off, n_q,
                               (unsigned long long *)sumk);
            HY_CHECK_LAUNCH("query_sumk_kernel");
        }
    }
    RegParams P{ax, ay, ids, cfirst, cu, cboff, qc, qb, mini_pos, mp_off, qlen, name_hash, rep_len, ref_len, n_q, o->seed, k,
                o->mask_level, o->pri_ratio, o->mask_len, o->best_n, o->max_gap, o->min_chain_score, (U128 *)z, regs, w, cov,
                tmp, n_regs, c_mlen, c_blen, c_st, c_last, c_fv, sumk, skip_q, kRegWave, kRegSmall, nullptr, 64};
    // tests / A-B: HYMET_REG_WAVE (chains above which a query takes the wave kernel),
    // HYMET_REG_LDS (chains up to which the wave kernel works in LDS; 32: every wave query on the
    // global-scratch path from 33 chains: a query's share of that scratch, 2n entries, holds
    // its power-of-two working size only from there)
    const char *ew = getenv("HYMET_REG_WAVE"), *el = getenv("HYMET_REG_LDS");
    if (ew && atoi(ew) >= 0) P.wave_min = atoi(ew);
    if (el) P.lds_max = std::max(32, std::min(kRegSmall, atoi(el)));
    if (const char *ep = getenv("HYMET_REG_PRIM")) P.prim_regs = std::max(0, std::min(64, atoi(ep)));
    ProfScope _ps(ctx, "mm_regions", (double)NC * (8.0 + 8.0 + 4.0 * 5) + (double)n_q * 64.0);  // chain + stats reads, reg writes
    static const bool reg_stats = getenv("HYMET_REG_STATS") != nullptr;  // diagnostic: chains per query
    if (reg_stats) {
        std::vector<int64_t> hq(n_q + 1);
        HY_HIP(hipMemcpyAsync(hq.data(), qc, 8 * (size_t)(n_q + 1), hipMemcpyDeviceToHost, st));
        HY_HIP(hipStreamSynchronize(st));
        int64_t h[8] = {0}, mx = 0, tot = 0, big_tot = 0;
        for (int q = 0; q < n_q; q++) {
            const int64_t c = hq[q + 1] - hq[q];
            const int b = c <= 48 ? 0 : c <= 256 ? 1 : c <= 1024 ? 2 : c <= 2048 ? 3 : c <= 8192 ? 4 : 5;
            h[b]++, mx = c > mx ? c : mx, tot += c;
            if (c > 2048) big_tot += c;
        }
        fprintf(stderr, "[regions] n_q %d anchors %lld chains %lld max %lld | <=48 %lld <=256 %lld <=1k %lld <=2k %lld <=8k %lld >8k %lld (chains in >2k: %lld)\n",
                n_q, (long long)NB, (long long)tot, (long long)mx, (long long)h[0], (long long)h[1], (long long)h[2], (long long)h[3],
                (long long)h[4], (long long)h[5], (long long)big_tot);
    }
    if (getenv("HYMET_REG_PROF")) {
        HY_HIP(hipMalloc((void **)&P.prof, 8 * 8));
        HY_HIP(hipMemsetAsync(P.prof, 0, 8 * 8, st));
    }
    DevBuf big, gscr;
    HY_HIP(big.alloc(4 * (size_t)n_q, st));
    HY_HIP(gscr.alloc((size_t)kRegScrStride * (size_t)(NC + 1), st));
    int32_t *n_big = ctx->dctr + kCtrRegBig;  // self-clearing (regions_wave_kernel's last block)
    hipLaunchKernelGGL(regions_kernel, dim3((unsigned)cdiv(n_q, 64)), dim3(64), 0, st, P, big.as<int32_t>(), n_big);
    HY_CHECK_LAUNCH("regions_kernel");
    // the listed queries of many chains, one wave each: regions in 13 KB of LDS (up to
    // kRegSmall chains), beyond that in a global scratch area
    hipLaunchKernelGGL(regions_wave_kernel, dim3((unsigned)std::min<int64_t>(n_q, 12 * (int64_t)ctx->n_cu)), dim3(64),
                       (size_t)kRegSmall * kRegEntryBytes, st, P, (const int32_t *)big.as<int32_t>(), n_big,
                       mb_dev(ctx, kMbRegBig), gscr.as<unsigned char>());
    HY_CHECK_LAUNCH("regions_wave_kernel");
    if (P.prof) {  // diagnostic: section cycles of the wave kernel's queries
        unsigned long long h[8];
        HY_HIP(hipMemcpyAsync(h, P.prof, sizeof h, hipMemcpyDeviceToHost, st));
        HY_HIP(hipStreamSynchronize(st));
        fprintf(stderr, "[regprof] queries %llu chains %llu | Mcycles keys %.1f sort+fill %.1f parent %.1f select %.1f est %.1f filter+mapq %.1f\n",
                h[6], h[7], h[0] / 1e6, h[1] / 1e6, h[2] / 1e6, h[3] / 1e6, h[4] / 1e6, h[5] / 1e6);
        (void)hipFree(P.prof);
    }
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet
