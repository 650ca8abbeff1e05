// Mapping of query contigs against one minimizer-index part with minimap2's asm10 settings
// (replaces `minimap2 -x asm10 reference.mmi input/ *.fna`, scripts/minimap2.sh:23;
// SURVEY.md §3.4, §8a rows A2-A4).  Stage by stage (map.c mm_map_frag):
//   1 sketch every query (mm_sketch_kernel, rid 0)
//   2 mm_seed_mz_flt: per-query over-represented minimizers (an LDS bucket screen per query;
//     a (query, x) radix sort + run count only for the queries it cannot clear)
//   3 seeds: CSR lookup of every minimizer (two adjacent loads), then one thread per query
//     replays mm_seed_select / mm_collect_matches (high-occurrence streaks, rep_len,
//     mini_pos) -- sequential by nature but O(minimizers) and parallel over queries
//   4 anchors: exclusive scan of seed occurrence counts, one thread per seed writes them
//   5 sort anchors by (query, strand, target, tpos, qpos): the grouped per-query sort of
//     mm_asort.hip (block sorts in LDS; the library's LSD radix sort only for groups of
//     more than 16384 anchors)
//   6 groups (query, strand, target) -> chain_groups_kernel (one wave per group) ->
//     backtrack_groups_kernel -> chains ordered by first anchor (compact_a)
//   7 long-join re-chain of the chained anchors with bw_long for the queries that need it
//   8 one thread per query: mm_gen_regs, mm_set_parent, mm_select_sub, mm_est_err,
//     mm_filter_strand_retained, mm_set_mapq
// Canonical tie-breaks T1-T4 are those of oracle/mm_oracle.c.
#include "mm_common.hpp"
#include "sort.hpp"

#include <algorithm>
#include <type_traits>
#include <utility>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

struct hymet_mm_result {
    int n_q = 0;
    std::vector<int64_t> reg_off;   // n_q + 1
    std::vector<int32_t> rep_len;   // n_q
    std::vector<hymet_mm_reg> regs;
};

namespace hymet {
namespace mm {

int launch_chain(hymet_ctx *ctx, const int32_t *ax, const uint64_t *ay, const int64_t *g_start, const uint8_t *g_qfirst,
                 const int32_t *order, int32_t n_work, int32_t *f, int64_t *p, int32_t *t_global, int max_dist,
                 int max_dist_inner, int bw, int max_chn_skip, int cap_rmq_size, float pen_gap, float pen_skip,
                 int64_t n_anchors, int64_t n_groups);
int launch_backtrack(hymet_ctx *ctx, const int64_t *g_start, const int32_t *f, const int64_t *p, int32_t *t,
                     const int32_t *z_cnt, const int32_t *z_idx, int32_t n_groups, const int32_t *order, int32_t n_work,
                     int min_cnt, int min_sc, int max_drop, int64_t *chain_ids, uint64_t *chain_u, int64_t *chain_first,
                     int32_t *n_chains, int64_t n_anchors);

namespace {

__device__ __forceinline__ int upper_idx(const int64_t *off, int n, int64_t v) {  // last s with off[s] <= v
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= v) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// qid[i] = query of entry i; also ones[i] = 1 (i < n) and zq[q] = 0 (q < n_q) when given
// (grid: max(n, n_q) threads)
__global__ void fill_qid_kernel(const int64_t *off, int n_q, int64_t n, uint32_t *qid, uint32_t *ones, int32_t *zq) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        qid[i] = (uint32_t)upper_idx(off, n_q, i);
        if (ones) ones[i] = 1u;
    }
    if (zq && i < n_q) zq[i] = 0;
}

// per query: its chain anchors when the long join re-chains it, else 0; entry n_q = 0 (the
// scan's total slot); *any = 1 when some query is flagged (the host zeroes the word first)
__global__ void flagged_len_kernel(const uint32_t *flag, const int64_t *qb, int n_q, uint32_t *cnt, int64_t *any) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q > n_q) return;
    if (q == n_q) {
        cnt[q] = 0;
        return;
    }
    const bool f = flag[q] != 0;
    cnt[q] = f ? (uint32_t)(qb[q + 1] - qb[q]) : 0u;
    if (f) *any = 1;
}

__global__ void iota_u32_kernel(uint32_t *a, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (uint32_t)i;
}

template <typename T>
__global__ void gather_kernel(const T *__restrict__ src, const uint32_t *__restrict__ idx, T *__restrict__ dst, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

// seed.c mm_seed_mz_flt: runs of equal (query, x) in the sorted order
__global__ void mzflt_runs_kernel(const uint32_t *sq, const uint64_t *sx, const uint32_t *sidx, const int64_t *qm_off,
                                  int64_t n, int q_occ_max, float q_occ_frac, uint32_t *keep) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    if (p > 0 && sq[p] == sq[p - 1] && sx[p] == sx[p - 1]) return;  // not a run start
    int64_t e = p + 1;
    while (e < n && sq[e] == sq[p] && sx[e] == sx[p]) e++;
    const uint32_t q = sq[p];
    const int64_t nq = qm_off[q + 1] - qm_off[q];
    if (nq <= q_occ_max) return;  // mm_seed_mz_flt returns early for this query
    const int32_t cnt = (int32_t)(e - p);
    if (cnt > q_occ_max && (float)cnt > (float)nq * q_occ_frac)
        for (int64_t j = p; j < e; j++) keep[sidx[j]] = 0;
}

// mm_seed_mz_flt screen, one block per query: its minimizers are counted into 4096 LDS
// buckets by hash.  A bucket's count bounds the count of every x in it, so a query whose
// buckets all stay at or below q_occ_max has no run to drop (exactly: the filter needs
// cnt > q_occ_max); the others get cnt[q] = their minimizer count and go to the exact (q, x)
// sort.  Also sets keep = 1 for every minimizer.  Block n_q writes the scan's total slot.
constexpr int kMzBuckets = 4096;
__global__ __launch_bounds__(256) void mzflt_screen_kernel(const uint64_t *mx, const int64_t *qm_off, int n_q, int q_occ_max,
                                                           uint32_t *keep, uint32_t *cnt, int64_t *any) {
    __shared__ uint32_t h[kMzBuckets];
    __shared__ int hit;
    const int q = blockIdx.x;
    if (q == n_q) {
        if (threadIdx.x == 0) cnt[q] = 0;
        return;
    }
    const int64_t s = qm_off[q], nq = qm_off[q + 1] - s;
    for (int64_t e = threadIdx.x; e < nq; e += 256) keep[s + e] = 1u;
    if (nq <= q_occ_max) {  // mm_seed_mz_flt returns early for this query
        if (threadIdx.x == 0) cnt[q] = 0;
        return;
    }
    for (int b = threadIdx.x; b < kMzBuckets; b += 256) h[b] = 0;
    if (threadIdx.x == 0) hit = 0;
    __syncthreads();
    bool over = false;
    for (int64_t e = threadIdx.x; e < nq; e += 256)
        over |= atomicAdd(&h[(uint32_t)(mx[s + e] >> 8) & (kMzBuckets - 1)], 1u) >= (uint32_t)q_occ_max;
    if (over) hit = 1;
    __syncthreads();
    if (threadIdx.x == 0) {
        cnt[q] = hit ? (uint32_t)nq : 0u;
        if (hit) *any = 1;
    }
}

// the flagged queries' minimizers as one list: global index and query per list entry
__global__ __launch_bounds__(256) void mzflt_list_kernel(const int64_t *qm_off, const uint32_t *cnt, const int64_t *coff,
                                                         uint32_t *gidx, uint32_t *sq) {
    const int q = blockIdx.x;
    const uint32_t nq = cnt[q];
    if (nq == 0) return;
    const int64_t s = qm_off[q], d = coff[q];
    for (uint32_t e = threadIdx.x; e < nq; e += 256) {
        gidx[d + e] = (uint32_t)(s + e);
        sq[d + e] = (uint32_t)q;
    }
}

// out[i] = src[idx[i]] as u64 (x of a list entry) and gout[i] = gidx[perm[i]]
__global__ void mzflt_gather_kernel(const uint32_t *perm, const uint32_t *gidx, const uint64_t *mx, uint32_t *gout,
                                    uint64_t *xout, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = gidx[perm[i]];
    gout[i] = g;
    xout[i] = mx[g];
}

// (also completes the exclusive scan: pos[n] = the kept total)
__global__ void compact_mz_kernel(const uint64_t *x, const uint64_t *y, const uint32_t *keep, int64_t *pos, int64_t n,
                                  uint64_t *ox, uint64_t *oy) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == n - 1) pos[n] = pos[i] + keep[i];
    if (i < n && keep[i]) {
        ox[pos[i]] = x[i];
        oy[pos[i]] = y[i];
    }
}

__global__ void sample_off_kernel(const int64_t *pos, const int64_t *qm_off, int n_q, int64_t total, int64_t *out) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q > n_q) return;
    out[q] = q == n_q ? total : pos[qm_off[q]];
}

// occurrences of every minimizer (one thread each)
__global__ void seed_count_kernel(const uint64_t *mx, int64_t n, const uint32_t *koff, int64_t n_buckets,
                                  uint32_t *seed_n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = mx[i] >> 8;
    uint32_t c = 0;
    if ((int64_t)h < n_buckets) c = koff[h + 1] - koff[h];
    seed_n[i] = c;
}

// ---- mm_seed_select + mm_collect_matches (seed.c), flat over the batch's minimizers.
// The sequential per-query loop is decomposed:
//   * every seed is low (n <= max_occ) or high; one scan of packed (low, high) counts ranks
//     them, and the low / high seeds are listed in order;
//   * a streak (maximal run of high seeds) ends at a low seed or at its query's end: one
//     thread per such end selects the streak's mh kept seeds -- the mh smallest (n, seed
//     number) keys, mh = round((pe - ps) / dist) capped at 128 from the bounding low seeds'
//     positions -- and flags the rest (and every seed above max_max_occ) as filtered;
//   * rep_len = sum over filtered seeds of en - max(st, en of the query's previous filtered
//     seed), the union of their spans (ends increase along the query): one max-scan finds
//     each one's predecessor, one integer atomic per seed sums the query.
constexpr uint32_t kFlt = 0x80000000u;  // filtered flag, kept in bit 31 of seed_n (n < 2^31)

__global__ void seed_class_kernel(const uint32_t *seed_n, int64_t M, int max_occ, uint64_t *cls) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > M) return;
    if (i == M) {  // the scan's extra entry: rank[M] = the totals
        cls[M] = 0;
        return;
    }
    const uint32_t n = seed_n[i];
    const bool hi = (int)n > max_occ, lo = n > 0 && !hi;
    cls[i] = (uint64_t)(hi ? 1u : 0u) << 32 | (lo ? 1u : 0u);
}

__global__ void seed_list_kernel(const uint32_t *seed_n, const uint64_t *rank, int64_t M, int max_occ, int32_t *low_idx,
                                 int32_t *high_idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const uint32_t n = seed_n[i];
    if (!n) return;
    if ((int)n > max_occ) high_idx[rank[i] >> 32] = (int32_t)i;
    else low_idx[(uint32_t)rank[i]] = (int32_t)i;
}

struct StreakParams {
    const uint64_t *my;
    const uint32_t *qid;
    const int64_t *qm_off, *qlen;
    const uint64_t *rank;      // exclusive (low, high) counts, M + 1 entries
    const int32_t *low_idx, *high_idx;
    int64_t n_low;
    int n_q;
    int max_occ, max_max_occ, dist;
    uint32_t *seed_n;
    uint32_t *flt_high;        // per high rank: filtered
};

__global__ void streak_kernel(StreakParams P) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P.n_low + P.n_q) return;
    int q;
    int64_t e_idx = -1, p_idx = -1;  // ending low seed, previous low seed (minimizer indices)
    uint64_t re, rp;                 // (low, high) ranks at the streak's end and start
    if (t < P.n_low) {
        e_idx = P.low_idx[t];
        q = (int)P.qid[e_idx];
        re = P.rank[e_idx];
        if (t > 0 && P.qid[P.low_idx[t - 1]] == (uint32_t)q) p_idx = P.low_idx[t - 1];
    } else {
        q = (int)(t - P.n_low);
        re = P.rank[P.qm_off[q + 1]];
        const uint64_t r0 = P.rank[P.qm_off[q]];
        if ((uint32_t)re > (uint32_t)r0) p_idx = P.low_idx[(uint32_t)re - 1];
    }
    rp = p_idx >= 0 ? P.rank[p_idx] : P.rank[P.qm_off[q]];
    const int64_t h0 = (int64_t)(rp >> 32), h1 = (int64_t)(re >> 32);  // the streak's high ranks
    const int cnt = (int)(h1 - h0);
    if (cnt <= 0) return;
    const bool case_a = P.dist > 0 && P.max_max_occ > P.max_occ;
    bool keep_all = false, keep_none = false;
    uint64_t thr = 0;
    if (case_a) {
        const uint64_t rq0 = P.rank[P.qm_off[q]], rq1 = P.rank[P.qm_off[q + 1]];
        const int64_t n_seed = (int64_t)((uint32_t)rq1 - (uint32_t)rq0) + (int64_t)((rq1 >> 32) - (rq0 >> 32));
        if (n_seed <= 1) return;  // seed.c: nothing is filtered for a single seed
        const int32_t ps = p_idx >= 0 ? (int32_t)((uint32_t)P.my[p_idx] >> 1) : 0;
        const int32_t pe = e_idx >= 0 ? (int32_t)((uint32_t)P.my[e_idx] >> 1) : (int32_t)P.qlen[q];
        int32_t mh = (int32_t)((double)(pe - ps) / P.dist + .499);
        if (mh > 128) mh = 128;
        keep_all = mh >= cnt, keep_none = mh <= 0;
        if (!keep_all && !keep_none) {  // the mh-th smallest (n, index) key
            uint64_t lo = 0, hi = ~0ull;
            while (lo < hi) {
                const uint64_t mid = lo + (hi - lo) / 2;
                int c = 0;
                for (int64_t r = h0; r < h1; r++) {
                    const int32_t a = P.high_idx[r];
                    c += ((uint64_t)P.seed_n[a] << 32 | (uint32_t)a) <= mid;
                }
                if (c >= mh) hi = mid;
                else lo = mid + 1;
            }
            thr = lo;
        }
    }
    for (int64_t r = h0; r < h1; r++) {
        const int32_t a = P.high_idx[r];
        const uint32_t n = P.seed_n[a];
        bool flt = true;  // case B: every seed above max_occ
        if (case_a) {
            const bool chosen = keep_all || (!keep_none && ((uint64_t)n << 32 | (uint32_t)a) <= thr);
            flt = !chosen || (int)n > P.max_max_occ;
        }
        P.flt_high[r] = flt ? 1u : 0u;
    }
}

// previous filtered high seed: inclusive max-scan of (flt ? rank : -1)
__global__ void flt_mark_kernel(const uint32_t *flt_high, int64_t n_high, int32_t *v) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n_high) v[r] = flt_high[r] ? (int32_t)r : -1;
}

__global__ void rep_len_kernel(const uint32_t *flt_high, const int32_t *prev_max, const int32_t *high_idx, int64_t n_high,
                               const uint64_t *mx, const uint64_t *my, const uint32_t *qid, int32_t *rep_len,
                               uint32_t *seed_n) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_high || !flt_high[r]) return;
    const int32_t a = high_idx[r];
    const uint32_t q = qid[a];
    const int32_t en = (int32_t)((uint32_t)my[a] >> 1) + 1, st = en - (int32_t)(mx[a] & 0xff);
    int32_t en_prev = 0;
    const int32_t pr = r > 0 ? prev_max[r - 1] : -1;
    if (pr >= 0) {
        const int32_t b = high_idx[pr];
        if (qid[b] == q) en_prev = (int32_t)((uint32_t)my[b] >> 1) + 1;
    }
    atomicAdd(rep_len + q, en - max(st, en_prev));
    seed_n[a] = 0;  // filtered: not a seed any more
}

__global__ void nz_flag_kernel(const uint32_t *v, int64_t n, uint32_t *flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = v[i] ? 1u : 0u;
}

struct AnchorParams {
    const uint64_t *mx, *my;
    const uint32_t *seed_n;
    const int64_t *a_pos;     // anchor offset of every minimizer
    const uint32_t *qid;
    const int64_t *qlen;
    const uint32_t *koff;
    const uint64_t *ipos;
    int64_t n;
    int rb;                   // bits for rid
    uint64_t *ax, *ay, *k1, *k2;
    uint32_t *val;
    // mini_pos
    const int64_t *mp_pos;
    uint64_t *mini_pos;
};

__global__ void write_anchors_kernel(AnchorParams P) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const uint32_t n = P.seed_n[i];
    if (!n) return;
    const uint64_t mx = P.mx[i], my = P.my[i];
    const uint32_t q_pos = (uint32_t)my, q_span = (uint32_t)(mx & 0xff);
    P.mini_pos[P.mp_pos[i]] = (uint64_t)q_span << 32 | (q_pos >> 1);
    const uint32_t q = P.qid[i];
    const int32_t qlen = (int32_t)P.qlen[q];
    const uint32_t *kp = P.koff + (mx >> 8);
    const uint64_t *r = P.ipos + kp[0];
    int64_t a = P.a_pos[i];
    for (uint32_t k = 0; k < n; k++, a++) {
        const uint64_t rk = r[k];
        const uint32_t rpos = (uint32_t)rk >> 1;
        const uint32_t rid = (uint32_t)(rk >> 32);
        uint64_t x, y;
        uint32_t rev;
        if ((rk & 1) == (q_pos & 1)) {
            rev = 0;
            x = (rk & 0xffffffff00000000ULL) | rpos;
            y = (uint64_t)q_span << 32 | (q_pos >> 1);
        } else {
            rev = 1;
            x = 1ULL << 63 | (rk & 0xffffffff00000000ULL) | rpos;
            y = (uint64_t)q_span << 32 | (uint32_t)(qlen - (int32_t)((q_pos >> 1) + 1 - q_span) - 1);
        }
        P.ax[a] = x;
        P.ay[a] = y;
        P.k1[a] = (uint64_t)q << (1 + P.rb) | (uint64_t)rev << P.rb | rid;
        P.k2[a] = (uint64_t)rpos << 32 | (uint32_t)y;
        P.val[a] = (uint32_t)a;
    }
}

// Anchor keys (the default path): one 64-bit key per anchor packing exactly the sort order
// of (query, x) -- K = q | rev | rid | rpos, field widths from the batch (query count,
// index sequences, longest index sequence) -- and the low 32 bits of y as the value.  The
// high bits of y hold the span, which is k for every minimizer of a non-HPC sketch.  One
// block per 256 consecutive minimizers: the block stages their anchor offsets, position-list
// starts and query coordinates in LDS, then its 256 lanes sweep the block's anchors
// (contiguous in both the position lists and the output), finding each anchor's minimizer
// by binary search in LDS -- coalesced reads and writes where a lane per minimizer would
// write 20-60 scattered anchors.
struct AnchorKeyParams {
    const uint64_t *mx, *my;
    const uint32_t *seed_n;
    const int64_t *a_pos;     // anchor offset of every minimizer (M + 1 entries)
    const uint32_t *qid;
    const int64_t *qlen;
    const uint32_t *koff;
    const uint64_t *ipos;
    int64_t n;                // minimizers
    int rb, pb;               // bits for rid / rpos
    uint64_t *key;
    uint32_t *val;
    const int64_t *mp_pos;
    uint64_t *mini_pos;
};

__global__ __launch_bounds__(256) void write_anchor_keys_kernel(AnchorKeyParams P) {
    __shared__ int64_t s_a[257];
    __shared__ uint64_t s_r[256];   // start of the minimizer's position list
    __shared__ uint32_t s_yf[256], s_yr[256], s_strand[256];
    __shared__ uint64_t s_q[256];   // q << (1 + rb + pb)
    const int tid = threadIdx.x;
    const int64_t m0 = (int64_t)blockIdx.x * 256;
    const int cnt = (int)min((int64_t)256, P.n - m0);
    if (tid < cnt) {
        const int64_t i = m0 + tid;
        const uint32_t n = P.seed_n[i];
        const uint64_t mx = P.mx[i], my = P.my[i];
        const uint32_t q_pos = (uint32_t)my, q_span = (uint32_t)(mx & 0xff);
        const uint32_t q = P.qid[i];
        if (n) P.mini_pos[P.mp_pos[i]] = (uint64_t)q_span << 32 | (q_pos >> 1);
        s_a[tid] = P.a_pos[i];
        s_r[tid] = P.koff[mx >> 8];
        s_yf[tid] = q_pos >> 1;
        s_yr[tid] = (uint32_t)((int32_t)P.qlen[q] - (int32_t)((q_pos >> 1) + 1 - q_span) - 1);
        s_strand[tid] = q_pos & 1;
        s_q[tid] = (uint64_t)q << (1 + P.rb + P.pb);
    }
    if (tid == 0) s_a[cnt] = P.a_pos[m0 + cnt];
    __syncthreads();
    const int64_t a0 = s_a[0], a1 = s_a[cnt];
    const int sh_rev = P.rb + P.pb;
    for (int64_t a = a0 + tid; a < a1; a += 256) {
        int lo = 0, hi = cnt - 1;  // last s with s_a[s] <= a (its list is non-empty)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_a[mid] <= a) lo = mid;
            else hi = mid - 1;
        }
        const uint64_t rk = P.ipos[s_r[lo] + (a - s_a[lo])];
        const uint32_t rpos = (uint32_t)rk >> 1;
        const uint64_t rid = rk >> 32;
        const uint32_t rev = ((uint32_t)rk & 1) != s_strand[lo];
        P.key[a] = s_q[lo] | (uint64_t)rev << sh_rev | rid << P.pb | rpos;
        P.val[a] = rev ? s_yr[lo] : s_yf[lo];
    }
}

// sorted keys -> (x, y); runs of equal key (one query minimizer position hit by several
// query minimizers) are ordered by y here: the lane at a run's start writes the run's y
// values by insertion sort (runs are short and rare), the other lanes of the run skip y.
__global__ void anchor_unpack_kernel(const uint64_t *key, const uint32_t *val, int64_t n, int rb, int pb, uint64_t yhi,
                                     uint64_t *ax, uint64_t *ay) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    const uint64_t rev = k >> (rb + pb) & 1, rid = k >> pb & ((1ull << rb) - 1), rpos = k & ((1ull << pb) - 1);
    ax[i] = rev << 63 | rid << 32 | rpos;
    const bool prev_eq = i > 0 && key[i - 1] == k;
    const bool next_eq = i + 1 < n && key[i + 1] == k;
    if (!prev_eq && !next_eq) {
        ay[i] = yhi << 32 | val[i];
    } else if (!prev_eq) {
        int64_t e = i + 1;
        while (e + 1 < n && key[e + 1] == k) e++;
        for (int64_t a = i; a <= e; a++) {
            const uint64_t v = yhi << 32 | val[a];
            int64_t b = a;
            while (b > i && ay[b - 1] > v) {
                ay[b] = ay[b - 1];
                b--;
            }
            ay[b] = v;
        }
    }
}

// group = (query, strand, target): the key without its low `shift` (rpos) bits
__global__ void group_flag_x_kernel(const uint64_t *x, int64_t n, uint32_t *flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = (i == 0 || (x[i] >> 32) != (x[i - 1] >> 32)) ? 1u : 0u;
}

// Groups of an anchor set sorted by (query, x, y): a group starts at every non-empty query's
// first anchor and wherever x >> 32 (strand, target) changes.  The x changes come as a bitmap
// from whoever wrote the set -- the grouped sort's writers (AnchorOut::head), the long join's
// compaction, or head_bits_x_kernel for the other paths -- so numbering the groups reads one bit
// per anchor instead of x twice: pass 1 counts the heads per tile of kGTile anchors (64 per
// thread: two bitmap words), a scan of the tile counts, pass 2 writes g_start and each group's
// query-first flag.  A tile's query starts come from the query offsets into an LDS bitmap.
constexpr int kGTile = 16384;

__device__ __forceinline__ uint64_t group_tile_bits(const uint32_t *hb, int64_t n, const int64_t *qoff, int n_q, int64_t t0,
                                                    uint64_t *qs) {
    __shared__ int s_q0;
    const int tid = threadIdx.x;
    const int64_t t1 = min(t0 + kGTile, n);
    const int64_t a0 = t0 + 64 * (int64_t)tid;
    const uint64_t hw = a0 < n ? reinterpret_cast<const uint64_t *>(hb)[a0 >> 6] : 0;
    qs[tid] = 0;
    if (tid == 0) {  // first query whose range ends after t0
        int lo = 0, hi = n_q;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (qoff[mid + 1] <= t0) lo = mid + 1;
            else hi = mid;
        }
        s_q0 = lo;
    }
    __syncthreads();
    for (int q = s_q0 + tid; q < n_q; q += 256) {
        const int64_t a = qoff[q];
        if (a >= t1) break;
        if (a >= t0 && a < qoff[q + 1]) atomicOr((unsigned long long *)&qs[(a - t0) >> 6], 1ull << ((a - t0) & 63));
    }
    __syncthreads();
    const int64_t m = n - a0;  // anchors of this thread's 64 that exist
    const uint64_t live = m >= 64 ? ~0ull : m > 0 ? (1ull << m) - 1 : 0ull;
    return (hw | qs[tid]) & live;
}

__global__ __launch_bounds__(256) void group_heads_count_kernel(const uint32_t *hb, int64_t n, const int64_t *qoff, int n_q,
                                                          uint32_t *tile_cnt) {
    __shared__ uint64_t qs[kGTile / 64];
    __shared__ uint32_t ws[4];
    const uint64_t h = group_tile_bits(hb, n, qoff, n_q, (int64_t)blockIdx.x * kGTile, qs);
    uint32_t c = (uint32_t)__popcll(h);
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// g_start of every group, its query-first flag (lchain.c's krmq index-0 quirk) and the
// g_start[G] = n sentinel
__global__ __launch_bounds__(256) void group_heads_write_kernel(const uint32_t *hb, int64_t n, const int64_t *qoff, int n_q,
                                                          const int64_t *tile_off, int64_t *g_start, uint8_t *qfirst,
                                                          int64_t G) {
    __shared__ uint64_t qs[kGTile / 64];
    __shared__ uint32_t ws[4];
    const int64_t t0 = (int64_t)blockIdx.x * kGTile;
    uint64_t h = group_tile_bits(hb, n, qoff, n_q, t0, qs);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t c = (uint32_t)__popcll(h);
    uint32_t inc = c;  // exclusive scan of the threads' counts in anchor order
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    int64_t g = tile_off[blockIdx.x] + inc - c;
    for (int k = 0; k < w; k++) g += ws[k];
    const uint64_t qw = qs[threadIdx.x];
    const int64_t a0 = t0 + 64 * (int64_t)threadIdx.x;
    while (h) {
        const int b = __ffsll((unsigned long long)h) - 1;
        h &= h - 1;
        g_start[g] = a0 + b;
        qfirst[g] = (uint8_t)(qw >> b & 1);
        ++g;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) g_start[G] = n;
}

// x's low words of an anchor set written without them (the two-key, re-sort and test paths)
__global__ void x_low_kernel(const uint64_t *x, int64_t n, uint32_t *x32) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x32[i] = (uint32_t)x[i];
}

// the head bitmap of an anchor set written without one (the two-key and re-sort paths):
// x >> 32 differs from the previous anchor's, a wave's 64 anchors per 64-bit word
__global__ __launch_bounds__(256) void head_bits_x_kernel(const uint64_t *x, int64_t n, uint64_t *hb) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool hd = i < n && (i == 0 || (x[i] >> 32) != (x[i - 1] >> 32));
    const uint64_t b = __ballot(hd);
    if ((threadIdx.x & 63) == 0 && i < n) hb[i >> 6] = b;
}

__global__ void group_start_kernel(const uint32_t *flag, const int64_t *gpos, int64_t n, int64_t *g_start, int32_t *gid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t g = gpos[i] + flag[i] - 1;
    gid[i] = (int32_t)g;
    if (flag[i]) g_start[g] = i;
}

// largest group: the first of the size-descending list, or, when sizes tie at the 16-bit
// key's cap, the largest of that tied prefix
// (out: a mailbox word)
__global__ void max_group_kernel(const int64_t *g_start, const int32_t *order, int32_t G, int64_t *out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    int64_t best = 0;
    for (int32_t w = 0; w < G; w++) {
        const int g = order[w];
        const int64_t sz = g_start[g + 1] - g_start[g];
        best = max(best, sz);
        if (sz < 0xffff) break;
    }
    *out = best;
}

// groups of fewer than min_cnt anchors: f = 0, p = -1, t = 0 (the chaining kernels write all
// three for the anchors of every work group, so t needs no pass over the set)
__global__ void nonwork_fp_kernel(const int64_t *g_start, int32_t G, int min_cnt, int32_t *f, int64_t *p, int32_t *t) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const int64_t a0 = g_start[g], a1 = g_start[g + 1];
    if (a1 - a0 >= min_cnt) return;
    for (int64_t a = a0; a < a1; a++) f[a] = 0, p[a] = -1, t[a] = 0;
}

// also clears the per-group query-first flags and the z-order list counters
__global__ void group_size_kernel(const int64_t *g_start, int32_t G, int min_cnt, uint32_t *key, uint32_t *gidx,
                                  uint32_t *is_work, uint8_t *qfirst, int32_t *zlists) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < 8) zlists[g] = 0;
    if (g >= G) return;
    if (qfirst) qfirst[g] = 0;
    const int64_t sz = g_start[g + 1] - g_start[g];
    // descending size in 16 bits (two radix passes): groups above 65535 anchors tie at the
    // front, non-work groups (< min_cnt <= 3 anchors) come after every work group
    key[g] = 0xffffu - (uint32_t)min(sz, (int64_t)0xffff);
    gidx[g] = (uint32_t)g;
    is_work[g] = sz >= min_cnt ? 1u : 0u;
}

// ---- backtrack order: z = anchors with f >= min_sc, per group ascending (f, idx) (the
// backtrack walks it from the end: canonical T3).  A group's z entries are kept inside the
// group's own anchor range [g_start[g], g_start[g] + z_cnt[g]), so no global flag scan or
// offset table is needed.  The entries are nearly sorted already: f grows along a colinear
// chain, so a group is a few ascending runs (one per chain or chain piece).
//  * groups of <= kZLane anchors: one lane each, ranks by all-pairs comparison in registers;
//  * larger groups: one wave each reads the group's f once, compacts its z keys (ballot), finds
//    the descents between consecutive keys (the previous key by shuffle) and records the
//    starts of the first kZRuns runs.  A single run is already the order (the wave wrote it).
//    Groups of <= max_runs runs are merged by a flat kernel -- every entry's position is its
//    offset in its own run plus, per other run, a binary search (keys are unique).  Groups
//    with more runs go to a block bitonic sort in LDS (<= kZs entries) or one global radix
//    sort over all such larger groups (lists appended with atomics: the sorted result does
//    not depend on the list order).
constexpr int kZs = 2048;
constexpr int kZRuns = 16;
constexpr int kZmLds = 6144;   // merge groups staged in LDS up to this many entries (48 KB: three blocks per CU)
constexpr int kZmUnit = 2048;  // larger merge groups: units of this many entries, one block each
constexpr int kZLane = 16;
#ifndef HYMET_Z_DEPTH
#define HYMET_Z_DEPTH 8
#endif
constexpr int kZDepth = HYMET_Z_DEPTH;  // f chunks in flight per wave (zorder_wave_kernel)

struct ZParams {
    const int32_t *f;
    const int64_t *g_start;
    const int32_t *order;  // all groups by descending size (the chaining work list, whole)
    int32_t G;
    int min_sc, max_runs;
    int zm_lds, zm_unit;   // kZmLds / kZmUnit (HYMET_ZM_LDS / HYMET_ZM_UNIT in tests)
    uint64_t *zkey;        // n: (f << 32 | idx) at the group's compacted z positions
    int32_t *z_idx;        // n: the order, at the same positions
    int32_t *z_cnt;        // per group: number of z entries
    int32_t *z_runs;       // per group: ascending runs (0 when empty)
    int32_t *run_start;    // per group, kZRuns entries: run starts relative to g_start
    int32_t *lists;        // [0] split, [1] mid count, [2] big count, [3] merge count, [4..5] big total (i64),
                           // [6] merge-unit count
    int32_t *merge_list;   // groups of 2..max_runs runs, for the merge
    int64_t *mergeu_list;  // units (group << 32 | u) of kZmUnit entries of the merge groups above kZmLds
    int32_t *mid_list;     // groups for the block sort
    int32_t *big_list;     // groups for the radix path
    int64_t *big_off;      // their offsets in the radix arrays
    int64_t *mail;         // mailbox words: big count, big total (published by zmerge_kernel)
};

// first list position whose group has <= kZLane anchors
__global__ void zsplit_kernel(ZParams P) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t lo = 0, hi = P.G;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        const int g = P.order[mid];
        if (P.g_start[g + 1] - P.g_start[g] <= kZLane) hi = mid;
        else lo = mid + 1;
    }
    P.lists[0] = lo;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return (uint64_t)hi << 32 | lo;
}

// one wave per group of > kZLane anchors (grid-stride over the list prefix)
__global__ __launch_bounds__(256) void zorder_wave_kernel(ZParams P) {
    const int lane = threadIdx.x & 63;
    const int32_t split = P.lists[0];
    const int nw = (int)(gridDim.x * (blockDim.x >> 6));
    // list entries held per wave (lane i: the i-th pending group) and appended 64 at a time:
    // one returning atomic per listed group on the shared counters serialised (~1 ms per
    // launch over ~10^5 groups, as in query_scan_kernel before)
    int32_t pend[3] = {0, 0, 0};  // merge, mid, big
    int np[3] = {0, 0, 0};
    unsigned long long big_m = 0;  // z entries of this wave's big groups
    int32_t *const lst[3] = {P.merge_list, P.mid_list, P.big_list};
    auto flush = [&](int l) {
        if (np[l] == 0) return;
        int base = 0;
        if (lane == 0) base = atomicAdd(P.lists + (l == 0 ? 3 : l == 1 ? 1 : 2), np[l]);
        base = __shfl(base, 0, 64);
        if (lane < np[l]) lst[l][base + lane] = pend[l];
        np[l] = 0;
    };
    auto push = [&](int l, int g) {
        if (lane == np[l]) pend[l] = g;
        if (++np[l] == 64) flush(l);
    };
    // The wave's groups are w0, w0 + nw, w0 + 2 nw, ...; each round loads the next 64 of them
    // (list entry and bounds, lane r holding group r) in one round trip instead of two dependent
    // ones per group -- most groups are a single chunk of f, so those round trips were half the
    // wave's time.
    for (int wb = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); wb < split; wb += 64 * nw) {
        const int64_t wl = (int64_t)wb + (int64_t)lane * nw;
        int gl = 0;
        int64_t sl = 0, el = 0;
        if (wl < split) {
            gl = P.order[wl];
            sl = P.g_start[gl];
            el = P.g_start[gl + 1];
        }
        const int nr = (int)min((int64_t)64, ((int64_t)split - wb + nw - 1) / nw);  // groups this round
        for (int r = 0; r < nr; r++) {
            const int g = __builtin_amdgcn_readlane(gl, r);
            const int64_t g0 = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(sl >> 32), r) << 32 |
                                         (uint32_t)__builtin_amdgcn_readlane((int32_t)sl, r));
            const int64_t n = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(el >> 32), r) << 32 |
                                        (uint32_t)__builtin_amdgcn_readlane((int32_t)el, r)) - g0;
            int32_t *rs = P.run_start + (int64_t)g * kZRuns;
            int m = 0, K = 0;  // z entries so far, descents so far (wave-uniform)
            uint64_t last = 0;
            const uint64_t below = (1ull << lane) - 1;
            // kZDepth chunks of f loaded together: a group of tens of thousands of anchors is one
            // wave's serial walk, the launch's tail (one chunk ahead: a round trip per 64 anchors)
            for (int64_t base0 = 0; base0 < n; base0 += 64 * kZDepth) {
                int32_t fc[kZDepth];
#pragma unroll
                for (int d = 0; d < kZDepth; d++) {
                    const int64_t i = base0 + 64 * d + lane;
                    fc[d] = i < n ? P.f[g0 + i] : 0;
                }
#pragma unroll
                for (int d = 0; d < kZDepth; d++) {
                    const int64_t i = base0 + 64 * d + lane;
                    const bool ok = i < n;
                    const int32_t fv = fc[d];
                    const bool z = ok && fv >= P.min_sc;
                    const uint64_t bal = __ballot(z);
                    if (bal == 0) continue;
                    const uint64_t key = (uint64_t)(uint32_t)fv << 32 | (uint32_t)(g0 + i);
                    const uint64_t lower = bal & below;
                    const int pos = m + __popcll(lower);
                    const int prev = lower ? 63 - __clzll((long long)lower) : lane;
                    uint64_t pk = shfl64(key, prev);
                    if (!lower) pk = last;
                    const bool desc = z && pos > 0 && key < pk;
                    const uint64_t dbal = __ballot(desc);
                    if (z) P.z_idx[g0 + pos] = (int32_t)(g0 + i);
                    if (desc) {
                        const int r = K + 1 + __popcll(dbal & below);
                        if (r < kZRuns) rs[r] = pos;
                    }
                    K += __popcll(dbal);
                    m += __popcll(bal);
                    last = shfl64(key, 63 - __clzll((long long)bal));
                }
            }
            const int runs = m > 0 ? K + 1 : 0;
            if (lane == 0) {
                rs[0] = 0;
                P.z_cnt[g] = m;
                P.z_runs[g] = runs;
            }
            if (runs > 1) {
                // only the merge / sort paths read the keys: a group of one run (C4's colinear
                // chains: most of them) writes its order alone, 4 B per z entry instead of 12, and
                // the others write the keys in a second pass over f
                int m2 = 0;
                for (int64_t base0 = 0; base0 < n; base0 += 64 * kZDepth) {
                    int32_t fc[kZDepth];
#pragma unroll
                    for (int d = 0; d < kZDepth; d++) {
                        const int64_t i = base0 + 64 * d + lane;
                        fc[d] = i < n ? P.f[g0 + i] : 0;
                    }
#pragma unroll
                    for (int d = 0; d < kZDepth; d++) {
                        const int64_t i = base0 + 64 * d + lane;
                        const bool z = i < n && fc[d] >= P.min_sc;
                        const uint64_t bal = __ballot(z);
                        if (bal == 0) continue;
                        if (z) P.zkey[g0 + m2 + __popcll(bal & below)] = (uint64_t)(uint32_t)fc[d] << 32 | (uint32_t)(g0 + i);
                        m2 += __popcll(bal);
                    }
                }
            }
            // (wave-uniform conditions)
            if (runs > 1 && runs <= P.max_runs) {
                if (m <= P.zm_lds) {
                    push(0, g);
                } else {  // a long merge is split over blocks (one block walking it was the launch's tail)
                    const int nu = (m + P.zm_unit - 1) / P.zm_unit;
                    int base = 0;
                    if (lane == 0) base = atomicAdd(P.lists + 6, nu);
                    base = __shfl(base, 0, 64);
                    for (int u = lane; u < nu; u += 64) P.mergeu_list[base + u] = (int64_t)g << 32 | (uint32_t)u;
                }
            }
            if (runs > P.max_runs) {
                if (m <= kZs) {
                    push(1, g);
                } else {
                    // list rank only: the radix arrays' offsets are a scan of the counts in rank
                    // order (zbig_count_kernel), since the sorted keys come out rank-major
                    push(2, g);
                    big_m += (unsigned long long)m;
                }
            }
        }
    }
    flush(0), flush(1), flush(2);
    if (lane == 0 && big_m) atomicAdd((unsigned long long *)(P.lists + 4), big_m);
}

// one lane per group of <= kZLane anchors: rank = number of smaller keys
__global__ __launch_bounds__(256) void zorder_lane_kernel(ZParams P) {
    const int32_t w = P.lists[0] + (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (w >= P.G) return;
    const int g = P.order[w];
    const int64_t g0 = P.g_start[g];
    const int n = (int)(P.g_start[g + 1] - g0);
    uint64_t key[kZLane];
#pragma unroll
    for (int j = 0; j < kZLane; j++) {
        const int32_t fv = j < n ? P.f[g0 + j] : 0;
        key[j] = j < n && fv >= P.min_sc ? (uint64_t)(uint32_t)fv << 32 | (uint32_t)(g0 + j) : ~0ull;
    }
    int m = 0;
#pragma unroll
    for (int j = 0; j < kZLane; j++) {
        if (key[j] == ~0ull) continue;
        int r = 0;
#pragma unroll
        for (int k = 0; k < kZLane; k++) r += key[k] < key[j];
        P.z_idx[g0 + r] = (int32_t)(uint32_t)key[j];
        m++;
    }
    P.z_cnt[g] = m;
    P.z_runs[g] = m > 0 ? 1 : 0;  // complete
}

// groups of 2..max_runs ascending runs: merge by ranks, one block per listed group (grid-stride
// over the list; a flat pass over every anchor position read each one's group first).  An
// entry's position is its offset in its own run plus, per other run, the count of smaller keys
// there; a group of up to kZmLds entries is staged in LDS first (real repeats: groups of many
// runs and thousands of entries).  Each thread takes a stripe of consecutive entries: within a
// run the keys ascend, so each other run's count only moves forward from the previous entry's,
// found by an exponential search from there (mostly one compare) instead of a full binary search
// per entry and run; a new run (the key drops) restarts the counts at the run starts.
// entries [qa, qb) of a group of m entries in K runs (rs: K + 1 run bounds)
__device__ __forceinline__ void zmerge_group(const uint64_t *zk, const int32_t *rs, int K, int m, int qa, int qb,
                                             int32_t *out) {
    const int S = (qb - qa + (int)blockDim.x - 1) / (int)blockDim.x;  // entries per thread
    const int q0 = qa + (int)threadIdx.x * S, q1 = min(q0 + S, qb);
    if (q0 >= qb) return;
    int rsr[kZRuns + 1], lo[kZRuns];
#pragma unroll
    for (int k = 0; k <= kZRuns; k++) rsr[k] = k <= K ? rs[k] : m;
    int own = 0, own_s = 0;  // the run of entry q and its start (no dynamic register indexing)
#pragma unroll
    for (int k = 1; k < kZRuns; k++)
        if (k < K && rsr[k] <= q0) own = k, own_s = rsr[k];
    uint64_t prev = ~0ull;
    for (int q = q0; q < q1; q++) {
        const uint64_t key = zk[q];
        const bool restart = key < prev;  // the first entry, or the first of the next run
        prev = key;
        if (restart && q > q0) own++, own_s = q;  // a run start is exactly where the key drops
        int pos = q - own_s;                       // the offset in its own run
#pragma unroll
        for (int k = 0; k < kZRuns; k++) {
            if (k < K && k != own) {
                const int s1 = rsr[k + 1];
                int l = restart ? rsr[k] : lo[k];
                if (l < s1 && zk[l] < key) {  // first entry >= key in (l, s1]: gallop, then bisect
                    int b = 1;
                    while (l + b < s1 && zk[l + b] < key) {
                        l += b;
                        b <<= 1;
                    }
                    int a = l + 1, e = min(l + b, s1);
                    while (a < e) {
                        const int mid = (a + e) >> 1;
                        if (zk[mid] < key) a = mid + 1;
                        else e = mid;
                    }
                    l = a;
                }
                lo[k] = l;
                pos += l - rsr[k];
            }
        }
        out[pos] = (int32_t)(uint32_t)key;
    }
}

__global__ __launch_bounds__(256) void zmerge_kernel(ZParams P) {
    __shared__ uint64_t sk[kZmLds];
    __shared__ int32_t srs[kZRuns + 1];
    const int n_list = P.lists[3], n_units = P.lists[6];
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the lists are final (zorder_wave_kernel ran)
        P.mail[0] = P.lists[2];
        P.mail[1] = *reinterpret_cast<const int64_t *>(P.lists + 4);
    }
    // units of the long merges first (they were the tail), then the staged groups
    for (int w = blockIdx.x; w < n_units + n_list; w += gridDim.x) {
        const bool unit = w < n_units;
        const int64_t uw = unit ? P.mergeu_list[w] : 0;
        const int g = unit ? (int)(uw >> 32) : P.merge_list[w - n_units];
        const int K = P.z_runs[g];
        const int64_t z0 = P.g_start[g];
        const int m = P.z_cnt[g];
        const int32_t *rs = P.run_start + (int64_t)g * kZRuns;
        const uint64_t *zk = P.zkey + z0;
        __syncthreads();  // the previous group's readers are done with sk / srs
        if (threadIdx.x <= K) srs[threadIdx.x] = threadIdx.x < K ? rs[threadIdx.x] : m;
        if (!unit)
            for (int q = threadIdx.x; q < m; q += blockDim.x) sk[q] = zk[q];
        __syncthreads();
        if (unit) {
            const int qa = (int)(uint32_t)uw * P.zm_unit;
            zmerge_group(zk, srs, K, m, qa, min(qa + P.zm_unit, m), P.z_idx + z0);
        } else {
            zmerge_group(sk, srs, K, m, 0, m, P.z_idx + z0);
        }
    }
}

// one block per listed group of <= kZs z entries (grid-stride over the list)
__global__ __launch_bounds__(256) void zsort_block_kernel(ZParams P) {
    __shared__ uint64_t s[kZs];
    const int n_list = P.lists[1];
    for (int w = blockIdx.x; w < n_list; w += gridDim.x) {
        const int g = P.mid_list[w];
        const int64_t z0 = P.g_start[g];
        const int n = P.z_cnt[g];
        int np = 128;
        while (np < n) np <<= 1;
        for (int i = threadIdx.x; i < np; i += 256) s[i] = i < n ? P.zkey[z0 + i] : ~0ull;
        __syncthreads();
        for (int k = 2; k <= np; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = threadIdx.x; i < np; i += 256) {
                    const int ij = i ^ j;
                    if (ij > i) {
                        const uint64_t a = s[i], b = s[ij];
                        if (((i & k) == 0) == (a > b)) {
                            s[i] = b;
                            s[ij] = a;
                        }
                    }
                }
                __syncthreads();
            }
        for (int i = threadIdx.x; i < n; i += 256) P.z_idx[z0 + i] = (int32_t)(uint32_t)s[i];
        __syncthreads();
    }
}

// z entries of each large group, in list-rank order (scanned into big_off)
__global__ void zbig_count_kernel(ZParams P, int32_t n_big, uint32_t *cnt) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n_big) cnt[r] = (uint32_t)P.z_cnt[P.big_list[r]];
}

// entries of the large groups, list-major: key = rank << 32 | f, value = idx; group r's
// entries start at big_off[r] both before and after the sort (offsets ascend with the rank)
__global__ void zbig_gather_kernel(ZParams P, uint64_t *skey, uint32_t *sval) {
    const int r = blockIdx.x, g = P.big_list[r];
    const int64_t z0 = P.g_start[g], n = P.z_cnt[g], o = P.big_off[r];
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
        const uint64_t k = P.zkey[z0 + t];
        skey[o + t] = (uint64_t)r << 32 | (k >> 32);
        sval[o + t] = (uint32_t)k;
    }
}

__global__ void zbig_scatter_kernel(ZParams P, const uint32_t *sval) {
    const int r = blockIdx.x, g = P.big_list[r];
    const int64_t z0 = P.g_start[g], n = P.z_cnt[g], o = P.big_off[r];
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) P.z_idx[z0 + t] = (int32_t)sval[o + t];
}

// chain list entries: (key = first anchor index) -> sorted
__global__ void chain_list_kernel(const int64_t *g_start, const int32_t *n_chains, const int64_t *c_pos, int32_t G,
                                  const uint64_t *chain_u, const int64_t *chain_first, const int64_t *chain_ids,
                                  uint64_t *ckey, uint64_t *cu, int64_t *cfirst) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const int64_t g0 = g_start[g];
    int64_t o = c_pos[g];
    for (int c = 0; c < n_chains[g]; c++, o++) {
        const int64_t fo = chain_first[g0 + c];
        ckey[o] = (uint64_t)chain_ids[fo + (uint32_t)chain_u[g0 + c] - 1];  // stored end -> start
        cu[o] = chain_u[g0 + c];
        cfirst[o] = fo;
    }
}

// anchors per chain in the compacted copy; with a long join (qflag), chains of flagged
// queries are left out of the copy and counted in cnt2 instead (they are only marked)
__global__ void chain_cnt_kernel(const uint64_t *cu, const uint32_t *cq, const uint32_t *qflag, int64_t n, uint32_t *cnt,
                                 uint32_t *cnt2) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t m = (uint32_t)cu[i];
    const bool fl = qflag && qflag[cq[i]];
    cnt[i] = fl ? 0u : m;
    if (cnt2) cnt2[i] = fl ? m : 0u;
}

// long join, first pass (map.c's rmq rescue): a query is re-chained when it has more than one
// chain and its first chain (compact order) leaves too much of it uncovered -- read from the
// chain list before the copy
__global__ void rechain_flag_kernel(const uint64_t *ay, const int64_t *chain_ids, const uint64_t *cu, const int64_t *cfirst,
                                    const int64_t *qc, const int64_t *qlen, int n_q, int rescue_size, float rescue_ratio,
                                    uint32_t *flag) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_q) return;
    const int64_t c0 = qc[q], nc = qc[q + 1] - c0;
    uint32_t f = 0;
    if (nc > 1) {
        const int32_t m = (int32_t)cu[c0];
        const int64_t fo = cfirst[c0];  // backtrack stores end -> start
        const int32_t st = (int32_t)ay[chain_ids[fo + m - 1]], en = (int32_t)ay[chain_ids[fo]];
        const int32_t ql = (int32_t)qlen[q];
        if (ql - (en - st) > rescue_size || (float)(en - st) > __fmul_rn((float)ql, rescue_ratio)) f = 1;
    }
    flag[q] = f;
}

// per-query anchor offsets of a compacted copy: the offset of the query's first chain
__global__ void chain_qb_kernel(const int64_t *qc, const int64_t *bpos, int64_t n_chain, int64_t nb, int n_q, int64_t *qb) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q > n_q) return;
    const int64_t c = qc[q];
    qb[q] = c < n_chain ? bpos[c] : nb;
}

// anchors of chain c in start -> end order, and c per anchor (the chains of queries the long
// join re-chains have no anchors here: cnt 0)
__global__ __launch_bounds__(256) void chain_copy_kernel(const uint64_t *cu, const int64_t *cfirst, const int64_t *bpos,
                                                         const int64_t *chain_ids, const uint64_t *ax, const uint64_t *ay,
                                                         int64_t n_chain, int64_t nb, uint64_t *bx, uint64_t *by,
                                                         int32_t *bchain) {
    // flat over the output anchors (~48 B each, bandwidth-bound: C4 copies ~236 M per batch at
    // ~3.8 TB/s): the block's first chain c0 by binary search over bpos; the starts of the next
    // 256 chains are staged in LDS and each lane finds its chain by an 8-step search there (a
    // forward walk per lane cost up to 255 dependent loads where chains are short).  Chains
    // left out of the copy have no anchors, so more than 256 may start in the block: lanes
    // past the staged ones search bpos itself.
    __shared__ int64_t s_c0;
    __shared__ int32_t s_st[257];  // block-relative starts of chains c0 .. c0 + 256 (clamped)
    const int64_t b0 = (int64_t)blockIdx.x * blockDim.x;
    if (threadIdx.x == 0) {
        int64_t lo = 0, hi = n_chain - 1;  // last c with bpos[c] <= b0
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (bpos[mid] <= b0) lo = mid;
            else hi = mid - 1;
        }
        s_c0 = lo;
    }
    __syncthreads();
    const int64_t c0 = s_c0;
    for (int i = threadIdx.x; i < 257; i += blockDim.x) {
        const int64_t c = c0 + i;
        s_st[i] = c < n_chain ? (int32_t)min(bpos[c] - b0, (int64_t)256) : 256;
    }
    __syncthreads();
    const int64_t b = b0 + threadIdx.x;
    if (b >= nb) return;
    int lo = 0, hi = 256;  // last i with s_st[i] <= threadIdx.x (s_st[0] <= 0, nondecreasing)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_st[mid] <= (int)threadIdx.x) lo = mid;
        else hi = mid - 1;
    }
    int64_t c = c0 + lo;
    if (lo == 256) {  // last c with bpos[c] <= b beyond the staged chains
        int64_t l2 = c, h2 = n_chain - 1;
        while (l2 < h2) {
            const int64_t mid = (l2 + h2 + 1) >> 1;
            if (bpos[mid] <= b) l2 = mid;
            else h2 = mid - 1;
        }
        c = l2;
    }
    const int32_t m = (int32_t)cu[c];
    const int64_t a = chain_ids[cfirst[c] + m - 1 - (b - bpos[c])];  // backtrack stores end -> start
    bx[b] = ax[a];
    by[b] = ay[a];
    bchain[b] = (int32_t)c;
}

// Long-join anchors: the first pass's chain anchors (t == 2 after the backtrack) of the
// flagged queries.  Thread l of a 4096-anchor tile decides anchors [16 l, 16 l + 16) of the
// tile (16-byte loads of t; the query of the first by a binary search over the query
// offsets, then stepping over the few query starts inside the 16).
__device__ __forceinline__ uint32_t keep_bits16(const int32_t *t, int64_t n, const uint32_t *qflag, const int64_t *qoff,
                                                int n_q, int64_t e0) {
    if (e0 >= n) return 0u;
    int lo = 0, hi = n_q - 1;  // last q with qoff[q] <= e0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (qoff[mid] <= e0) lo = mid;
        else hi = mid - 1;
    }
    int q = lo;
    int64_t qend = qoff[q + 1];
    int32_t v[16];
    if (e0 + 16 <= n) {
        const int4 *p4 = reinterpret_cast<const int4 *>(t + e0);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int4 w = p4[u];
            v[4 * u] = w.x, v[4 * u + 1] = w.y, v[4 * u + 2] = w.z, v[4 * u + 3] = w.w;
        }
    } else {
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = e0 + u < n ? t[e0 + u] : 0;
    }
    uint32_t bits = 0, fl = qflag[q];
#pragma unroll
    for (int u = 0; u < 16; u++) {
        while (e0 + u >= qend && q + 1 < n_q) {  // a query starts here
            q++;
            qend = qoff[q + 1];
            fl = qflag[q];
        }
        bits |= (uint32_t)(v[u] == 2 && fl != 0) << u;
    }
    return bits;
}

// (also each tile's last kept anchor, or -1: the compaction's group heads compare a tile's
// first kept anchor with the one before it)
__global__ __launch_bounds__(256) void mark_count_kernel(const int32_t *t, int64_t n, const uint32_t *qflag,
                                                         const int64_t *qoff, int n_q, uint32_t *cnt, int64_t *last_kept) {
    __shared__ uint32_t ws[4];
    __shared__ int64_t wl[4];
    const int64_t e0 = (int64_t)blockIdx.x * 4096 + threadIdx.x * 16;
    const uint32_t kb = keep_bits16(t, n, qflag, qoff, n_q, e0);
    uint32_t c = __popc(kb);
    long long l = kb ? e0 + 31 - __clz((int)kb) : -1;
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor((int)c, o, 64);
        l = max(l, __shfl_xor(l, o, 64));
    }
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c, wl[threadIdx.x >> 6] = l;
    __syncthreads();
    if (threadIdx.x == 0) {
        cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
        last_kept[blockIdx.x] = max(max(wl[0], wl[1]), max(wl[2], wl[3]));
    }
}

// stable compaction of the kept anchors (x, y): the first-pass set is sorted by (query, x,
// y), so its kept subsequence is the long join's sorted anchor set -- no re-sort.  The keep
// bits are decided per 16 consecutive anchors (as in the count) into LDS; rows of 256
// anchors are then written lanes striped (coalesced), positions by ballot counts.
// The output's group heads (x >> 32 differs from the previous kept anchor's) go into its
// bitmap ohb (zeroed): the previous kept anchor is a lower lane of the same 64-anchor chunk
// (shuffle), else the last kept one of an earlier chunk of the tile (LDS), else the last kept
// anchor of an earlier tile (last_kept, from the count).
__global__ __launch_bounds__(256) void mark_compact_kernel(const int32_t *t, int64_t n, const uint32_t *qflag,
                                                           const int64_t *qoff, int n_q, const int64_t *tile_off,
                                                           const int64_t *last_kept, const uint64_t *ax, const uint64_t *ay,
                                                           uint64_t *ox, uint64_t *oy, uint32_t *ohb, uint32_t *ox32) {
    __shared__ uint32_t rc[64];       // kept per (row, wave), row-major
    __shared__ uint32_t nk[64];       // the same counts (rc becomes their exclusive scan)
    __shared__ uint32_t lx[64];       // x >> 32 of each (row, wave) chunk's last kept anchor
    __shared__ uint16_t kb[256];      // keep bits of anchors [16 l, 16 l + 16) of the tile
    const int64_t t0 = (int64_t)blockIdx.x * 4096;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    kb[threadIdx.x] = (uint16_t)keep_bits16(t, n, qflag, qoff, n_q, t0 + threadIdx.x * 16);
    __syncthreads();
    bool m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int r = j * 256 + threadIdx.x;  // tile-relative anchor
        m[j] = (kb[r >> 4] >> (r & 15)) & 1;
        const uint64_t b = __ballot(m[j]);
        if (lane == 0) rc[j * 4 + w] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    uint32_t v = 0, inc = 0;
    if (w == 0) nk[lane] = rc[lane];
    if (w == 0) {  // wave 0: exclusive scan of the 64 counts in element order
        v = rc[lane];
        inc = v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += o;
        }
    }
    __syncthreads();
    if (w == 0) rc[lane] = inc - v;
    __syncthreads();
    const int64_t base = tile_off[blockIdx.x];
    uint32_t xh[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint64_t b = __ballot(m[j]);
        xh[j] = 0;
        if (m[j]) {
            const int64_t e = t0 + j * 256 + threadIdx.x;
            const int64_t o = base + rc[j * 4 + w] + __popcll(b & ((1ull << lane) - 1));
            const uint64_t xv = ax[e];
            xh[j] = (uint32_t)(xv >> 32);
            ox[o] = xv;
            ox32[o] = (uint32_t)xv;
            oy[o] = ay[e];
        }
        if (b && lane == 63 - __clzll((long long)b)) lx[j * 4 + w] = xh[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint64_t b = __ballot(m[j]);
        const uint64_t below = b & ((1ull << lane) - 1);
        const int src = below ? 63 - __clzll((long long)below) : lane;
        const uint32_t xp = (uint32_t)__shfl((int)xh[j], src, 64);
        if (m[j]) {
            bool hd;
            if (below) {
                hd = xp != xh[j];
            } else {  // the chunk's first kept anchor
                int c = j * 4 + w - 1;
                while (c >= 0 && nk[c] == 0) --c;
                if (c >= 0) {
                    hd = lx[c] != xh[j];
                } else {  // the tile's first: the last kept anchor of an earlier tile
                    int64_t tt = (int64_t)blockIdx.x - 1;
                    while (tt >= 0 && last_kept[tt] < 0) --tt;
                    hd = tt < 0 || (uint32_t)(ax[last_kept[tt]] >> 32) != xh[j];
                }
            }
            if (hd) {
                const int64_t o = base + rc[j * 4 + w] + __popcll(below);
                atomicOr(ohb + (o >> 5), 1u << (o & 31));
            }
        }
    }
}

// query of each chain (from the sorted first-anchor key, via the anchor query offsets)
__global__ void chain_query_kernel(const uint64_t *ckey, int64_t n, const int64_t *a_off, int n_q, uint32_t *cq) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n) cq[c] = (uint32_t)upper_idx(a_off, n_q, (int64_t)ckey[c]);
}

__global__ void count_per_query_kernel(const uint32_t *cq, int64_t n, int n_q, int64_t *q_first) {
    // q_first[q] = first chain index of query q (lower bound), q_first[n_q] = n
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p > n) return;
    const int64_t qp = p == 0 ? -1 : (int64_t)cq[p - 1];
    const int64_t qc = p == n ? (int64_t)n_q : (int64_t)cq[p];
    for (int64_t q = qp + 1; q <= qc; q++) q_first[q] = p;
}

}  // namespace

// ---------------------------------------------------------------- host helpers
// HYMET_TRACE=1: whole-call wall time of hymet_mm_map, destructors included
struct CallTrace {
    bool on = getenv("HYMET_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    ~CallTrace() {
        if (on)
            fprintf(stderr, "[hymet_mm_map] %-22s %9.2f ms\n", "TOTAL (with frees)",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count());
    }
};
// HYMET_TRACE=1: per-phase wall times of hymet_mm_map (stream synchronised at each mark)
struct PhaseTrace {
    hymet_ctx *ctx;
    bool on;
    std::chrono::steady_clock::time_point t;
    explicit PhaseTrace(hymet_ctx *c) : ctx(c), on(getenv("HYMET_TRACE") != nullptr), t(std::chrono::steady_clock::now()) {}
    void mark(const char *what) {
        if (!on) return;
        (void)hipStreamSynchronize(ctx->stream);
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[hymet_mm_map] %-22s %9.2f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

// the library's stable LSD radix sort (sort.hpp), profiled under `tag`; keys / vals point at
// the sorted data on return
template <typename K, typename V, int RB = 0>
static int sort_pairs(hymet_ctx *ctx, K *&keys, K *&keys_alt, V *&vals, V *&vals_alt, int64_t n, int begin_bit, int end_bit,
                      const char *tag = "radix_sort") {
    if (n <= 1) return HYMET_OK;
    ProfScope _ps(ctx, tag, 2.0 * (double)n * (sizeof(K) + sizeof(V)) * (double)((end_bit - begin_bit + 7) / 8));
    return radix_sort_pairs(ctx, keys, keys_alt, vals, vals_alt, n, begin_bit, end_bit);
}

static int scan_flags(hymet_ctx *ctx, const uint32_t *flag, int64_t n, DevBuf &pos, int64_t *total) {
    HY_HIP(pos.alloc(8 * (size_t)(n + 1), ctx->stream));
    return exclusive_scan_u32_i64(ctx, flag, pos.as<int64_t>(), n, total);
}


#define LAUNCH1(kern, n, ...)                                                                           \
    do {                                                                                                \
        if ((n) > 0) {                                                                                  \
            hipLaunchKernelGGL(kern, dim3((unsigned)cdiv((n), 256)), dim3(256), 0, ctx->stream, __VA_ARGS__); \
            HY_CHECK_LAUNCH(#kern);                                                                     \
        }                                                                                               \
    } while (0)

// An anchor set sorted by (query, x, y): arrays + per-query offsets (device + host).
struct AnchorSet {
    DevBuf ax, ay;
    int64_t n = 0;
    DevBuf d_off;
    DevBuf hb;            // group-head bitmap (head_bits_bytes(n)): bit i where x >> 32 changes
    bool has_hb = false;  // hb written by whoever built the set; else chain_set derives it from x
    DevBuf ax32;          // x's low words (the chaining kernels read 4 B of x per anchor, not 8)
    bool has_x32 = false;
};

// Chains of an anchor set: compacted anchors (chain by chain, chains ordered by first
// anchor) + chain scores/counts + per-query chain offsets.
struct ChainSet {
    DevBuf cu, cboff;          // per chain: score<<32 | count; offset of its anchors in chain order
    DevBuf ids, cfirst;        // backtrack output (each chain end -> start) and each chain's first slot
    const uint64_t *ax = nullptr, *ay = nullptr;  // the chained anchor set (alive as long as the chains)
    DevBuf bx, by, bchain;     // a copy of the chained anchors in chain order (only for re-chain paths)
    DevBuf cq;                 // query of each chain
    int64_t n_anchor = 0, n_chain = 0;
    DevBuf d_qc, d_qb;  // n_q + 1 chain / chain-order anchor offsets per query
};

// A first pass followed by the long join (map.c's rmq rescue): chain_set flags the re-chained
// queries from its chain list; with mark_only their chains are not copied out (their regions
// are never built) but marked in the chained anchor set, which the long join compacts.
struct LeanJoin {
    const int64_t *qlen;
    int rescue_size;
    float rescue_ratio;
    bool mark_only;
    DevBuf flag;                 // per query: re-chained
    DevBuf mark;                 // mark_only: per anchor of the set (+16 bytes for 16-byte loads)
    DevBuf qb2;                  // mark_only: n_q + 1 offsets of the re-chained queries' chain anchors
    int64_t n2 = 0;
};

// sort raw anchors (x, y, k1 with k2 keys) into an AnchorSet
static int sort_anchor_set(hymet_ctx *ctx, DevBuf &x, DevBuf &y, DevBuf &k1, DevBuf &k2, DevBuf &val, int64_t n,
                           int key1_bits, AnchorSet &out) {
    DevBuf k2b, valb, k1g, k1b;
    HY_HIP(k2b.alloc(8 * (size_t)n, ctx->stream));
    HY_HIP(valb.alloc(4 * (size_t)n, ctx->stream));
    uint64_t *kk = k2.as<uint64_t>(), *kka = k2b.as<uint64_t>();
    uint32_t *vv = val.as<uint32_t>(), *vva = valb.as<uint32_t>();
    int rc = sort_pairs(ctx, kk, kka, vv, vva, n, 0, 64, "radix_sort_anchor_pos");
    if (rc) return rc;
    HY_HIP(k1g.alloc(8 * (size_t)n, ctx->stream));
    HY_HIP(k1b.alloc(8 * (size_t)n, ctx->stream));
    LAUNCH1(gather_kernel<uint64_t>, n, k1.as<uint64_t>(), vv, k1g.as<uint64_t>(), n);
    uint64_t *k1p = k1g.as<uint64_t>(), *k1a = k1b.as<uint64_t>();
    rc = sort_pairs(ctx, k1p, k1a, vv, vva, n, 0, key1_bits, "radix_sort_anchor_group");
    if (rc) return rc;
    HY_HIP(out.ax.alloc(8 * (size_t)n, ctx->stream));
    HY_HIP(out.ay.alloc(8 * (size_t)n, ctx->stream));
    LAUNCH1(gather_kernel<uint64_t>, n, x.as<uint64_t>(), vv, out.ax.as<uint64_t>(), n);
    LAUNCH1(gather_kernel<uint64_t>, n, y.as<uint64_t>(), vv, out.ay.as<uint64_t>(), n);
    out.n = n;
    return HYMET_OK;
}

// sort anchor keys (write_anchor_keys_kernel / rechain_keys_kernel) into an AnchorSet: the
// per-query grouped sort (mm_asort.hip), or one LSD radix sort over the key's significant
// bits where that does not apply (HYMET_ANCHOR_GSORT=0 forces it), then unpack to (x, y)
static int sort_anchor_keys(hymet_ctx *ctx, DevBuf &key, DevBuf &val, int64_t n, int end_bit, int rb, int pb, int yhi,
                            const int64_t *d_qoff, int n_q, int64_t max_qlen, AnchorSet &out) {
    DevBuf kb, vb;
    HY_HIP(kb.alloc(8 * (size_t)n, ctx->stream));
    HY_HIP(vb.alloc(4 * (size_t)n, ctx->stream));
    HY_HIP(out.ax.alloc(8 * (size_t)n, ctx->stream));
    HY_HIP(out.ay.alloc(8 * (size_t)n, ctx->stream));
    out.n = n;
    uint64_t *kk = key.as<uint64_t>(), *kka = kb.as<uint64_t>();
    uint32_t *vv = val.as<uint32_t>(), *vva = vb.as<uint32_t>();
    static const bool gsort = [] {
        const char *e = getenv("HYMET_ANCHOR_GSORT");
        return !(e && e[0] == '0');
    }();
    if (gsort) {
        HY_HIP(out.hb.alloc(head_bits_bytes(n), ctx->stream));
        HY_HIP(out.ax32.alloc(4 * (size_t)n, ctx->stream));
        const int rc = grouped_anchor_sort(ctx, kk, vv, n, d_qoff, n_q, rb, pb, (uint64_t)yhi, max_qlen, kka, vva,
                                           out.ax.as<uint64_t>(), out.ay.as<uint64_t>(), out.hb.as<uint32_t>(),
                                           out.ax32.as<uint32_t>());
        if (rc == HYMET_OK) {
            out.has_hb = out.has_x32 = true;
            return HYMET_OK;
        }
        if (rc != 1) return rc;
    }
    int rc = sort_pairs<uint64_t, uint32_t>(ctx, kk, kka, vv, vva, n, 0, end_bit, "radix_sort_anchors");
    if (rc) return rc;
    {
        ProfScope _ps(ctx, "mm_anchor_unpack", 28.0 * (double)n);  // key + value read, x + y write
        LAUNCH1(anchor_unpack_kernel, n, kk, vv, n, rb, pb, (uint64_t)yhi, out.ax.as<uint64_t>(), out.ay.as<uint64_t>());
    }
    return HYMET_OK;
}

// chaining + backtrack + compact_a over an anchor set
static int chain_set(hymet_ctx *ctx, const hymet_mm_opt *opt, float pen_gap, float pen_skip, int bw, AnchorSet &A,
                     int n_q, ChainSet &C, LeanJoin *lj = nullptr, bool copy = false) {
    const int64_t n = A.n;
    C.ax = A.ax.as<uint64_t>(), C.ay = A.ay.as<uint64_t>();
    if (n == 0) {
        HY_HIP(C.d_qc.alloc(8 * (size_t)(n_q + 1), ctx->stream));
        HY_HIP(C.d_qb.alloc(8 * (size_t)(n_q + 1), ctx->stream));
        HY_HIP(hipMemsetAsync(C.d_qc.p, 0, 8 * (size_t)(n_q + 1), ctx->stream));
        HY_HIP(hipMemsetAsync(C.d_qb.p, 0, 8 * (size_t)(n_q + 1), ctx->stream));
        return HYMET_OK;
    }
    // groups: (query, strand, target) runs, from the set's head bitmap by tiles (count, scan of
    // the tile counts, write)
    if (!A.has_hb) {
        HY_HIP(A.hb.alloc(head_bits_bytes(n), ctx->stream));
        LAUNCH1(head_bits_x_kernel, n, A.ax.as<uint64_t>(), n, A.hb.as<uint64_t>());
        A.has_hb = true;
    }
    if (!A.has_x32) {
        HY_HIP(A.ax32.alloc(4 * (size_t)n, ctx->stream));
        LAUNCH1(x_low_kernel, n, A.ax.as<uint64_t>(), n, A.ax32.as<uint32_t>());
        A.has_x32 = true;
    }
    DevBuf tcnt, toff;
    const int64_t ntile = cdiv(n, kGTile);
    HY_HIP(tcnt.alloc(4 * (size_t)(ntile + 1), ctx->stream));
    HY_HIP(toff.alloc(8 * (size_t)(ntile + 1), ctx->stream));
    hipLaunchKernelGGL(group_heads_count_kernel, dim3((unsigned)ntile), dim3(256), 0, ctx->stream, A.hb.as<uint32_t>(), n,
                       A.d_off.as<int64_t>(), n_q, tcnt.as<uint32_t>());
    HY_CHECK_LAUNCH("group_heads_count_kernel");
    int64_t G = 0;
    int rc = exclusive_scan_u32_i64(ctx, tcnt.as<uint32_t>(), toff.as<int64_t>(), ntile, &G);
    if (rc) return rc;
    DevBuf g_start, t, qfirst;
    HY_HIP(g_start.alloc(8 * (size_t)(G + 1), ctx->stream));
    HY_HIP(qfirst.alloc((size_t)G, ctx->stream));
    HY_HIP(t.alloc(4 * (size_t)n, ctx->stream));  // zeroed by the chaining kernels (and nonwork_fp_kernel) as they go
    if (!HYMET_CHAIN_TZERO) HY_HIP(hipMemsetAsync(t.p, 0, 4 * (size_t)n, ctx->stream));
    hipLaunchKernelGGL(group_heads_write_kernel, dim3((unsigned)ntile), dim3(256), 0, ctx->stream, A.hb.as<uint32_t>(), n,
                       A.d_off.as<int64_t>(), n_q, toff.as<int64_t>(), g_start.as<int64_t>(), qfirst.as<uint8_t>(), G);
    HY_CHECK_LAUNCH("group_heads_write_kernel");
    // work list: groups with >= min_cnt anchors, biggest first
    DevBuf skey, sidx, swork, skey2, sidx2, zlists;
    HY_HIP(skey.alloc(4 * (size_t)G, ctx->stream));
    HY_HIP(sidx.alloc(4 * (size_t)G, ctx->stream));
    HY_HIP(swork.alloc(4 * (size_t)G, ctx->stream));
    HY_HIP(skey2.alloc(4 * (size_t)G, ctx->stream));
    HY_HIP(sidx2.alloc(4 * (size_t)G, ctx->stream));
    HY_HIP(zlists.alloc(32, ctx->stream));
    LAUNCH1(group_size_kernel, std::max<int64_t>(G, 8), g_start.as<int64_t>(), (int32_t)G, opt->min_cnt, skey.as<uint32_t>(),
            sidx.as<uint32_t>(), swork.as<uint32_t>(), (uint8_t *)nullptr, zlists.as<int32_t>());
    // drop non-work groups: key of those = 0xffffffff (sorted last), count them on the host
    {
        DevBuf wpos;
        int64_t n_work = 0;
        rc = scan_flags(ctx, swork.as<uint32_t>(), G, wpos, &n_work);
        if (rc) return rc;
        uint32_t *kp = skey.as<uint32_t>(), *ka = skey2.as<uint32_t>(), *vp = sidx.as<uint32_t>(), *va = sidx2.as<uint32_t>();
        rc = sort_pairs(ctx, kp, ka, vp, va, G, 0, 16, "radix_sort_groups");
        if (rc) return rc;
        {  // the chaining kernel packs local predecessor indices in 24 bits
            LAUNCH1(max_group_kernel, 1, g_start.as<int64_t>(), (const int32_t *)vp, (int32_t)G, mb_dev(ctx, kMbGmax));
            HY_HIP(hipStreamSynchronize(ctx->stream));
            const int64_t big = mb_read(ctx, kMbGmax);
            HY_ARG(big < (1ll << 24) - 1, "hymet_mm_map: an anchor group exceeds 2^24 anchors");
            static const bool stats = getenv("HYMET_CHAIN_STATS") != nullptr;  // profiling: tail size per launch
            if (stats) fprintf(stderr, "[chain] bw %d anchors %lld groups %lld work %lld largest %lld\n", bw, (long long)n,
                               (long long)G, (long long)n_work, (long long)big);
        }
        DevBuf f, p;
        HY_HIP(f.alloc(4 * (size_t)n, ctx->stream));
        HY_HIP(p.alloc(8 * (size_t)n, ctx->stream));
        // the chaining kernels write f/p (and t = 0) of every anchor of a work group; the rest
        // (groups of fewer than min_cnt anchors) get f = 0, p = -1, t = 0 here instead of
        // memsets of all n
        LAUNCH1(nonwork_fp_kernel, G, g_start.as<int64_t>(), (int32_t)G, opt->min_cnt, f.as<int32_t>(), p.as<int64_t>(),
                t.as<int32_t>());
        rc = launch_chain(ctx, A.ax32.as<int32_t>(), A.ay.as<uint64_t>(), g_start.as<int64_t>(), qfirst.as<uint8_t>(),
                          (const int32_t *)vp,
                          (int32_t)n_work, f.as<int32_t>(), p.as<int64_t>(), t.as<int32_t>(), opt->max_gap,
                          opt->rmq_inner_dist, bw, opt->max_chain_skip, opt->rmq_size_cap, pen_gap, pen_skip, n, G);
        if (rc) return rc;
        // z = anchors with f >= min_sc ordered by (group, f, idx), inside each group's range
        DevBuf zkey, zidx, z_cnt, z_runs, run_start, merge_list, mergeu_list, mid_list, big_list, big_off;
        HY_HIP(zkey.alloc(8 * (size_t)n, ctx->stream));
        HY_HIP(zidx.alloc(4 * (size_t)n, ctx->stream));
        HY_HIP(z_cnt.alloc(4 * (size_t)G, ctx->stream));
        HY_HIP(z_runs.alloc(4 * (size_t)G, ctx->stream));
        HY_HIP(run_start.alloc(4 * (size_t)G * kZRuns, ctx->stream));
        HY_HIP(merge_list.alloc(4 * (size_t)G, ctx->stream));
        // HYMET_ZM_LDS / HYMET_ZM_UNIT (tests): stage merge groups up to that many entries, split
        // the others into units of that many
        const char *el = getenv("HYMET_ZM_LDS"), *eu = getenv("HYMET_ZM_UNIT");
        const int zm_lds = el ? std::max(0, std::min(kZmLds, atoi(el))) : kZmLds;
        const int zm_unit = eu ? std::max(1, atoi(eu)) : kZmUnit;
        HY_HIP(mergeu_list.alloc(8 * (size_t)(n / zm_unit + G + 16), ctx->stream));  // >= sum of cdiv(m, unit)
        HY_HIP(mid_list.alloc(4 * (size_t)G, ctx->stream));
        HY_HIP(big_list.alloc(4 * (size_t)G, ctx->stream));
        HY_HIP(big_off.alloc(8 * (size_t)G, ctx->stream));
        const int32_t *vi = zidx.as<int32_t>();
        {
            ProfScope _ps(ctx, "mm_z_order", 16.0 * (double)n);  // f read, key + idx written (z entries <= anchors)
            // HYMET_Z_RUNS (tests): merge groups of at most that many runs, sort the others
            const char *ev = getenv("HYMET_Z_RUNS");
            const int max_runs = ev ? std::max(1, std::min(kZRuns, atoi(ev))) : kZRuns;
            ZParams Z{f.as<int32_t>(), g_start.as<int64_t>(), (const int32_t *)vp, (int32_t)G, opt->min_chain_score,
                      max_runs, zm_lds, zm_unit, zkey.as<uint64_t>(), zidx.as<int32_t>(), z_cnt.as<int32_t>(), z_runs.as<int32_t>(),
                      run_start.as<int32_t>(), zlists.as<int32_t>(), merge_list.as<int32_t>(), mergeu_list.as<int64_t>(),
                      mid_list.as<int32_t>(), big_list.as<int32_t>(),
                      big_off.as<int64_t>(), mb_dev(ctx, kMbZBig)};
            hipLaunchKernelGGL(zsplit_kernel, dim3(1), dim3(64), 0, ctx->stream, Z);
            HY_CHECK_LAUNCH("zsplit_kernel");
            const int64_t nwb = std::min<int64_t>(cdiv(G, 4), (int64_t)ctx->n_cu * 8);
            hipLaunchKernelGGL(zorder_wave_kernel, dim3((unsigned)std::max<int64_t>(nwb, 1)), dim3(256), 0, ctx->stream, Z);
            HY_CHECK_LAUNCH("zorder_wave_kernel");
            LAUNCH1(zorder_lane_kernel, G, Z);
            const int64_t nb = std::min<int64_t>(G, (int64_t)ctx->n_cu * 8);
            hipLaunchKernelGGL(zmerge_kernel, dim3((unsigned)nb), dim3(256), 0, ctx->stream, Z);
            HY_CHECK_LAUNCH("zmerge_kernel");
            hipLaunchKernelGGL(zsort_block_kernel, dim3((unsigned)nb), dim3(256), 0, ctx->stream, Z);
            HY_CHECK_LAUNCH("zsort_block_kernel");
            HY_HIP(hipStreamSynchronize(ctx->stream));
            const int64_t n_big = mb_read(ctx, kMbZBig), nz_big = mb_read(ctx, kMbZBigTotal);
            if (n_big > 0) {
                DevBuf bcnt;
                HY_HIP(bcnt.alloc(4 * (size_t)(n_big + 1), ctx->stream));
                LAUNCH1(zbig_count_kernel, n_big, Z, (int32_t)n_big, bcnt.as<uint32_t>());
                int64_t nz_scan = 0;
                rc = exclusive_scan_u32_i64(ctx, bcnt.as<uint32_t>(), big_off.as<int64_t>(), n_big, &nz_scan);
                if (rc) return rc;
                if (nz_scan != nz_big) return hymet::fail(HYMET_E_INTERNAL, "hymet_mm_map: z list count mismatch");
                DevBuf sk, sk2, sv, sv2;
                HY_HIP(sk.alloc(8 * (size_t)nz_big, ctx->stream));
                HY_HIP(sk2.alloc(8 * (size_t)nz_big, ctx->stream));
                HY_HIP(sv.alloc(4 * (size_t)nz_big, ctx->stream));
                HY_HIP(sv2.alloc(4 * (size_t)nz_big, ctx->stream));
                hipLaunchKernelGGL(zbig_gather_kernel, dim3((unsigned)n_big), dim3(256), 0, ctx->stream, Z, sk.as<uint64_t>(),
                                   sv.as<uint32_t>());
                HY_CHECK_LAUNCH("zbig_gather_kernel");
                uint64_t *kp = sk.as<uint64_t>(), *ka = sk2.as<uint64_t>();
                uint32_t *vp2 = sv.as<uint32_t>(), *va2 = sv2.as<uint32_t>();
                rc = sort_pairs(ctx, kp, ka, vp2, va2, nz_big, 0, 32 + bits_for(n_big), "radix_sort_z_big");
                if (rc) return rc;
                hipLaunchKernelGGL(zbig_scatter_kernel, dim3((unsigned)n_big), dim3(256), 0, ctx->stream, Z,
                                   (const uint32_t *)vp2);
                HY_CHECK_LAUNCH("zbig_scatter_kernel");
            }
        }
        DevBuf chain_ids, chain_u, chain_first, n_chains;
        HY_HIP(chain_ids.alloc(8 * (size_t)n, ctx->stream));
        HY_HIP(chain_u.alloc(8 * (size_t)n, ctx->stream));
        HY_HIP(chain_first.alloc(8 * (size_t)n, ctx->stream));
        HY_HIP(n_chains.alloc(4 * (size_t)G, ctx->stream));
        if (getenv("HYMET_TRACE_BT")) {  // diagnostic: backtrack time vs the largest groups
            std::vector<int64_t> gs(G + 1);
            std::vector<int32_t> zc(G);
            HY_HIP(hipMemcpyAsync(gs.data(), g_start.p, 8 * (size_t)(G + 1), hipMemcpyDeviceToHost, ctx->stream));
            HY_HIP(hipMemcpyAsync(zc.data(), z_cnt.p, 4 * (size_t)G, hipMemcpyDeviceToHost, ctx->stream));
            HY_HIP(hipStreamSynchronize(ctx->stream));
            int64_t mg = 0, mz = 0, big = 0, nz = 0;
            for (int64_t g = 0; g < G; g++) {
                mg = std::max(mg, gs[g + 1] - gs[g]);
                mz = std::max(mz, (int64_t)zc[g]);
                nz += zc[g];
                big += gs[g + 1] - gs[g] > 10000;
            }
            fprintf(stderr, "[bt] G=%lld n=%lld nz=%lld max_group=%lld max_z=%lld groups>10k=%lld", (long long)G,
                    (long long)n, (long long)nz, (long long)mg, (long long)mz, (long long)big);
        }
        const auto bt0 = std::chrono::steady_clock::now();
        rc = launch_backtrack(ctx, g_start.as<int64_t>(), f.as<int32_t>(), p.as<int64_t>(), t.as<int32_t>(),
                              z_cnt.as<int32_t>(), (const int32_t *)vi, (int32_t)G, (const int32_t *)vp, (int32_t)n_work,
                              opt->min_cnt, opt->min_chain_score, bw,
                              chain_ids.as<int64_t>(), chain_u.as<uint64_t>(), chain_first.as<int64_t>(),
                              n_chains.as<int32_t>(), n);
        if (rc) return rc;
        if (getenv("HYMET_DEBUG_BT")) {  // diagnostic: z order and chain disjointness per group
            HY_HIP(hipStreamSynchronize(ctx->stream));
            std::vector<int64_t> gs(G + 1), hid(n), hcf(n);
            std::vector<int32_t> zc(G), zi(n), hf(n), nch(G), zr(G);
            std::vector<uint64_t> hcu(n);
            HY_HIP(hipMemcpy(gs.data(), g_start.p, 8 * (size_t)(G + 1), hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(zc.data(), z_cnt.p, 4 * (size_t)G, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(zr.data(), z_runs.p, 4 * (size_t)G, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(zi.data(), zidx.p, 4 * (size_t)n, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(hf.data(), f.p, 4 * (size_t)n, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(nch.data(), n_chains.p, 4 * (size_t)G, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(hid.data(), chain_ids.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(hcu.data(), chain_u.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
            HY_HIP(hipMemcpy(hcf.data(), chain_first.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
            std::vector<int32_t> seen(n, -1);
            int64_t bad_z = 0, bad_c = 0;
            for (int64_t g = 0; g < G; g++) {
                const int64_t g0 = gs[g], gn = gs[g + 1] - g0;
                int64_t want = 0;
                for (int64_t a = g0; a < g0 + gn; a++) want += hf[a] >= opt->min_chain_score;
                bool zok = zc[g] == want || gn < opt->min_cnt;
                for (int64_t t = 0; zok && t < zc[g]; t++) {
                    const int64_t a = zi[g0 + t];
                    if (a < g0 || a >= g0 + gn || hf[a] < opt->min_chain_score) zok = false;
                    else if (t > 0) {
                        const int64_t b = zi[g0 + t - 1];
                        if (!(hf[b] < hf[a] || (hf[b] == hf[a] && b < a))) zok = false;
                    }
                }
                if (!zok && bad_z++ < 5)
                    fprintf(stderr, "[bt] group %lld size %lld: z order wrong (z_cnt %d want %lld runs %d)\n", (long long)g,
                            (long long)gn, zc[g], (long long)want, zr[g]);
                for (int c = 0; c < nch[g]; c++) {
                    const int64_t fo = hcf[g0 + c];
                    const int32_t m = (int32_t)hcu[g0 + c];
                    for (int32_t j = 0; j < m; j++) {
                        const int64_t a = hid[fo + j];
                        if (a < g0 || a >= g0 + gn || seen[a] == (int32_t)g) {
                            if (bad_c++ < 5)
                                fprintf(stderr, "[bt] group %lld size %lld chain %d/%d anchor %lld %s (z runs %d)\n",
                                        (long long)g, (long long)gn, c, nch[g], (long long)a,
                                        (a < g0 || a >= g0 + gn) ? "outside the group" : "in two chains", zr[g]);
                        } else {
                            seen[a] = (int32_t)g;
                        }
                    }
                }
            }
            fprintf(stderr, "[bt] groups %lld anchors %lld: z errors %lld, chain overlaps %lld\n", (long long)G, (long long)n,
                    (long long)bad_z, (long long)bad_c);
        }
        if (getenv("HYMET_TRACE_BT")) {
            HY_HIP(hipStreamSynchronize(ctx->stream));
            fprintf(stderr, " bt=%.2f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - bt0).count());
        }
        // chain list sorted by first anchor index (compact_a order)
        DevBuf cpos;
        int64_t NC = 0;
        rc = scan_flags(ctx, (const uint32_t *)n_chains.p, G, cpos, &NC);
        if (rc) return rc;
        C.n_chain = NC;
        DevBuf ckey, cfirst, ckey2, cu2, cfirst2;
        HY_HIP(ckey.alloc(8 * (size_t)(NC + 1), ctx->stream));
        HY_HIP(C.cu.alloc(8 * (size_t)(NC + 1), ctx->stream));
        HY_HIP(cfirst.alloc(8 * (size_t)(NC + 1), ctx->stream));
        LAUNCH1(chain_list_kernel, G, g_start.as<int64_t>(), n_chains.as<int32_t>(), cpos.as<int64_t>(), (int32_t)G,
                chain_u.as<uint64_t>(), chain_first.as<int64_t>(), chain_ids.as<int64_t>(), ckey.as<uint64_t>(),
                C.cu.as<uint64_t>(), cfirst.as<int64_t>());
        // sort chains by first anchor: pairs (key, perm) then gather
        DevBuf perm, perm2, ckeyb;
        HY_HIP(perm.alloc(4 * (size_t)(NC + 1), ctx->stream));
        HY_HIP(perm2.alloc(4 * (size_t)(NC + 1), ctx->stream));
        HY_HIP(ckeyb.alloc(8 * (size_t)(NC + 1), ctx->stream));
        LAUNCH1(iota_u32_kernel, NC, perm.as<uint32_t>(), NC);
        uint64_t *ck = ckey.as<uint64_t>(), *cka = ckeyb.as<uint64_t>();
        uint32_t *pp = perm.as<uint32_t>(), *ppa = perm2.as<uint32_t>();
        rc = sort_pairs(ctx, ck, cka, pp, ppa, NC, 0, bits_for(n), "radix_sort_chains");
        if (rc) return rc;
        DevBuf cu_s, cf_s;
        HY_HIP(cu_s.alloc(8 * (size_t)(NC + 1), ctx->stream));
        HY_HIP(cf_s.alloc(8 * (size_t)(NC + 1), ctx->stream));
        LAUNCH1(gather_kernel<uint64_t>, NC, C.cu.as<uint64_t>(), pp, cu_s.as<uint64_t>(), NC);
        LAUNCH1(gather_kernel<int64_t>, NC, cfirst.as<int64_t>(), pp, cf_s.as<int64_t>(), NC);
        C.cu.swap(cu_s);
        // per-query chain offsets
        DevBuf &cq = C.cq;
        HY_HIP(cq.alloc(4 * (size_t)(NC + 1), ctx->stream));
        LAUNCH1(chain_query_kernel, NC, ck, NC, A.d_off.as<int64_t>(), n_q, cq.as<uint32_t>());
        HY_HIP(C.d_qc.alloc(8 * (size_t)(n_q + 1), ctx->stream));
        hipLaunchKernelGGL(count_per_query_kernel, dim3((unsigned)cdiv(NC + 1, 256)), dim3(256), 0, ctx->stream,
                           cq.as<uint32_t>(), NC, n_q, C.d_qc.as<int64_t>());
        HY_CHECK_LAUNCH("count_per_query_kernel");
        // long join: the re-chained queries, from the chain list
        const uint32_t *qflag = nullptr;
        if (lj) {
            HY_HIP(lj->flag.alloc(4 * (size_t)n_q, ctx->stream));
            LAUNCH1(rechain_flag_kernel, n_q, A.ay.as<uint64_t>(), chain_ids.as<int64_t>(), C.cu.as<uint64_t>(),
                    cf_s.as<int64_t>(), C.d_qc.as<int64_t>(), lj->qlen, n_q, lj->rescue_size, lj->rescue_ratio,
                    lj->flag.as<uint32_t>());
            if (lj->mark_only) qflag = lj->flag.as<uint32_t>();
        }
        // anchors of every chain (but those only marked), compacted in chain order
        DevBuf ccnt, ccnt2;
        HY_HIP(ccnt.alloc(4 * (size_t)(NC + 1), ctx->stream));
        if (qflag) HY_HIP(ccnt2.alloc(4 * (size_t)(NC + 1), ctx->stream));
        LAUNCH1(chain_cnt_kernel, NC, C.cu.as<uint64_t>(), cq.as<uint32_t>(), qflag, NC, ccnt.as<uint32_t>(),
                qflag ? ccnt2.as<uint32_t>() : nullptr);
        int64_t NB = 0;
        rc = scan_flags(ctx, ccnt.as<uint32_t>(), NC, C.cboff, &NB);
        if (rc) return rc;
        C.n_anchor = NB;
        if (copy) {  // the re-sort / two-key long-join paths read the chained anchors as a copy
            HY_HIP(C.bx.alloc(8 * (size_t)(NB + 1), ctx->stream));
            HY_HIP(C.by.alloc(8 * (size_t)(NB + 1), ctx->stream));
            HY_HIP(C.bchain.alloc(4 * (size_t)(NB + 1), ctx->stream));
            if (NC > 0 && NB > 0)
                LAUNCH1(chain_copy_kernel, NB, C.cu.as<uint64_t>(), cf_s.as<int64_t>(), C.cboff.as<int64_t>(),
                        chain_ids.as<int64_t>(), A.ax.as<uint64_t>(), A.ay.as<uint64_t>(), NC, NB, C.bx.as<uint64_t>(),
                        C.by.as<uint64_t>(), C.bchain.as<int32_t>());
        }
        HY_HIP(C.d_qb.alloc(8 * (size_t)(n_q + 1), ctx->stream));
        LAUNCH1(chain_qb_kernel, n_q + 1, C.d_qc.as<int64_t>(), C.cboff.as<int64_t>(), NC, NB, n_q, C.d_qb.as<int64_t>());
        if (qflag) {  // the re-chained queries' chain anchors: per-query counts, and t handed over
            DevBuf boff2;
            int64_t NB2 = 0;
            rc = scan_flags(ctx, ccnt2.as<uint32_t>(), NC, boff2, &NB2);
            if (rc) return rc;
            // the backtrack left t == 2 on every kept chain's anchors: the long join selects
            // those of its queries straight from t (no pass over the chains)
            lj->mark.swap(t);
            HY_HIP(lj->qb2.alloc(8 * (size_t)(n_q + 1), ctx->stream));
            LAUNCH1(chain_qb_kernel, n_q + 1, C.d_qc.as<int64_t>(), boff2.as<int64_t>(), NC, NB2, n_q, lj->qb2.as<int64_t>());
            lj->n2 = NB2;
        }
        // regions and chain statistics read the chains in place
        C.ids.swap(chain_ids);
        C.cfirst.swap(cf_s);
    }
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet

namespace hymet {
namespace mm {
int launch_regions(hymet_ctx *ctx, const uint64_t *ax, const uint64_t *ay, const int64_t *ids, const int64_t *cfirst,
                   const uint64_t *cu, const int64_t *cboff,
                   const int64_t *qc, const int64_t *qb, const uint64_t *mini_pos, const int64_t *mp_off, const int64_t *qlen,
                   const uint32_t *name_hash, const int32_t *rep_len, const int64_t *ref_len, int n_q, const hymet_mm_opt *o,
                   int k, void *z, hymet_mm_reg *regs, int32_t *w, uint64_t *cov, int32_t *tmp, int32_t *n_regs,
                   int64_t NB, int64_t NC, int64_t NM, const uint32_t *cq,
                   const MiniWord *mtab, const int64_t *qbase, const uint32_t *skip_q, uint64_t *sumk, bool sumk_done);

namespace {
// query position -> index among the query's seeded minimizers (mini_pos order), for
// mm_est_err's get_mini_idx (MiniWord): pass 1 sets the start bits, pass 2 writes each word's
// base (every seeded minimizer of the word writes the same value: its index less the start
// bits below it)
__global__ __launch_bounds__(256) void mini_bits_kernel(const uint64_t *my, const uint32_t *seed_n, const uint32_t *qid,
                                                        const int64_t *qbase, int64_t M, MiniWord *tab) {
    // consecutive minimizers of a query share words: the bits of a run of lanes on one word
    // are OR-ed across the run and set by one atomic (device-scope atomics are the costly part)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool on = i < M && seed_n[i];
    const int64_t b = on ? qbase[qid[i]] + ((uint32_t)my[i] >> 1) : -64 * (int64_t)(lane + 1);  // distinct dummy words
    const int64_t w = b >> 6;
    uint64_t bits = on ? 1ull << (b & 63) : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // OR over the lanes of the same word (runs are contiguous)
        const int64_t wo = __shfl_down(w, d, 64);
        const uint64_t bo = __shfl_down(bits, d, 64);
        if (lane + d < 64 && wo == w) bits |= bo;
    }
    const int64_t wp = __shfl_up(w, 1, 64);
    if (on && (lane == 0 || wp != w)) atomicOr((unsigned long long *)&tab[w].bits, bits);
}
__global__ void mini_base_kernel(const uint64_t *my, const uint32_t *seed_n, const uint32_t *qid, const int64_t *qm_off,
                                 const int64_t *mp_pos, const int64_t *qbase, int64_t M, MiniWord *tab) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M || !seed_n[i]) return;
    const uint32_t q = qid[i];
    const int64_t b = qbase[q] + ((uint32_t)my[i] >> 1);
    const uint64_t bits = tab[b >> 6].bits;
    tab[b >> 6].base = (uint32_t)(mp_pos[i] - mp_pos[qm_off[q]]) - (uint32_t)__popcll(bits & ((1ull << (b & 63)) - 1));
}

// re-chain input: the chained anchors of flagged queries (query-major), with sort keys
__global__ void rechain_gather_kernel(const uint64_t *bx, const uint64_t *by, const int64_t *qb, const uint32_t *qflag,
                                      const int64_t *new_off, int n_q, int rb, uint64_t *x, uint64_t *y, uint64_t *k1,
                                      uint64_t *k2, uint32_t *val) {
    const int q = blockIdx.x;
    if (q >= n_q || !qflag[q]) return;
    const int64_t b0 = qb[q], b1 = qb[q + 1], o = new_off[q];
    for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        const int64_t a = o + (i - b0);
        const uint64_t ax = bx[i], ay = by[i];
        x[a] = ax;
        y[a] = ay;
        k1[a] = (uint64_t)q << (1 + rb) | (ax >> 63) << rb | (ax << 1 >> 33);
        k2[a] = (uint64_t)(uint32_t)ax << 32 | (uint32_t)ay;
        val[a] = (uint32_t)a;
    }
}

// one thread per re-chain anchor (flat: a block per query left the long queries' blocks as
// the tail); the block's first query by one binary search, each lane's by a short forward walk
__global__ __launch_bounds__(256) void rechain_keys_kernel(const uint64_t *bx, const uint64_t *by, const int64_t *qb,
                                                           const int64_t *new_off, int n_q, int64_t n, int rb, int pb,
                                                           uint64_t *key, uint32_t *val) {
    __shared__ int s_q0;
    const int64_t a0 = (int64_t)blockIdx.x * blockDim.x;
    if (threadIdx.x == 0) s_q0 = upper_idx(new_off, n_q, a0);
    __syncthreads();
    const int64_t a = a0 + threadIdx.x;
    if (a >= n) return;
    int q = s_q0;
    while (q + 1 < n_q && new_off[q + 1] <= a) q++;  // last q with new_off[q] <= a
    const int64_t i = qb[q] + (a - new_off[q]);
    const uint64_t ax = bx[i];
    key[a] = (uint64_t)q << (1 + rb + pb) | (ax >> 63) << (rb + pb) | (ax << 1 >> 33) << pb | (uint32_t)ax;
    val[a] = (uint32_t)by[i];
}

// per query: regions kept (first-pass chains, or the long-join re-chain's for flagged queries)
__global__ void reg_count_kernel(const uint32_t *flag, const int32_t *n1, const int32_t *n2, int n_q, uint32_t *cnt) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n_q) cnt[q] = (uint32_t)((flag && flag[q]) ? n2[q] : n1[q]);
}

// one thread per query: copy its region records to their PAF positions (+ line metadata)
struct RegOut {
    hymet_mm_reg *regs;
    int32_t *q, *part, *rl, *t;  // optional (accumulator sink)
    int32_t q_base, part_id, t_base;
};
__global__ void reg_gather_kernel(const uint32_t *flag, const int32_t *n1, const int32_t *n2, const int64_t *qc1,
                                  const int64_t *qc2, const hymet_mm_reg *r1, const hymet_mm_reg *r2, const int64_t *off,
                                  const int32_t *rep_len, int n_q, RegOut o) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_q) return;
    const bool use2 = flag && flag[q];
    const hymet_mm_reg *src = use2 ? r2 + qc2[q] : r1 + qc1[q];
    const int nr = use2 ? n2[q] : n1[q];
    const int64_t d = off[q];
    for (int i = 0; i < nr; i++) {
        const hymet_mm_reg r = src[i];
        o.regs[d + i] = r;
        if (o.q) {
            o.q[d + i] = o.q_base + q;
            o.part[d + i] = o.part_id;
            o.rl[d + i] = rep_len[q];
            o.t[d + i] = o.t_base + r.rid;
        }
    }
}

__global__ void qlen_sizes_kernel(const int64_t *off, int n_q, const uint32_t *flag, uint32_t *sz) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n_q) sz[q] = flag[q] ? (uint32_t)(off[q + 1] - off[q]) : 0u;
}
}  // namespace
}  // namespace mm
}  // namespace hymet

using namespace hymet;
using namespace hymet::mm;

// where hymet_mm_map puts a batch's PAF records: host vectors (hymet_mm_result) or the
// device-resident accumulator of a run (hymet_paf_acc)
struct MapSink {
    hymet_mm_result *res = nullptr;
    hymet_paf_acc *acc = nullptr;
    int32_t q_base = 0, part_id = 0, t_base = 0;
};

static int acc_reserve(hymet_ctx *ctx, hymet_paf_acc *a, int64_t need) {
    if (need <= a->cap) return HYMET_OK;
    const int64_t cap = std::max<int64_t>(need, std::max<int64_t>(a->cap * 3 / 2, 1 << 16));
    hipStream_t st = ctx->stream;
    DevBuf nregs, nq, npart, nrl, nt;
    HY_HIP(nregs.alloc(sizeof(hymet_mm_reg) * (size_t)cap, st));
    HY_HIP(nq.alloc(4 * (size_t)cap, st));
    HY_HIP(npart.alloc(4 * (size_t)cap, st));
    HY_HIP(nrl.alloc(4 * (size_t)cap, st));
    HY_HIP(nt.alloc(4 * (size_t)cap, st));
    if (a->n) {
        HY_HIP(hipMemcpyAsync(nregs.p, a->regs.p, sizeof(hymet_mm_reg) * (size_t)a->n, hipMemcpyDeviceToDevice, st));
        HY_HIP(hipMemcpyAsync(nq.p, a->q.p, 4 * (size_t)a->n, hipMemcpyDeviceToDevice, st));
        HY_HIP(hipMemcpyAsync(npart.p, a->part.p, 4 * (size_t)a->n, hipMemcpyDeviceToDevice, st));
        HY_HIP(hipMemcpyAsync(nrl.p, a->rl.p, 4 * (size_t)a->n, hipMemcpyDeviceToDevice, st));
        HY_HIP(hipMemcpyAsync(nt.p, a->t.p, 4 * (size_t)a->n, hipMemcpyDeviceToDevice, st));
    }
    a->regs.swap(nregs);
    a->q.swap(nq);
    a->part.swap(npart);
    a->rl.swap(nrl);
    a->t.swap(nt);
    a->cap = cap;
    return HYMET_OK;
}

static int mm_map_impl(hymet_ctx *ctx, const hymet_mm_index *idx, const hymet_mm_opt *opt, const uint32_t *d_2b,
                       const uint32_t *d_mask, const int64_t *h_starts, const int64_t *h_lens, const uint32_t *h_name_hash,
                       const uint32_t *d_name_hash, int32_t n_q, MapSink &sink) {
    CallTrace call_trace;
    HY_ARG(ctx && idx && opt && d_2b && d_mask, "hymet_mm_map: null argument");
    HY_ARG(n_q >= 0, "hymet_mm_map: n_q < 0");
    HY_ARG(h_name_hash || d_name_hash, "hymet_mm_map: no query name hashes");
    HY_ARG(opt->mid_occ > 0, "hymet_mm_map: opt->mid_occ must be resolved (hymet_mm_index_max_occ + clamps)");
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    hymet_mm_result *res = sink.res;
    if (res) {
        res->n_q = n_q;
        res->reg_off.assign(n_q + 1, 0);
        res->rep_len.assign(n_q, 0);
    }
    if (n_q == 0) return HYMET_OK;
    const int k = idx->k, w = idx->w;
    const float pen_gap = (float)(opt->chain_gap_scale * 0.01 * k);
    const float pen_skip = (float)(opt->chain_skip_scale * 0.01 * k);
    int rc;
    PhaseTrace tr(ctx);
    // ---------------------------------------------------------------- 1 sketch
    DevBuf mx, my, qm_off;
    int64_t M = 0;
    rc = sketch_sequences(ctx, d_2b, d_mask, h_starts, h_lens, n_q, w, k, 0, mx, my, &M, &qm_off);
    if (rc) return rc;
    DevBuf d_qlen, d_hash_buf;
    HY_HIP(d_qlen.alloc(8 * (size_t)n_q, st));
    HY_HIP(hipMemcpyAsync(d_qlen.p, h_lens, 8 * (size_t)n_q, hipMemcpyHostToDevice, st));
    const uint32_t *d_hash = d_name_hash;  // the caller's device copy when it has one
    if (!d_hash) {
        HY_HIP(d_hash_buf.alloc(4 * (size_t)n_q, st));
        HY_HIP(hipMemcpyAsync(d_hash_buf.p, h_name_hash, 4 * (size_t)n_q, hipMemcpyHostToDevice, st));
        d_hash = d_hash_buf.as<uint32_t>();
    }
    // ------------------------------------------------------- 2 mm_seed_mz_flt
    bool need_flt = false;
    DevBuf keep, fcnt, fcoff;
    int64_t MF = 0;  // minimizers of the queries the screen could not clear
    if (opt->q_occ_frac > 0.0f && M > 0 && opt->mid_occ > 0) {  // only queries with more than mid_occ minimizers are filtered
        HY_HIP(keep.alloc(4 * (size_t)M, st));
        HY_HIP(fcnt.alloc(4 * (size_t)(n_q + 1), st));
        ctx->mbox_h[kMbFlag] = 0;
        hipLaunchKernelGGL(mzflt_screen_kernel, dim3((unsigned)n_q + 1), dim3(256), 0, st, mx.as<uint64_t>(), qm_off.as<int64_t>(),
                           n_q, opt->mid_occ, keep.as<uint32_t>(), fcnt.as<uint32_t>(), mb_dev(ctx, kMbFlag));
        HY_CHECK_LAUNCH("mzflt_screen_kernel");
        HY_HIP(hipStreamSynchronize(st));
        if (mb_read(ctx, kMbFlag) != 0) {
            HY_HIP(fcoff.alloc(8 * (size_t)(n_q + 1), st));
            rc = exclusive_scan_u32_i64(ctx, fcnt.as<uint32_t>(), fcoff.as<int64_t>(), n_q + 1, &MF);
            if (rc) return rc;
        }
    }
    tr.mark("sketch");
    if (MF > 0) {
        // the exact filter over the flagged queries' minimizers only: list entries sorted by x,
        // then stably by query, runs of equal (q, x) counted
        need_flt = true;
        DevBuf gidx, sx, sx2, sidx, sidx2, sq0, sq, sq2, kpos, nx, ny, gx, gg;
        HY_HIP(gidx.alloc(4 * (size_t)MF, st));
        HY_HIP(sq0.alloc(4 * (size_t)MF, st));
        hipLaunchKernelGGL(mzflt_list_kernel, dim3((unsigned)n_q), dim3(256), 0, st, qm_off.as<int64_t>(), fcnt.as<uint32_t>(),
                           fcoff.as<int64_t>(), gidx.as<uint32_t>(), sq0.as<uint32_t>());
        HY_CHECK_LAUNCH("mzflt_list_kernel");
        HY_HIP(sx.alloc(8 * (size_t)MF, st));
        HY_HIP(sx2.alloc(8 * (size_t)MF, st));
        HY_HIP(sidx.alloc(4 * (size_t)MF, st));
        HY_HIP(sidx2.alloc(4 * (size_t)MF, st));
        LAUNCH1(gather_kernel<uint64_t>, MF, mx.as<uint64_t>(), gidx.as<uint32_t>(), sx.as<uint64_t>(), MF);
        LAUNCH1(iota_u32_kernel, MF, sidx.as<uint32_t>(), MF);
        uint64_t *kx = sx.as<uint64_t>(), *kxa = sx2.as<uint64_t>();
        uint32_t *vi = sidx.as<uint32_t>(), *via = sidx2.as<uint32_t>();
        rc = sort_pairs(ctx, kx, kxa, vi, via, MF, 0, 2 * k + 8, "radix_sort_mz");
        if (rc) return rc;
        HY_HIP(sq.alloc(4 * (size_t)MF, st));
        HY_HIP(sq2.alloc(4 * (size_t)MF, st));
        LAUNCH1(gather_kernel<uint32_t>, MF, sq0.as<uint32_t>(), vi, sq.as<uint32_t>(), MF);
        uint32_t *kq = sq.as<uint32_t>(), *kqa = sq2.as<uint32_t>();
        rc = sort_pairs(ctx, kq, kqa, vi, via, MF, 0, bits_for(n_q), "radix_sort_mz");
        if (rc) return rc;
        HY_HIP(gx.alloc(8 * (size_t)MF, st));
        HY_HIP(gg.alloc(4 * (size_t)MF, st));
        LAUNCH1(mzflt_gather_kernel, MF, vi, gidx.as<uint32_t>(), mx.as<uint64_t>(), gg.as<uint32_t>(), gx.as<uint64_t>(), MF);
        LAUNCH1(mzflt_runs_kernel, MF, kq, gx.as<uint64_t>(), gg.as<uint32_t>(), qm_off.as<int64_t>(), MF, opt->mid_occ,
                opt->q_occ_frac, keep.as<uint32_t>());
        int64_t M2 = 0;
        rc = scan_flags(ctx, keep.as<uint32_t>(), M, kpos, &M2);
        if (rc) return rc;
        HY_HIP(nx.alloc(8 * (size_t)(M2 + 1), st));
        HY_HIP(ny.alloc(8 * (size_t)(M2 + 1), st));
        LAUNCH1(compact_mz_kernel, M, mx.as<uint64_t>(), my.as<uint64_t>(), keep.as<uint32_t>(), kpos.as<int64_t>(), M,
                nx.as<uint64_t>(), ny.as<uint64_t>());
        DevBuf nqm;
        HY_HIP(nqm.alloc(8 * (size_t)(n_q + 1), st));
        hipLaunchKernelGGL(sample_off_kernel, dim3((unsigned)cdiv(n_q + 1, 256)), dim3(256), 0, st, kpos.as<int64_t>(),
                           qm_off.as<int64_t>(), n_q, M2, nqm.as<int64_t>());
        HY_CHECK_LAUNCH("sample_off_kernel");
        mx.swap(nx);
        my.swap(ny);
        qm_off.swap(nqm);
        M = M2;
    }
    tr.mark("mz_flt");
    // ------------------------------------------------------------- 3 seeds
    DevBuf seed_n, rep_len, qid;
    HY_HIP(seed_n.alloc(4 * (size_t)(M + 1), st));
    HY_HIP(rep_len.alloc(4 * (size_t)n_q, st));
    HY_HIP(qid.alloc(4 * (size_t)(M + 1), st));
    LAUNCH1(fill_qid_kernel, std::max<int64_t>(M, n_q), qm_off.as<int64_t>(), n_q, M, qid.as<uint32_t>(), nullptr,
            rep_len.as<int32_t>());
    {
        ProfScope _ps(ctx, "mm_seed_count", (double)M * (8.0 + 8.0 + 4.0));  // minimizer, 2 offsets, count
        LAUNCH1(seed_count_kernel, M, mx.as<uint64_t>(), M, idx->d_koff, idx->n_buckets, seed_n.as<uint32_t>());
    }
    if (M > 0) {
        ProfScope _ps(ctx, "mm_seed_select", (double)M * (4.0 + 8.0 + 8.0 + 8.0));  // count, class, rank, list
        DevBuf cls, rank;
        HY_HIP(cls.alloc(8 * (size_t)(M + 1), st));
        HY_HIP(rank.alloc(8 * (size_t)(M + 1), st));
        LAUNCH1(seed_class_kernel, M + 1, seed_n.as<uint32_t>(), M, opt->mid_occ, cls.as<uint64_t>());
        DevBuf spart;
        {  // exclusive scan of packed (low, high) counts over M + 1 entries: rank[M] = totals
            rc = scan_u64(ctx, cls.as<uint64_t>(), rank.as<uint64_t>(), M + 1, spart, mb_dev(ctx, kMbScan));
            if (rc) return rc;
        }
        HY_HIP(hipStreamSynchronize(st));
        const uint64_t tot = (uint64_t)mb_read(ctx, kMbScan);
        const int64_t n_low = (uint32_t)tot, n_high = (int64_t)(tot >> 32);
        if (n_high > 0) {
            DevBuf low_idx, high_idx, flt_high, vmax, pmax;
            HY_HIP(low_idx.alloc(4 * (size_t)(n_low + 1), st));
            HY_HIP(high_idx.alloc(4 * (size_t)n_high, st));
            HY_HIP(flt_high.alloc(4 * (size_t)n_high, st));
            LAUNCH1(seed_list_kernel, M, seed_n.as<uint32_t>(), rank.as<uint64_t>(), M, opt->mid_occ,
                    low_idx.as<int32_t>(), high_idx.as<int32_t>());
            StreakParams S{my.as<uint64_t>(), qid.as<uint32_t>(), qm_off.as<int64_t>(), d_qlen.as<int64_t>(),
                           rank.as<uint64_t>(), low_idx.as<int32_t>(), high_idx.as<int32_t>(), n_low, n_q, opt->mid_occ,
                           opt->max_max_occ, opt->occ_dist, seed_n.as<uint32_t>(), flt_high.as<uint32_t>()};
            HY_HIP(hipMemsetAsync(flt_high.p, 0, 4 * (size_t)n_high, st));
            LAUNCH1(streak_kernel, n_low + n_q, S);
            HY_HIP(vmax.alloc(4 * (size_t)n_high, st));
            HY_HIP(pmax.alloc(4 * (size_t)n_high, st));
            LAUNCH1(flt_mark_kernel, n_high, flt_high.as<uint32_t>(), n_high, vmax.as<int32_t>());
            {
                DevBuf mpart;
                rc = inclusive_max_scan_i32(ctx, vmax.as<int32_t>(), pmax.as<int32_t>(), n_high, mpart);
                if (rc) return rc;
            }
            LAUNCH1(rep_len_kernel, n_high, flt_high.as<uint32_t>(), pmax.as<int32_t>(), high_idx.as<int32_t>(), n_high,
                    mx.as<uint64_t>(), my.as<uint64_t>(), qid.as<uint32_t>(), rep_len.as<int32_t>(), seed_n.as<uint32_t>());
        }
    }
    tr.mark("seeds");
    // ------------------------------------------------------------ 4 anchors
    DevBuf a_pos, mflag, mp_pos, mini_pos, mp_off;
    int64_t A = 0, NM = 0;
    rc = scan_flags(ctx, seed_n.as<uint32_t>(), M, a_pos, &A);
    if (rc) return rc;
    HY_HIP(mflag.alloc(4 * (size_t)(M + 1), st));
    LAUNCH1(nz_flag_kernel, M, seed_n.as<uint32_t>(), M, mflag.as<uint32_t>());
    rc = scan_flags(ctx, mflag.as<uint32_t>(), M, mp_pos, &NM);
    if (rc) return rc;
    HY_HIP(hipMemcpyAsync(a_pos.as<int64_t>() + M, &A, 8, hipMemcpyHostToDevice, st));
    HY_HIP(hipMemcpyAsync(mp_pos.as<int64_t>() + M, &NM, 8, hipMemcpyHostToDevice, st));
    HY_HIP(mini_pos.alloc(8 * (size_t)(NM + 1), st));
    HY_HIP(mp_off.alloc(8 * (size_t)(n_q + 1), st));
    hipLaunchKernelGGL(sample_off_kernel, dim3((unsigned)cdiv(n_q + 1, 256)), dim3(256), 0, st, mp_pos.as<int64_t>(),
                       qm_off.as<int64_t>(), n_q, NM, mp_off.as<int64_t>());
    HY_CHECK_LAUNCH("sample_off_kernel");
    // mm_est_err's minimizer lookup table (filled once seed_n is final, below): each query's
    // bases at a 64-aligned offset, 16 B per 64 bases
    DevBuf d_qbase, pos_tab;
    std::vector<int64_t> qbase(n_q + 1, 0);  // lives until the call returns (async H2D source)
    int64_t max_qlen = 1;
    {
        for (int q = 0; q < n_q; q++) {
            qbase[q + 1] = qbase[q] + ((h_lens[q] + 63) & ~(int64_t)63);
            max_qlen = std::max<int64_t>(max_qlen, h_lens[q]);
        }
        HY_HIP(d_qbase.alloc(8 * (size_t)(n_q + 1), st));
        HY_HIP(hipMemcpyAsync(d_qbase.p, qbase.data(), 8 * (size_t)(n_q + 1), hipMemcpyHostToDevice, st));
        const size_t n_words = (size_t)(qbase[n_q] >> 6) + 1;
        HY_HIP(pos_tab.alloc(sizeof(MiniWord) * n_words, st));
        HY_HIP(hipMemsetAsync(pos_tab.p, 0, sizeof(MiniWord) * n_words, st));
        LAUNCH1(mini_bits_kernel, M, my.as<uint64_t>(), seed_n.as<uint32_t>(), qid.as<uint32_t>(), d_qbase.as<int64_t>(), M,
                pos_tab.as<MiniWord>());
        LAUNCH1(mini_base_kernel, M, my.as<uint64_t>(), seed_n.as<uint32_t>(), qid.as<uint32_t>(), qm_off.as<int64_t>(),
                mp_pos.as<int64_t>(), d_qbase.as<int64_t>(), M, pos_tab.as<MiniWord>());
    }
    AnchorSet S1;
    HY_HIP(S1.d_off.alloc(8 * (size_t)(n_q + 1), st));
    hipLaunchKernelGGL(sample_off_kernel, dim3((unsigned)cdiv(n_q + 1, 256)), dim3(256), 0, st, a_pos.as<int64_t>(),
                       qm_off.as<int64_t>(), n_q, A, S1.d_off.as<int64_t>());
    HY_CHECK_LAUNCH("sample_off_kernel");
    const int rb = bits_for(idx->n_seq);
    const int key1_bits = bits_for(n_q) + 1 + rb;
    HY_ARG(key1_bits <= 64, "hymet_mm_map: too many queries x targets for the sort key");
    int64_t max_len = 1;
    for (int64_t l : idx->h_len) max_len = std::max(max_len, l);
    const int pb = bits_for(max_len - 1);
    // one-key anchor sort when (query, strand, rid, rpos) fits 64 bits (always, short of
    // ~2^20 queries per batch against chromosome-scale targets); else the two-key path
    const bool key_path = key1_bits + pb <= 64 && !getenv("HYMET_ANCHOR_LEGACY");
    if (key_path) {
        DevBuf key, val;
        HY_HIP(key.alloc(8 * (size_t)(A + 1), st));
        HY_HIP(val.alloc(4 * (size_t)(A + 1), st));
        AnchorKeyParams P{mx.as<uint64_t>(), my.as<uint64_t>(), seed_n.as<uint32_t>(), a_pos.as<int64_t>(),
                          qid.as<uint32_t>(), d_qlen.as<int64_t>(), idx->d_koff, idx->d_pos, M, rb, pb,
                          key.as<uint64_t>(), val.as<uint32_t>(), mp_pos.as<int64_t>(), mini_pos.as<uint64_t>()};
        {
            ProfScope _ps(ctx, "mm_anchors", (double)A * (8.0 + 12.0));  // position fetch + key/value write
            if (M > 0) {
                hipLaunchKernelGGL(write_anchor_keys_kernel, dim3((unsigned)cdiv(M, 256)), dim3(256), 0, st, P);
                HY_CHECK_LAUNCH("write_anchor_keys_kernel");
            }
        }
        rc = sort_anchor_keys(ctx, key, val, A, key1_bits + pb, rb, pb, k, S1.d_off.as<int64_t>(), n_q, max_qlen, S1);
        if (rc) return rc;
    } else {
        DevBuf x, y, k1, k2, val;
        HY_HIP(x.alloc(8 * (size_t)(A + 1), st));
        HY_HIP(y.alloc(8 * (size_t)(A + 1), st));
        HY_HIP(k1.alloc(8 * (size_t)(A + 1), st));
        HY_HIP(k2.alloc(8 * (size_t)(A + 1), st));
        HY_HIP(val.alloc(4 * (size_t)(A + 1), st));
        AnchorParams P{mx.as<uint64_t>(), my.as<uint64_t>(), seed_n.as<uint32_t>(), a_pos.as<int64_t>(), qid.as<uint32_t>(),
                       d_qlen.as<int64_t>(), idx->d_koff, idx->d_pos, M, rb, x.as<uint64_t>(), y.as<uint64_t>(),
                       k1.as<uint64_t>(), k2.as<uint64_t>(), val.as<uint32_t>(), mp_pos.as<int64_t>(), mini_pos.as<uint64_t>()};
        ProfScope _ps(ctx, "mm_anchors", (double)A * (8.0 + 36.0));  // position fetch + anchor/key writes
        LAUNCH1(write_anchors_kernel, M, P);
        // ------------------------------------------------------- 5 sort
        rc = sort_anchor_set(ctx, x, y, k1, k2, val, A, key1_bits, S1);
        if (rc) return rc;
    }
    tr.mark("anchors+sort");
    // HYMET_DUMP_ANCHORS=path (profiling, tools/chain_prof): the first call's sorted first-pass
    // anchors as (x, y) pairs with x>>32 replaced by the (query, strand, target) group ordinal;
    // HYMET_DUMP_ANCHORS2=path: the same for the long-join re-chain's anchors
    auto dump_anchors = [&](const char *path, AnchorSet &S, bool &dumped) -> int {
        if (!path || dumped || S.n == 0) return HYMET_OK;
        dumped = true;
        const char *mx = getenv("HYMET_DUMP_MAX");  // anchors to dump (default 2^24)
        const int64_t nd = std::min<int64_t>(S.n, mx ? atoll(mx) : (1 << 24));
        std::vector<uint64_t> hx(nd), hy(nd);
        std::vector<int64_t> qo(n_q + 1);
        HY_HIP(hipMemcpyAsync(hx.data(), S.ax.p, 8 * (size_t)nd, hipMemcpyDeviceToHost, st));
        HY_HIP(hipMemcpyAsync(hy.data(), S.ay.p, 8 * (size_t)nd, hipMemcpyDeviceToHost, st));
        HY_HIP(hipMemcpyAsync(qo.data(), S.d_off.p, 8 * (size_t)(n_q + 1), hipMemcpyDeviceToHost, st));
        HY_HIP(hipStreamSynchronize(st));
        if (FILE *fp = fopen(path, "wb")) {
            uint64_t gid = 0;
            int q = 0;
            std::vector<uint64_t> buf;
            buf.reserve(1 << 21);
            for (int64_t a = 0; a < nd; a++) {
                bool qs = false;  // a query's first anchor
                while (q < n_q && qo[q + 1] <= a) q++, qs = true;
                if (a && (qs || (hx[a] >> 32) != (hx[a - 1] >> 32))) gid++;
                buf.push_back(gid << 32 | (uint32_t)hx[a]);
                buf.push_back(hy[a]);
                if (buf.size() >= (1u << 21)) fwrite(buf.data(), 8, buf.size(), fp), buf.clear();
            }
            fwrite(buf.data(), 8, buf.size(), fp);
            fclose(fp);
        }
        return HYMET_OK;
    };
    static bool dumped1 = false, dumped2 = false;
    rc = dump_anchors(getenv("HYMET_DUMP_ANCHORS"), S1, dumped1);
    if (rc) return rc;
    // ------------------------------------------------ 6 chain (+ 7 long join)
    ChainSet C1;
    const bool long_join = opt->bw_long > opt->bw;
    const bool resort = getenv("HYMET_RECHAIN_SORT") != nullptr;  // tests: the re-sort path
    LeanJoin lj{d_qlen.as<int64_t>(), opt->rmq_rescue_size, opt->rmq_rescue_ratio, key_path && !resort};
    rc = chain_set(ctx, opt, pen_gap, pen_skip, opt->bw, S1, n_q, C1, long_join ? &lj : nullptr, long_join && !lj.mark_only);
    if (rc) return rc;
    tr.mark("chain_set 1");
    ChainSet *CF = &C1;
    ChainSet C2;
    AnchorSet S2;  // the long join's anchors: its chains (C2) are read in place until the regions
    DevBuf flag;  // queries re-chained by the long join (their first-pass regions are not built)
    if (long_join && C1.n_chain > 0) {
        flag.swap(lj.flag);
        // anchors of flagged queries only: their per-query offsets, built on the device (the
        // total and whether any query is flagged come back through the mailbox)
        const DevBuf &qbuf = lj.mark_only ? lj.qb2 : C1.d_qb;
        DevBuf fcnt;
        HY_HIP(fcnt.alloc(4 * (size_t)(n_q + 1), st));
        ctx->mbox_h[kMbFlag] = 0;
        LAUNCH1(flagged_len_kernel, n_q + 1, flag.as<uint32_t>(), qbuf.as<int64_t>(), n_q, fcnt.as<uint32_t>(),
                mb_dev(ctx, kMbFlag));
        int64_t A2 = 0;
        rc = scan_flags(ctx, fcnt.as<uint32_t>(), n_q + 1, S2.d_off, &A2);  // (syncs the stream)
        if (rc) return rc;
        const bool any = mb_read(ctx, kMbFlag) != 0;
        if (any) {
            if (lj.mark_only) {
                // the flagged queries' chain anchors (t == 2 from the backtrack), compacted out of
                // the first-pass set in its (key, y) order -- already the long join's sorted set
                const int64_t n1 = S1.n, nt = cdiv(n1, 4096);
                DevBuf &mark = lj.mark;
                DevBuf tcnt, toff, tlast;
                HY_HIP(tcnt.alloc(4 * (size_t)(nt + 1), st));
                HY_HIP(toff.alloc(8 * (size_t)(nt + 1), st));
                HY_HIP(tlast.alloc(8 * (size_t)(nt + 1), st));
                hipLaunchKernelGGL(mark_count_kernel, dim3((unsigned)nt), dim3(256), 0, st, mark.as<int32_t>(), n1,
                                   flag.as<uint32_t>(), S1.d_off.as<int64_t>(), n_q, tcnt.as<uint32_t>(), tlast.as<int64_t>());
                HY_CHECK_LAUNCH("mark_count_kernel");
                int64_t got = 0;
                rc = exclusive_scan_u32_i64(ctx, tcnt.as<uint32_t>(), toff.as<int64_t>(), nt, &got);
                if (rc) return rc;
                if (got != A2 || got != lj.n2) {
                    if (getenv("HYMET_DEBUG_LJ2")) {  // diagnostic: per-query marks vs chain anchors
                        std::vector<int32_t> hm(n1);
                        std::vector<int64_t> qo(n_q + 1), qb(n_q + 1);
                        std::vector<uint32_t> h_flag(n_q);
                        HY_HIP(hipMemcpy(hm.data(), mark.p, 4 * (size_t)n1, hipMemcpyDeviceToHost));
                        HY_HIP(hipMemcpy(qo.data(), S1.d_off.p, 8 * (size_t)(n_q + 1), hipMemcpyDeviceToHost));
                        HY_HIP(hipMemcpy(qb.data(), qbuf.p, 8 * (size_t)(n_q + 1), hipMemcpyDeviceToHost));
                        HY_HIP(hipMemcpy(h_flag.data(), flag.p, 4 * (size_t)n_q, hipMemcpyDeviceToHost));
                        int shown = 0;
                        for (int q = 0; q < n_q; q++) {
                            int64_t mk = 0;
                            for (int64_t a = qo[q]; a < qo[q + 1]; a++) mk += hm[a] == 2 && h_flag[q];
                            const int64_t want = qb[q + 1] - qb[q];
                            if ((h_flag[q] ? want : 0) != mk && shown++ < 10)
                                fprintf(stderr, "[lj2] q %d flag %u anchors %lld marks %lld chain anchors %lld\n", q, h_flag[q],
                                        (long long)(qo[q + 1] - qo[q]), (long long)mk, (long long)want);
                        }
                        fprintf(stderr, "[lj2] got %lld A2 %lld n2 %lld n1 %lld\n", (long long)got, (long long)A2,
                                (long long)lj.n2, (long long)n1);
                    }
                    return hymet::fail(HYMET_E_INTERNAL, "hymet_mm_map: long-join anchor count mismatch");
                }
                HY_HIP(S2.ax.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(S2.ay.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(S2.hb.alloc(head_bits_bytes(A2), st));
                HY_HIP(S2.ax32.alloc(4 * (size_t)(A2 + 1), st));
                HY_HIP(hipMemsetAsync(S2.hb.p, 0, head_bits_bytes(A2), st));
                hipLaunchKernelGGL(mark_compact_kernel, dim3((unsigned)nt), dim3(256), 0, st, mark.as<int32_t>(), n1,
                                   flag.as<uint32_t>(), S1.d_off.as<int64_t>(), n_q, toff.as<int64_t>(), tlast.as<int64_t>(),
                                   S1.ax.as<uint64_t>(), S1.ay.as<uint64_t>(), S2.ax.as<uint64_t>(), S2.ay.as<uint64_t>(),
                                   S2.hb.as<uint32_t>(), S2.ax32.as<uint32_t>());
                HY_CHECK_LAUNCH("mark_compact_kernel");
                S2.n = A2;
                S2.has_hb = S2.has_x32 = true;
                rc = dump_anchors(getenv("HYMET_DUMP_ANCHORS2"), S2, dumped2);
                if (rc) return rc;
            } else if (key_path) {
                DevBuf key, val;
                HY_HIP(key.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(val.alloc(4 * (size_t)(A2 + 1), st));
                LAUNCH1(rechain_keys_kernel, A2, C1.bx.as<uint64_t>(), C1.by.as<uint64_t>(), C1.d_qb.as<int64_t>(),
                        S2.d_off.as<int64_t>(), n_q, A2, rb, pb, key.as<uint64_t>(), val.as<uint32_t>());
                rc = sort_anchor_keys(ctx, key, val, A2, key1_bits + pb, rb, pb, k, S2.d_off.as<int64_t>(), n_q, max_qlen, S2);
                if (rc) return rc;
                rc = dump_anchors(getenv("HYMET_DUMP_ANCHORS2"), S2, dumped2);
                if (rc) return rc;
            } else {
                DevBuf x, y, k1, k2, val;
                HY_HIP(x.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(y.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(k1.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(k2.alloc(8 * (size_t)(A2 + 1), st));
                HY_HIP(val.alloc(4 * (size_t)(A2 + 1), st));
                hipLaunchKernelGGL(rechain_gather_kernel, dim3((unsigned)n_q), dim3(256), 0, st, C1.bx.as<uint64_t>(),
                                   C1.by.as<uint64_t>(), C1.d_qb.as<int64_t>(), flag.as<uint32_t>(), S2.d_off.as<int64_t>(), n_q,
                                   rb, x.as<uint64_t>(), y.as<uint64_t>(), k1.as<uint64_t>(), k2.as<uint64_t>(), val.as<uint32_t>());
                HY_CHECK_LAUNCH("rechain_gather_kernel");
                rc = sort_anchor_set(ctx, x, y, k1, k2, val, A2, key1_bits, S2);
                if (rc) return rc;
            }
            rc = chain_set(ctx, opt, pen_gap, pen_skip, opt->bw_long, S2, n_q, C2);
            if (rc) return rc;
            // merge: flagged queries take C2's chains, the others keep C1's
            CF = nullptr;
        }
    }
    tr.mark("long join");
    // -------------------------------------------------------------- 8 regions
    // region records stay in HBM: per chain set, records at the set's chain offsets + counts
    DevBuf sumk;  // per query: sum of its minimizer spans (avg_k), computed by the first call
    HY_HIP(sumk.alloc(8 * (size_t)(n_q + 1), st));
    bool sumk_done = false;
    auto run_regions = [&](ChainSet &C, DevBuf &rg, DevBuf &nr, const uint32_t *skip_q) -> int {
        const int64_t NC = C.n_chain;
        DevBuf z, wv, cov, tmp;
        HY_HIP(z.alloc(16 * (size_t)(NC + 1), st));
        HY_HIP(rg.alloc(sizeof(hymet_mm_reg) * (size_t)(NC + 1), st));
        HY_HIP(wv.alloc(4 * (size_t)(NC + 1), st));
        HY_HIP(cov.alloc(8 * (size_t)(NC + 1), st));
        HY_HIP(tmp.alloc(4 * (size_t)(NC + 1), st));
        HY_HIP(nr.alloc(4 * (size_t)n_q, st));
        return launch_regions(ctx, C.ax, C.ay, C.ids.as<int64_t>(), C.cfirst.as<int64_t>(), C.cu.as<uint64_t>(),
                              C.cboff.as<int64_t>(),
                              C.d_qc.as<int64_t>(), C.d_qb.as<int64_t>(), mini_pos.as<uint64_t>(), mp_off.as<int64_t>(),
                              d_qlen.as<int64_t>(), d_hash, rep_len.as<int32_t>(), idx->d_len, n_q, opt, k,
                              z.p, rg.as<hymet_mm_reg>(), wv.as<int32_t>(), cov.as<uint64_t>(), tmp.as<int32_t>(),
                              nr.as<int32_t>(), C.n_anchor, NC, NM, C.cq.as<uint32_t>(),
                              pos_tab.as<MiniWord>(), d_qbase.as<int64_t>(), skip_q, sumk.as<uint64_t>(),
                              std::exchange(sumk_done, true));
    };
    DevBuf rg1, nr1, rg2, nr2;
    rc = run_regions(C1, rg1, nr1, CF ? nullptr : flag.as<uint32_t>());
    if (rc) return rc;
    if (!CF) {
        rc = run_regions(C2, rg2, nr2, nullptr);
        if (rc) return rc;
    }
    // PAF order within the batch: query by query, each query's regions as selected
    DevBuf cnt, off;
    HY_HIP(cnt.alloc(4 * (size_t)(n_q + 1), st));
    const uint32_t *fl = CF ? nullptr : flag.as<uint32_t>();
    const int32_t *n2p = CF ? nr1.as<int32_t>() : nr2.as<int32_t>();
    const int64_t *qc2 = CF ? C1.d_qc.as<int64_t>() : C2.d_qc.as<int64_t>();
    const hymet_mm_reg *r2p = CF ? rg1.as<hymet_mm_reg>() : rg2.as<hymet_mm_reg>();
    LAUNCH1(reg_count_kernel, n_q, fl, nr1.as<int32_t>(), n2p, n_q, cnt.as<uint32_t>());
    int64_t N = 0;
    rc = scan_flags(ctx, cnt.as<uint32_t>(), n_q, off, &N);
    if (rc) return rc;
    HY_HIP(hipMemcpyAsync(off.as<int64_t>() + n_q, &N, 8, hipMemcpyHostToDevice, st));
    RegOut o{};
    DevBuf tmp_regs;
    if (sink.acc) {
        hymet_paf_acc *a = sink.acc;
        rc = acc_reserve(ctx, a, a->n + N);
        if (rc) return rc;
        o = RegOut{a->regs.as<hymet_mm_reg>() + a->n, a->q.as<int32_t>() + a->n, a->part.as<int32_t>() + a->n,
                   a->rl.as<int32_t>() + a->n, a->t.as<int32_t>() + a->n, sink.q_base, sink.part_id, sink.t_base};
    } else {
        HY_HIP(tmp_regs.alloc(sizeof(hymet_mm_reg) * (size_t)(N + 1), st));
        o.regs = tmp_regs.as<hymet_mm_reg>();
    }
    {
        ProfScope _ps(ctx, "mm_paf_records", (double)N * (2.0 * sizeof(hymet_mm_reg) + 16.0));
        LAUNCH1(reg_gather_kernel, n_q, fl, nr1.as<int32_t>(), n2p, C1.d_qc.as<int64_t>(), qc2, rg1.as<hymet_mm_reg>(),
                r2p, off.as<int64_t>(), rep_len.as<int32_t>(), n_q, o);
    }
    if (sink.acc) {
        sink.acc->n += N;
    } else {
        res->regs.resize(N);
        if (N) HY_HIP(hipMemcpyAsync(res->regs.data(), tmp_regs.p, sizeof(hymet_mm_reg) * (size_t)N, hipMemcpyDeviceToHost, st));
        HY_HIP(hipMemcpyAsync(res->reg_off.data(), off.p, 8 * (size_t)(n_q + 1), hipMemcpyDeviceToHost, st));
        HY_HIP(hipMemcpyAsync(res->rep_len.data(), rep_len.p, 4 * (size_t)n_q, hipMemcpyDeviceToHost, st));
    }
    // host vectors above are async copy sources/targets
    HY_HIP(hipStreamSynchronize(st));
    tr.mark("regions");
    return HYMET_OK;
}

extern "C" {

int hymet_mm_map(hymet_ctx *ctx, const hymet_mm_index *idx, const hymet_mm_opt *opt, const uint32_t *d_2b,
                 const uint32_t *d_mask, const int64_t *h_starts, const int64_t *h_lens, const uint32_t *h_name_hash,
                 int32_t n_q, hymet_mm_result **out) {
    HY_ARG(out != nullptr, "hymet_mm_map: null argument");
    MapSink sink;
    sink.res = new hymet_mm_result();
    *out = sink.res;
    return mm_map_impl(ctx, idx, opt, d_2b, d_mask, h_starts, h_lens, h_name_hash, nullptr, n_q, sink);
}

int hymet_paf_acc_create(hymet_ctx *ctx, hymet_paf_acc **out) {
    HY_ARG(ctx && out, "hymet_paf_acc_create: null argument");
    hymet_paf_acc *a = new hymet_paf_acc();
    a->device = ctx->device;
    *out = a;
    return HYMET_OK;
}

int hymet_paf_acc_reset(hymet_paf_acc *acc) {
    HY_ARG(acc, "hymet_paf_acc_reset: null argument");
    acc->n = 0;
    return HYMET_OK;
}

int hymet_paf_acc_destroy(hymet_paf_acc *acc) {
    if (acc) {
        (void)hipSetDevice(acc->device);
        delete acc;
    }
    return HYMET_OK;
}

int hymet_paf_acc_info(const hymet_paf_acc *acc, int64_t *n_lines, void **d_regs, void **d_q, void **d_part, void **d_rl,
                       void **d_t) {
    HY_ARG(acc && n_lines, "hymet_paf_acc_info: null argument");
    *n_lines = acc->n;
    if (d_regs) *d_regs = acc->regs.p;
    if (d_q) *d_q = acc->q.p;
    if (d_part) *d_part = acc->part.p;
    if (d_rl) *d_rl = acc->rl.p;
    if (d_t) *d_t = acc->t.p;
    return HYMET_OK;
}

int hymet_paf_acc_append(hymet_ctx *ctx, hymet_paf_acc *dst, const hymet_paf_acc *src, int64_t begin, int64_t end) {
    HY_ARG(ctx && dst && src && dst != src, "hymet_paf_acc_append: null or aliased argument");
    HY_ARG(begin >= 0 && end >= begin && end <= src->n, "hymet_paf_acc_append: line range outside the source");
    const int64_t m = end - begin;
    if (m == 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    int rc = acc_reserve(ctx, dst, dst->n + m);
    if (rc) return rc;
    hipStream_t st = ctx->stream;
    const int64_t d = dst->n;
    HY_HIP(hipMemcpyAsync(dst->regs.as<hymet_mm_reg>() + d, src->regs.as<hymet_mm_reg>() + begin, sizeof(hymet_mm_reg) * (size_t)m,
                          hipMemcpyDeviceToDevice, st));
    HY_HIP(hipMemcpyAsync(dst->q.as<int32_t>() + d, src->q.as<int32_t>() + begin, 4 * (size_t)m, hipMemcpyDeviceToDevice, st));
    HY_HIP(hipMemcpyAsync(dst->part.as<int32_t>() + d, src->part.as<int32_t>() + begin, 4 * (size_t)m, hipMemcpyDeviceToDevice,
                          st));
    HY_HIP(hipMemcpyAsync(dst->rl.as<int32_t>() + d, src->rl.as<int32_t>() + begin, 4 * (size_t)m, hipMemcpyDeviceToDevice, st));
    HY_HIP(hipMemcpyAsync(dst->t.as<int32_t>() + d, src->t.as<int32_t>() + begin, 4 * (size_t)m, hipMemcpyDeviceToDevice, st));
    dst->n += m;
    return HYMET_OK;
}

int hymet_paf_acc_copy(hymet_ctx *ctx, const hymet_paf_acc *acc, int32_t *h_q, int32_t *h_part, int32_t *h_t) {
    HY_ARG(ctx && acc, "hymet_paf_acc_copy: null argument");
    if (acc->n <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (h_q) HY_HIP(hipMemcpyAsync(h_q, acc->q.p, 4 * (size_t)acc->n, hipMemcpyDeviceToHost, st));
    if (h_part) HY_HIP(hipMemcpyAsync(h_part, acc->part.p, 4 * (size_t)acc->n, hipMemcpyDeviceToHost, st));
    if (h_t) HY_HIP(hipMemcpyAsync(h_t, acc->t.p, 4 * (size_t)acc->n, hipMemcpyDeviceToHost, st));
    HY_HIP(hipStreamSynchronize(st));
    return HYMET_OK;
}

int hymet_paf_acc_field(hymet_ctx *ctx, const hymet_paf_acc *acc, int field, int32_t *h_out) {
    HY_ARG(ctx && acc && h_out && field >= 0 && field < (int)(sizeof(hymet_mm_reg) / 4), "hymet_paf_acc_field: bad argument");
    if (acc->n <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    const char *src = static_cast<const char *>(acc->regs.p) + 4 * (size_t)field;
    HY_HIP(hipMemcpy2DAsync(h_out, 4, src, sizeof(hymet_mm_reg), 4, (size_t)acc->n, hipMemcpyDeviceToHost, ctx->stream));
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}

int hymet_mm_map_acc(hymet_ctx *ctx, const hymet_mm_index *idx, const hymet_mm_opt *opt, const uint32_t *d_2b,
                     const uint32_t *d_mask, const int64_t *h_starts, const int64_t *h_lens, const uint32_t *d_name_hash,
                     int32_t n_q, int32_t q_base, int32_t part_id, int32_t t_base, hymet_paf_acc *acc) {
    HY_ARG(acc && d_name_hash, "hymet_mm_map_acc: null argument");
    MapSink sink;
    sink.acc = acc;
    sink.q_base = q_base;
    sink.part_id = part_id;
    sink.t_base = t_base;
    return mm_map_impl(ctx, idx, opt, d_2b, d_mask, h_starts, h_lens, nullptr, d_name_hash, n_q, sink);
}

int hymet_mm_chain_dp(hymet_ctx *ctx, const uint64_t *h_x, const uint64_t *h_y, int64_t n, int max_dist,
                      int max_dist_inner, int bw, int max_chn_skip, int cap_rmq_size, float pen_gap, float pen_skip,
                      int32_t *h_f, int64_t *h_p) {
    HY_ARG(ctx && (n == 0 || (h_x && h_y && h_f && h_p)), "hymet_mm_chain_dp: null argument");
    HY_ARG(n >= 0 && n < INT32_MAX, "hymet_mm_chain_dp: n out of range");
    if (n == 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    DevBuf x, y, flag, gpos, gid, g_start, qfirst, skey, sidx, swork, skey2, sidx2, f, p, t;
    HY_HIP(x.alloc(8 * (size_t)n, st));
    HY_HIP(y.alloc(8 * (size_t)n, st));
    HY_HIP(hipMemcpyAsync(x.p, h_x, 8 * (size_t)n, hipMemcpyHostToDevice, st));
    HY_HIP(hipMemcpyAsync(y.p, h_y, 8 * (size_t)n, hipMemcpyHostToDevice, st));
    HY_HIP(flag.alloc(4 * (size_t)n, st));
    LAUNCH1(group_flag_x_kernel, n, x.as<uint64_t>(), n, flag.as<uint32_t>());
    int64_t G = 0;
    int rc = scan_flags(ctx, flag.as<uint32_t>(), n, gpos, &G);
    if (rc) return rc;
    HY_HIP(g_start.alloc(8 * (size_t)(G + 1), st));
    HY_HIP(gid.alloc(4 * (size_t)n, st));
    LAUNCH1(group_start_kernel, n, flag.as<uint32_t>(), gpos.as<int64_t>(), n, g_start.as<int64_t>(), gid.as<int32_t>());
    HY_HIP(hipMemcpyAsync(g_start.as<int64_t>() + G, &n, 8, hipMemcpyHostToDevice, st));
    HY_HIP(qfirst.alloc((size_t)G, st));
    DevBuf zl;
    HY_HIP(zl.alloc(32, st));
    for (DevBuf *b : {&skey, &sidx, &swork, &skey2, &sidx2}) HY_HIP(b->alloc(4 * (size_t)G, st));
    LAUNCH1(group_size_kernel, std::max<int64_t>(G, 8), g_start.as<int64_t>(), (int32_t)G, 1, skey.as<uint32_t>(),
            sidx.as<uint32_t>(), swork.as<uint32_t>(), qfirst.as<uint8_t>(), zl.as<int32_t>());
    HY_HIP(hipMemsetAsync(qfirst.p, 1, 1, st));  // one query: group 0 holds anchor 0
    uint32_t *kp = skey.as<uint32_t>(), *ka = skey2.as<uint32_t>(), *vp = sidx.as<uint32_t>(), *va = sidx2.as<uint32_t>();
    rc = sort_pairs(ctx, kp, ka, vp, va, G, 0, 16, "radix_sort_groups");
    if (rc) return rc;
    {  // the chaining kernel packs local predecessor indices in 24 bits
        DevBuf gmax;
        HY_HIP(gmax.alloc(8, st));
        LAUNCH1(max_group_kernel, 1, g_start.as<int64_t>(), (const int32_t *)vp, (int32_t)G, gmax.as<int64_t>());
        int64_t big = 0;
        HY_HIP(hipMemcpyAsync(&big, gmax.p, 8, hipMemcpyDeviceToHost, st));
        HY_HIP(hipStreamSynchronize(st));
        HY_ARG(big < (1ll << 24) - 1, "hymet_mm_chain_dp: an anchor group exceeds 2^24 anchors");
    }
    HY_HIP(f.alloc(4 * (size_t)n, st));
    HY_HIP(p.alloc(8 * (size_t)n, st));
    HY_HIP(t.alloc(4 * (size_t)n, st));
    HY_HIP(hipMemsetAsync(f.p, 0, 4 * (size_t)n, st));
    HY_HIP(hipMemsetAsync(p.p, 0xFF, 8 * (size_t)n, st));
    HY_HIP(hipMemsetAsync(t.p, 0, 4 * (size_t)n, st));
    DevBuf x32;
    HY_HIP(x32.alloc(4 * (size_t)n, st));
    LAUNCH1(x_low_kernel, n, x.as<uint64_t>(), n, x32.as<uint32_t>());
    rc = launch_chain(ctx, x32.as<int32_t>(), y.as<uint64_t>(), g_start.as<int64_t>(), qfirst.as<uint8_t>(),
                      (const int32_t *)vp, (int32_t)G, f.as<int32_t>(), p.as<int64_t>(), t.as<int32_t>(), max_dist,
                      max_dist_inner, bw, max_chn_skip, cap_rmq_size, pen_gap, pen_skip, n, G);
    if (rc) return rc;
    HY_HIP(hipMemcpyAsync(h_f, f.p, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
    HY_HIP(hipMemcpyAsync(h_p, p.p, 8 * (size_t)n, hipMemcpyDeviceToHost, st));
    HY_HIP(hipStreamSynchronize(st));
    return HYMET_OK;
}

int hymet_mm_result_size(const hymet_mm_result *res, int64_t *n_regs) {
    HY_ARG(res && n_regs, "hymet_mm_result_size: null argument");
    *n_regs = (int64_t)res->regs.size();
    return HYMET_OK;
}

int hymet_mm_result_copy(const hymet_mm_result *res, int64_t *h_off, int32_t *h_rep_len, hymet_mm_reg *h_regs) {
    HY_ARG(res, "hymet_mm_result_copy: null result");
    if (h_off) memcpy(h_off, res->reg_off.data(), 8 * (size_t)(res->n_q + 1));
    if (h_rep_len && res->n_q) memcpy(h_rep_len, res->rep_len.data(), 4 * (size_t)res->n_q);
    if (h_regs && !res->regs.empty()) memcpy(h_regs, res->regs.data(), sizeof(hymet_mm_reg) * res->regs.size());
    return HYMET_OK;
}

int hymet_mm_result_destroy(hymet_mm_result *res) {
    delete res;
    return HYMET_OK;
}

}  // extern "C"
