// Weighted-LCA classification of every query.
//
//   scripts/classification_cami.py:290-308  _process_one   (tw[tid] += cov * ref_counts[t])
//   scripts/classification_cami.py:251-288  _weighted_lca  (per rank: name weights over tw in
//                                                            insertion order, first max, conf *= best/denom)
//   scripts/classification.py:83-157        legacy: exact-match shortcut, total-weight
//                                            normalisation, first "rank:" part per lineage
//
// Host side (hymet_amd/classify.py) turns strings into integers once per distinct target /
// taxid: target -> taxid index (the reference's identifier lookup), taxid -> per-rank name
// ids.  The device then does the per-PAF-line arithmetic in double, in the reference's
// iteration order, so every confidence is bit-identical (built with -ffp-contract=off).
//
// lca_refcount_kernel: global per-target PAF line counts (atomics; an int32 histogram).
// lca_wave_kernel: one wave per query (row), lines of the query in PAF order (CSR).  The
// reference's insertion-ordered dicts (taxid -> weight, then per rank name -> weight) become
// LDS hash tables whose entries are numbered in first-appearance order; every floating-point
// sum is still taken sequentially in the reference's order (lines, then taxids, then names),
// lane-parallel only across distinct keys.  A thread per query with linear-search dicts cost
// O(lines x taxids) per query: 550 ms per step at CAMI-high, ~350 lines and ~350 distinct
// strain taxids per contig.  Rows of more than kLcaLines lines take lca_row_seq, the
// one-thread form, on global scratch sized by the line count.
#include "common.hpp"
#include "mm_common.hpp"
#include "sort.hpp"


namespace {

constexpr int kRanks = 8;

struct LcaParams {
    int mode;                    // 0 = classification_cami, 1 = classification (legacy)
    int n_q;
    const int64_t *q_off;        // n_q + 1: the query's lines in PAF order
    const int32_t *line_t;       // target index per line (-1: no target)
    const int64_t *line_blen;
    const int64_t *line_qlen;
    const uint8_t *line_exact;   // legacy: query == target and coverage >= 0.99
    const int32_t *ref_counts;   // per target
    const int32_t *t_tax;        // target -> taxid index (-1 = no mapping)
    const int32_t *tax_names;    // taxid index * 8 + rank -> name id (-1 = empty); cami
    const uint8_t *tax_in_hier;  // legacy: taxid present in the hierarchy
    int32_t *scr_tid;            // scratch per line
    double *scr_w;
    int32_t *scr_nm;
    double *scr_nw;
    int32_t *out_depth;          // chosen ranks (0 = Unknown / root), -1 = exact shortcut
    int32_t *out_names;          // n_q * 8
    double *out_conf;
    int32_t *out_tax;            // legacy exact shortcut: taxid index
};

__global__ void lca_refcount_kernel(const int32_t *line_t, int64_t n, int32_t *counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && line_t[i] >= 0) atomicAdd(&counts[line_t[i]], 1);
}

__device__ void lca_row_seq(const LcaParams &P, int q) {
    const int64_t l0 = P.q_off[q], l1 = P.q_off[q + 1];
    int32_t *tids = P.scr_tid + l0;
    double *tw = P.scr_w + l0;
    int32_t *nm = P.scr_nm + l0;
    double *nw = P.scr_nw + l0;
    int nt = 0;
    P.out_tax[q] = -1;
    if (P.mode == 1) {  // legacy exact shortcut: first exact line whose target has a taxid
        for (int64_t l = l0; l < l1; l++) {
            const int32_t t = P.line_t[l];
            if (P.line_exact[l] && t >= 0 && P.t_tax[t] >= 0) {
                const int32_t tid = P.t_tax[t];
                if (P.tax_in_hier[tid]) {
                    P.out_depth[q] = -1;
                    P.out_tax[q] = tid;
                    P.out_conf[q] = 1.0;
                    return;
                }
                break;  // classification.py:145-151: only exact_matches[0] is tried
            }
        }
    }
    bool any = false;
    double total = 0.0;
    for (int64_t l = l0; l < l1; l++) {
        const int32_t t = P.line_t[l];
        if (t < 0) continue;
        const int32_t tid = P.t_tax[t];
        if (tid < 0) continue;
        any = true;
        const int64_t ql = P.line_qlen[l];
        const double cov = ql > 0 ? (double)P.line_blen[l] / (double)ql : 0.0;
        const double w = cov * (double)P.ref_counts[t];
        int j = 0;
        while (j < nt && tids[j] != tid) j++;
        if (j == nt) {
            tids[nt] = tid;
            tw[nt] = 0.0;
            nt++;
        }
        tw[j] += w;
        total += w;
    }
    P.out_depth[q] = 0;
    P.out_conf[q] = 0.0;
    if (!any) return;
    if (P.mode == 0) {
        double tot = 0.0;  // sum(taxid_weights.values())
        for (int j = 0; j < nt; j++) tot += tw[j];
        if (!(tot > 0.0)) return;
        double conf = 1.0;
        int depth = 0;
        for (int r = 0; r < kRanks; r++) {
            int nn = 0;
            double denom = 0.0;
            for (int j = 0; j < nt; j++) {
                const int32_t name = P.tax_names[(int64_t)tids[j] * kRanks + r];
                if (name < 0) continue;  // no hierarchy row or empty name at this rank
                int e = 0;
                while (e < nn && nm[e] != name) e++;
                if (e == nn) {
                    nm[nn] = name;
                    nw[nn] = 0.0;
                    nn++;
                }
                nw[e] += tw[j];
                denom += tw[j];
            }
            if (!(denom > 0.0) || nn == 0) break;
            int b = 0;
            for (int e = 1; e < nn; e++)
                if (nw[e] > nw[b]) b = e;  // max(): first maximal item wins
            P.out_names[q * kRanks + r] = nm[b];
            conf *= nw[b] / denom;
            depth = r + 1;
        }
        P.out_depth[q] = depth;
        P.out_conf[q] = depth ? (conf < 1.0 ? conf : 1.0) : 0.0;
    } else {
        if (total == 0.0) return;
        // lineages = [(parts, w / total) for tid in tw if tid in hierarchy]
        int nl = 0;
        for (int j = 0; j < nt; j++)
            if (P.tax_in_hier[tids[j]]) nl++;
        if (nl == 0) return;
        double conf = 1.0;
        int depth = 0;
        for (int r = 0; r < kRanks; r++) {
            int nn = 0;
            for (int j = 0; j < nt; j++) {
                if (!P.tax_in_hier[tids[j]]) continue;
                const int32_t part = P.tax_names[(int64_t)tids[j] * kRanks + r];  // first "rank:" part
                if (part < 0) continue;
                const double wn = tw[j] / total;
                int e = 0;
                while (e < nn && nm[e] != part) e++;
                if (e == nn) {
                    nm[nn] = part;
                    nw[nn] = 0.0;
                    nn++;
                }
                nw[e] += wn;
            }
            if (nn == 0) break;
            int b = 0;
            for (int e = 1; e < nn; e++)
                if (nw[e] > nw[b]) b = e;
            P.out_names[q * kRanks + r] = nm[b];
            conf *= nw[b];
            depth = r + 1;
        }
        P.out_depth[q] = depth;
        P.out_conf[q] = depth ? (conf < 1.0 ? conf : 1.0) : 0.0;
    }
}

constexpr int kLcaLines = 512;            // rows of up to this many lines run in LDS
constexpr int kLcaSlots = 2 * kLcaLines;  // open-addressing slots (a power of two)

__device__ __forceinline__ double lca_rld(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}

// One 64-lane round of inserts into an insertion-ordered LDS dict: lanes with `act` look up
// `key` (>= 0); keys not seen before are numbered cnt, cnt + 1, ... in the order of their
// first occurrence `pos` (lane order within the round = the reference's iteration order).
// Returns the key's number (-1 for inactive lanes).  One wave per block: __syncthreads orders
// the LDS accesses of the round.
__device__ __forceinline__ int lca_dict_round(int32_t *skey, int32_t *sfirst, int32_t *sidx, int32_t key, int32_t pos,
                                              bool act, int &cnt) {
    const int lane = threadIdx.x;
    uint32_t h = 0;
    if (act) {
        h = ((uint32_t)key * 2654435761u) >> 22;  // 10 bits: kLcaSlots
        for (;;) {
            const int32_t cur = atomicCAS(&skey[h], -1, key);
            if (cur == -1 || cur == key) break;
            h = (h + 1) & (kLcaSlots - 1);
        }
        atomicMin(&sfirst[h], pos);
    }
    __syncthreads();
    const bool first = act && sidx[h] == -1 && sfirst[h] == pos;
    const uint64_t mf = __ballot(first);
    if (first) sidx[h] = cnt + __popcll(mf & ((1ull << lane) - 1));
    __syncthreads();
    const int idx = act ? sidx[h] : -1;
    cnt += __popcll(mf);
    return idx;
}

__device__ __forceinline__ void lca_dict_reset(int32_t *skey, int32_t *sfirst, int32_t *sidx) {
    __syncthreads();
    for (int s = threadIdx.x; s < kLcaSlots; s += 64) skey[s] = -1, sfirst[s] = INT32_MAX, sidx[s] = -1;
    __syncthreads();
}

// sums[i] for i = base + lane < n_out: the values val[k] (k in [0, n_in), ascending) whose
// idx[k] == i, added in k order from 0.0 -- the reference's `d[key] += v` over its loop
__device__ __forceinline__ double lca_sum_by(const int32_t *idx, const double *val, int n_in, int base) {
    const int lane = threadIdx.x;
    const int me = base + lane;
    double acc = 0.0;
    for (int kb = 0; kb < n_in; kb += 64) {
        const int k = kb + lane;
        const int ik = k < n_in ? idx[k] : -1;
        const double vk = k < n_in ? val[k] : 0.0;
        for (uint64_t m = __ballot(ik >= base && ik < base + 64); m; m &= m - 1) {
            const int u = __ffsll((unsigned long long)m) - 1;
            const double v = lca_rld(vk, u);
            if (__builtin_amdgcn_readlane(ik, u) == me) acc += v;
        }
    }
    return acc;
}

// first maximal (value, index) over lanes: larger value, ties -> smaller index (max() over an
// insertion-ordered dict); e < 0 = none
__device__ __forceinline__ void lca_first_max(double &v, int &e) {
    for (int d = 1; d < 64; d <<= 1) {
        const double ov = __hiloint2double(__shfl_xor(__double2hiint(v), d, 64), __shfl_xor(__double2loint(v), d, 64));
        const int oe = __shfl_xor(e, d, 64);
        if (oe >= 0 && (e < 0 || ov > v || (ov == v && oe < e))) v = ov, e = oe;
    }
}

__global__ __launch_bounds__(64) void lca_wave_kernel(LcaParams P) {
    __shared__ int32_t skey[kLcaSlots], sfirst[kLcaSlots], sidx[kLcaSlots];
    __shared__ int32_t line_j[kLcaLines], j_tid[kLcaLines], j_e[kLcaLines], e_name[kLcaLines];
    __shared__ double line_w[kLcaLines], j_w[kLcaLines];
    const int q = blockIdx.x, lane = threadIdx.x;
    const int64_t l0 = P.q_off[q], l1 = P.q_off[q + 1];
    const int m = (int)(l1 - l0);
    if (l1 - l0 > kLcaLines) {
        if (lane == 0) lca_row_seq(P, q);
        return;
    }
    if (lane == 0) P.out_tax[q] = -1;
    if (P.mode == 1) {  // legacy exact shortcut: only the first exact line with a taxid is tried
        for (int kb = 0; kb < m; kb += 64) {
            const int k = kb + lane;
            int32_t tid = -1;
            if (k < m) {
                const int32_t t = P.line_t[l0 + k];
                if (P.line_exact[l0 + k] && t >= 0) tid = P.t_tax[t];
            }
            const uint64_t mx = __ballot(tid >= 0);
            if (mx) {
                const int32_t tid0 = __builtin_amdgcn_readlane(tid, __ffsll((unsigned long long)mx) - 1);
                if (P.tax_in_hier[tid0]) {
                    if (lane == 0) P.out_depth[q] = -1, P.out_tax[q] = tid0, P.out_conf[q] = 1.0;
                    return;
                }
                break;  // classification.py:145-151
            }
        }
    }
    // taxid dict in line order: line_j = the line's taxid number, line_w its weight
    lca_dict_reset(skey, sfirst, sidx);
    int nt = 0;
    bool any = false;
    for (int kb = 0; kb < m; kb += 64) {
        const int k = kb + lane;
        int32_t t = -1, tid = -1;
        double w = 0.0;
        if (k < m) {
            t = P.line_t[l0 + k];
            if (t >= 0) tid = P.t_tax[t];
            if (tid >= 0) {
                const int64_t ql = P.line_qlen[l0 + k];
                const double cov = ql > 0 ? (double)P.line_blen[l0 + k] / (double)ql : 0.0;
                w = cov * (double)P.ref_counts[t];
            }
        }
        const bool valid = tid >= 0;
        any = any || __ballot(valid) != 0;
        const int j = lca_dict_round(skey, sfirst, sidx, tid, k, valid, nt);
        if (valid) j_tid[j] = tid;
        if (k < m) line_j[k] = j, line_w[k] = w;
    }
    if (lane == 0) P.out_depth[q] = 0, P.out_conf[q] = 0.0;
    if (!any) return;
    __syncthreads();
    for (int jb = 0; jb < nt; jb += 64) {  // tw[j] += w over the lines, in line order
        const double acc = lca_sum_by(line_j, line_w, m, jb);
        if (jb + lane < nt) j_w[jb + lane] = acc;
    }
    __syncthreads();
    double conf = 1.0;
    int depth = 0;
    if (P.mode == 0) {
        double tot = 0.0;  // sum(taxid_weights.values()), dict order
        for (int jb = 0; jb < nt; jb += 64) {
            const double v = jb + lane < nt ? j_w[jb + lane] : 0.0;
            for (int u = 0; u < min(64, nt - jb); u++) tot += lca_rld(v, u);
        }
        if (!(tot > 0.0)) return;
        for (int r = 0; r < kRanks; r++) {
            lca_dict_reset(skey, sfirst, sidx);
            int nn = 0;
            double denom = 0.0;
            for (int jb = 0; jb < nt; jb += 64) {
                const int j = jb + lane;
                const int32_t name = j < nt ? P.tax_names[(int64_t)j_tid[j] * kRanks + r] : -1;
                const bool ok = name >= 0;  // no hierarchy row or empty name at this rank: skipped
                const double wj = j < nt ? j_w[j] : 0.0;
                const int e = lca_dict_round(skey, sfirst, sidx, name, j, ok, nn);
                if (ok) e_name[e] = name;
                if (j < nt) j_e[j] = e;
                for (uint64_t mm = __ballot(ok); mm; mm &= mm - 1) denom += lca_rld(wj, __ffsll((unsigned long long)mm) - 1);
            }
            if (!(denom > 0.0) || nn == 0) break;
            __syncthreads();
            double bv = 0.0;
            int be = -1;
            for (int eb = 0; eb < nn; eb += 64) {
                const double acc = lca_sum_by(j_e, j_w, nt, eb);
                if (eb + lane < nn && (be < 0 || acc > bv)) bv = acc, be = eb + lane;
            }
            lca_first_max(bv, be);
            if (lane == 0) P.out_names[q * kRanks + r] = e_name[be];
            conf *= bv / denom;
            depth = r + 1;
        }
    } else {
        double total = 0.0;  // sum of the weights of every line with a taxid, line order
        for (int kb = 0; kb < m; kb += 64) {
            const int k = kb + lane;
            const bool v = k < m && line_j[k] >= 0;
            const double w = v ? line_w[k] : 0.0;
            for (uint64_t mm = __ballot(v); mm; mm &= mm - 1) total += lca_rld(w, __ffsll((unsigned long long)mm) - 1);
        }
        if (total == 0.0) return;
        int nl = 0;
        for (int jb = 0; jb < nt; jb += 64) {  // wn = w / total per lineage in the hierarchy
            const int j = jb + lane;
            const bool inh = j < nt && P.tax_in_hier[j_tid[j]];
            nl += __popcll(__ballot(inh));
            if (j < nt) line_w[j] = j_w[j] / total;
        }
        if (nl == 0) return;
        __syncthreads();
        for (int r = 0; r < kRanks; r++) {
            lca_dict_reset(skey, sfirst, sidx);
            int nn = 0;
            for (int jb = 0; jb < nt; jb += 64) {
                const int j = jb + lane;
                const int32_t tid = j < nt ? j_tid[j] : -1;
                const int32_t part = tid >= 0 && P.tax_in_hier[tid] ? P.tax_names[(int64_t)tid * kRanks + r] : -1;
                const bool ok = part >= 0;
                const int e = lca_dict_round(skey, sfirst, sidx, part, j, ok, nn);
                if (ok) e_name[e] = part;
                if (j < nt) j_e[j] = e;
            }
            if (nn == 0) break;
            __syncthreads();
            double bv = 0.0;
            int be = -1;
            for (int eb = 0; eb < nn; eb += 64) {
                const double acc = lca_sum_by(j_e, line_w, nt, eb);
                if (eb + lane < nn && (be < 0 || acc > bv)) bv = acc, be = eb + lane;
            }
            lca_first_max(bv, be);
            if (lane == 0) P.out_names[q * kRanks + r] = e_name[be];
            conf *= bv;
            depth = r + 1;
        }
    }
    if (lane == 0) {
        P.out_depth[q] = depth;
        P.out_conf[q] = depth ? (conf < 1.0 ? conf : 1.0) : 0.0;
    }
}

// ---------------------------------------------------------------- accumulator path
// The fused path's PAF never leaves HBM (hymet_paf_acc): rows (queries with >= 1 line) are
// ordered by first appearance = (index part of the query's first line, query index), which
// is the insertion order of classification_cami.py's query_map (:181-208, written :333-339)
// for minimap2's part-major, query-ordered output; each row's lines keep PAF order.
constexpr int32_t kNoPart = 0x7fffffff;

__global__ void acc_first_kernel(const int32_t *q, const int32_t *part, int64_t n, int32_t *first_part, uint32_t *cnt) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    atomicMin(&first_part[q[l]], part[l]);
    atomicAdd(&cnt[q[l]], 1u);
}

__global__ void acc_keys_kernel(const int32_t *first_part, int32_t n_q, uint64_t *key, int32_t *n_rows) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    const int32_t p = q < n_q ? first_part[q] : kNoPart;
    const bool none = p == kNoPart || p == 0x7f7f7f7f;
    if (q < n_q) key[q] = none ? ~0ull : ((uint64_t)(uint32_t)p << 32 | (uint32_t)q);
    const uint64_t m = __ballot(!none);  // one atomic per wave on the shared counter
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(n_rows, __popcll(m));
}

__global__ void acc_rows_kernel(const uint64_t *key, int32_t n_rows, const uint32_t *cnt, int32_t *row_q, int32_t *row_part,
                                int32_t *row_of, uint32_t *row_cnt) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const int32_t q = (int32_t)(uint32_t)key[r];
    row_q[r] = q;
    row_part[r] = (int32_t)(key[r] >> 32);
    row_of[q] = r;
    row_cnt[r] = cnt[q];
}

__global__ void acc_line_keys_kernel(const int32_t *q, int64_t n, const int32_t *row_of, uint32_t *key, uint32_t *val) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    key[l] = (uint32_t)row_of[q[l]];
    val[l] = (uint32_t)l;
}

struct AccLineParams {
    const uint32_t *perm;         // CSR position -> accumulator line
    int64_t n;
    const hymet_mm_reg *regs;
    const int32_t *q, *t;
    const int64_t *qlen;          // per query
    int mode;
    const uint8_t *qname_pool;    // legacy exact test: query name == target name
    const int64_t *qname_off;
    const uint8_t *tname_pool;
    const int64_t *tname_off;
    int32_t *line_t;
    int64_t *line_blen, *line_qlen;
    uint8_t *line_exact;
};

__global__ void acc_line_gather_kernel(AccLineParams P) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const uint32_t l = P.perm[i];
    const int32_t q = P.q[l], t = P.t[l];
    const int64_t bl = P.regs[l].blen, ql = P.qlen[q];
    P.line_t[i] = t;
    P.line_blen[i] = bl;
    P.line_qlen[i] = ql;
    uint8_t ex = 0;
    if (P.mode == 1) {  // classification.py:52-53: query_id == ref_id and coverage >= 0.99
        const int64_t a0 = P.qname_off[q], a1 = P.qname_off[q + 1], b0 = P.tname_off[t], b1 = P.tname_off[t + 1];
        bool same = a1 - a0 == b1 - b0;
        for (int64_t j = 0; same && j < a1 - a0; j++) same = P.qname_pool[a0 + j] == P.tname_pool[b0 + j];
        const double cov = ql > 0 ? (double)bl / (double)ql : 0.0;
        ex = same && cov >= 0.99;
    }
    P.line_exact[i] = ex;
}

}  // namespace

extern "C" {

int hymet_acc_ref_counts(hymet_ctx *ctx, const hymet_paf_acc *acc, int32_t *d_counts) {
    HY_ARG(ctx && acc && d_counts, "hymet_acc_ref_counts: null argument");
    if (acc->n <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    hymet::ProfScope _ps(ctx, "lca_refcount", 8.0 * (double)acc->n);
    hipLaunchKernelGGL(lca_refcount_kernel, dim3((unsigned)hymet::cdiv(acc->n, 256)), dim3(256), 0, ctx->stream,
                       acc->t.as<int32_t>(), acc->n, d_counts);
    HY_CHECK_LAUNCH("lca_refcount_kernel");
    return HYMET_OK;
}

int hymet_acc_classify(hymet_ctx *ctx, const hymet_paf_acc *acc, int mode, int32_t n_q, const int64_t *d_qlen,
                       const int32_t *d_ref_counts, const int32_t *d_t_tax, const int32_t *d_tax_names,
                       const uint8_t *d_tax_in_hier, const uint8_t *d_qname_pool, const int64_t *d_qname_off,
                       const uint8_t *d_tname_pool, const int64_t *d_tname_off, int32_t *d_row_q, int32_t *d_row_part,
                       int32_t *d_row_depth, int32_t *d_row_names, double *d_row_conf, int32_t *d_row_tax,
                       int32_t *n_rows) {
    using hymet::mm::DevBuf;
    HY_ARG(ctx && acc && n_rows && d_qlen, "hymet_acc_classify: null argument");
    HY_ARG(mode == 0 || mode == 1, "hymet_acc_classify: mode must be 0 (classification_cami) or 1 (classification)");
    HY_ARG(mode == 0 || (d_qname_pool && d_qname_off && d_tname_pool && d_tname_off),
           "hymet_acc_classify: the legacy exact-match test needs the query and target name pools");
    *n_rows = 0;
    const int64_t n = acc->n;
    if (n_q <= 0 || n <= 0) return HYMET_OK;
    HY_ARG(n < (int64_t)UINT32_MAX, "hymet_acc_classify: more than 2^32 PAF lines");
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    hymet::ProfScope _ps(ctx, "lca_rows", 40.0 * (double)n);
    DevBuf first, cnt, key, key2, nr;
    HY_HIP(first.alloc(4 * (size_t)n_q, st));
    HY_HIP(cnt.alloc(4 * (size_t)n_q, st));
    HY_HIP(key.alloc(8 * (size_t)n_q, st));
    HY_HIP(key2.alloc(8 * (size_t)n_q, st));
    HY_HIP(nr.alloc(4, st));
    HY_HIP(hipMemsetAsync(first.p, 0x7f, 4 * (size_t)n_q, st));  // 0x7f7f7f7f > any part id
    HY_HIP(hipMemsetAsync(cnt.p, 0, 4 * (size_t)n_q, st));
    HY_HIP(hipMemsetAsync(nr.p, 0, 4, st));
    const unsigned gl = (unsigned)hymet::cdiv(n, 256), gq = (unsigned)hymet::cdiv(n_q, 256);
    hipLaunchKernelGGL(acc_first_kernel, dim3(gl), dim3(256), 0, st, acc->q.as<int32_t>(), acc->part.as<int32_t>(), n,
                       first.as<int32_t>(), cnt.as<uint32_t>());
    HY_CHECK_LAUNCH("acc_first_kernel");
    // 0x7f7f7f7f marks "no line": normalise to kNoPart inside the key kernel
    hipLaunchKernelGGL(acc_keys_kernel, dim3(gq), dim3(256), 0, st, first.as<int32_t>(), n_q, key.as<uint64_t>(),
                       nr.as<int32_t>());
    HY_CHECK_LAUNCH("acc_keys_kernel");
    uint64_t *sorted_key = key.as<uint64_t>();
    {  // rows by (first part, query); the values ride along unused
        DevBuf dv, dv2;
        HY_HIP(dv.alloc(4 * (size_t)n_q, st));
        HY_HIP(dv2.alloc(4 * (size_t)n_q, st));
        uint64_t *kka = key2.as<uint64_t>();
        uint32_t *vv = dv.as<uint32_t>(), *vva = dv2.as<uint32_t>();
        const int rc = hymet::mm::radix_sort_pairs(ctx, sorted_key, kka, vv, vva, n_q, 0, 64);
        if (rc) return rc;
    }
    int32_t R = 0;
    HY_HIP(hipMemcpyAsync(&R, nr.p, 4, hipMemcpyDeviceToHost, st));
    HY_HIP(hipStreamSynchronize(st));
    *n_rows = R;
    if (R == 0) return HYMET_OK;
    DevBuf row_of, row_cnt, row_off, lk, lk2, lv, lv2, lt, lb, lq, le;
    HY_HIP(row_of.alloc(4 * (size_t)n_q, st));
    HY_HIP(row_cnt.alloc(4 * (size_t)(R + 1), st));
    HY_HIP(row_off.alloc(8 * (size_t)(R + 1), st));
    hipLaunchKernelGGL(acc_rows_kernel, dim3((unsigned)hymet::cdiv(R, 256)), dim3(256), 0, st, sorted_key, R,
                       cnt.as<uint32_t>(), d_row_q, d_row_part, row_of.as<int32_t>(), row_cnt.as<uint32_t>());
    HY_CHECK_LAUNCH("acc_rows_kernel");
    {
        DevBuf part;
        HY_HIP(hipMemsetAsync(row_cnt.as<uint32_t>() + R, 0, 4, st));
        const int rc = hymet::mm::scan_u32_i64(ctx, row_cnt.as<uint32_t>(), row_off.as<int64_t>(), R + 1, part);
        if (rc) return rc;
    }
    // lines grouped by row, PAF order kept inside a row (stable LSD sort by row)
    HY_HIP(lk.alloc(4 * (size_t)n, st));
    HY_HIP(lk2.alloc(4 * (size_t)n, st));
    HY_HIP(lv.alloc(4 * (size_t)n, st));
    HY_HIP(lv2.alloc(4 * (size_t)n, st));
    hipLaunchKernelGGL(acc_line_keys_kernel, dim3(gl), dim3(256), 0, st, acc->q.as<int32_t>(), n, row_of.as<int32_t>(),
                       lk.as<uint32_t>(), lv.as<uint32_t>());
    HY_CHECK_LAUNCH("acc_line_keys_kernel");
    int bits = 1;
    while ((1ll << bits) < R) bits++;
    uint32_t *sorted_v = lv.as<uint32_t>();
    {
        uint32_t *kk = lk.as<uint32_t>(), *kka = lk2.as<uint32_t>(), *vva = lv2.as<uint32_t>();
        const int rc = hymet::mm::radix_sort_pairs(ctx, kk, kka, sorted_v, vva, n, 0, bits);
        if (rc) return rc;
    }
    HY_HIP(lt.alloc(4 * (size_t)n, st));
    HY_HIP(lb.alloc(8 * (size_t)n, st));
    HY_HIP(lq.alloc(8 * (size_t)n, st));
    HY_HIP(le.alloc((size_t)n, st));
    AccLineParams A{sorted_v, n, acc->regs.as<hymet_mm_reg>(), acc->q.as<int32_t>(), acc->t.as<int32_t>(), d_qlen,
                    mode, d_qname_pool, d_qname_off, d_tname_pool, d_tname_off, lt.as<int32_t>(), lb.as<int64_t>(),
                    lq.as<int64_t>(), le.as<uint8_t>()};
    hipLaunchKernelGGL(acc_line_gather_kernel, dim3(gl), dim3(256), 0, st, A);
    HY_CHECK_LAUNCH("acc_line_gather_kernel");
    DevBuf s_tid, s_w, s_nm, s_nw;
    HY_HIP(s_tid.alloc(4 * (size_t)n, st));
    HY_HIP(s_w.alloc(8 * (size_t)n, st));
    HY_HIP(s_nm.alloc(4 * (size_t)n, st));
    HY_HIP(s_nw.alloc(8 * (size_t)n, st));
    HY_HIP(hipMemsetAsync(d_row_names, 0, 4 * 8 * (size_t)R, st));
    LcaParams P{mode,          R,               row_off.as<int64_t>(), lt.as<int32_t>(),   lb.as<int64_t>(),
                lq.as<int64_t>(), le.as<uint8_t>(), d_ref_counts,      d_t_tax,            d_tax_names,
                d_tax_in_hier, s_tid.as<int32_t>(), s_w.as<double>(),  s_nm.as<int32_t>(), s_nw.as<double>(),
                d_row_depth,   d_row_names,     d_row_conf,            d_row_tax};
    hipLaunchKernelGGL(lca_wave_kernel, dim3((unsigned)R), dim3(64), 0, st, P);
    HY_CHECK_LAUNCH("lca_wave_kernel");
    return HYMET_OK;
}

int hymet_lca_ref_counts(hymet_ctx *ctx, const int32_t *d_line_t, int64_t n_lines, int32_t *d_counts) {
    HY_ARG(ctx && (n_lines == 0 || (d_line_t && d_counts)), "hymet_lca_ref_counts: null argument");
    if (n_lines <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    hymet::ProfScope _ps(ctx, "lca_refcount");
    hipLaunchKernelGGL(lca_refcount_kernel, dim3((unsigned)hymet::cdiv(n_lines, 256)), dim3(256), 0, ctx->stream, d_line_t,
                       n_lines, d_counts);
    HY_CHECK_LAUNCH("lca_refcount_kernel");
    return HYMET_OK;
}

int hymet_lca(hymet_ctx *ctx, int mode, int32_t n_q, const int64_t *d_q_off, const int32_t *d_line_t,
              const int64_t *d_line_blen, const int64_t *d_line_qlen, const uint8_t *d_line_exact,
              const int32_t *d_ref_counts, const int32_t *d_t_tax, const int32_t *d_tax_names,
              const uint8_t *d_tax_in_hier, int32_t *d_scr_tid, double *d_scr_w, int32_t *d_scr_nm, double *d_scr_nw,
              int32_t *d_out_depth, int32_t *d_out_names, double *d_out_conf, int32_t *d_out_tax) {
    HY_ARG(ctx && d_q_off, "hymet_lca: null argument");
    HY_ARG(mode == 0 || mode == 1, "hymet_lca: mode must be 0 (classification_cami) or 1 (classification)");
    if (n_q <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    LcaParams P{mode,          n_q,          d_q_off,     d_line_t,    d_line_blen,   d_line_qlen, d_line_exact,
                d_ref_counts,  d_t_tax,      d_tax_names, d_tax_in_hier, d_scr_tid,   d_scr_w,     d_scr_nm,
                d_scr_nw,      d_out_depth,  d_out_names, d_out_conf,  d_out_tax};
    hymet::ProfScope _ps(ctx, "lca");
    hipLaunchKernelGGL(lca_wave_kernel, dim3((unsigned)n_q), dim3(64), 0, ctx->stream, P);
    HY_CHECK_LAUNCH("lca_wave_kernel");
    return HYMET_OK;
}

}  // extern "C"
