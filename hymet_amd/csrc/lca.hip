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
// lca_kernel: one thread per query, lines of the query in PAF order (CSR); insertion-ordered
// "dicts" are arrays in a per-query scratch slice sized by its line count.
#include "common.hpp"

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

__global__ __launch_bounds__(64) void lca_kernel(LcaParams P) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P.n_q) return;
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

}  // namespace

extern "C" {

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
    hipLaunchKernelGGL(lca_kernel, dim3((unsigned)hymet::cdiv(n_q, 64)), dim3(64), 0, ctx->stream, P);
    HY_CHECK_LAUNCH("lca_kernel");
    return HYMET_OK;
}

}  // extern "C"
