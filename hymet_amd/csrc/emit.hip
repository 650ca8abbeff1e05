// Text output of the fused path, written in HBM and copied out once:
//
//   * resultados.paf lines (minimap2 format.c mm_write_paf3 + write_tags, no CIGAR: the
//     reference maps without -c, scripts/minimap2.sh:23) from a hymet_paf_acc;
//   * classified_sequences.tsv rows (classification_cami.py:333-339 / classification.py
//     main_process: csv.writer, tab-delimited, minimal quoting, CRLF, "%.4f" confidences)
//     from the device LCA rows.
//
// Two passes over the records (byte length per record, exclusive scan, write), one thread
// per record.  Numbers are formatted exactly: decimal integers, and "%.4f" by correctly
// rounded fixed-point conversion of the double's binary value (round half to even, as glibc
// printf and Python's float formatting do), using 128-bit integer arithmetic.
#include "common.hpp"
#include "mm_common.hpp"


namespace {

struct Out {
    char *p;
    int64_t n;
    __device__ __forceinline__ void put(char c) {
        if (p) p[n] = c;
        n++;
    }
    __device__ __forceinline__ void puts(const char *s) {
        while (*s) put(*s++);
    }
    __device__ __forceinline__ void span(const uint8_t *s, int64_t len) {
        for (int64_t i = 0; i < len; i++) put((char)s[i]);
    }
};

__device__ void put_i64(Out &o, int64_t v) {
    char buf[24];
    int n = 0;
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do {
        buf[n++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (v < 0) o.put('-');
    while (n) o.put(buf[--n]);
}

// "%.4f" of v (finite), correctly rounded with ties to even
__device__ void put_fixed4(Out &o, double v) {
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    if (bits >> 63) o.put('-');
    const int ex = (int)((bits >> 52) & 0x7ff);
    const uint64_t man = bits & ((1ull << 52) - 1);
    uint64_t N = 0;  // round(|v| * 10^4)
    if (ex != 0) {
        const uint64_t m = man | (1ull << 52);
        const int e = ex - 1075;  // |v| = m * 2^e
        const unsigned __int128 P = (unsigned __int128)m * 10000u;
        if (e >= 0) {
            N = (uint64_t)(P << e);  // |v| >= 2^52: not produced by this path's values
        } else if (-e < 127) {
            const int sh = -e;
            const unsigned __int128 q = P >> sh, rem = P - (q << sh), half = (unsigned __int128)1 << (sh - 1);
            N = (uint64_t)q;
            if (rem > half || (rem == half && (N & 1))) N++;
        }
    }  // subnormals and zero round to 0
    put_i64(o, (int64_t)(N / 10000));
    o.put('.');
    const uint32_t f = (uint32_t)(N % 10000);
    o.put((char)('0' + f / 1000));
    o.put((char)('0' + f / 100 % 10));
    o.put((char)('0' + f / 10 % 10));
    o.put((char)('0' + f % 10));
}

// ------------------------------------------------------------------------------ PAF
struct PafParams {
    int64_t n;
    const hymet_mm_reg *regs;
    const int32_t *q, *rl, *t;
    const uint8_t *qname;      // pool of query names, qname_off[q]..qname_off[q+1]
    const int64_t *qname_off;
    const int64_t *qlen;
    const uint8_t *tname;
    const int64_t *tname_off;
    const int64_t *tlen;
    const int64_t *line_off;   // write pass
    char *out;
};

__device__ int64_t paf_line(const PafParams &P, int64_t l, char *dst) {
    Out o{dst, 0};
    const hymet_mm_reg r = P.regs[l];
    const int32_t q = P.q[l], t = P.t[l];
    const bool prim = r.id == r.parent;
    o.span(P.qname + P.qname_off[q], P.qname_off[q + 1] - P.qname_off[q]);
    o.put('\t');
    put_i64(o, P.qlen[q]);
    o.put('\t');
    put_i64(o, r.qs);
    o.put('\t');
    put_i64(o, r.qe);
    o.put('\t');
    o.put(r.rev ? '-' : '+');
    o.put('\t');
    o.span(P.tname + P.tname_off[t], P.tname_off[t + 1] - P.tname_off[t]);
    o.put('\t');
    put_i64(o, P.tlen[t]);
    o.put('\t');
    put_i64(o, r.rs);
    o.put('\t');
    put_i64(o, r.re);
    o.put('\t');
    put_i64(o, r.mlen);
    o.put('\t');
    put_i64(o, r.blen);
    o.put('\t');
    put_i64(o, r.mapq);
    o.puts(prim ? "\ttp:A:P\tcm:i:" : "\ttp:A:S\tcm:i:");
    put_i64(o, r.cnt);
    o.puts("\ts1:i:");
    put_i64(o, r.score);
    if (prim) {
        o.puts("\ts2:i:");
        put_i64(o, r.subsc);
    }
    const float d = r.div;
    if (d >= 0.0f && d <= 1.0f) {
        o.puts("\tdv:f:");
        if (d == 0.0f) o.put('0');
        else put_fixed4(o, (double)d);
    }
    o.puts("\trl:i:");
    put_i64(o, P.rl[l]);
    o.put('\n');
    return o.n;
}

__global__ void paf_len_kernel(PafParams P, uint32_t *len) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l < P.n) len[l] = (uint32_t)paf_line(P, l, nullptr);
}

__global__ void paf_write_kernel(PafParams P) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l < P.n) paf_line(P, l, P.out + P.line_off[l]);
}

// ------------------------------------------------------------------------------ TSV
__constant__ char kRank[8][13] = {"superkingdom", "phylum", "class", "order", "family", "genus", "species", "strain"};

struct TsvParams {
    int mode;  // 0 classification_cami, 1 classification (legacy)
    int32_t n;
    const int32_t *row_q, *row_depth, *row_names, *row_tax;
    const double *row_conf;
    const uint8_t *qname;
    const int64_t *qname_off;
    const uint8_t *label;      // label pool (CAMI: names; legacy: raw "rank:..." parts)
    const int64_t *label_off;
    const uint8_t *taxlin;     // legacy exact shortcut: per taxid, raw lineage / level strings
    const int64_t *taxlin_off;
    const uint8_t *taxlvl;
    const int64_t *taxlvl_off;
    const int64_t *row_off;
    char *out;
};

__device__ __forceinline__ bool special(uint8_t c) { return c == '\t' || c == '"' || c == '\r' || c == '\n'; }

// csv QUOTE_MINIMAL: quote a field holding the delimiter, the quote char or a line break;
// inside quotes '"' doubles.  `each(f)` feeds the field's bytes to f.
template <typename Each>
__device__ void csv_field(Out &o, Each each) {
    bool q = false;
    each([&](uint8_t c) { q |= special(c); });
    if (!q) {
        each([&](uint8_t c) { o.put((char)c); });
        return;
    }
    o.put('"');
    each([&](uint8_t c) {
        if (c == '"') o.put('"');
        o.put((char)c);
    });
    o.put('"');
}

__device__ int64_t tsv_row(const TsvParams &P, int32_t r, char *dst) {
    Out o{dst, 0};
    const int32_t q = P.row_q[r], d = P.row_depth[r];
    const int64_t a0 = P.qname_off[q], a1 = P.qname_off[q + 1];
    csv_field(o, [&](auto f) {
        for (int64_t i = a0; i < a1; i++) f(P.qname[i]);
    });
    o.put('\t');
    double conf = P.row_conf[r];
    if (d == 0) {
        o.puts("Unknown\troot\t");
        conf = 0.0;
    } else if (d < 0) {  // legacy exact shortcut: the taxid's raw lineage and its level
        const int32_t tx = P.row_tax[r];
        csv_field(o, [&](auto f) {
            for (int64_t i = P.taxlin_off[tx]; i < P.taxlin_off[tx + 1]; i++) f(P.taxlin[i]);
        });
        o.put('\t');
        csv_field(o, [&](auto f) {
            for (int64_t i = P.taxlvl_off[tx]; i < P.taxlvl_off[tx + 1]; i++) f(P.taxlvl[i]);
        });
        o.put('\t');
        conf = 1.0;
    } else {
        const int32_t *nm = P.row_names + (int64_t)r * 8;
        const int mode = P.mode;
        csv_field(o, [&](auto f) {
            for (int i = 0; i < d; i++) {
                if (i) {
                    f(';');
                    if (mode == 0) f(' ');
                }
                if (mode == 0) {  // "rank:name" joined by "; " (classification_cami.py:286)
                    for (const char *s = kRank[i]; *s; s++) f((uint8_t)*s);
                    f(':');
                }
                for (int64_t j = P.label_off[nm[i]]; j < P.label_off[nm[i] + 1]; j++) f(P.label[j]);
            }
        });
        o.put('\t');
        o.puts(kRank[d - 1]);  // deepest rank (legacy: determine_taxonomic_level of rank:-parts)
        o.put('\t');
    }
    put_fixed4(o, conf);
    o.put('\r');
    o.put('\n');
    return o.n;
}

__global__ void tsv_len_kernel(TsvParams P, uint32_t *len) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < P.n) len[r] = (uint32_t)tsv_row(P, r, nullptr);
}

__global__ void tsv_write_kernel(TsvParams P) {
    const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < P.n) tsv_row(P, r, P.out + P.row_off[r]);
}

// exclusive scan of per-record lengths into offsets (n + 1 entries); total on the host
int scan_lengths(hymet_ctx *ctx, hymet::mm::DevBuf &len, int64_t n, hymet::mm::DevBuf &off, int64_t *total) {
    hipStream_t st = ctx->stream;
    HY_HIP(off.alloc(8 * (size_t)(n + 1), st));
    HY_HIP(hipMemsetAsync(len.as<uint32_t>() + n, 0, 4, st));
    hymet::mm::DevBuf tmp;
    const int rc = hymet::mm::scan_u32_i64(ctx, len.as<uint32_t>(), off.as<int64_t>(), n + 1, tmp);
    if (rc) return rc;
    HY_HIP(hipMemcpyAsync(total, off.as<int64_t>() + n, 8, hipMemcpyDeviceToHost, st));
    HY_HIP(hipStreamSynchronize(st));
    return HYMET_OK;
}

}  // namespace

using hymet::mm::DevBuf;

extern "C" {

int hymet_emit_paf(hymet_ctx *ctx, const hymet_paf_acc *acc, const uint8_t *d_qname, const int64_t *d_qname_off,
                   const int64_t *d_qlen, const uint8_t *d_tname, const int64_t *d_tname_off, const int64_t *d_tlen,
                   char *d_out, int64_t cap, int64_t *n_bytes, int64_t *d_line_off) {
    HY_ARG(ctx && acc && n_bytes, "hymet_emit_paf: null argument");
    *n_bytes = 0;
    const int64_t n = acc->n;
    if (n <= 0) return HYMET_OK;
    HY_ARG(d_qname && d_qname_off && d_qlen && d_tname && d_tname_off && d_tlen, "hymet_emit_paf: null name/length table");
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    DevBuf len, off;
    HY_HIP(len.alloc(4 * (size_t)(n + 1), st));
    PafParams P{n, acc->regs.as<hymet_mm_reg>(), acc->q.as<int32_t>(), acc->rl.as<int32_t>(), acc->t.as<int32_t>(),
                d_qname, d_qname_off, d_qlen, d_tname, d_tname_off, d_tlen, nullptr, nullptr};
    const unsigned g = (unsigned)hymet::cdiv(n, 256);
    int64_t total = 0;
    {
        hymet::ProfScope _ps(ctx, "emit_paf_len", 104.0 * (double)n);
        hipLaunchKernelGGL(paf_len_kernel, dim3(g), dim3(256), 0, st, P, len.as<uint32_t>());
        HY_CHECK_LAUNCH("paf_len_kernel");
        int rc = scan_lengths(ctx, len, n, off, &total);
        if (rc) return rc;
    }
    *n_bytes = total;
    if (total > cap) return hymet::fail(HYMET_E_CAPACITY, "hymet_emit_paf: output buffer too small");
    HY_ARG(d_out, "hymet_emit_paf: null output");
    P.line_off = off.as<int64_t>();
    P.out = d_out;
    {
        hymet::ProfScope _ps(ctx, "emit_paf", 104.0 * (double)n + (double)total);
        hipLaunchKernelGGL(paf_write_kernel, dim3(g), dim3(256), 0, st, P);
        HY_CHECK_LAUNCH("paf_write_kernel");
    }
    if (d_line_off) HY_HIP(hipMemcpyAsync(d_line_off, off.p, 8 * (size_t)(n + 1), hipMemcpyDeviceToDevice, st));
    HY_HIP(hipStreamSynchronize(st));
    return HYMET_OK;
}

int hymet_emit_tsv(hymet_ctx *ctx, int mode, int32_t n_rows, const int32_t *d_row_q, const int32_t *d_row_depth,
                   const int32_t *d_row_names, const double *d_row_conf, const int32_t *d_row_tax, const uint8_t *d_qname,
                   const int64_t *d_qname_off, const uint8_t *d_label, const int64_t *d_label_off, const uint8_t *d_taxlin,
                   const int64_t *d_taxlin_off, const uint8_t *d_taxlvl, const int64_t *d_taxlvl_off, char *d_out,
                   int64_t cap, int64_t *n_bytes) {
    HY_ARG(ctx && n_bytes, "hymet_emit_tsv: null argument");
    HY_ARG(mode == 0 || mode == 1, "hymet_emit_tsv: mode must be 0 or 1");
    *n_bytes = 0;
    if (n_rows <= 0) return HYMET_OK;
    HY_ARG(d_row_q && d_row_depth && d_row_names && d_row_conf && d_row_tax && d_qname && d_qname_off && d_label &&
               d_label_off, "hymet_emit_tsv: null row table");
    HY_ARG(mode == 0 || (d_taxlin && d_taxlin_off && d_taxlvl && d_taxlvl_off), "hymet_emit_tsv: legacy needs taxid strings");
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    DevBuf len, off;
    HY_HIP(len.alloc(4 * (size_t)(n_rows + 1), st));
    TsvParams P{mode,    n_rows,  d_row_q,  d_row_depth,  d_row_names, d_row_tax,   d_row_conf, d_qname,
                d_qname_off, d_label, d_label_off, d_taxlin, d_taxlin_off, d_taxlvl, d_taxlvl_off, nullptr, nullptr};
    const unsigned g = (unsigned)hymet::cdiv(n_rows, 256);
    int64_t total = 0;
    hymet::ProfScope _ps(ctx, "emit_tsv", 64.0 * (double)n_rows);
    hipLaunchKernelGGL(tsv_len_kernel, dim3(g), dim3(256), 0, st, P, len.as<uint32_t>());
    HY_CHECK_LAUNCH("tsv_len_kernel");
    int rc = scan_lengths(ctx, len, n_rows, off, &total);
    if (rc) return rc;
    *n_bytes = total;
    if (total > cap) return hymet::fail(HYMET_E_CAPACITY, "hymet_emit_tsv: output buffer too small");
    HY_ARG(d_out, "hymet_emit_tsv: null output");
    P.row_off = off.as<int64_t>();
    P.out = d_out;
    hipLaunchKernelGGL(tsv_write_kernel, dim3(g), dim3(256), 0, st, P);
    HY_CHECK_LAUNCH("tsv_write_kernel");
    HY_HIP(hipStreamSynchronize(st));
    return HYMET_OK;
}

}  // extern "C"
