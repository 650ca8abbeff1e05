// Minimizer sketching + the direct-address minimizer index (replaces `minimap2 -I2g -d`,
// scripts/minimap2.sh:12).
//
// mm_sketch_kernel<W, WRITE>: one thread = one 512-position chunk of one sequence.  The
// thread replays minimap2's sequential robust-winnowing sketch (sketch.c mm_sketch) from
// a warm-up point w+k+16 bases before its chunk, emitting only the pushes made while it is
// inside the chunk (and the end-of-sequence flush).  After warm-up the winnowing state
// (window contents, current minimum = rightmost minimum of the window, the valid-base run)
// equals the state of a single pass over the whole sequence, so the concatenated chunk
// outputs are bit-identical to mm_sketch, push order included.  The
// window lives in registers as a shift register (W compile-time), so the oldest slot is
// index 0 and "the minimum left the window" is min_step == step - W.
// Two launches: count (WRITE=false) -> exclusive scan -> write (WRITE=true); or, for query
// batches, one write launch into fixed per-chunk slots (slot_cap entries, counted on the
// way) -> scan of the counts -> a compaction copy (the winnowing replay runs once).
//
// Index: minimizer (hash = x>>8, y) pairs are sorted by (hash, y) with the library's stable
// LSD radix sort (sort.hpp): y first (32 + bits_for(n_seq) bits), then the hash (2k bits);
// the sorted pairs are copied into idx->d_hash / idx->d_pos and laid out as a CSR over ALL
// 4^k hash values (k <= 15: 2^30+1 uint32
// offsets = 4.3 GB per index part, which MI355X's 288 GB HBM affords), so a seed lookup is
// two adjacent loads instead of a hash-table probe chain.
#include "mm_common.hpp"

#include "sort.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace hymet {
namespace mm {
namespace {

template <int W, bool WRITE>
__global__ __launch_bounds__(256) void mm_sketch_kernel(SketchParams P) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= P.n_chunks) return;
    // sequence owning chunk g: last s with chunk_off[s] <= g
    int lo = 0, hi = P.n_seq - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (P.chunk_off[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    const int s = lo;
    const int64_t L = P.seq_len[s];
    const int64_t cst = (g - P.chunk_off[s]) * kChunk;
    const int64_t cen = min(cst + kChunk, L);
    const int64_t wst = max((int64_t)0, cst - P.warm);
    const int64_t base = P.seq_start[s];
    const int k = P.k;
    const uint64_t shift1 = 2 * (k - 1), mask = (1ULL << 2 * k) - 1;
    const uint64_t ridhi = P.rid_mode ? ((uint64_t)s << 32) : 0;
    uint64_t km0 = 0, km1 = 0;
    int l = 0, kmer_span = 0;
    uint64_t bx[W], by[W];
#pragma unroll
    for (int j = 0; j < W; j++) bx[j] = by[j] = kMax64;
    uint64_t minx = kMax64, miny = kMax64;
    int64_t step = 0, min_step = -W;
    uint32_t cnt = 0;
    const int64_t out0 = WRITE ? (P.slot_cap ? g * P.slot_cap : P.out_off[g]) : 0;
    const uint32_t lim = P.slot_cap ? (uint32_t)P.slot_cap : 0xffffffffu;
    uint32_t cw = 0, mw = 0;
    auto push = [&](uint64_t x, uint64_t y) {
        if (WRITE && cnt < lim) {
            P.out_x[out0 + cnt] = x;
            P.out_y[out0 + cnt] = y;
        }
        cnt++;
    };
    for (int64_t i = wst; i < cen; ++i) {
        const int64_t pi = base + i;
        if (i == wst || (pi & 15) == 0) cw = P.w2b[pi >> 4];
        if (i == wst || (pi & 31) == 0) mw = P.wm[pi >> 5];
        const bool emit = i >= cst;
        const uint32_t c = (cw >> (2 * (pi & 15))) & 3u;
        const bool bad = (mw >> (pi & 31)) & 1u;
        uint64_t ix = kMax64, iy = kMax64;
        if (!bad) {
            kmer_span = l + 1 < k ? l + 1 : k;
            km0 = (km0 << 2 | c) & mask;
            km1 = (km1 >> 2) | (uint64_t)(3u ^ c) << shift1;
            if (km0 == km1) continue;  // symmetric k-mer: no window slot (sketch.c)
            const int z = km0 < km1 ? 0 : 1;
            ++l;
            if (l >= k && kmer_span < 256) {
                ix = hash64m(z ? km1 : km0, mask) << 8 | (uint64_t)kmer_span;
                iy = ridhi | (uint64_t)(uint32_t)i << 1 | (uint64_t)z;
            }
        } else {
            l = 0;
            kmer_span = 0;
        }
        // buf[buf_pos] = info  ==  shift the register file, newest at W-1
#pragma unroll
        for (int j = 0; j < W - 1; j++) {
            bx[j] = bx[j + 1];
            by[j] = by[j + 1];
        }
        bx[W - 1] = ix;
        by[W - 1] = iy;
        if (l == W + k - 1 && minx != kMax64 && emit) {  // first window: identical k-mers
#pragma unroll
            for (int j = 0; j < W - 1; j++)
                if (minx == bx[j] && by[j] != miny) push(bx[j], by[j]);
        }
        if (ix <= minx) {
            if (l >= W + k && minx != kMax64 && emit) push(minx, miny);
            minx = ix;
            miny = iy;
            min_step = step;
        } else if (min_step == step - W) {  // the minimum just left the window
            if (l >= W + k - 1 && minx != kMax64 && emit) push(minx, miny);
            minx = kMax64;
#pragma unroll
            for (int j = 0; j < W; j++)
                if (minx >= bx[j]) {
                    minx = bx[j];
                    miny = by[j];
                    min_step = step - (W - 1 - j);
                }
            if (l >= W + k - 1 && minx != kMax64 && emit) {
#pragma unroll
                for (int j = 0; j < W; j++)
                    if (minx == bx[j] && miny != by[j]) push(bx[j], by[j]);
            }
        }
        ++step;
    }
    if (cen == L && minx != kMax64) push(minx, miny);
    if (!WRITE || P.slot_cap) P.counts[g] = cnt;
    if (WRITE && P.slot_cap && cnt > lim) atomicOr(P.overflow, 1u);
}

// one-pass mode: chunk g's slot entries to its place in the packed output
__global__ __launch_bounds__(64) void sketch_compact_kernel(const uint64_t *sx, const uint64_t *sy, const uint32_t *cnt,
                                                            const int64_t *off, int slot_cap, uint64_t *ox, uint64_t *oy) {
    const int64_t g = blockIdx.x;
    const int64_t s0 = g * slot_cap, o = off[g];
    for (uint32_t j = threadIdx.x; j < cnt[g]; j += 64) {
        ox[o + j] = sx[s0 + j];
        oy[o + j] = sy[s0 + j];
    }
}

__global__ void bucket_hist_kernel(const uint64_t *__restrict__ x, int64_t n, uint32_t *__restrict__ cnt,
                                   uint32_t *__restrict__ hash_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = (uint32_t)(x[i] >> 8);
    hash_out[i] = h;
    atomicAdd(&cnt[h], 1u);
}

// per-key occurrence histogram: nearly every key occurs once or a few times, so small counts
// go to a block-local LDS histogram (count 1 to a per-thread register) and only the rare
// large ones to global atomics (one global counter for all of them stalled ~0.5 s on C4)
__global__ __launch_bounds__(256) void occ_hist_kernel(const uint32_t *__restrict__ koff, int64_t n_buckets, uint32_t *hist,
                                                       int cap) {
    __shared__ uint32_t sh[256];
    sh[threadIdx.x] = 0;
    __syncthreads();
    uint32_t ones = 0;
    for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n_buckets;
         h += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t c = koff[h + 1] - koff[h];
        if (c == 1) ones++;
        else if (c > 1 && c < 256) atomicAdd(&sh[c], 1u);
        else if (c >= 256) atomicAdd(&hist[c < (uint32_t)cap ? c : (uint32_t)cap], 1u);
    }
    for (int o = 32; o > 0; o >>= 1) ones += __shfl_xor(ones, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&sh[1], ones);
    __syncthreads();
    if (sh[threadIdx.x]) atomicAdd(&hist[threadIdx.x], sh[threadIdx.x]);
}

}  // namespace

int launch_sketch(hymet_ctx *ctx, int w, bool write, const SketchParams &P) {
    if (P.n_chunks <= 0) return HYMET_OK;
    ProfScope _ps(ctx, write ? "mm_sketch_write" : "mm_sketch_count", (double)P.n_chunks * (kChunk * 0.375 + 4.0));
    const dim3 grid((unsigned)cdiv(P.n_chunks, 256)), block(256);
    switch (w) {
#define HY_W(WW)                                                                                   \
    case WW:                                                                                       \
        if (write) hipLaunchKernelGGL((mm_sketch_kernel<WW, true>), grid, block, 0, ctx->stream, P); \
        else hipLaunchKernelGGL((mm_sketch_kernel<WW, false>), grid, block, 0, ctx->stream, P);    \
        break;
        HY_W(2) HY_W(3) HY_W(4) HY_W(5) HY_W(6) HY_W(7) HY_W(8) HY_W(9) HY_W(10) HY_W(11) HY_W(12)
        HY_W(13) HY_W(14) HY_W(15) HY_W(16) HY_W(17) HY_W(18) HY_W(19) HY_W(20) HY_W(24) HY_W(25) HY_W(28) HY_W(32)
#undef HY_W
    default:
        return fail(HYMET_E_ARG, "minimizer window w must be one of 2..20, 24, 25, 28, 32");
    }
    HY_CHECK_LAUNCH("mm_sketch_kernel");
    return HYMET_OK;
}

int sketch_sequences(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                     const int64_t *h_lens, int n_seq, int w, int k, int rid_mode, DevBuf &d_x, DevBuf &d_y,
                     int64_t *n_out, DevBuf *d_seq_off) {
    *n_out = 0;
    if (k < 1 || k > 28) return fail(HYMET_E_ARG, "k must be in 1..28 (minimap2)");
    std::vector<int64_t> coff(n_seq + 1, 0);
    for (int i = 0; i < n_seq; i++) coff[i + 1] = coff[i] + (h_lens[i] + kChunk - 1) / kChunk;
    const int64_t n_chunks = coff[n_seq];
    DevBuf d_starts, d_lens, d_coff, d_cnt, d_off;
    HY_HIP(d_starts.alloc(8 * (size_t)n_seq, ctx->stream));
    HY_HIP(d_lens.alloc(8 * (size_t)n_seq, ctx->stream));
    HY_HIP(d_coff.alloc(8 * (size_t)(n_seq + 1), ctx->stream));
    HY_HIP(hipMemcpyAsync(d_starts.p, h_starts, 8 * (size_t)n_seq, hipMemcpyHostToDevice, ctx->stream));
    HY_HIP(hipMemcpyAsync(d_lens.p, h_lens, 8 * (size_t)n_seq, hipMemcpyHostToDevice, ctx->stream));
    HY_HIP(hipMemcpyAsync(d_coff.p, coff.data(), 8 * (size_t)(n_seq + 1), hipMemcpyHostToDevice, ctx->stream));
    HY_HIP(d_cnt.alloc(4 * (size_t)(n_chunks + 1), ctx->stream));
    HY_HIP(d_off.alloc(8 * (size_t)(n_chunks + 1), ctx->stream));
    SketchParams P{};
    P.w2b = d_2b;
    P.wm = d_mask;
    P.seq_start = d_starts.as<int64_t>();
    P.seq_len = d_lens.as<int64_t>();
    P.chunk_off = d_coff.as<int64_t>();
    P.n_chunks = n_chunks;
    P.n_seq = n_seq;
    P.k = k;
    P.warm = w + k + 16;
    P.rid_mode = rid_mode;
    P.counts = d_cnt.as<uint32_t>();
    int64_t total = 0;
    int rc = HYMET_OK;
    // one pass into per-chunk slots when they fit a modest scratch (query batches; the index
    // build's gigabases take the two-pass path).  A chunk pushes each window minimum once, so
    // it holds at most its 512 positions plus the warm-up window's: slot_cap never overflows
    // in practice, and an overflow falls back to the two passes.
    constexpr int kSlotCap = kChunk + 64;
    bool done = false;
    if (n_chunks > 0 && (double)n_chunks * kSlotCap * 16.0 <= 2.0e9 && !getenv("HYMET_SKETCH_TWO_PASS")) {
        DevBuf sx, sy;
        HY_HIP(sx.alloc(8 * (size_t)n_chunks * kSlotCap, ctx->stream));
        HY_HIP(sy.alloc(8 * (size_t)n_chunks * kSlotCap, ctx->stream));
        HY_HIP(hipMemsetAsync(d_cnt.as<uint32_t>() + n_chunks, 0, 4, ctx->stream));
        SketchParams Q = P;
        Q.slot_cap = kSlotCap;
        Q.overflow = d_cnt.as<uint32_t>() + n_chunks;
        Q.out_x = sx.as<uint64_t>();
        Q.out_y = sy.as<uint64_t>();
        rc = launch_sketch(ctx, w, true, Q);
        if (rc) return rc;
        uint32_t ovf = 0;
        HY_HIP(hipMemcpyAsync(&ovf, Q.overflow, 4, hipMemcpyDeviceToHost, ctx->stream));
        rc = exclusive_scan_u32_i64(ctx, d_cnt.as<uint32_t>(), d_off.as<int64_t>(), n_chunks, &total);
        if (rc) return rc;
        if (!ovf) {
            HY_HIP(d_x.alloc(8 * (size_t)total, ctx->stream));
            HY_HIP(d_y.alloc(8 * (size_t)total, ctx->stream));
            hipLaunchKernelGGL(sketch_compact_kernel, dim3((unsigned)n_chunks), dim3(64), 0, ctx->stream, sx.as<uint64_t>(),
                               sy.as<uint64_t>(), d_cnt.as<uint32_t>(), d_off.as<int64_t>(), kSlotCap, d_x.as<uint64_t>(),
                               d_y.as<uint64_t>());
            HY_CHECK_LAUNCH("sketch_compact_kernel");
            done = true;
        }
    }
    if (!done) {
        rc = launch_sketch(ctx, w, false, P);
        if (rc) return rc;
        rc = exclusive_scan_u32_i64(ctx, d_cnt.as<uint32_t>(), d_off.as<int64_t>(), n_chunks, &total);
        if (rc) return rc;
        HY_HIP(d_x.alloc(8 * (size_t)total, ctx->stream));
        HY_HIP(d_y.alloc(8 * (size_t)total, ctx->stream));
        P.out_off = d_off.as<int64_t>();
        P.out_x = d_x.as<uint64_t>();
        P.out_y = d_y.as<uint64_t>();
        rc = launch_sketch(ctx, w, true, P);
        if (rc) return rc;
    }
    if (d_seq_off) {
        // per-sequence offsets = chunk offsets sampled at each sequence's first chunk
        std::vector<int64_t> so(n_seq + 1);
        std::vector<int64_t> choff(n_chunks + 1);
        if (n_chunks) HY_HIP(hipMemcpyAsync(choff.data(), d_off.p, 8 * (size_t)n_chunks, hipMemcpyDeviceToHost, ctx->stream));
        HY_HIP(hipStreamSynchronize(ctx->stream));
        choff[n_chunks] = total;
        for (int i = 0; i <= n_seq; i++) so[i] = choff[coff[i]];
        HY_HIP(d_seq_off->alloc(8 * (size_t)(n_seq + 1), ctx->stream));
        HY_HIP(hipMemcpyAsync(d_seq_off->p, so.data(), 8 * (size_t)(n_seq + 1), hipMemcpyHostToDevice, ctx->stream));
        HY_HIP(hipStreamSynchronize(ctx->stream));
    }
    *n_out = total;
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet

using namespace hymet;
using namespace hymet::mm;

extern "C" {

int hymet_mm_sketch(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                    const int64_t *h_lens, int32_t n_seq, int w, int k, int rid_mode, uint64_t *h_x, uint64_t *h_y,
                    int64_t cap, int64_t *n_out) {
    HY_ARG(ctx && d_2b && d_mask && n_out, "hymet_mm_sketch: null argument");
    HY_HIP(hipSetDevice(ctx->device));
    DevBuf dx, dy;
    int64_t n = 0;
    int rc = sketch_sequences(ctx, d_2b, d_mask, h_starts, h_lens, n_seq, w, k, rid_mode, dx, dy, &n, nullptr);
    if (rc) return rc;
    *n_out = n;
    if (n > cap) return fail(HYMET_E_CAPACITY, "hymet_mm_sketch: output capacity too small");
    if (n) {
        HY_HIP(hipMemcpyAsync(h_x, dx.p, 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
        HY_HIP(hipMemcpyAsync(h_y, dy.p, 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    }
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}

int hymet_mm_index_build(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                         const int64_t *h_lens, int32_t n_seq, int w, int k, hymet_mm_index **out) {
    HY_ARG(ctx && d_2b && d_mask && out, "hymet_mm_index_build: null argument");
    HY_ARG(k >= 1 && k <= 15, "hymet_mm_index_build: direct-address index supports k <= 15 (minimap2 default 15)");
    HY_ARG(n_seq >= 0, "hymet_mm_index_build: n_seq < 0");
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    DevBuf dx, dy;
    int64_t n = 0;
    int rc = sketch_sequences(ctx, d_2b, d_mask, h_starts, h_lens, n_seq, w, k, 1, dx, dy, &n, nullptr);
    if (rc) return rc;
    HY_ARG(n < (1ll << 32), "hymet_mm_index_build: more than 2^32 minimizers in one index part");
    const int64_t nb = 1ll << (2 * k);
    hymet_mm_index *idx = new hymet_mm_index();
    idx->w = w, idx->k = k, idx->n_seq = n_seq, idx->n_pos = n, idx->n_buckets = nb, idx->device = ctx->device;
    idx->h_len.assign(h_lens, h_lens + n_seq);
    auto cleanup = [&](int code) {
        hymet_mm_index_destroy(idx);
        return code;
    };
    if (hipMalloc(&idx->d_koff, 4 * (size_t)(nb + 1)) != hipSuccess || hipMalloc(&idx->d_pos, 8 * (size_t)(n + 1)) != hipSuccess ||
        hipMalloc(&idx->d_hash, 4 * (size_t)(n + 1)) != hipSuccess || hipMalloc(&idx->d_len, 8 * (size_t)(n_seq + 1)) != hipSuccess)
        return cleanup(fail(HYMET_E_HIP, "hymet_mm_index_build: out of device memory"));
    if (n_seq) {
        if (hipMemcpyAsync(idx->d_len, h_lens, 8 * (size_t)n_seq, hipMemcpyHostToDevice, st) != hipSuccess)
            return cleanup(fail(HYMET_E_HIP, "copy lengths"));
    }
    // bucket histogram (counts) -> CSR offsets
    DevBuf cnt, hsh, hsh2, pos2;
    if (cnt.alloc(4 * (size_t)(nb + 1), st) || hsh.alloc(4 * (size_t)(n + 1), st) || hsh2.alloc(4 * (size_t)(n + 1), st) ||
        pos2.alloc(8 * (size_t)(n + 1), st))
        return cleanup(fail(HYMET_E_HIP, "hymet_mm_index_build: out of device memory (scratch)"));
    if (hipMemsetAsync(cnt.p, 0, 4 * (size_t)(nb + 1), st)) return cleanup(fail(HYMET_E_HIP, "memset"));
    if (n) {
        hipLaunchKernelGGL(bucket_hist_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, dx.as<uint64_t>(), n,
                           cnt.as<uint32_t>(), hsh.as<uint32_t>());
        if (hipGetLastError() != hipSuccess) return cleanup(fail(HYMET_E_HIP, "bucket_hist_kernel"));
    }
    {
        DevBuf part;
        if (scan_u32(ctx, cnt.as<uint32_t>(), idx->d_koff, nb + 1, part)) return cleanup(fail(HYMET_E_HIP, "scan"));
    }
    // sort (hash, y): y first, then a stable pass on the hash (2k bits); y = seq << 32 | pos << 1 | strand
    if (n) {
        uint64_t *ky = dy.as<uint64_t>(), *kya = pos2.as<uint64_t>();
        uint32_t *vh = hsh.as<uint32_t>(), *vha = hsh2.as<uint32_t>();
        const int ybits = 32 + bits_for(n_seq);
        if (radix_sort_pairs(ctx, ky, kya, vh, vha, n, 0, std::min(64, ybits))) return cleanup(fail(HYMET_E_HIP, "sort"));
        // hashes are keys now: the sorted ones in vh; the y's ride along
        uint32_t *kh = vh, *kha = vha;
        uint64_t *vy = ky, *vya = kya;
        if (radix_sort_pairs(ctx, kh, kha, vy, vya, n, 0, 2 * k)) return cleanup(fail(HYMET_E_HIP, "sort"));
        if (hipMemcpyAsync(idx->d_hash, kh, 4 * (size_t)n, hipMemcpyDeviceToDevice, st) ||
            hipMemcpyAsync(idx->d_pos, vy, 8 * (size_t)n, hipMemcpyDeviceToDevice, st))
            return cleanup(fail(HYMET_E_HIP, "copy"));
    }
    if (hipStreamSynchronize(st) != hipSuccess) return cleanup(fail(HYMET_E_HIP, "hymet_mm_index_build: sync"));
    *out = idx;
    return HYMET_OK;
}

int hymet_mm_index_destroy(hymet_mm_index *idx) {
    if (!idx) return HYMET_OK;
    (void)hipSetDevice(idx->device);
    if (idx->d_koff) (void)hipFree(idx->d_koff);
    if (idx->d_pos) (void)hipFree(idx->d_pos);
    if (idx->d_hash) (void)hipFree(idx->d_hash);
    if (idx->d_len) (void)hipFree(idx->d_len);
    delete idx;
    return HYMET_OK;
}

int hymet_mm_index_info(const hymet_mm_index *idx, int32_t *w, int32_t *k, int32_t *n_seq, int64_t *n_pos) {
    HY_ARG(idx, "hymet_mm_index_info: null index");
    if (w) *w = idx->w;
    if (k) *k = idx->k;
    if (n_seq) *n_seq = idx->n_seq;
    if (n_pos) *n_pos = idx->n_pos;
    return HYMET_OK;
}

// index.c mm_idx_cal_max_occ: ((1-f) * n_keys)-th smallest per-key count, + 1
int hymet_mm_index_max_occ(hymet_ctx *ctx, const hymet_mm_index *idx, float frac, int32_t *out) {
    HY_ARG(ctx && idx && out, "hymet_mm_index_max_occ: null argument");
    if (frac <= 0.f) {
        *out = INT32_MAX;
        return HYMET_OK;
    }
    HY_HIP(hipSetDevice(ctx->device));
    const int cap = 1 << 20;
    DevBuf hist;
    HY_HIP(hist.alloc(4 * (size_t)(cap + 1), ctx->stream));
    HY_HIP(hipMemsetAsync(hist.p, 0, 4 * (size_t)(cap + 1), ctx->stream));
    hipLaunchKernelGGL(occ_hist_kernel, dim3(ctx->n_cu * 8), dim3(256), 0, ctx->stream, idx->d_koff, idx->n_buckets,
                       hist.as<uint32_t>(), cap);
    HY_CHECK_LAUNCH("occ_hist_kernel");
    std::vector<uint32_t> h(cap + 1);
    HY_HIP(hipMemcpyAsync(h.data(), hist.p, 4 * (size_t)(cap + 1), hipMemcpyDeviceToHost, ctx->stream));
    HY_HIP(hipStreamSynchronize(ctx->stream));
    uint64_t n_keys = 0;
    for (int c = 1; c <= cap; c++) n_keys += h[c];
    if (n_keys == 0) {
        *out = INT32_MAX;
        return HYMET_OK;
    }
    const uint64_t kk = (uint64_t)(uint32_t)((1. - frac) * (double)n_keys);
    uint64_t acc = 0;
    int val = cap;
    for (int c = 1; c <= cap; c++) {
        acc += h[c];
        if (acc > kk) {
            val = c;
            break;
        }
    }
    HY_ARG(val < cap, "hymet_mm_index_max_occ: occurrence above histogram range");
    *out = val + 1;
    return HYMET_OK;
}

// ------------------------------------------------------- persisted index (minimap2.sh:10)
// A part on disk: "HYMETIX1", int32 w, k, n_seq, pad, int64 n_pos, int64 len[n_seq],
// uint32 bucket[n_pos], uint64 pos[n_pos] (sorted by (bucket, pos) as in HBM).  The direct-
// address offsets are rebuilt on load from the sorted buckets (no sort, no sketch).
static const char kIxMagic[8] = {'H', 'Y', 'M', 'E', 'T', 'I', 'X', '1'};

int hymet_mm_index_save(hymet_ctx *ctx, const hymet_mm_index *idx, const char *path, int append, int64_t *end_offset) {
    HY_ARG(ctx && idx && path, "hymet_mm_index_save: null argument");
    HY_HIP(hipSetDevice(ctx->device));
    FILE *fp = fopen(path, append ? "ab" : "wb");
    if (!fp) return fail(HYMET_E_ARG, std::string("hymet_mm_index_save: cannot open ") + path);
    const int32_t hdr[4] = {idx->w, idx->k, idx->n_seq, 0};
    const int64_t n = idx->n_pos;
    bool ok = fwrite(kIxMagic, 1, 8, fp) == 8 && fwrite(hdr, 4, 4, fp) == 4 && fwrite(&n, 8, 1, fp) == 1 &&
              (idx->n_seq == 0 || fwrite(idx->h_len.data(), 8, (size_t)idx->n_seq, fp) == (size_t)idx->n_seq);
    const int64_t chunk = 1 << 24;
    std::vector<uint64_t> buf;
    for (int pass = 0; ok && pass < 2; pass++) {  // buckets, then positions, streamed in chunks
        const size_t es = pass == 0 ? 4 : 8;
        buf.resize((size_t)std::min<int64_t>(n, chunk) + 1);
        for (int64_t a = 0; ok && a < n; a += chunk) {
            const int64_t m = std::min<int64_t>(chunk, n - a);
            const void *src = pass == 0 ? (const void *)(idx->d_hash + a) : (const void *)(idx->d_pos + a);
            if (hipMemcpy(buf.data(), src, es * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess) {
                fclose(fp);
                return fail(HYMET_E_HIP, "hymet_mm_index_save: copy");
            }
            ok = fwrite(buf.data(), es, (size_t)m, fp) == (size_t)m;
        }
    }
    if (end_offset) *end_offset = (int64_t)ftell(fp);
    if (fclose(fp) != 0 || !ok) return fail(HYMET_E_ARG, std::string("hymet_mm_index_save: write failed: ") + path);
    return HYMET_OK;
}

__global__ void koff_gap_kernel(const uint32_t *__restrict__ hash, int64_t n, uint32_t *__restrict__ koff) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t prev = i ? (int64_t)hash[i - 1] : -1;
    for (int64_t b = prev + 1; b <= (int64_t)hash[i]; b++) koff[b] = (uint32_t)i;  // first entry of buckets (prev, h]
}

__global__ void koff_tail_kernel(int64_t from, int64_t to, uint32_t v, uint32_t *__restrict__ koff) {
    for (int64_t b = from + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= to; b += (int64_t)gridDim.x * blockDim.x)
        koff[b] = v;
}

int hymet_mm_index_load(hymet_ctx *ctx, const char *path, int64_t offset, hymet_mm_index **out, int64_t *end_offset) {
    HY_ARG(ctx && path && out, "hymet_mm_index_load: null argument");
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    FILE *fp = fopen(path, "rb");
    if (!fp) return fail(HYMET_E_ARG, std::string("hymet_mm_index_load: cannot open ") + path);
    char mg[8];
    int32_t hdr[4];
    int64_t n = 0;
    if (fseeko(fp, offset, SEEK_SET) != 0 || fread(mg, 1, 8, fp) != 8 || memcmp(mg, kIxMagic, 8) != 0 ||
        fread(hdr, 4, 4, fp) != 4 || fread(&n, 8, 1, fp) != 1 || hdr[1] < 1 || hdr[1] > 15 || hdr[2] < 0 || n < 0 ||
        n >= (1ll << 32)) {
        fclose(fp);
        return fail(HYMET_E_ARG, std::string("hymet_mm_index_load: not a hymet index part: ") + path);
    }
    hymet_mm_index *idx = new hymet_mm_index();
    idx->w = hdr[0], idx->k = hdr[1], idx->n_seq = hdr[2], idx->n_pos = n, idx->n_buckets = 1ll << (2 * hdr[1]);
    idx->device = ctx->device;
    idx->h_len.resize(idx->n_seq);
    auto bad = [&](int code, const char *what) {
        fclose(fp);
        hymet_mm_index_destroy(idx);
        return fail(code, std::string("hymet_mm_index_load: ") + what);
    };
    if (idx->n_seq && fread(idx->h_len.data(), 8, (size_t)idx->n_seq, fp) != (size_t)idx->n_seq) return bad(HYMET_E_ARG, "truncated");
    const int64_t nb = idx->n_buckets;
    if (hipMalloc(&idx->d_koff, 4 * (size_t)(nb + 1)) != hipSuccess || hipMalloc(&idx->d_pos, 8 * (size_t)(n + 1)) != hipSuccess ||
        hipMalloc(&idx->d_hash, 4 * (size_t)(n + 1)) != hipSuccess || hipMalloc(&idx->d_len, 8 * (size_t)(idx->n_seq + 1)) != hipSuccess)
        return bad(HYMET_E_HIP, "out of device memory");
    if (idx->n_seq && hipMemcpy(idx->d_len, idx->h_len.data(), 8 * (size_t)idx->n_seq, hipMemcpyHostToDevice) != hipSuccess)
        return bad(HYMET_E_HIP, "copy lengths");
    const int64_t chunk = 1 << 24;
    std::vector<uint64_t> buf((size_t)std::min<int64_t>(std::max<int64_t>(n, 1), chunk));
    for (int pass = 0; pass < 2; pass++) {
        const size_t es = pass == 0 ? 4 : 8;
        for (int64_t a = 0; a < n; a += chunk) {
            const int64_t m = std::min<int64_t>(chunk, n - a);
            if (fread(buf.data(), es, (size_t)m, fp) != (size_t)m) return bad(HYMET_E_ARG, "truncated");
            void *dst = pass == 0 ? (void *)(idx->d_hash + a) : (void *)(idx->d_pos + a);
            if (hipMemcpy(dst, buf.data(), es * (size_t)m, hipMemcpyHostToDevice) != hipSuccess) return bad(HYMET_E_HIP, "copy");
        }
    }
    if (end_offset) *end_offset = (int64_t)ftello(fp);
    fclose(fp);
    // offsets: koff[b] = first entry of bucket >= b; koff[nb] = n
    if (n > 0) {
        uint32_t last = 0;
        if (hipMemcpy(&last, idx->d_hash + n - 1, 4, hipMemcpyDeviceToHost) != hipSuccess) return bad(HYMET_E_HIP, "copy");
        hipLaunchKernelGGL(koff_gap_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, idx->d_hash, n, idx->d_koff);
        hipLaunchKernelGGL(koff_tail_kernel, dim3(ctx->n_cu * 8), dim3(256), 0, st, (int64_t)last + 1, nb, (uint32_t)n,
                           idx->d_koff);
    } else {
        hipLaunchKernelGGL(koff_tail_kernel, dim3(ctx->n_cu * 8), dim3(256), 0, st, (int64_t)0, nb, 0u, idx->d_koff);
    }
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
        hymet_mm_index_destroy(idx);
        return fail(HYMET_E_HIP, "hymet_mm_index_load: offsets kernel");
    }
    *out = idx;
    return HYMET_OK;
}

// host copies of the sorted (bucket, y) arrays, for tests
int hymet_mm_index_export(hymet_ctx *ctx, const hymet_mm_index *idx, uint32_t *h_hash, uint64_t *h_pos) {
    HY_ARG(ctx && idx && h_hash && h_pos, "hymet_mm_index_export: null argument");
    HY_HIP(hipSetDevice(ctx->device));
    if (idx->n_pos) {
        HY_HIP(hipMemcpyAsync(h_hash, idx->d_hash, 4 * (size_t)idx->n_pos, hipMemcpyDeviceToHost, ctx->stream));
        HY_HIP(hipMemcpyAsync(h_pos, idx->d_pos, 8 * (size_t)idx->n_pos, hipMemcpyDeviceToHost, ctx->stream));
    }
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}

}  // extern "C"
