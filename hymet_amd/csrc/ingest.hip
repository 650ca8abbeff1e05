// Device half of the FASTA ingest (the host half is fasta.cpp).
//
// One contiguous byte range of a FASTA file (a shard of whole records) is uploaded as is;
// these kernels turn it into the ASCII sequence pool every stage reads (records joined by one
// 'N', hymet_amd.seqio.DevicePool layout; hymet_pack then packs it per alphabet) and compute
// the khash X31 hash of every record name (map.c mm_map_frag seeds its tie-break hash with
// it).  Line breaks are dropped by a two-pass stream compaction over 8 KiB chunks of each
// record's sequence range: count kept bytes per chunk, exclusive scan, write.  HBM-bound:
// ~2 B moved per input byte.
#include "common.hpp"
#include "mm_common.hpp"


namespace {

constexpr int kChunk = 8192;   // raw bytes per chunk
constexpr int kThreads = 256;  // 32 bytes per thread

struct ChunkRef {
    int64_t raw;      // first raw byte of the chunk (relative to the uploaded range)
    int32_t len;      // raw bytes in the chunk
    int32_t rec;      // record (relative to the shard)
    int64_t first;    // index of the record's first chunk
};

__device__ __forceinline__ bool kept(uint8_t c) { return c != '\n' && c != '\r'; }

__global__ __launch_bounds__(kThreads) void chunk_count_kernel(const uint8_t *__restrict__ raw, const ChunkRef *__restrict__ ch,
                                                               int64_t n_chunks, uint32_t *__restrict__ cnt) {
    const int64_t c = blockIdx.x;
    if (c >= n_chunks) return;
    const ChunkRef r = ch[c];
    const int b = threadIdx.x * 32;
    uint32_t k = 0;
    for (int j = 0; j < 32; j++) k += (b + j < r.len) && kept(raw[r.raw + b + j]);
    __shared__ uint32_t red[kThreads / 64];
    for (int o = 32; o > 0; o >>= 1) k += __shfl_down(k, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = k;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < kThreads / 64; w++) s += red[w];
        cnt[c] = s;
    }
}

__global__ __launch_bounds__(kThreads) void chunk_write_kernel(const uint8_t *__restrict__ raw, const ChunkRef *__restrict__ ch,
                                                               int64_t n_chunks, const int64_t *__restrict__ pref,
                                                               const int64_t *__restrict__ pool_start, uint8_t *__restrict__ pool) {
    const int64_t c = blockIdx.x;
    if (c >= n_chunks) return;
    const ChunkRef r = ch[c];
    const int b = threadIdx.x * 32;
    uint8_t v[32];
    uint32_t k = 0;
    for (int j = 0; j < 32; j++) {
        v[j] = (b + j < r.len) ? raw[r.raw + b + j] : (uint8_t)'\n';
        k += kept(v[j]);
    }
    // block exclusive scan of the per-thread kept counts
    __shared__ uint32_t wsum[kThreads / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = k;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < wv; w++) base += wsum[w];
    int64_t o = pool_start[r.rec] + (pref[c] - pref[r.first]) + base + (inc - k);
    for (int j = 0; j < 32; j++)
        if (kept(v[j])) pool[o++] = v[j];
}

__global__ void separator_kernel(const int64_t *__restrict__ pool_start, const int64_t *__restrict__ nbases, int64_t n_rec,
                                 uint8_t *__restrict__ pool) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r + 1 < n_rec) pool[pool_start[r] + nbases[r]] = 'N';
}

__global__ void name_hash_kernel(const uint8_t *__restrict__ raw, const int64_t *__restrict__ name_off,
                                 const int32_t *__restrict__ name_len, int64_t n, uint32_t *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t *s = raw + name_off[r];
    const int L = name_len[r];
    uint32_t h = 0;
    if (L > 0) {  // khash __ac_X31_hash_string over signed chars
        h = (uint32_t)(int32_t)(int8_t)s[0];
        for (int i = 1; i < L; i++) h = (h << 5) - h + (uint32_t)(int32_t)(int8_t)s[i];
    }
    out[r] = h;
}

}  // namespace

using hymet::mm::DevBuf;

extern "C" int hymet_fasta_compact(hymet_ctx *ctx, const uint8_t *d_raw, int64_t raw_len, int64_t raw_base,
                                   const int64_t *h_seq_off, const int64_t *h_seq_end, const int64_t *h_nbases,
                                   int64_t n_rec, uint8_t *d_pool, int64_t pool_len, int64_t *d_pool_start) {
    HY_ARG(ctx && (n_rec == 0 || (d_raw && h_seq_off && h_seq_end && h_nbases && d_pool && d_pool_start)),
           "hymet_fasta_compact: null argument");
    if (n_rec <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    std::vector<int64_t> pstart(n_rec);
    int64_t pos = 0;
    std::vector<ChunkRef> chunks;
    chunks.reserve((size_t)(raw_len / kChunk + n_rec + 1));
    for (int64_t r = 0; r < n_rec; r++) {
        const int64_t a = h_seq_off[r] - raw_base, e = h_seq_end[r] - raw_base;
        HY_ARG(a >= 0 && e >= a && e <= raw_len, "hymet_fasta_compact: a record lies outside the uploaded range");
        pstart[r] = pos;
        pos += h_nbases[r] + 1;
        const int64_t first = (int64_t)chunks.size();
        for (int64_t b = a; b < e; b += kChunk)
            chunks.push_back({b, (int32_t)std::min<int64_t>(kChunk, e - b), (int32_t)r, first});
    }
    HY_ARG(pos - 1 == pool_len, "hymet_fasta_compact: pool_len != sum(nbases) + n_rec - 1");
    const int64_t C = (int64_t)chunks.size();
    HY_HIP(hipMemcpyAsync(d_pool_start, pstart.data(), 8 * (size_t)n_rec, hipMemcpyHostToDevice, st));
    DevBuf d_ch, d_cnt, d_pref, d_nb, tmp;
    if (C > 0) {
        hymet::ProfScope _ps(ctx, "fasta_compact", 2.0 * (double)raw_len);
        HY_HIP(d_ch.alloc(sizeof(ChunkRef) * (size_t)C, st));
        HY_HIP(d_cnt.alloc(4 * (size_t)(C + 1), st));
        HY_HIP(d_pref.alloc(8 * (size_t)(C + 1), st));
        HY_HIP(hipMemcpyAsync(d_ch.p, chunks.data(), sizeof(ChunkRef) * (size_t)C, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(chunk_count_kernel, dim3((unsigned)C), dim3(kThreads), 0, st, d_raw, d_ch.as<ChunkRef>(), C,
                           d_cnt.as<uint32_t>());
        HY_CHECK_LAUNCH("chunk_count_kernel");
        const int rc = hymet::mm::scan_u32_i64(ctx, d_cnt.as<uint32_t>(), d_pref.as<int64_t>(), C, tmp);
        if (rc) return rc;
        hipLaunchKernelGGL(chunk_write_kernel, dim3((unsigned)C), dim3(kThreads), 0, st, d_raw, d_ch.as<ChunkRef>(), C,
                           d_pref.as<int64_t>(), d_pool_start, d_pool);
        HY_CHECK_LAUNCH("chunk_write_kernel");
    }
    HY_HIP(d_nb.alloc(8 * (size_t)n_rec, st));
    HY_HIP(hipMemcpyAsync(d_nb.p, h_nbases, 8 * (size_t)n_rec, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(separator_kernel, dim3((unsigned)hymet::cdiv(n_rec, 256)), dim3(256), 0, st, d_pool_start,
                       d_nb.as<int64_t>(), n_rec, d_pool);
    HY_CHECK_LAUNCH("separator_kernel");
    // the host vectors are sources of async copies: wait before they go out of scope
    HY_HIP(hipStreamSynchronize(st));
    return HYMET_OK;
}

extern "C" int hymet_name_hash(hymet_ctx *ctx, const uint8_t *d_raw, const int64_t *d_name_off, const int32_t *d_name_len,
                               int64_t n, uint32_t *d_hash) {
    HY_ARG(ctx && (n == 0 || (d_raw && d_name_off && d_name_len && d_hash)), "hymet_name_hash: null argument");
    if (n <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(name_hash_kernel, dim3((unsigned)hymet::cdiv(n, 256)), dim3(256), 0, ctx->stream, d_raw, d_name_off,
                       d_name_len, n, d_hash);
    HY_CHECK_LAUNCH("name_hash_kernel");
    return HYMET_OK;
}
