// Shared device/host helpers for the minimizer index and mapper (minimap2 restatement).
#pragma once
#include "common.hpp"

#include <cstring>
#include <vector>

namespace hymet {
namespace mm {

constexpr uint64_t kMax64 = ~0ull;
constexpr int kChunk = 512;  // sequence positions per sketch thread

// sketch.c hash64: invertible integer hash restricted to 2k bits
__host__ __device__ __forceinline__ uint64_t hash64m(uint64_t key, uint64_t mask) {
    key = (~key + (key << 21)) & mask;
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8)) & mask;
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4)) & mask;
    key = key ^ key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}
// hit.c hash64 (Thomas Wang, full 64 bits)
__host__ __device__ __forceinline__ uint64_t hash64(uint64_t key) {
    key = (~key + (key << 21));
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8));
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4));
    key = key ^ key >> 28;
    key = (key + (key << 31));
    return key;
}

// Device scratch from the library's caching allocator (hymet::scratch_alloc), returned to the
// cache at scope exit.  The cache is per stream and all work of a context runs on its one
// stream, so a block handed back while kernels that use it are still queued can be reissued
// at once: the next user is queued behind them.
// mm_est_err's get_mini_idx as a table lookup: per 64 query bases (each query's range padded
// to a multiple of 64), a bit per base where a seeded minimizer starts and the query-relative
// index of the word's first such minimizer; index(x) = base + popcount(bits below x).  16 B per
// 64 bases (a dense int32 per base was 4 B per base: 240 MB per 60 Mbp batch, a memset and a
// gather over ~20 cache lines per wave of chain anchors)
struct MiniWord {
    uint64_t bits;
    uint32_t base;
    uint32_t pad;
};
__device__ __forceinline__ int32_t mini_word_idx(const MiniWord &e, int32_t x) {
    const uint64_t below = (1ull << (x & 63)) - 1;
    return (e.bits >> (x & 63) & 1) ? (int32_t)(e.base + (uint32_t)__popcll(e.bits & below)) : -1;
}

struct DevBuf {
    void *p = nullptr;
    size_t n = 0, cls = 0;
    hipStream_t st = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    hipError_t alloc(size_t bytes, hipStream_t stream) {
        release();
        n = bytes;
        st = stream;
        return scratch_alloc(bytes == 0 ? 16 : bytes, stream, &p, &cls);
    }
    void release() {
        if (p) scratch_free(p, st, cls);
        p = nullptr;
        n = 0;
    }
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
    // exchange whole buffers: the size class travels with the pointer (the scratch cache
    // files a block under its class when it is released)
    void swap(DevBuf &o) {
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(cls, o.cls);
        std::swap(st, o.st);
    }
};

struct SketchParams {
    const uint32_t *w2b;
    const uint32_t *wm;
    const int64_t *seq_start;  // pool offset of every sequence
    const int64_t *seq_len;
    const int64_t *chunk_off;  // n_seq + 1: first chunk of every sequence
    int64_t n_chunks;
    int n_seq;
    int k;
    int warm;
    int rid_mode;  // 0: rid = 0 (queries) ; 1: rid = sequence index (index build)
    uint32_t *counts;          // per chunk (count pass)
    const int64_t *out_off;    // per chunk (write pass)
    uint64_t *out_x;
    uint64_t *out_y;
    int slot_cap;              // > 0: one-pass mode -- chunk g writes at g * slot_cap and its count
    uint32_t *overflow;        // one-pass mode: set when a chunk exceeds slot_cap
};

// Count (WRITE=false) or emit (WRITE=true) the minimizers of every chunk; defined in
// mm_sketch.hip and used by the index builder and the mapper.
int launch_sketch(hymet_ctx *ctx, int w, bool write, const SketchParams &P);

// exclusive scan of n uint32 counts into int64 offsets (scan.hip); returns the total through
// *total (synchronises the stream)
int exclusive_scan_u32_i64(hymet_ctx *ctx, const uint32_t *in, int64_t *out, int64_t n, int64_t *total);
// the same, asynchronous: `part` (scratch, kept alive by the caller) ends with the total at
// index ceil(n / 4096)
int scan_u32_i64(hymet_ctx *ctx, const uint32_t *in, int64_t *out, int64_t n, DevBuf &part, int64_t *mail = nullptr);
// exclusive scan of n uint64 values (asynchronous; part ends with the total at ceil(n / 4096))
// mailbox words (hymet_ctx::mbox_h) by use; each is read right after the sync that follows
// the kernel storing it, so uses that never overlap may share a word
enum : int { kMbScan = 0, kMbGmax = 1, kMbZBig = 2, kMbZBigTotal = 3, kMbFlag = 4, kMbRegBig = 5, kMbRegBig2 = 6, kMbQClass = 8,
             kMbGroups = 20, kMbGClass = 24 };
// self-clearing device counters (hymet_ctx::dctr): counters at [base, base + n), ticket at base + n
enum : int { kCtrQClass = 0, kCtrGroups = 16, kCtrGClass = 24, kCtrScan = 40, kCtrMaxScan = 41, kCtrRegBig = 42, kCtrRegBig2 = 44 };

// Called by every thread of every block after the block's last update of cnt[0, n): the last
// block to arrive stores the totals into the mailbox words mail[0, n) and zeroes the counters
// and the ticket, leaving them ready for the next launch (no memset, no copy back).
__device__ __forceinline__ void publish_counters(int32_t *cnt, int n, int64_t *mail) {
    __shared__ bool last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(reinterpret_cast<uint32_t *>(cnt + n), 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    if ((int)threadIdx.x < n) mail[threadIdx.x] = atomicExch(cnt + threadIdx.x, 0);
    if (threadIdx.x == 0) atomicExch(cnt + n, 0);
}

// bits needed to hold v (at least 1)
inline int bits_for(int64_t v) {
    int b = 0;
    while (b < 63 && (1ll << b) <= v) b++;
    return b < 1 ? 1 : b;
}
// exclusive scan of uint32 counts into uint32 offsets (totals below 2^32)
int scan_u32(hymet_ctx *ctx, const uint32_t *in, uint32_t *out, int64_t n, DevBuf &part, int64_t *mail = nullptr);
int scan_u64(hymet_ctx *ctx, const uint64_t *in, uint64_t *out, int64_t n, DevBuf &part, int64_t *mail = nullptr);
// inclusive running maximum of n int32 values (asynchronous)
int inclusive_max_scan_i32(hymet_ctx *ctx, const int32_t *in, int32_t *out, int64_t n, DevBuf &part);

// Per-query grouped sort of anchor keys (mm_asort.hip): key/val (n, query-major, query offsets
// d_qoff[n_q + 1]) into the sorted anchor set okey (k1) / ax / ay (oval: scratch).  Returns 1
// with nothing written where it does not apply (the caller's device sort then runs).
// t (the backtrack's marks, zero before it runs) cleared by a fill of every anchor in chain_set
// (0), or by the chaining kernels as each anchor is decided (1: the extra store per anchor made
// the first-pass wave kernel ~3 % slower on the C4 dump, 6.65-6.81 vs 6.84-7.11 ms, while the
// fill overlaps the other mapping stream's kernels; profiles/r06_tzero/)
#ifndef HYMET_CHAIN_TZERO
#define HYMET_CHAIN_TZERO 0
#endif

// hb: the set's group-head bitmap (head_bits_bytes(n); AnchorOut::head); ax32: x's low words.
int grouped_anchor_sort(hymet_ctx *ctx, const uint64_t *key, const uint32_t *val, int64_t n, const int64_t *d_qoff, int n_q,
                        int rb, int pb, uint64_t yhi, int64_t max_qlen, uint64_t *okey, uint32_t *oval, uint64_t *ax,
                        uint64_t *ay, uint32_t *hb, uint32_t *ax32);
// bytes of an anchor set's group-head bitmap: one bit per anchor, in whole 64-bit words (the
// group kernels read two words per thread)
inline size_t head_bits_bytes(int64_t n) { return 8 * (size_t)((n + 63) / 64 + 1); }

// Minimizers of a packed set of sequences: host-side chunk bookkeeping + both passes.
// On success d_x / d_y hold *n_out minimizers in sequence order (sequence-major); if
// d_seq_off is non-null it receives n_seq+1 per-sequence offsets (device, int64).
int sketch_sequences(hymet_ctx *ctx, const uint32_t *d_2b, const uint32_t *d_mask, const int64_t *h_starts,
                     const int64_t *h_lens, int n_seq, int w, int k, int rid_mode, DevBuf &d_x, DevBuf &d_y,
                     int64_t *n_out, DevBuf *d_seq_off);

}  // namespace mm
}  // namespace hymet

// opaque index handle (include/hymet_gpu.h)
struct hymet_mm_index {
    int w = 10, k = 15, n_seq = 0;
    int64_t n_pos = 0;
    int64_t n_buckets = 0;   // 4^k direct-address buckets
    uint32_t *d_koff = nullptr;   // n_buckets + 1 offsets into d_pos
    uint64_t *d_pos = nullptr;    // y = rid<<32 | pos<<1 | strand, sorted per bucket
    uint32_t *d_hash = nullptr;   // bucket of every d_pos entry (kept for export / stats)
    int64_t *d_len = nullptr;     // sequence lengths
    std::vector<int64_t> h_len;
    int device = 0;
};

// Device-resident PAF lines of a whole run (include/hymet_gpu.h hymet_paf_acc): every
// hymet_mm_map_acc call appends its batch's lines, so the buffer holds resultados.paf's
// lines in minimap2's order (index part by part, queries in input order, regions by score)
// as records -- the classifier and the PAF text writer read them in place.
struct hymet_paf_acc {
    int device = 0;
    int64_t n = 0, cap = 0;
    hymet::mm::DevBuf regs;  // hymet_mm_reg per line
    hymet::mm::DevBuf q;     // int32 query index in the run
    hymet::mm::DevBuf part;  // int32 index part
    hymet::mm::DevBuf rl;    // int32 rep_len of the line's query in that part (rl:i tag)
    hymet::mm::DevBuf t;     // int32 target index in the run (part's first target + rid)
};
