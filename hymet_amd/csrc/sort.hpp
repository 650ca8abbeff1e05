// Stable LSD radix sort of (key, value) pairs on the device -- the library's own sort for
// every pass that orders by a packed integer key (minimizers by hash, groups by size, chains
// by first anchor, the long segments of the grouped anchor sort, PAF lines by LCA row).
//
// One 8-bit digit per pass over bits [begin_bit, end_bit):
//   rs_hist    per 2048-element tile, the 256-bin digit histogram (LDS counters, one
//              wave-aggregated increment per distinct digit of a wave) -> counts[digit][tile]
//   scan       exclusive scan of the digit-major counts (scan.hip): the output offset of
//              every (digit, tile)
//   rs_scatter the tile again, in 8 rounds of 256 elements: an element's rank among the
//              equal digits before it = its wave's lower lanes with that digit (8 ballots)
//              + the earlier waves' and rounds' counts; keys and values are staged in LDS in
//              digit order and written out as contiguous runs (coalesced)
// Passes ping-pong between the two buffers; `keys` / `vals` point at the sorted data on
// return (the rocPRIM double-buffer contract it replaces).  No per-call state to initialise,
// no host synchronisation.
#pragma once
#include "mm_common.hpp"

namespace hymet {
namespace mm {
namespace rsort {

constexpr int kBlock = 256;
constexpr int kRounds = 8;
constexpr int kTile = kBlock * kRounds;  // 2048

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K k, int shift, uint32_t mask) {
    return (uint32_t)(k >> shift) & mask;
}

// lanes of this wave holding the same digit (8 ballots; all 64 lanes take part)
__device__ __forceinline__ uint64_t same_digit(uint32_t d, bool valid) {
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const uint64_t on = __ballot(valid && ((d >> b) & 1));
        m &= ((d >> b) & 1) ? on : ~on;
    }
    return valid ? m : 0ull;
}

template <typename K>
__global__ __launch_bounds__(kBlock) void rs_hist(const K *__restrict__ keys, int64_t n, int shift, uint32_t mask,
                                                  int64_t n_tiles, uint32_t *__restrict__ counts) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kTile;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
        const int64_t e = base + r * kBlock + threadIdx.x;
        const bool v = e < n;
        const uint32_t d = v ? digit_of(keys[e], shift, mask) : 0u;
        const uint64_t m = same_digit(d, v);
        if (v && lane == __ffsll((unsigned long long)m) - 1) atomicAdd(&h[d], (uint32_t)__popcll(m));
    }
    __syncthreads();
    counts[(int64_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

template <typename K, typename V>
__global__ __launch_bounds__(kBlock) void rs_scatter(const K *__restrict__ keys, const V *__restrict__ vals, int64_t n,
                                                     int shift, uint32_t mask, int64_t n_tiles,
                                                     const uint32_t *__restrict__ counts,
                                                     const int64_t *__restrict__ offs, K *__restrict__ okeys,
                                                     V *__restrict__ ovals) {
    __shared__ uint32_t run[256];       // elements of each digit placed so far (tile-local)
    __shared__ uint32_t wc[4][256];     // this round's count per (wave, digit)
    __shared__ uint32_t tstart[256];    // tile-local start of each digit's run
    __shared__ K sk[kTile];
    __shared__ V sv[kTile];
    __shared__ uint8_t sd[kTile];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kTile;
    const int m_tile = (int)min<int64_t>(kTile, n - base);
    // tile-local digit starts: exclusive scan of this tile's histogram over the 256 digits
    {
        const uint32_t c = counts[(int64_t)threadIdx.x * n_tiles + blockIdx.x];
        uint32_t inc = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= d) inc += o;
        }
        if (lane == 63) run[w] = inc;  // wave totals (run[] is reset below)
        __syncthreads();
        uint32_t before = 0;
        for (int ww = 0; ww < w; ww++) before += run[ww];
        tstart[threadIdx.x] = before + inc - c;
        __syncthreads();
    }
    run[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < 4 * 256; i += kBlock) (&wc[0][0])[i] = 0;
    __syncthreads();
#pragma unroll 1
    for (int r = 0; r < kRounds; r++) {
        const int li = r * kBlock + threadIdx.x;  // tile-relative element
        const bool v = li < m_tile;
        K k = 0;
        V val = 0;
        uint32_t d = 0;
        if (v) {
            k = keys[base + li];
            val = vals[base + li];
            d = digit_of(k, shift, mask);
        }
        const uint64_t m = same_digit(d, v);
        const uint32_t rk = (uint32_t)__popcll(m & ((1ull << lane) - 1));
        if (v && rk == 0) wc[w][d] = (uint32_t)__popcll(m);
        __syncthreads();
        if (v) {
            uint32_t before = run[d];
            for (int ww = 0; ww < w; ww++) before += wc[ww][d];
            const uint32_t pos = tstart[d] + before + rk;
            sk[pos] = k;
            sv[pos] = val;
            sd[pos] = (uint8_t)d;
        }
        __syncthreads();
        {
            const int d2 = threadIdx.x;
            run[d2] += wc[0][d2] + wc[1][d2] + wc[2][d2] + wc[3][d2];
            wc[0][d2] = wc[1][d2] = wc[2][d2] = wc[3][d2] = 0;
        }
        __syncthreads();
    }
    // staged in digit order: element p of digit d goes to offs[d][tile] + (p - tstart[d])
    for (int p = threadIdx.x; p < m_tile; p += kBlock) {
        const uint32_t d = sd[p];
        const int64_t o = offs[(int64_t)d * n_tiles + blockIdx.x] + (p - (int64_t)tstart[d]);
        okeys[o] = sk[p];
        ovals[o] = sv[p];
    }
}

}  // namespace rsort

// sort (keys, vals) by key bits [begin_bit, end_bit), stably; on return keys / vals point at
// the sorted buffers and keys_alt / vals_alt at the others
template <typename K, typename V>
int radix_sort_pairs(hymet_ctx *ctx, K *&keys, K *&keys_alt, V *&vals, V *&vals_alt, int64_t n, int begin_bit,
                     int end_bit) {
    using namespace rsort;
    if (n <= 1 || end_bit <= begin_bit) return HYMET_OK;
    hipStream_t st = ctx->stream;
    const int64_t n_tiles = cdiv(n, kTile);
    DevBuf counts, offs, part;
    HY_HIP(counts.alloc(4 * (size_t)(256 * n_tiles), st));
    HY_HIP(offs.alloc(8 * (size_t)(256 * n_tiles), st));
    for (int shift = begin_bit; shift < end_bit; shift += 8) {
        const int nb = min(8, end_bit - shift);
        const uint32_t mask = (1u << nb) - 1u;
        hipLaunchKernelGGL((rs_hist<K>), dim3((unsigned)n_tiles), dim3(kBlock), 0, st, keys, n, shift, mask, n_tiles,
                           counts.as<uint32_t>());
        HY_CHECK_LAUNCH("rs_hist");
        int rc = scan_u32_i64(ctx, counts.as<uint32_t>(), offs.as<int64_t>(), 256 * n_tiles, part);
        if (rc) return rc;
        hipLaunchKernelGGL((rs_scatter<K, V>), dim3((unsigned)n_tiles), dim3(kBlock), 0, st, keys, vals, n, shift, mask,
                           n_tiles, counts.as<uint32_t>(), offs.as<int64_t>(), keys_alt, vals_alt);
        HY_CHECK_LAUNCH("rs_scatter");
        std::swap(keys, keys_alt);
        std::swap(vals, vals_alt);
    }
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet
