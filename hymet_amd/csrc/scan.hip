// Exclusive prefix sum of uint32 counts into int64 offsets -- the scan behind every
// count-then-write pass of the library (seed and anchor offsets, group starts, region and
// text offsets).  Reduce-then-scan over tiles of 4096 counts, in two launches: per-tile sums,
// whose LAST block to finish (told by a ticket, an agent-scope atomic add) scans the tile
// sums into tile offsets; then every tile re-read and scanned in LDS with its offset.
// 16 B of HBM traffic per count (4 + 4 read, 8 written), no per-call state to initialise
// (the ticket is a self-clearing context counter).  There is no one-block middle launch: a
// one-block kernel behind a full-grid one waited for a free CU slot while the other mapping
// stream's persistent chaining grid held every CU (round 3: 1,159 such launches, 231 ms of
// waiting per two-stream step).
#include "mm_common.hpp"

namespace hymet {
namespace mm {
namespace {

constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const int lo = __shfl_up((int)(uint32_t)v, d, 64), hi = __shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return (uint64_t)(uint32_t)hi << 32 | (uint32_t)lo;
}

// inclusive scan across the 64 lanes of a wave
__device__ __forceinline__ uint64_t wave_incl(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = shfl_up64(v, d);
        if (lane >= d) v += o;
    }
    return v;
}

// exclusive scan of one value per thread over a block of NW waves; *total gets the sum
template <int NW>
__device__ __forceinline__ uint64_t block_excl(uint64_t v, uint64_t *ws, uint64_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t inc = wave_incl(v);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        if (i < w) before += ws[i];
        all += ws[i];
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

// The hand-off of the tile sums to the last block: lane 0 of every block stores its sum with
// an sc1 store, waits for it (vmcnt(0)), then adds to the ticket; the block whose add returns
// nb - 1 reads every sum with sc1 loads.  No fence, no dependence on dispatch order.
// Why this is sound on gfx950 without a release/acquire pair (the LLVM AMDGPU memory model
// for the GFX942 family, which gfx950 belongs to):
//   * a relaxed atomic store / load at agent scope is emitted as global_store / global_load
//     with sc1 set: it bypasses the XCD-private L2 caching of the line and is performed at the
//     device's coherence point, so it is coherent across the eight XCDs by itself;
//   * the store's vmcnt decrement happens when that write is acknowledged at the coherence
//     point, so the s_waitcnt vmcnt(0) orders the completed store before the ticket's atomic
//     RMW, which is itself performed at the coherence point;
//   * the last block issues its sc1 loads only after its own RMW returned nb - 1 (the value
//     is consumed through LDS and s_barrier), i.e. after every other block's RMW, each of
//     which followed that block's completed store.
// A release fetch_add would add buffer_wbl2 (an L2 write-back of the whole XCD's dirty lines)
// per block -- the cost DESIGN.md §3 measured for agent-scope fences in the backtrack kernel
// -- for no ordering the sc1 accesses do not already give.  The guide's measured hand-off
// table (MI355X_MICROARCH.md, inter-workgroup visibility, first row) is this pattern;
// tests/test_sort_gpu.py runs it at ~9,800 tiles per call under a concurrent second stream.
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(int32_t *p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_sc1(const int32_t *p) {
    return __hip_atomic_load(const_cast<int32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane 0 publishes this block's partial; returns true (block-uniform) in the last block
template <typename T>
__device__ __forceinline__ bool publish_part(T *part, T v, uint32_t *ticket) {
    __shared__ bool last;
    if (threadIdx.x == 0) {
        st_sc1(part + blockIdx.x, v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    return last;
}

// the last block: exclusive scan of the nb tile sums in place (rounds of 1024), part[nb] =
// total, *mail = total; the ticket is cleared for the next call
__device__ void scan_parts_last(uint64_t *part, int64_t nb, int64_t *mail, uint32_t *ticket) {
    __shared__ uint64_t ws[kScanBlock / 64];
    uint64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += 4 * kScanBlock) {
        const int64_t b = b0 + 4 * (int64_t)threadIdx.x;
        uint64_t v[4], s = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            v[j] = b + j < nb ? ld_sc1(part + b + j) : 0;
            s += v[j];
        }
        uint64_t total;
        uint64_t run = carry + block_excl<kScanBlock / 64>(s, ws, &total);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (b + j < nb) part[b + j] = run;
            run += v[j];
        }
        carry += total;
    }
    if (threadIdx.x == 0) {
        part[nb] = carry;
        if (mail) *mail = (int64_t)carry;
        atomicExch(ticket, 0u);
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(const uint32_t *__restrict__ in, int64_t n,
                                                                 uint64_t *__restrict__ part, uint32_t *ticket,
                                                                 int64_t *mail) {
    __shared__ uint64_t ws[kScanBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    uint64_t s = 0;
    if (base + kScanTile <= n && ((uintptr_t)in & 15) == 0) {  // full tile: 16-byte loads
        const uint4 *v = reinterpret_cast<const uint4 *>(in + base);
#pragma unroll
        for (int j = 0; j < kScanItems / 4; j++) {
            const uint4 q = v[j * kScanBlock + threadIdx.x];
            s += (uint64_t)q.x + q.y + q.z + q.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {
            const int64_t i = base + j * kScanBlock + threadIdx.x;
            if (i < n) s += in[i];
        }
    }
    uint64_t total;
    (void)block_excl<kScanBlock / 64>(s, ws, &total);
    if (publish_part(part, total, ticket)) scan_parts_last(part, gridDim.x, mail, ticket);
}

__device__ __forceinline__ int pad16(int e) { return e + (e >> 4); }

// O = int64_t (offsets) or uint32_t (the index's bucket offsets, sums below 2^32)
template <typename O>
__global__ __launch_bounds__(kScanBlock) void scan_down_kernel(const uint32_t *__restrict__ in, int64_t n,
                                                               const uint64_t *__restrict__ part, O *__restrict__ out) {
    __shared__ uint32_t sv[kScanTile + kScanTile / 16];
    __shared__ O so[kScanTile + kScanTile / 16];
    __shared__ uint64_t ws[kScanBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    const int t = threadIdx.x;
    const bool full = base + kScanTile <= n && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0;
    if (full) {  // 16-byte loads, striped
        const uint4 *v = reinterpret_cast<const uint4 *>(in + base);
#pragma unroll
        for (int j = 0; j < kScanItems / 4; j++) {
            const int q = j * kScanBlock + t;
            const uint4 w = v[q];
            const int e = 4 * q;  // 4 consecutive counts: one pad word per 16 keeps them together
            sv[pad16(e)] = w.x, sv[pad16(e) + 1] = w.y, sv[pad16(e) + 2] = w.z, sv[pad16(e) + 3] = w.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {  // coalesced, striped
            const int e = j * kScanBlock + t;
            sv[pad16(e)] = base + e < n ? in[base + e] : 0u;
        }
    }
    __syncthreads();
    uint32_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {  // thread t owns counts t*16 .. t*16+15
        v[j] = sv[pad16(t * kScanItems + j)];
        s += v[j];
    }
    uint64_t total;
    uint64_t run = part[blockIdx.x] + block_excl<kScanBlock / 64>(s, ws, &total);
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        so[pad16(t * kScanItems + j)] = (O)run;
        run += v[j];
    }
    __syncthreads();
    if (full && sizeof(O) == 8) {  // 16-byte stores, striped
        longlong2 *o = reinterpret_cast<longlong2 *>(out + base);
#pragma unroll
        for (int j = 0; j < kScanItems / 2; j++) {
            const int q = j * kScanBlock + t, e = 2 * q;
            o[q] = make_longlong2((long long)so[pad16(e)], (long long)so[pad16(e) + 1]);
        }
    } else if (full) {
        uint4 *o = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
        for (int j = 0; j < kScanItems / 4; j++) {
            const int q = j * kScanBlock + t, e = 4 * q;
            o[q] = make_uint4((uint32_t)so[pad16(e)], (uint32_t)so[pad16(e) + 1], (uint32_t)so[pad16(e) + 2],
                              (uint32_t)so[pad16(e) + 3]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {
            const int e = j * kScanBlock + t;
            if (base + e < n) out[base + e] = so[pad16(e)];
        }
    }
}

// uint64 -> uint64 variant (packed counters, e.g. two 32-bit counts per word): thread t of a
// tile owns 16 consecutive entries
__global__ __launch_bounds__(kScanBlock) void scan_reduce64_kernel(const uint64_t *__restrict__ in, int64_t n,
                                                                   uint64_t *__restrict__ part, uint32_t *ticket,
                                                                   int64_t *mail) {
    __shared__ uint64_t ws[kScanBlock / 64];
    const int64_t b = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) s += b + j < n ? in[b + j] : 0ull;
    uint64_t total;
    (void)block_excl<kScanBlock / 64>(s, ws, &total);
    if (publish_part(part, total, ticket)) scan_parts_last(part, gridDim.x, mail, ticket);
}

__global__ __launch_bounds__(kScanBlock) void scan_down64_kernel(const uint64_t *__restrict__ in, int64_t n,
                                                                 const uint64_t *__restrict__ part,
                                                                 uint64_t *__restrict__ out) {
    __shared__ uint64_t ws[kScanBlock / 64];
    const int64_t b = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    uint64_t v[kScanItems], s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        v[j] = b + j < n ? in[b + j] : 0ull;
        s += v[j];
    }
    uint64_t total;
    uint64_t run = part[blockIdx.x] + block_excl<kScanBlock / 64>(s, ws, &total);
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        if (b + j < n) out[b + j] = run;
        run += v[j];
    }
}

// inclusive running maximum of int32 values: per-tile maxima, one block scanning them
// (exclusive, seeded with INT32_MIN), then every tile re-scanned with its carry
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v = max(v, o);
    }
    return v;
}

// exclusive block max-scan of one value per thread (INT32_MIN before the first); *all = block max
template <int NW>
__device__ __forceinline__ int32_t block_excl_max(int32_t v, int32_t *ws, int32_t *all) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int32_t inc = wave_incl_max(v);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    int32_t before = INT32_MIN, a = INT32_MIN;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        if (i < w) before = max(before, ws[i]);
        a = max(a, ws[i]);
    }
    __syncthreads();
    *all = a;
    int32_t ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = INT32_MIN;
    return max(before, ex);
}

__global__ __launch_bounds__(kScanBlock) void max_reduce_kernel(const int32_t *__restrict__ in, int64_t n,
                                                                int32_t *__restrict__ part, uint32_t *ticket) {
    __shared__ int32_t ws[kScanBlock / 64];
    const int64_t b = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int32_t m = INT32_MIN;
#pragma unroll
    for (int j = 0; j < kScanItems; j++)
        if (b + j < n) m = max(m, in[b + j]);
    int32_t all;
    (void)block_excl_max<kScanBlock / 64>(m, ws, &all);
    if (!publish_part(part, all, ticket)) return;
    // last block: exclusive max-scan of the tile maxima in place (rounds of 1024)
    const int64_t nb = gridDim.x;
    int32_t carry = INT32_MIN;
    for (int64_t b0 = 0; b0 < nb; b0 += 4 * kScanBlock) {
        const int64_t q = b0 + 4 * (int64_t)threadIdx.x;
        int32_t v[4], mm = INT32_MIN;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            v[j] = q + j < nb ? ld_sc1(part + q + j) : INT32_MIN;
            mm = max(mm, v[j]);
        }
        int32_t blk;
        int32_t run = max(carry, block_excl_max<kScanBlock / 64>(mm, ws, &blk));
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (q + j < nb) part[q + j] = run;
            run = max(run, v[j]);
        }
        carry = max(carry, blk);
    }
    if (threadIdx.x == 0) atomicExch(ticket, 0u);
}

__global__ __launch_bounds__(kScanBlock) void max_down_kernel(const int32_t *__restrict__ in, int64_t n,
                                                              const int32_t *__restrict__ part, int32_t *__restrict__ out) {
    __shared__ int32_t ws[kScanBlock / 64];
    const int64_t b = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int32_t v[kScanItems], m = INT32_MIN;
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        v[j] = b + j < n ? in[b + j] : INT32_MIN;
        m = max(m, v[j]);
    }
    int32_t all;
    int32_t run = max(part[blockIdx.x], block_excl_max<kScanBlock / 64>(m, ws, &all));
#pragma unroll
    for (int j = 0; j < kScanItems; j++) {
        run = max(run, v[j]);
        if (b + j < n) out[b + j] = run;
    }
}

}  // namespace

int inclusive_max_scan_i32(hymet_ctx *ctx, const int32_t *in, int32_t *out, int64_t n, DevBuf &part) {
    if (n <= 0) return HYMET_OK;
    hipStream_t st = ctx->stream;
    const int64_t nb = cdiv(n, kScanTile);
    HY_HIP(part.alloc(4 * (size_t)(nb + 1), st));
    hipLaunchKernelGGL(max_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<int32_t>(),
                       reinterpret_cast<uint32_t *>(ctx->dctr + kCtrMaxScan));
    HY_CHECK_LAUNCH("max_reduce_kernel");
    hipLaunchKernelGGL(max_down_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<int32_t>(), out);
    HY_CHECK_LAUNCH("max_down_kernel");
    return HYMET_OK;
}

int scan_u64(hymet_ctx *ctx, const uint64_t *in, uint64_t *out, int64_t n, DevBuf &part, int64_t *mail) {
    if (n <= 0) return HYMET_OK;
    hipStream_t st = ctx->stream;
    const int64_t nb = cdiv(n, kScanTile);
    HY_HIP(part.alloc(8 * (size_t)(nb + 1), st));
    hipLaunchKernelGGL(scan_reduce64_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<uint64_t>(),
                       reinterpret_cast<uint32_t *>(ctx->dctr + kCtrScan), mail);
    HY_CHECK_LAUNCH("scan_reduce64_kernel");
    hipLaunchKernelGGL(scan_down64_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<uint64_t>(), out);
    HY_CHECK_LAUNCH("scan_down64_kernel");
    return HYMET_OK;
}

int scan_u32_i64(hymet_ctx *ctx, const uint32_t *in, int64_t *out, int64_t n, DevBuf &part, int64_t *mail) {
    if (n <= 0) return HYMET_OK;
    hipStream_t st = ctx->stream;
    const int64_t nb = cdiv(n, kScanTile);
    HY_HIP(part.alloc(8 * (size_t)(nb + 1), st));
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<uint64_t>(),
                       reinterpret_cast<uint32_t *>(ctx->dctr + kCtrScan), mail);
    HY_CHECK_LAUNCH("scan_reduce_kernel");
    hipLaunchKernelGGL(scan_down_kernel<int64_t>, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<uint64_t>(), out);
    HY_CHECK_LAUNCH("scan_down_kernel");
    return HYMET_OK;
}

int scan_u32(hymet_ctx *ctx, const uint32_t *in, uint32_t *out, int64_t n, DevBuf &part, int64_t *mail) {
    if (n <= 0) return HYMET_OK;
    hipStream_t st = ctx->stream;
    const int64_t nb = cdiv(n, kScanTile);
    HY_HIP(part.alloc(8 * (size_t)(nb + 1), st));
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<uint64_t>(),
                       reinterpret_cast<uint32_t *>(ctx->dctr + kCtrScan), mail);
    HY_CHECK_LAUNCH("scan_reduce_kernel");
    hipLaunchKernelGGL(scan_down_kernel<uint32_t>, dim3((unsigned)nb), dim3(kScanBlock), 0, st, in, n, part.as<uint64_t>(), out);
    HY_CHECK_LAUNCH("scan_down_kernel");
    return HYMET_OK;
}

int exclusive_scan_u32_i64(hymet_ctx *ctx, const uint32_t *in, int64_t *out, int64_t n, int64_t *total) {
    *total = 0;
    if (n <= 0) return HYMET_OK;
    DevBuf part;
    int rc = scan_u32_i64(ctx, in, out, n, part, mb_dev(ctx, kMbScan));
    if (rc) return rc;
    HY_HIP(hipStreamSynchronize(ctx->stream));
    *total = mb_read(ctx, kMbScan);
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet

// ---- C ABI: the library's radix sort, for tests and callers that sort packed keys
#include "sort.hpp"

extern "C" int hymet_scan_u32(hymet_ctx *ctx, const uint32_t *d_in, int64_t *d_out, int64_t n, int mode, int64_t *total) {
    HY_ARG(ctx && (n == 0 || (d_in && d_out)) && (mode == 0 || mode == 1), "hymet_scan_u32: bad argument");
    HY_HIP(hipSetDevice(ctx->device));
    using namespace hymet::mm;
    if (mode == 1) {
        DevBuf part;
        const int rc = inclusive_max_scan_i32(ctx, reinterpret_cast<const int32_t *>(d_in), reinterpret_cast<int32_t *>(d_out), n,
                                              part);
        if (rc) return rc;
        HY_HIP(hipStreamSynchronize(ctx->stream));
        return HYMET_OK;
    }
    int64_t t = 0;
    const int rc = exclusive_scan_u32_i64(ctx, d_in, d_out, n, &t);
    if (total) *total = t;
    return rc;
}

extern "C" int hymet_sort_pairs_u64(hymet_ctx *ctx, uint64_t *d_keys, uint32_t *d_vals, int64_t n, int begin_bit,
                                    int end_bit) {
    HY_ARG(ctx && (n == 0 || (d_keys && d_vals)), "hymet_sort_pairs_u64: null argument");
    HY_ARG(begin_bit >= 0 && end_bit <= 64 && begin_bit <= end_bit, "hymet_sort_pairs_u64: bad bit range");
    if (n <= 1) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    using namespace hymet::mm;
    DevBuf k2, v2;
    HY_HIP(k2.alloc(8 * (size_t)n, ctx->stream));
    HY_HIP(v2.alloc(4 * (size_t)n, ctx->stream));
    uint64_t *kk = d_keys, *kka = k2.as<uint64_t>();
    uint32_t *vv = d_vals, *vva = v2.as<uint32_t>();
    const int rc = radix_sort_pairs(ctx, kk, kka, vv, vva, n, begin_bit, end_bit);
    if (rc) return rc;
    if (kk != d_keys) {
        HY_HIP(hipMemcpyAsync(d_keys, kk, 8 * (size_t)n, hipMemcpyDeviceToDevice, ctx->stream));
        HY_HIP(hipMemcpyAsync(d_vals, vv, 4 * (size_t)n, hipMemcpyDeviceToDevice, ctx->stream));
    }
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}
