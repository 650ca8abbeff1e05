// Screen-table insert variants on 1e8 random 64-bit keys (tools/insert_bench.hip; A/B only):
//   k8      8-byte key slots, 2^28 slots (2 GB), CAS only
//   k16     16-byte slots (4 GB), CAS only
//   k16st   16-byte slots, CAS + the owner's store of the second word (the product kernel)
//   k8c     8-byte key slots + a separate 4-byte canonical array (1 GB), CAS + owner store there
//   k16h    16-byte slots at 2^27 slots (2 GB, load 0.75), CAS + owner store
// Each is timed with HIP events over 5 launches after a warm-up; keys regenerated per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint64_t kEmpty = ~0ull;
__device__ __forceinline__ uint64_t home_slot(uint64_t h, int shift) { return (h * 0x9E3779B97F4A7C15ull) >> shift; }

template <int W, bool ST, bool SEP>
__global__ __launch_bounds__(256) void ins(const uint64_t *__restrict__ hs, int64_t n, unsigned long long *tab,
                                           uint32_t *canon, uint64_t mask, int shift, int64_t *slot_of) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = hs[i];
    uint64_t s = home_slot(h, shift);
    for (;;) {
        const unsigned long long prev = atomicCAS(&tab[W * s], kEmpty, (unsigned long long)h);
        if (prev == kEmpty) {
            if (ST && W == 2) tab[2 * s + 1] = (unsigned long long)(uint32_t)i | ((unsigned long long)(uint32_t)i << 32);
            if (SEP) canon[s] = (uint32_t)i;
            break;
        }
        if (prev == h) break;
        s = (s + 1) & mask;
    }
    slot_of[i] = (int64_t)s;
}

template <int W, bool ST, bool SEP>
int run(const char *name, const uint64_t *d_h, int64_t n, int lg, unsigned long long *tab, uint32_t *canon,
        int64_t *slot_of) {
    const int64_t ns = 1ll << lg;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float tot = 0;
    for (int r = 0; r < 6; r++) {
        CK(hipMemset(tab, 0xFF, (size_t)ns * 8 * W));
        if (SEP) CK(hipMemset(canon, 0xFF, (size_t)ns * 4));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((ins<W, ST, SEP>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d_h, n, tab, canon,
                           (uint64_t)(ns - 1), 64 - lg, slot_of);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r) tot += ms;
    }
    printf("%-6s slots 2^%d x %2d B: %.2f ms per insert of %lld keys\n", name, lg, 8 * W, tot / 5, (long long)n);
    return 0;
}

int main() {
    const int64_t n = 100000000;
    std::vector<uint64_t> h(n);
    std::mt19937_64 g(7);
    for (auto &x : h) x = g() >> 1;
    uint64_t *d_h;
    unsigned long long *tab;
    uint32_t *canon;
    int64_t *slot_of;
    CK(hipMalloc(&d_h, 8 * n));
    CK(hipMalloc(&tab, 16ull << 28));
    CK(hipMalloc(&canon, 4ull << 28));
    CK(hipMalloc(&slot_of, 8 * n));
    CK(hipMemcpy(d_h, h.data(), 8 * n, hipMemcpyHostToDevice));
    if (run<1, false, false>("k8", d_h, n, 28, tab, canon, slot_of)) return 1;
    if (run<2, false, false>("k16", d_h, n, 28, tab, canon, slot_of)) return 1;
    if (run<2, true, false>("k16st", d_h, n, 28, tab, canon, slot_of)) return 1;
    if (run<1, false, true>("k8c", d_h, n, 28, tab, canon, slot_of)) return 1;
    if (run<2, true, false>("k16h", d_h, n, 27, tab, canon, slot_of)) return 1;
    return 0;
}
