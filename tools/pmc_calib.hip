// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// library's kernels use (MI355X_MICROARCH.md: only 16 B/lane streaming reads and writes are
// calibrated there; "calibrate on a known byte count in your own access pattern").
// Each kernel streams exactly 2 GiB (past the 256 MiB Infinity Cache) with one access width
// per lane: 4, 8 or 16 bytes, reads (summed into one word per thread so nothing is dropped)
// or writes.  Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes);
// tools/pmc_summary.py divides the known bytes by the counters.
//   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBytes = size_t(2) << 30;

template <typename T>
__global__ __launch_bounds__(256) void calib_read(const T *__restrict__ a, size_t n, unsigned long long *out) {
    unsigned long long s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        s += reinterpret_cast<const unsigned int *>(&v)[0];
    }
    if (s == 0x123456789ull) out[0] = s;  // practically never: keeps the loads
}

template <typename T>
__global__ __launch_bounds__(256) void calib_write(T *__restrict__ a, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        unsigned int *w = reinterpret_cast<unsigned int *>(&v);
        for (size_t k = 0; k < sizeof(T) / 4; k++) w[k] = (unsigned int)(i + k);
        a[i] = v;
    }
}

// Scattered reads (round 5): one T per `Stride`-byte slot of the 2 GiB buffer, the slots visited
// in a pseudo-random order (k * 0x9E3779B1 mod the slot count: a bijection, no index array to
// stream), one access per lane per step -- the chaining / backtrack kernels' pattern (window
// heads, predecessor walks).  Each slot is read once, so the bytes the memory system must move
// are (slots x min(Stride, line)) and the bytes the kernel uses are (slots x sizeof(T)); the
// counters tell which of the two FETCH_SIZE follows for scattered traffic.
template <typename T, int Stride>
__global__ __launch_bounds__(256) void calib_gather(const unsigned char *__restrict__ a, size_t slots, unsigned long long *out) {
    unsigned long long s = 0;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < slots; k += (size_t)gridDim.x * blockDim.x) {
        const size_t slot = (k * 0x9E3779B1ull) & (slots - 1);
        const T v = *reinterpret_cast<const T *>(a + slot * Stride);
        s += reinterpret_cast<const unsigned int *>(&v)[0];
    }
    if (s == 0x123456789ull) out[0] = s;
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main() {
    void *buf;
    unsigned long long *out;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(buf, 1, kBytes));
    const dim3 grid(256 * 8 * 4), block(256);
    hipLaunchKernelGGL(calib_write<unsigned int>, grid, block, 0, 0, (unsigned int *)buf, kBytes / 4);
    hipLaunchKernelGGL(calib_write<uint2>, grid, block, 0, 0, (uint2 *)buf, kBytes / 8);
    hipLaunchKernelGGL(calib_write<uint4>, grid, block, 0, 0, (uint4 *)buf, kBytes / 16);
    hipLaunchKernelGGL(calib_read<unsigned int>, grid, block, 0, 0, (const unsigned int *)buf, kBytes / 4, out);
    hipLaunchKernelGGL(calib_read<uint2>, grid, block, 0, 0, (const uint2 *)buf, kBytes / 8, out);
    hipLaunchKernelGGL(calib_read<uint4>, grid, block, 0, 0, (const uint4 *)buf, kBytes / 16, out);
    const unsigned char *b = (const unsigned char *)buf;
    hipLaunchKernelGGL((calib_gather<unsigned int, 128>), grid, block, 0, 0, b, kBytes / 128, out);
    hipLaunchKernelGGL((calib_gather<uint2, 128>), grid, block, 0, 0, b, kBytes / 128, out);
    hipLaunchKernelGGL((calib_gather<unsigned int, 64>), grid, block, 0, 0, b, kBytes / 64, out);
    hipLaunchKernelGGL((calib_gather<unsigned int, 32>), grid, block, 0, 0, b, kBytes / 32, out);
    hipLaunchKernelGGL((calib_gather<uint4, 256>), grid, block, 0, 0, b, kBytes / 256, out);
    CK(hipDeviceSynchronize());
    printf("calibration kernels: %zu bytes each (read / write at 4, 8, 16 B per lane)\n", kBytes);
    printf("gather kernels: one T per Stride-byte slot, random slot order: <u32,128> %zu, <u64,128> %zu, <u32,64> %zu, "
           "<u32,32> %zu, <u128,256> %zu accesses\n", kBytes / 128, kBytes / 128, kBytes / 64, kBytes / 32, kBytes / 256);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
