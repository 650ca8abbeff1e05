// ASCII -> packed 2-bit bases + invalid-base bitmask (HBM layout shared by every stage).
//
// Layout (DESIGN.md "Data layout in HBM"): base i of the pool lives at bits 2*(i%16) of
// d_2b[i/16] and its invalid flag at bit i%32 of d_mask[i/32].  One thread packs 32 bases
// with two 16-byte loads: 1 B/base in, 0.375 B/base out.
#include "common.hpp"

namespace {

// 0..3 = A,C,G,T ; 4 = invalid.  [0] Mash (upper-cased, alphabet ACGT: CommandScreen
// hashSequence), [1] Mash with preserveCase, [2] minimap2 seq_nt4_table (A/C/G/T/U, any case).
__constant__ uint8_t kCode[3][256];

__global__ __launch_bounds__(256) void pack_kernel(const uint8_t *__restrict__ ascii, int64_t n, int alpha,
                                                   uint32_t *__restrict__ w2b, uint32_t *__restrict__ wm) {
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t b0 = t * 32;
    if (b0 >= n) return;
    const uint8_t *tab = kCode[alpha];
    uint32_t lo = 0, hi = 0, m = 0;
    if (b0 + 32 <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(ascii + b0);
        uint4 a = p[0], b = p[1];
        uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < 32; j++) {
            uint32_t c = tab[(w[j >> 2] >> (8 * (j & 3))) & 0xFF];
            uint32_t bad = c >> 2;
            c &= 3;
            if (j < 16) lo |= c << (2 * j);
            else hi |= c << (2 * (j - 16));
            m |= bad << j;
        }
    } else {
        for (int j = 0; j < 32; j++) {
            uint32_t c = (b0 + j < n) ? tab[ascii[b0 + j]] : 4u;
            uint32_t bad = c >> 2;
            c &= 3;
            if (j < 16) lo |= c << (2 * j);
            else hi |= c << (2 * (j - 16));
            m |= bad << j;
        }
    }
    int64_t nw2 = (n + 15) / 16;
    w2b[2 * t] = lo;
    if (2 * t + 1 < nw2) w2b[2 * t + 1] = hi;
    wm[t] = m;
}

bool g_tables_ready[64] = {false};

int ensure_tables(int dev) {
    if (g_tables_ready[dev]) return HYMET_OK;
    uint8_t h[3][256];
    for (int a = 0; a < 3; a++)
        for (int i = 0; i < 256; i++) h[a][i] = 4;
    const char *up = "ACGT";
    for (int j = 0; j < 4; j++) {
        h[0][(uint8_t)up[j]] = j;
        h[0][(uint8_t)up[j] + 32] = j;  // upper-cased before the alphabet test
        h[1][(uint8_t)up[j]] = j;       // preserveCase: lower case is outside the alphabet
        h[2][(uint8_t)up[j]] = j;
        h[2][(uint8_t)up[j] + 32] = j;
    }
    h[2][(uint8_t)'U'] = 3;
    h[2][(uint8_t)'u'] = 3;
    HY_HIP(hipMemcpyToSymbol(HIP_SYMBOL(kCode), h, sizeof(h)));
    g_tables_ready[dev] = true;
    return HYMET_OK;
}

}  // namespace

extern "C" int hymet_pack(hymet_ctx *ctx, const uint8_t *d_ascii, int64_t n, int alphabet, uint32_t *d_2b,
                          uint32_t *d_mask) {
    HY_ARG(ctx && d_ascii && d_2b && d_mask, "hymet_pack: null argument");
    HY_ARG(alphabet >= 0 && alphabet <= 2, "hymet_pack: alphabet must be 0, 1 or 2");
    HY_ARG(((uintptr_t)d_ascii & 15) == 0, "hymet_pack: d_ascii must be 16-byte aligned");
    if (n <= 0) return HYMET_OK;
    HY_HIP(hipSetDevice(ctx->device));
    int rc = ensure_tables(ctx->device);
    if (rc) return rc;
    int64_t nthreads = (n + 31) / 32;
    hymet::ProfScope _ps(ctx, "pack", 1.375 * (double)n);  // ASCII read, 2-bit + mask write
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)hymet::cdiv(nthreads, 256)), dim3(256), 0, ctx->stream, d_ascii, n,
                       alphabet, d_2b, d_mask);
    HY_CHECK_LAUNCH("pack_kernel");
    return HYMET_OK;
}
