// Section-level cycle profile of chain_groups_kernel (s_memtime around each stage of the
// per-anchor loop) on ONE group.  Build (tools/chain_prof.sh):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -DHYMET_CHAIN_PROF -I include \
//         tools/chain_prof.hip -o tools/chain_prof
// Input: raw n x (x, y) uint64 anchors (tools/bench_chain.py --dump FILE).
#include "../hymet_amd/csrc/mm_chain.hip"

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

using namespace hymet::mm;

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                       \
        }                                                                   \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: chain_prof anchors.bin bw\n");
        return 2;
    }
    FILE *fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    fseek(fp, 0, SEEK_END);
    const long bytes = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    std::vector<uint64_t> a((size_t)bytes / 16 * 2);
    if (fread(a.data(), 16, a.size() / 2, fp) != a.size() / 2) return 2;
    fclose(fp);
    const int64_t n = (int64_t)a.size() / 2;
    const int bw = atoi(argv[2]);
    std::vector<uint64_t> hx(n), hy(n);
    for (int64_t i = 0; i < n; i++) hx[i] = a[2 * i], hy[i] = a[2 * i + 1];
    uint64_t *dx, *dy;
    int64_t *gs, *dp;
    int32_t *order, *cnt, *df, *dt;
    uint8_t *qf;
    int4 *sum;
    const size_t ns = (size_t)(n >> 6) + (size_t)n / 2 + 4;
    CK(hipMalloc(&dx, 8 * n));
    CK(hipMalloc(&dy, 8 * n));
    CK(hipMalloc(&gs, 16));
    CK(hipMalloc(&dp, 8 * n));
    CK(hipMalloc(&order, 4));
    CK(hipMalloc(&cnt, 4 * kChainCtrPad * kChainStripes));  // the striped work counters (zeroed by the split kernel)
    CK(hipMalloc(&df, 4 * n));
    CK(hipMalloc(&dt, 4 * n));
    CK(hipMalloc(&qf, 1));
    CK(hipMalloc(&sum, 16 * kGSumInts * ns));
    CK(hipMemcpy(dx, hx.data(), 8 * n, hipMemcpyHostToDevice));
    int32_t *dx32;  // the chaining kernels read x's low words
    {
        std::vector<int32_t> h32(n);
        for (int64_t i = 0; i < n; i++) h32[i] = (int32_t)hx[i];
        CK(hipMalloc(&dx32, 4 * n));
        CK(hipMemcpy(dx32, h32.data(), 4 * n, hipMemcpyHostToDevice));
    }
    CK(hipMemcpy(dy, hy.data(), 8 * n, hipMemcpyHostToDevice));
    // groups = runs of equal x >> 32, work list by size descending, group 0 holds anchor 0
    std::vector<int64_t> h_gs;
    for (int64_t i = 0; i < n; i++)
        if (i == 0 || (hx[i] >> 32) != (hx[i - 1] >> 32)) h_gs.push_back(i);
    const int G = (int)h_gs.size();
    h_gs.push_back(n);
    {  // group-size distribution: groups and anchors per size class
        const int64_t lim[] = {3, 8, 16, 32, 64, 128, 256, 1024, 4096, 16384, INT64_MAX};
        int64_t ng[11] = {0}, na[11] = {0};
        for (int g = 0; g < G; g++) {
            const int64_t s = h_gs[g + 1] - h_gs[g];
            int c = 0;
            while (s > lim[c]) c++;
            ng[c]++, na[c] += s;
        }
        for (int c = 0; c < 11; c++)
            printf("groups <= %6lld: %8lld groups (%5.1f%%), %10lld anchors (%5.1f%%)\n", (long long)(c < 10 ? lim[c] : -1),
                   (long long)ng[c], 100.0 * ng[c] / G, (long long)na[c], 100.0 * na[c] / n);
    }
    std::vector<int32_t> h_order(G);
    for (int g = 0; g < G; g++) h_order[g] = g;
    std::sort(h_order.begin(), h_order.end(), [&](int a, int b) { return h_gs[a + 1] - h_gs[a] > h_gs[b + 1] - h_gs[b]; });
    // the library's work list holds groups of >= min_cnt (3) anchors only
    int nwork = 0;
    while (nwork < G && h_gs[h_order[nwork] + 1] - h_gs[h_order[nwork]] >= 3) nwork++;
    int32_t *split;
    CK(hipMalloc(&split, 4));
    std::vector<uint8_t> h_qf(G, 0);
    h_qf[0] = 1;
    CK(hipFree(gs));
    CK(hipFree(order));
    CK(hipFree(qf));
    CK(hipMalloc(&gs, 8 * (G + 1)));
    CK(hipMalloc(&order, 4 * G));
    CK(hipMalloc(&qf, G));
    CK(hipMemcpy(gs, h_gs.data(), 8 * (G + 1), hipMemcpyHostToDevice));
    CK(hipMemcpy(order, h_order.data(), 4 * G, hipMemcpyHostToDevice));
    CK(hipMemcpy(qf, h_qf.data(), G, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    // waves per CU as the library launches them (launch_chain: 16), HYMET_CHAIN_PROF_WPC overrides
    const char *wpc = getenv("HYMET_CHAIN_PROF_WPC");
    const int nblk = std::min(nwork, prop.multiProcessorCount * (wpc ? atoi(wpc) : 16));
    {
        int per_cu = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, chain_groups_kernel<0>, 64, kChainLds);
        printf("occupancy: %d waves per CU at %zu B of LDS per wave\n", per_cu, (size_t)kChainLds);
    }
    int max_dist = 10000 < bw ? bw : 10000;
    for (int rep = 0; rep < 2; rep++) {
        unsigned long long z[32] = {0};
#ifdef HYMET_CHAIN_PROF
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_prof), z, sizeof(z)));
#endif
        CK(hipMemset(cnt, 0, 4));
        CK(hipMemset(df, 0, 4 * n));
        CK(hipMemset(dp, 0xFF, 8 * n));
        CK(hipMemset(dt, 0, 4 * n));  // t arrives zeroed (overflow stamps are i + 1)
        ChainParams P{dx32, dy, gs, qf, order, nwork, cnt, df, dp, dt, sum, max_dist, 1000, bw, 25, 100000, 0.12f, 0.0f, nullptr};
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
#ifdef HYMET_CHAIN_GTIME
        uint64_t *gt;
        CK(hipMalloc(&gt, 8 * (size_t)G));
        CK(hipMemset(gt, 0, 8 * (size_t)G));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_gtime), &gt, sizeof(gt)));
        int4 *gc;
        CK(hipMalloc(&gc, 16 * (size_t)G));
        CK(hipMemset(gc, 0, 16 * (size_t)G));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_gcnt), &gc, sizeof(gc)));
#endif
        CK(hipEventRecord(e0, 0));
        if (getenv("HYMET_CHAIN_PROF_WAVE_ONLY")) {
            hipLaunchKernelGGL(chain_groups_kernel<0>, dim3(nblk), dim3(64), kChainLds, 0, P);
            CK(hipGetLastError());
        } else if (launch_chain_raw(0, P, nblk, split) != 0) {
            return 1;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
#ifdef HYMET_CHAIN_PROF
        CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(g_chain_prof), sizeof(z)));
#endif
#ifdef HYMET_CHAIN_GTIME
        {  // per-group wall time (wall_clock64 ticks) by size class
            std::vector<uint64_t> h(G);
            CK(hipMemcpy(h.data(), gt, 8 * (size_t)G, hipMemcpyDeviceToHost));
            CK(hipFree(gt));
            std::vector<int4> hc(G);
            CK(hipMemcpy(hc.data(), gc, 16 * (size_t)G, hipMemcpyDeviceToHost));
            CK(hipFree(gc));
            int wclk = 100000;  // kHz
            (void)hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);
            const int64_t lim[] = {3, 8, 16, 32, 64, 128, 256, 1024, 4096, 16384, INT64_MAX};
            double tc[11] = {0}, na[11] = {0}, mx[11] = {0}, it[11] = {0}, ba[11] = {0}, bn[11] = {0}, bx[11] = {0};
            double tot = 0;
            for (int g = 0; g < G; g++) {
                const int64_t sz = h_gs[g + 1] - h_gs[g];
                int c = 0;
                while (sz > lim[c]) c++;
                const double us = h[g] / (wclk / 1000.0);
                tc[c] += us, na[c] += sz, tot += us, mx[c] = std::max(mx[c], us);
                it[c] += hc[g].x, ba[c] += hc[g].y, bn[c] += hc[g].z, bx[c] += hc[g].w;
            }
            printf("wave-time %.1f ms total over %d groups (kernel wall x waves = %.1f ms)\n", tot / 1e3, G, ms * nblk);
            for (int c = 0; c < 11; c++)
                if (na[c] > 0)
                    printf("  groups <= %6lld: %7.1f%% of wave-time, %8.3f us/anchor, max group %8.1f us; per anchor: "
                           "%.3f iterations, %.4f batch attempts, %.4f batches, %.3f in batches; %.2f us/iteration\n",
                           (long long)(c < 10 ? lim[c] : -1), 100.0 * tc[c] / tot, tc[c] / na[c], mx[c], it[c] / na[c],
                           ba[c] / na[c], bn[c] / na[c], bx[c] / na[c], tc[c] / std::max(1.0, it[c]));
        }
#endif
        {  // f / p digest: variants must agree bit for bit
            std::vector<int32_t> hf(n);
            std::vector<int64_t> hp(n);
            CK(hipMemcpy(hf.data(), df, 4 * n, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hp.data(), dp, 8 * n, hipMemcpyDeviceToHost));
            uint64_t h = 1469598103934665603ull;
            for (int64_t i = 0; i < n; i++) h = (h ^ (uint64_t)(uint32_t)hf[i]) * 1099511628211ull, h = (h ^ (uint64_t)hp[i]) * 1099511628211ull;
            printf("fp digest %016llx\n", (unsigned long long)h);
        }
        const char *names[8] = {"i0-advance", "st+head", "st_in", "rmq", "walk", "winner+cert", "st_in-probe", "loop/batch"};
        double tot = 0;
        for (int k = 0; k < 8; k++) tot += (double)z[k];
        printf("n=%lld groups=%d bw=%d kernel %.2f ms = %.0f ns/anchor; %.0f cycles/anchor\n", (long long)n, G, bw, ms, ms * 1e6 / n,
               tot / n);
        for (int k = 0; k < 8; k++)
            if (z[k]) printf("  %-12s %8.0f cyc/anchor  %5.1f%%\n", names[k], (double)z[k] / n, 100.0 * z[k] / tot);
        const char *cn[8] = {"global fetch", "list ins general", "list erase general", "rmq full path", "walk",
                             "head suffix", "cert y-fail", "batches"};
        printf("  %-20s %8.4f per anchor\n", "no try: same x", (double)z[8 + 9] / n);
        for (int k = 0; k < 8; k++) printf("  %-20s %8.4f per anchor\n", cn[k], (double)z[8 + k] / n);
        const char *cn2[12] = {"batch attempts", "pre: cert", "pre: b0 != prev", "pre: walk", "fail: x same", "fail: y range",
                               "fail: gap/width", "fail: cand", "fail: walk", "fail: list", "accepted", "no try: empty window"};
        for (int k = 0; k < 12; k++) printf("  %-20s %8.4f per anchor\n", cn2[k], (double)z[16 + k] / n);
        const char *cn3[4] = {"head changes", "head chg repeated", "no try: back-off", "loop iterations"};
        for (int k = 0; k < 4; k++) printf("  %-20s %8.4f per anchor\n", cn3[k], (double)z[28 + k] / n);
    }
    return 0;
}
