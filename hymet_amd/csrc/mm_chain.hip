// Collinear chaining of anchors (minimap2 lchain.c mg_lchain_rmq + mg_chain_backtrack, as
// driven by `-x asm10`: --rmq, -r1k,100k, -g10k).
//
// chain_groups_kernel: one WAVE per (query, strand, target) group -- mg_lchain_rmq never
// chains across a change of x>>32, so groups are independent.  Groups are pulled from a
// size-descending work list with one atomic per group (biggest first, no tail of giants).
// Per anchor i the wave
//   * slides the outer window [st, i0) (x within max_dist) and the inner window
//     [st_in, i0) (x within max_dist_inner); the inner window is also kept as a (y, idx)
//     sorted list in LDS (the krmq inner tree's in-order sequence), plus an LDS ring of
//     "visited in this iteration" stamps (the t[] array restricted to the window, which is
//     the only part of t[] the skip heuristic ever reads);
//   * RMQ: every lane scans a strided slice of the outer window for the minimum priority
//     -(f_j + 0.5*gap*(x_j+y_j)) with y_j in the krmq closed interval
//     [(y_i-max_dist, INT32_MAX), (y_i, 0)], then a wave min-reduction (ties -> larger j:
//     canonical tie-break T2);
//   * if the RMQ winner is not an exact extension, walks the inner list downwards in
//     chunks of 64: candidate scores are computed lane-parallel, the order-dependent
//     n_skip / t[] logic is resolved in program order.
// All floating point follows lchain.c exactly (float mg_log2 / penalty, double priority;
// built with -ffp-contract=off).
//
// backtrack_groups_kernel: one thread per group replays mg_chain_backtrack on the group's
// anchors ordered by (f, idx) descending (canonical T3).
#include "mm_common.hpp"

namespace hymet {
namespace mm {
namespace {

constexpr int kInnerCap = 1024;  // LDS inner-window capacity per wave (entries)
constexpr int kWavesPerBlock = 4;

struct ChainParams {
    const uint64_t *ax;
    const uint64_t *ay;
    const int64_t *g_start;   // group g = anchors [g_start[g], g_start[g+1])
    const int32_t *order;     // work list of group ids (size-descending)
    int32_t n_work;
    int32_t *work_counter;
    int32_t *f;
    int64_t *p;
    int32_t *t_global;        // overflow path only
    int max_dist, max_dist_inner, bw, max_chn_skip, cap_rmq_size;
    float pen_gap, pen_skip;
};

__device__ __forceinline__ float mg_log2(float x) {
    union {
        float f;
        uint32_t i;
    } z = {x};
    float log_2 = (float)(((z.i >> 23) & (int)(0xff)) - 128);
    z.i &= ~(255u << 23);
    z.i += 127u << 23;
    log_2 += (-0.34484843f * z.f + 2.02466578f) * z.f - 0.67487759f;
    return log_2;
}

__device__ __forceinline__ int32_t comput_sc(uint64_t xi, uint64_t yi_, uint64_t xj, uint64_t yj_, float pen_gap,
                                             float pen_skip, int32_t *exact, int32_t *width) {
    const int32_t dq = (int32_t)yi_ - (int32_t)yj_;
    const int32_t dr = (int32_t)(xi - xj);
    const int32_t dd = dr > dq ? dr - dq : dq - dr;
    *width = dd;
    const int32_t dg = dr < dq ? dr : dq;
    const int32_t q_span = (int32_t)(yj_ >> 32 & 0xff);
    int32_t sc = q_span < dg ? q_span : dg;
    *exact = (dd == 0 && dg <= q_span);
    if (dd || dq > q_span) {
        const float lin_pen = __fadd_rn(__fmul_rn(pen_gap, (float)dd), __fmul_rn(pen_skip, (float)dg));
        const float log_pen = dd >= 1 ? mg_log2((float)(dd + 1)) : 0.0f;
        sc -= (int)__fadd_rn(lin_pen, __fmul_rn(.5f, log_pen));
    }
    return sc;
}

__device__ __forceinline__ double prio(int32_t f, uint64_t x, uint64_t y, float pen_gap) {
    const int32_t s = (int32_t)((uint32_t)x + (uint32_t)y);
    const double c = 0.5 * (double)pen_gap;
    return -((double)f + __dmul_rn(c, (double)s));
}

__device__ __forceinline__ bool key_less(int32_t ya, int32_t ja, int32_t yb, int32_t jb) {
    return ya < yb || (ya == yb && ja < jb);
}

__global__ __launch_bounds__(256) void chain_groups_kernel(ChainParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    int2 *lst = reinterpret_cast<int2 *>(smem) + wv * kInnerCap;                       // (y, local idx)
    int32_t *stamp = reinterpret_cast<int32_t *>(smem + kWavesPerBlock * kInnerCap * sizeof(int2)) + wv * kInnerCap;
    for (;;) {
        int w = 0;
        if (lane == 0) w = atomicAdd(P.work_counter, 1);
        w = __shfl(w, 0, 64);
        if (w >= P.n_work) break;
        const int g = P.order[w];
        const int64_t g0 = P.g_start[g], g1 = P.g_start[g + 1];
        int ni = 0;           // entries in lst (== i0 - st_in while !overflow)
        bool overflow = false;
        for (int e = lane; e < kInnerCap; e += 64) stamp[e] = -1;
        int64_t i0 = g0, st = g0, st_in = g0;
        for (int64_t i = g0; i < g1; ++i) {
            const uint64_t xi = P.ax[i], yi_ = P.ay[i];
            const int32_t yi = (int32_t)yi_;
            int32_t max_f = (int32_t)(yi_ >> 32 & 0xff);
            int64_t max_j = -1;
            if (i0 < i && P.ax[i0] != xi) {
                for (int64_t j = i0; j < i; ++j) {  // insert into the inner tree
                    if (P.max_dist_inner <= 0) break;
                    if (!overflow && ni >= kInnerCap) overflow = true;
                    if (overflow) continue;
                    const int32_t yj = (int32_t)P.ay[j], jl = (int32_t)(j - g0);
                    int c = 0;
                    for (int e = lane; e < ni; e += 64) c += key_less(lst[e].x, lst[e].y, yj, jl);
                    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                    for (int top = ni - 1; top >= c; top -= 64) {  // shift [c, ni) right by one
                        const int e = top - lane;
                        int2 v;
                        if (e >= c) v = lst[e];
                        __builtin_amdgcn_wave_barrier();
                        if (e >= c) lst[e + 1] = v;
                        __builtin_amdgcn_wave_barrier();
                    }
                    if (lane == 0) lst[c] = make_int2(yj, jl);
                    __builtin_amdgcn_wave_barrier();
                    ni++;
                }
                i0 = i;
            }
            while (st < i && (xi > P.ax[st] + (uint64_t)P.max_dist || (i0 > st ? i0 - st : 0) > P.cap_rmq_size)) ++st;
            if (P.max_dist_inner > 0) {
                while (st_in < i && (xi > P.ax[st_in] + (uint64_t)P.max_dist_inner ||
                                     (i0 > st_in ? i0 - st_in : 0) > P.cap_rmq_size)) {
                    if (st_in < i0 && !overflow) {  // erase from the inner list
                        const int32_t yj = (int32_t)P.ay[st_in], jl = (int32_t)(st_in - g0);
                        int c = 0;
                        for (int e = lane; e < ni; e += 64) c += key_less(lst[e].x, lst[e].y, yj, jl);
                        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                        for (int b = c; b < ni - 1; b += 64) {  // shift (c, ni) left by one
                            const int e = b + lane + 1;
                            int2 v;
                            if (e < ni) v = lst[e];
                            __builtin_amdgcn_wave_barrier();
                            if (e < ni) lst[e - 1] = v;
                            __builtin_amdgcn_wave_barrier();
                        }
                        ni--;
                    }
                    ++st_in;
                }
            }
            // ---- RMQ over the outer window
            double bp = 0.0;
            int64_t bj = -1;
            for (int64_t j = st + lane; j < i0; j += 64) {
                const int32_t yj = (int32_t)P.ay[j];
                const bool in = (yj > yi - P.max_dist) && (yj < yi || (yj == yi && j == 0));
                if (!in) continue;
                const double pr = prio(P.f[j], P.ax[j], P.ay[j], P.pen_gap);
                if (bj < 0 || pr < bp || (pr == bp && j > bj)) bp = pr, bj = j;
            }
            for (int o = 32; o > 0; o >>= 1) {
                const double op = __shfl_xor(bp, o, 64);
                const int64_t oj = __shfl_xor(bj, o, 64);
                if (oj >= 0 && (bj < 0 || op < bp || (op == bp && oj > bj))) bp = op, bj = oj;
            }
            if (bj >= 0) {
                int32_t exact, width;
                const int32_t sc = P.f[bj] + comput_sc(xi, yi_, P.ax[bj], P.ay[bj], P.pen_gap, P.pen_skip, &exact, &width);
                if (width <= P.bw && sc > max_f) max_f = sc, max_j = bj;
                const int64_t n_inner = i0 > st_in ? i0 - st_in : 0;
                if (!exact && n_inner > 0 && yi > 0) {
                    int n_skip = 0;
                    bool done = false;
                    const int32_t ylo = yi - P.max_dist_inner;
                    if (!overflow) {
                        // last list position with y <= yi - 1
                        int c = 0;
                        for (int e = lane; e < ni; e += 64) c += lst[e].x < yi;
                        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
                        for (int pos = c - 1; pos >= 0 && !done; pos -= 64) {
                            const int e = pos - lane;
                            int32_t yj = INT32_MIN, jl = 0, sc_l = 0, w_l = INT32_MAX;
                            int64_t pj = -1;
                            if (e >= 0) {
                                const int2 v = lst[e];
                                yj = v.x, jl = v.y;
                                const int64_t j = g0 + jl;
                                int32_t ex;
                                sc_l = P.f[j] + comput_sc(xi, yi_, P.ax[j], P.ay[j], P.pen_gap, P.pen_skip, &ex, &w_l);
                                pj = P.p[j];
                            }
                            const int nl = min(64, pos + 1);
                            for (int l = 0; l < nl; ++l) {
                                const int32_t yl = __shfl(yj, l, 64);
                                if (yl < ylo) {
                                    done = true;
                                    break;
                                }
                                const int32_t wl = __shfl(w_l, l, 64);
                                if (wl > P.bw) continue;
                                const int32_t sl = __shfl(sc_l, l, 64);
                                const int32_t jll = __shfl(jl, l, 64);
                                const int64_t pl = __shfl(pj, l, 64);
                                const int64_t j = g0 + jll;
                                if (sl > max_f) {
                                    max_f = sl, max_j = j;
                                    if (n_skip > 0) --n_skip;
                                } else if (stamp[(int)((j - g0) % kInnerCap)] == (int32_t)i && j >= st_in && j < i0) {
                                    if (++n_skip > P.max_chn_skip) {
                                        done = true;
                                        break;
                                    }
                                }
                                if (pl >= 0 && pl >= st_in && pl < i0) {
                                    __builtin_amdgcn_wave_barrier();
                                    if (lane == 0) stamp[(int)((pl - g0) % kInnerCap)] = (int32_t)i;
                                    __builtin_amdgcn_wave_barrier();
                                }
                            }
                        }
                    } else {
                        // overflow path: next candidate = largest (y, idx) below the previous one
                        int32_t cy = yi, cj = INT32_MIN;  // exclusive upper bound (yi - 1, +inf) == (yi, -inf)
                        bool first = true;
                        for (;;) {
                            int32_t by = INT32_MIN, bjl = INT32_MIN;
                            for (int64_t j = st_in + lane; j < i0; j += 64) {
                                const int32_t yj = (int32_t)P.ay[j];
                                const int32_t jl = (int32_t)(j - g0);
                                const bool below = first ? (yj <= yi - 1) : key_less(yj, jl, cy, cj);
                                if (below && (bjl == INT32_MIN || key_less(by, bjl, yj, jl))) by = yj, bjl = jl;
                            }
                            for (int o = 32; o > 0; o >>= 1) {
                                const int32_t oy = __shfl_xor(by, o, 64), oj = __shfl_xor(bjl, o, 64);
                                if (oj != INT32_MIN && (bjl == INT32_MIN || key_less(by, bjl, oy, oj))) by = oy, bjl = oj;
                            }
                            if (bjl == INT32_MIN) break;
                            first = false;
                            cy = by, cj = bjl;
                            if (by < ylo) break;
                            const int64_t j = g0 + bjl;
                            int32_t ex, wl;
                            const int32_t sl = P.f[j] + comput_sc(xi, yi_, P.ax[j], P.ay[j], P.pen_gap, P.pen_skip, &ex, &wl);
                            if (wl <= P.bw) {
                                if (sl > max_f) {
                                    max_f = sl, max_j = j;
                                    if (n_skip > 0) --n_skip;
                                } else if (P.t_global[j] == (int32_t)i) {
                                    if (++n_skip > P.max_chn_skip) break;
                                }
                                const int64_t pl = P.p[j];
                                if (pl >= 0) P.t_global[pl] = (int32_t)i;  // every lane writes: program order
                            }
                        }
                    }
                }
            }
            P.f[i] = max_f;  // every lane stores: later loads by any lane follow its own store
            P.p[i] = max_j;
        }
    }
}

struct BacktrackParams {
    const int64_t *g_start;
    const int32_t *f;
    const int64_t *p;
    int32_t *t;
    const int64_t *z_off;   // per group: start of its (f, idx)-ascending z list
    const int32_t *z_idx;   // anchor indices ordered by (group, f, idx) ascending
    int32_t n_groups;
    int min_cnt, min_sc, max_drop;
    // outputs (per group region = its anchor range)
    int64_t *chain_ids;     // anchor ids of each chain, start -> end, packed in the group's range
    uint64_t *chain_u;      // score<<32 | count, packed at the group's range start
    int64_t *chain_first;   // offset in chain_ids of each chain
    int32_t *n_chains;      // per group
};

__device__ int64_t bk_end(int32_t max_drop, int64_t zi, int32_t zf, const int32_t *f, const int64_t *p, int32_t *t) {
    int64_t i = zi, end_i = -1, max_i = i;
    int32_t max_s = 0;
    if (i < 0 || t[i] != 0) return i;
    do {
        int32_t s;
        t[i] = 2;
        end_i = i = p[i];
        s = i < 0 ? zf : zf - f[i];
        if (s > max_s) max_s = s, max_i = i;
        else if (max_s - s > max_drop) break;
    } while (i >= 0 && t[i] == 0);
    for (i = zi; i >= 0 && i != end_i; i = p[i]) t[i] = 0;
    return max_i;
}

__global__ __launch_bounds__(64) void backtrack_groups_kernel(BacktrackParams P) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= P.n_groups) return;
    const int64_t g0 = P.g_start[g], g1 = P.g_start[g + 1];
    for (int64_t i = g0; i < g1; i++) P.t[i] = 0;
    int64_t wpos = g0;  // next free slot in chain_ids
    int nc = 0;
    const int64_t z0 = P.z_off[g], z1 = P.z_off[g + 1];
    for (int64_t k = z1 - 1; k >= z0; --k) {
        const int64_t zi = P.z_idx[k];
        if (P.t[zi] != 0) continue;
        const int32_t zf = P.f[zi];
        const int64_t end_i = bk_end(P.max_drop, zi, zf, P.f, P.p, P.t);
        int64_t i = zi, nv = 0;
        for (; i != end_i; i = P.p[i]) {
            P.chain_ids[wpos + nv] = i;  // end -> start for now
            P.t[i] = 1;
            nv++;
        }
        const int32_t sc = i < 0 ? zf : zf - P.f[i];
        if (sc >= P.min_sc && nv > 0 && nv >= P.min_cnt) {
            for (int64_t a = 0, b = nv - 1; a < b; a++, b--) {  // start -> end
                const int64_t tmp = P.chain_ids[wpos + a];
                P.chain_ids[wpos + a] = P.chain_ids[wpos + b];
                P.chain_ids[wpos + b] = tmp;
            }
            P.chain_u[g0 + nc] = (uint64_t)(uint32_t)sc << 32 | (uint32_t)nv;
            P.chain_first[g0 + nc] = wpos;
            nc++;
            wpos += nv;
        }
    }
    P.n_chains[g] = nc;
}

}  // namespace

int launch_chain(hymet_ctx *ctx, const uint64_t *ax, const uint64_t *ay, const int64_t *g_start, const int32_t *order,
                 int32_t n_work, int32_t *f, int64_t *p, int32_t *t_global, int max_dist, int max_dist_inner, int bw,
                 int max_chn_skip, int cap_rmq_size, float pen_gap, float pen_skip, int64_t n_anchors) {
    if (n_work <= 0) return HYMET_OK;
    DevBuf cnt;
    HY_HIP(cnt.alloc(4, ctx->stream));
    HY_HIP(hipMemsetAsync(cnt.p, 0, 4, ctx->stream));
    if (max_dist < bw) max_dist = bw;
    if (max_dist_inner <= 0 || max_dist_inner >= max_dist) max_dist_inner = 0;
    ChainParams P{ax, ay, g_start, order, n_work, cnt.as<int32_t>(), f, p, t_global, max_dist, max_dist_inner, bw,
                  max_chn_skip, cap_rmq_size, pen_gap, pen_skip};
    const size_t lds = kWavesPerBlock * kInnerCap * (sizeof(int2) + sizeof(int32_t));
    int64_t blocks = cdiv(n_work, kWavesPerBlock);
    const int64_t cap = (int64_t)ctx->n_cu * 6;
    if (blocks > cap) blocks = cap;
    ProfScope _ps(ctx, "mm_chain", 28.0 * (double)n_anchors);  // x,y read + f,p write per anchor
    hipLaunchKernelGGL(chain_groups_kernel, dim3((unsigned)blocks), dim3(64 * kWavesPerBlock), lds, ctx->stream, P);
    HY_CHECK_LAUNCH("chain_groups_kernel");
    return HYMET_OK;
}

int launch_backtrack(hymet_ctx *ctx, const int64_t *g_start, const int32_t *f, const int64_t *p, int32_t *t,
                     const int64_t *z_off, const int32_t *z_idx, int32_t n_groups, int min_cnt, int min_sc,
                     int max_drop, int64_t *chain_ids, uint64_t *chain_u, int64_t *chain_first, int32_t *n_chains) {
    if (n_groups <= 0) return HYMET_OK;
    BacktrackParams P{g_start, f, p, t, z_off, z_idx, n_groups, min_cnt, min_sc, max_drop, chain_ids, chain_u, chain_first,
                      n_chains};
    ProfScope _ps(ctx, "mm_backtrack");
    hipLaunchKernelGGL(backtrack_groups_kernel, dim3((unsigned)cdiv(n_groups, 64)), dim3(64), 0, ctx->stream, P);
    HY_CHECK_LAUNCH("backtrack_groups_kernel");
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet
