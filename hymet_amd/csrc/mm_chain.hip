// Collinear chaining of anchors (minimap2 lchain.c mg_lchain_rmq + mg_chain_backtrack, as
// driven by `-x asm10`: --rmq, -r1k,100k, -g10k).
//
// chain_groups_kernel: one WAVE (= one block) per (query, strand, target) group --
// mg_lchain_rmq never chains across a change of x>>32, so groups are independent.  Groups
// are pulled from a size-descending work list with one atomic per group (biggest first).
// The DP is sequential along the group, so the kernel is latency-bound: it keeps the
// per-anchor chain of dependent operations short (register-cached deque ends, lane-parallel
// probes, DPP/permlane reductions, no LDS round trip where a register will do) and the LDS
// footprint small (~15 KB) so that ~10 groups run per CU.
//   * anchors are fetched 64 at a time with one coalesced load (double buffered) and handed
//     out with lane shuffles; the last kRing anchors sit in an LDS ring as one int4
//     (x, y, f, (p+1) | span<<24);
//   * RMQ window = anchors [st, i0) (x within max_dist: 10 kbp on the first pass, bw_long =
//     100 kbp on the long-join re-chain, ~18k anchors), cut into blocks of 64.  Every
//     complete block gets a summary: its argmin priority -(f_j + 0.5*gap*(x_j+y_j)) (ties ->
//     larger index, canonical T2), the y of that argmin and the block's y range; a monotone
//     deque over the summaries gives the best complete block of the window in O(1), and the
//     head block (partial, oldest) is cached with its suffix argmins.
//     FAST PATH: scan the newest 64 window entries with the krmq range test
//     [(y_i-max_dist, INT32_MAX), (y_i, 0)] and reduce; if neither the deque front nor the
//     head suffix beats that candidate -- ignoring y, so a fortiori with it -- it is the
//     exact RMQ answer.  On colinear chains the newest anchors carry the best priority.
//     FULL PATH: take the summary of every block whose y range meets the query and whose
//     argmin lies inside it (then it is the argmin of the block's in-range subset), scan
//     entries of the partial head/tail blocks and of blocks whose argmin is out of range;
//   * the inner window (x within rmq_inner_dist) is a (y, idx) sorted ring-deque in LDS (the
//     krmq inner tree's in-order sequence; colinear inserts append, colinear erases pop the
//     front); the walk's "visited in this iteration" stamps (lchain.c's t[]) go to t_global
//     as i + 1 (the walk is rare on real anchors; t arrives zeroed and is re-zeroed after a
//     group that stamped it).  A candidate of the
//     inner walk scores at most f_j + span_j, so when a monotone max-deque over the window
//     says max(f_j + span_j) <= max_f the walk cannot change max_f/max_j and is skipped.
//     Otherwise the walk is evaluated 64 candidates at a time: scores lane-parallel, the
//     running max by a prefix-max scan, t[] marks by one LDS write round (a mark always
//     points to a later candidate in walk order), and the saturating n_skip counter by a
//     prefix scan of max-plus maps -- the same decisions as the sequential loop, including
//     where it breaks.
// All floating point follows lchain.c exactly (float mg_log2 / penalty, double priority;
// built with -ffp-contract=off).
//
// backtrack_groups_kernel: one thread per group replays mg_chain_backtrack on the group's
// anchors ordered by (f, idx) descending (canonical T3).
#include "mm_common.hpp"

#include <cstdlib>
#include <string>

namespace hymet {
namespace mm {
namespace {

// Occupancy: the kernel is latency-bound, so it is sized for 16 resident waves per CU --
// registers capped at 128 VGPRs (4 waves per SIMD) and ~9.75 KB of LDS per wave.  Measured
// on C4: 8 -> 12 -> 16 waves/CU took mm_chain 2198 -> 1873 -> 1744 ms per step.  Every ring
// and deque has an HBM or slow-path fallback when it overflows.
#ifndef HYMET_CHAIN_RING
#define HYMET_CHAIN_RING 128
#endif
#ifndef HYMET_CHAIN_SUMRING
#define HYMET_CHAIN_SUMRING 16
#endif
#ifndef HYMET_CHAIN_BDQ
#define HYMET_CHAIN_BDQ 32
#endif
#ifndef HYMET_CHAIN_IDQ
#define HYMET_CHAIN_IDQ 64
#endif
// A colinear batch's pre-batch best B from the O(1) window sources when they decide it.
#ifndef HYMET_CHAIN_B0FAST
#define HYMET_CHAIN_B0FAST 1
#endif
// Block summaries of colinear blocks (y increasing) by one DPP prefix min and popcounts
// instead of a shuffle scan and a readlane loop over the records (~64 per colinear block).
#ifndef HYMET_CHAIN_CBFAST
#define HYMET_CHAIN_CBFAST 1
#endif
// Colinear batch commits: the inner max-deque's records and the tail block's argmin from the
// batch's monotone values in O(1) when f + span rises and the priority falls along the batch.
#ifndef HYMET_CHAIN_MONO
#define HYMET_CHAIN_MONO 1
#endif
// Window-start blocks passed whole are skipped by their last x (an LDS ring) instead of loaded.
#ifndef HYMET_CHAIN_BLX
#define HYMET_CHAIN_BLX 0
#endif
// A batch starts at any anchor whose window best B lies in its range (not only after B = i-1).
#ifndef HYMET_CHAIN_B0ANY
#define HYMET_CHAIN_B0ANY 1
#endif
// First back-off step of the batch attempts after a failed or short batch.
#ifndef HYMET_CHAIN_SPEC_GAP0
#define HYMET_CHAIN_SPEC_GAP0 2
#endif
// Inner-window entries leaving as a prefix of the (y, idx) list are popped, not compacted.
#ifndef HYMET_CHAIN_IPOP
#define HYMET_CHAIN_IPOP 1
#endif
// Colinear batches skip the prefix min of priorities and the prefix max of f + span.
#ifndef HYMET_CHAIN_BMONO
#define HYMET_CHAIN_BMONO 1
#endif
// Batch f / p global stores issued at the end of the commit instead of its start.
#ifndef HYMET_CHAIN_LATE_FP
#define HYMET_CHAIN_LATE_FP 1
#endif
// Head cache prefetch: when the head cache takes block b, block b + 1's entries are loaded
// into registers, so the next window-start block change does not wait on HBM.
#ifndef HYMET_CHAIN_HCPF
#define HYMET_CHAIN_HCPF 0
#endif
// Lean head cache: when the window start enters a block beyond the ring, load only its x (the
// window-start probes) and the block's suffix records (kept with its summary), not every
// entry's (x, y, f, p); entries are fetched in full only when a y-bounded scan needs them.
#ifndef HYMET_CHAIN_HLEAN
#define HYMET_CHAIN_HLEAN 0
#endif
// Entries fetched from HBM (head cache, window scans, the winner) without p: only the inner
// walk reads an entry's predecessor, and it fetches through the ring or HBM (fetch_p)
#ifndef HYMET_CHAIN_HNOP
#define HYMET_CHAIN_HNOP 1
#endif
// A window that anchor i-1 leaves empties whole (x never decreases along a group): st / st_in
// jump to i and the deques and the inner list are cleared in O(1), instead of one probe round
// (and a head-cache load beyond the rings) per 64 entries passed.
#ifndef HYMET_CHAIN_DRAIN
#define HYMET_CHAIN_DRAIN 1
#endif
// A committed batch also inserts its last anchor into the window structures when the next
// anchor's x differs (lchain.c inserts [i0, i) once x changes): the next iteration then has
// nothing to insert (step 1 is skipped) instead of one insert_one per batch.
#ifndef HYMET_CHAIN_INSALL
#define HYMET_CHAIN_INSALL 1
#endif
// A colinear batch is cut at the first anchor whose y does not rise: no anchor from there on
// can commit (the batch needs py < ky lane to lane), and Y -- the y bound B is taken under --
// becomes the y of the last anchor that can.  Without the cut, a stray anchor inside the
// 64-anchor window past a chain's end set Y to its random y, every chain anchor above it
// failed `ky <= Y`, and the rest of the chain was single-stepped behind the back-off.
#ifndef HYMET_CHAIN_YPREFIX
#define HYMET_CHAIN_YPREFIX 1
#endif
// Wave-uniform loop state pinned to scalar registers (readfirstlane at the derivation points):
// branches on it become scalar branches instead of exec-mask bookkeeping (first pass 11.55 ->
// 11.27 ms, long join 7.27 -> 7.07 ms on the real-anchor dump; VALU -9 % per anchor).
#ifndef HYMET_CHAIN_UNI
#define HYMET_CHAIN_UNI 1
#endif
#ifndef HYMET_CHAIN_WPE  // waves per SIMD the register allocation targets (0: compiler's choice)
#define HYMET_CHAIN_WPE 4
#endif
constexpr int kRing = HYMET_CHAIN_RING;  // LDS ring of recent anchors, int4 each (2 KB)
constexpr int kRingMask = kRing - 1;
constexpr int kStair = 4;       // staircase entries kept per block summary
constexpr int kSumInts = kStair + 1;  // int4 words per block summary: staircase + (ymin, ymax, n|trunc, -)
// HBM summaries add the block's last kSufRec suffix records: the lanes better than every later
// lane (the argmins of the suffixes [k, 64)), lane 63 first, as ring entries (x, y, f, pw)
constexpr int kSufRec = HYMET_CHAIN_HLEAN ? 4 : 0;
constexpr int kGSumInts = kSumInts + kSufRec;
constexpr int kSumRing = HYMET_CHAIN_SUMRING;  // LDS ring of the last complete block summaries (1.25 KB)
#ifndef HYMET_CHAIN_INNER
#define HYMET_CHAIN_INNER 256
#endif
constexpr int kInnerCap = HYMET_CHAIN_INNER;  // LDS inner-window list (ring-deque): 2 KB at 256
constexpr int kXRing = 256;  // LDS ring of the last 256 anchors' x (1 KB): the window-start probes
constexpr int kBdq = HYMET_CHAIN_BDQ;  // block-argmin deque, 2 int4 per element (1 KB)
constexpr int kIdq = HYMET_CHAIN_IDQ;  // inner max-deque (idx, f + span) (0.5 KB)
constexpr int kBlx = 64;  // LDS ring of the last 64 complete blocks' last x (0.25 KB)
constexpr size_t kChainLds = kRing * sizeof(int4) + kSumRing * kSumInts * sizeof(int4) + 64 * 2 * sizeof(int4) +
                             kInnerCap * sizeof(int2) + kXRing * sizeof(int32_t) + kBdq * 2 * sizeof(int4) + kIdq * sizeof(int2) +
                             (HYMET_CHAIN_BLX ? kBlx * sizeof(int32_t) : 0);
constexpr int kNegInf = -(1 << 29);
constexpr int kSpecGap0 = HYMET_CHAIN_SPEC_GAP0;

// ISA section markers (static instruction counts by section: build with -DHYMET_CHAIN_MARKS -S)
#ifdef HYMET_CHAIN_MARKS
#define AMARK(name) asm volatile("; @@ " #name)
#else
#define AMARK(name)
#endif
// Section cycle counters for tools/chain_prof (built with -DHYMET_CHAIN_PROF); no-ops otherwise.
#ifdef HYMET_CHAIN_PROF
__device__ unsigned long long g_chain_prof[32];
#define CPROF_DECL uint64_t _pt = clock64(), _pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, _pcnt[24] = {0};
#define CCOUNT(k) (_pcnt[k]++)
#define CPROF(k)                       \
    do {                               \
        const uint64_t _n = clock64(); \
        _pacc[k] += _n - _pt;          \
        _pt = _n;                      \
    } while (0)
#define CPROF_FLUSH                                                                  \
    do {                                                                             \
        if (lane == 0)                                                               \
            for (int _k = 0; _k < 24; _k++) { if (_k < 8) atomicAdd(&g_chain_prof[_k], _pacc[_k]); atomicAdd(&g_chain_prof[8 + _k], _pcnt[_k]); } \
    } while (0)
#else
#define CPROF_DECL
#define CCOUNT(k)
#define CPROF(k)
#define CPROF_FLUSH
#endif
// Per-group wall cycles for tools/chain_prof (-DHYMET_CHAIN_GTIME): two clock reads per group,
// cheap enough not to change the schedule (the section counters above do: ~10x slower).
#ifdef HYMET_CHAIN_GTIME
__device__ uint64_t *g_chain_gtime;
__device__ int4 *g_chain_gcnt;  // per group: loop iterations, batch attempts, batches, batch anchors
#define GTIME_START                         \
    const uint64_t _gt0 = wall_clock64();   \
    int4 _gc = make_int4(0, 0, 0, 0);
#define GCNT(f, v) (_gc.f += (v))
#define GTIME_STOP                                                                \
    do {                                                                          \
        if (lane == 0 && g_chain_gtime) g_chain_gtime[g] = wall_clock64() - _gt0; \
        if (lane == 0 && g_chain_gcnt) g_chain_gcnt[g] = _gc;                      \
    } while (0)
#else
#define GTIME_START
#define GTIME_STOP
#define GCNT(f, v)
#endif

// the wave kernel's work counters: kChainStripes of them, kChainCtrPad ints (256 B) apart
#ifndef HYMET_CHAIN_STRIPES
#define HYMET_CHAIN_STRIPES 8
#endif
constexpr int kChainStripes = HYMET_CHAIN_STRIPES, kChainCtrPad = 64;

struct ChainParams {
    const int32_t *ax;        // x's low word (target position) per anchor: x >> 32 is the group's constant
    const uint64_t *ay;
    const int64_t *g_start;   // group g = anchors [g_start[g], g_start[g+1])
    const uint8_t *g_qfirst;  // group g starts its query's anchor array (the krmq index-0 quirk)
    const int32_t *order;     // work list of group ids (size-descending)
    int32_t n_work;
    int32_t *work_counter;
    int32_t *f;
    int64_t *p;
    int32_t *t_global;        // overflow path only
    int4 *sum;                // block summaries of every group (group g at ((g_start[g] >> 6) + g) * kGSumInts)
    int max_dist, max_dist_inner, bw, max_chn_skip, cap_rmq_size;
    float pen_gap, pen_skip;
    const int32_t *work_end;  // device: the wave kernel takes work items [0, *work_end) (null: n_work)
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

// lchain.c comput_sc on the low 32 bits (x>>32 is constant inside a group)
__device__ __forceinline__ int32_t comput_sc(int32_t xi, int32_t yi, int32_t xj, int32_t yj, int32_t q_span,
                                             float pen_gap, float pen_skip, int32_t *exact, int32_t *width) {
    const int32_t dq = yi - yj;
    const int32_t dr = (int32_t)((uint32_t)xi - (uint32_t)xj);
    const int32_t dd = dr > dq ? dr - dq : dq - dr;
    *width = dd;
    const int32_t dg = dr < dq ? dr : dq;
    int32_t sc = q_span < dg ? q_span : dg;
    *exact = (dd == 0 && dg <= q_span);
    if (dd || dq > q_span) {
        const float lin_pen = __fadd_rn(__fmul_rn(pen_gap, (float)dd), __fmul_rn(pen_skip, (float)dg));
        const float log_pen = dd >= 1 ? mg_log2((float)(dd + 1)) : 0.0f;
        sc -= (int)__fadd_rn(lin_pen, __fmul_rn(.5f, log_pen));
    }
    return sc;
}

__device__ __forceinline__ double prio(int32_t f, int32_t x, int32_t y, double c) {
    const int32_t s = (int32_t)((uint32_t)x + (uint32_t)y);
    return -__dadd_rn((double)f, __dmul_rn(c, (double)s));
}

__device__ __forceinline__ bool key_less(int32_t ya, int32_t ja, int32_t yb, int32_t jb) {
    return ya < yb || (ya == yb && ja < jb);
}

// (pr, j) beats (bp, bj): smaller priority, ties -> larger index; bj < 0 = none
__device__ __forceinline__ bool better(double pr, int32_t j, double bp, int32_t bj) {
    return j >= 0 && (bj < 0 || pr < bp || (pr == bp && j > bj));
}

// ---- wave-wide reductions without LDS: DPP within rows of 16, permlane swaps across rows
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}

// partner value across rows: xor 16 (permlane16_swap) / xor 32 (permlane32_swap)
__device__ __forceinline__ int xrow16(int v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? r[0] : r[1];
}
__device__ __forceinline__ int xrow32(int v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? r[0] : r[1];
}

template <int STEP>
__device__ __forceinline__ int xstep(int v) {
    if constexpr (STEP == 0) return dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    if constexpr (STEP == 1) return dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    if constexpr (STEP == 2) return dpp<0x141>(v);  // row_half_mirror
    if constexpr (STEP == 3) return dpp<0x140>(v);  // row_mirror
    if constexpr (STEP == 4) return xrow16(v);
    return xrow32(v);
}

template <int STEP>
__device__ __forceinline__ void argmin_step(double &p, int32_t &j, int32_t &y) {
    const int lo = xstep<STEP>(__double2loint(p)), hi = xstep<STEP>(__double2hiint(p));
    const int oj = xstep<STEP>(j), oy = xstep<STEP>(y);
    const double op = __hiloint2double(hi, lo);
    if (better(op, oj, p, j)) p = op, j = oj, y = oy;
}

// every lane ends with the wave's best (p, j) and the payload y of that lane
__device__ __forceinline__ void wave_argmin(double &p, int32_t &j, int32_t &y) {
    argmin_step<0>(p, j, y);
    argmin_step<1>(p, j, y);
    argmin_step<2>(p, j, y);
    argmin_step<3>(p, j, y);
    argmin_step<4>(p, j, y);
    argmin_step<5>(p, j, y);
}

template <int STEP>
__device__ __forceinline__ void minmax_step(int32_t &mn, int32_t &mx) {
    mn = min(mn, xstep<STEP>(mn));
    mx = max(mx, xstep<STEP>(mx));
}
__device__ __forceinline__ void wave_minmax(int32_t &mn, int32_t &mx) {
    minmax_step<0>(mn, mx);
    minmax_step<1>(mn, mx);
    minmax_step<2>(mn, mx);
    minmax_step<3>(mn, mx);
    minmax_step<4>(mn, mx);
    minmax_step<5>(mn, mx);
}

// Values this wave wrote earlier (f, p, t, block summaries) are re-read through L2: an
// agent-scope relaxed load cannot hit a line the CU's L1 cached before the store.
template <typename T>
__device__ __forceinline__ T ld_l2(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int4 ld_l2(const int4 *p) {
    const int32_t *q = reinterpret_cast<const int32_t *>(p);
    return make_int4(ld_l2(q), ld_l2(q + 1), ld_l2(q + 2), ld_l2(q + 3));
}

// ---- wave prefix scans with DPP: row_shr within rows of 16, row_bcast15/31 across rows
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ int dppu(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xF, false);
}
// value of lane l-1 (lane 0: first)
__device__ __forceinline__ int shr1(int v, int first) {
    const int r = dppu<0x138>(0, v);  // wave_shr:1
    return threadIdx.x == 0 ? first : r;
}
__device__ __forceinline__ int scan_max(int v) {  // inclusive prefix max
    v = max(v, dppu<0x111>(INT32_MIN, v));
    v = max(v, dppu<0x112>(INT32_MIN, v));
    v = max(v, dppu<0x114>(INT32_MIN, v));
    v = max(v, dppu<0x118>(INT32_MIN, v));
    v = max(v, dppu<0x142, 0xA>(INT32_MIN, v));
    v = max(v, dppu<0x143, 0xC>(INT32_MIN, v));
    return v;
}
// inclusive scan of the maps f -> max(f + a, b) (left to right)
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ void mp_step(int &a, int &b) {
    const int ao = dppu<CTRL, ROWMASK>(0, a), bo = dppu<CTRL, ROWMASK>(kNegInf, b);
    b = max(bo + a, b);
    a = ao + a;
}
__device__ __forceinline__ void scan_maxplus(int &a, int &b) {
    mp_step<0x111>(a, b);
    mp_step<0x112>(a, b);
    mp_step<0x114>(a, b);
    mp_step<0x118>(a, b);
    mp_step<0x142, 0xA>(a, b);
    mp_step<0x143, 0xC>(a, b);
}
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ double min_step(double v) {
    const double id = 1e300;
    const int lo = dppu<CTRL, ROWMASK>(__double2loint(id), __double2loint(v));
    const int hi = dppu<CTRL, ROWMASK>(__double2hiint(id), __double2hiint(v));
    const double o = __hiloint2double(hi, lo);
    return o < v ? o : v;
}
__device__ __forceinline__ double scan_min_d(double v) {  // inclusive prefix min
    v = min_step<0x111>(v);
    v = min_step<0x112>(v);
    v = min_step<0x114>(v);
    v = min_step<0x118>(v);
    v = min_step<0x142, 0xA>(v);
    v = min_step<0x143, 0xC>(v);
    return v;
}

// ---- constant-offset lane exchanges without ds_bpermute: the compiler hoists a bpermute's
// lane-address computation out of the loops and keeps it live (or spills it) for the whole
// kernel -- ~20 VGPRs here -- while DPP / permlane forms need no address register.
// lane l + 1's value (lane 63: its own), as __shfl_down(v, 1): DPP wave_shl:1
__device__ __forceinline__ int down1(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xF, 0xF, false); }
__device__ __forceinline__ double down1d(double v) {
    return __hiloint2double(down1(__double2hiint(v)), down1(__double2loint(v)));
}
// lane 63 - l's value: row_mirror inside rows of 16, then row r <- row 3 - r
__device__ __forceinline__ int rev64(int v) { return xrow16(xrow32(dpp<0x140>(v))); }
__device__ __forceinline__ double rev64d(double v) {
    return __hiloint2double(rev64(__double2hiint(v)), rev64(__double2loint(v)));
}
// sum over the wave, in every lane (butterflies: quad swaps, half-row and row mirrors, row swaps)
__device__ __forceinline__ int wave_sum(int v) {
    v += xstep<0>(v);
    v += xstep<1>(v);
    v += xstep<2>(v);
    v += xstep<3>(v);
    v += xstep<4>(v);
    v += xstep<5>(v);
    return v;
}
// inclusive prefix argmin of (p, j, y) by better(): ties -> larger j, j < 0 = none
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ void pargmin_step(double &p, int32_t &j, int32_t &y) {
    const int lo = dppu<CTRL, ROWMASK>(0, __double2loint(p)), hi = dppu<CTRL, ROWMASK>(0, __double2hiint(p));
    const int oj = dppu<CTRL, ROWMASK>(-1, j), oy = dppu<CTRL, ROWMASK>(0, y);
    const double op = __hiloint2double(hi, lo);
    if (better(op, oj, p, j)) p = op, j = oj, y = oy;
}
__device__ __forceinline__ void prefix_argmin(double &p, int32_t &j, int32_t &y) {
    pargmin_step<0x111>(p, j, y);
    pargmin_step<0x112>(p, j, y);
    pargmin_step<0x114>(p, j, y);
    pargmin_step<0x118>(p, j, y);
    pargmin_step<0x142, 0xA>(p, j, y);
    pargmin_step<0x143, 0xC>(p, j, y);
}
// argmin over lanes [l, 64) (the suffix), in lane l
__device__ __forceinline__ void suffix_argmin(double &p, int32_t &j, int32_t &y) {
    double rp = rev64d(p);
    int32_t rj = rev64(j), ry = rev64(y);
    prefix_argmin(rp, rj, ry);
    p = rev64d(rp), j = rev64(rj), y = rev64(ry);
}
// max over lanes [l, 64), in lane l
__device__ __forceinline__ int suffix_max(int v) { return rev64(scan_max(rev64(v))); }

struct Ent {
    int32_t x, y, f, pw;  // pw = (p_local + 1) | span << 24
    __device__ int32_t p() const { return (pw & 0xFFFFFF) - 1; }
    __device__ int32_t sp() const { return (int32_t)((uint32_t)pw >> 24); }
};

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
#if HYMET_CHAIN_UNI
__device__ __forceinline__ int32_t U(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double Ud(double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)), __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
#else
__device__ __forceinline__ int32_t U(int32_t v) { return v; }
__device__ __forceinline__ double Ud(double v) { return v; }
#endif
// HYMET_CHAIN_UNI2: values every lane loads from the same LDS word (deque ends, list ends, the
// head suffix record, entries passed to insert_one) are wave-uniform but look divergent to the
// compiler, which then keeps the loop state derived from them (deque indices, list length) in
// VGPRs and runs their loops under exec masks; readfirstlane makes them SGPRs
#ifndef HYMET_CHAIN_UNI2
#define HYMET_CHAIN_UNI2 0
#endif
#if HYMET_CHAIN_UNI2
__device__ __forceinline__ int32_t UL(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int4 UL4(int4 v) { return make_int4(UL(v.x), UL(v.y), UL(v.z), UL(v.w)); }
__device__ __forceinline__ int2 UL2(int2 v) { return make_int2(UL(v.x), UL(v.y)); }
#else
__device__ __forceinline__ int32_t UL(int32_t v) { return v; }
__device__ __forceinline__ int4 UL4(int4 v) { return v; }
__device__ __forceinline__ int2 UL2(int2 v) { return v; }
#endif
__device__ __forceinline__ double rld(double v, int l) {
    return __hiloint2double(rl(__double2hiint(v), l), rl(__double2loint(v), l));
}
__device__ __forceinline__ int4 pack_st(double pr, int32_t j, int32_t y) {
    return make_int4(__double2loint(pr), __double2hiint(pr), j, y);
}
__device__ __forceinline__ double st_pr(const int4 &v) { return __hiloint2double(v.y, v.x); }

// First-pass groups of at most kMidMax anchors (and more than the lane kernel's kSmall) are
// chained by a wave with one LANE PER ANCHOR, the whole group in registers (chain_mid_group):
// the window trees become 64-bit lane masks, the RMQ one wave argmin, the inner walk one pass
// in the (y, idx) order through the same prefix scans the wave kernel's walk uses.  The
// general path single-steps these groups (repeat hits that do not chain colinearly) at
// ~2.2 us per anchor through its LDS list / deque / block-summary upkeep; this path takes
// ~1 us (tools/chain_prof on the real-anchor dumps, f/p digests identical: C4 first pass
// 10.53 -> 10.18 ms with the drain, Zymo backbones 19.53 -> 17.48 ms).  The long join's
// groups are chained anchors, which the general path commits in colinear batches: there the
// lane-per-anchor path measured 2-6 % slower, so it serves the first pass only.  0 disables.
#ifndef HYMET_CHAIN_MID
#define HYMET_CHAIN_MID 64
#endif
// chain_mid_group skips the inner walk when no inner-tree entry's f + span exceeds max_f
#ifndef HYMET_CHAIN_MIDSKIP
#define HYMET_CHAIN_MIDSKIP 1
#endif
constexpr int kMidMax = HYMET_CHAIN_MID;

// mg_lchain_rmq on one group of n <= 64 anchors, lane l = anchor l (lchain.c; the same
// decisions as chain_small_kernel's lane replay and the general path).  scr: 128 ints of LDS.
__device__ __forceinline__ void chain_mid_group(const ChainParams &P, int64_t g0, int n, bool qfirst, double c,
                                                int32_t *scr) {
    const int lane = threadIdx.x;
    const bool act = lane < n;
    const int jl = act ? lane : n - 1;
    const uint64_t yv = P.ay[g0 + jl];
    const int32_t X = P.ax[g0 + jl], Y = (int32_t)yv, SP = (int32_t)(yv >> 32 & 0xff);
    // walk order: the anchors by (y, idx) descending; lane w of the walk holds anchor wa
    int rank = 0;
    for (int m = 0; m < n; ++m) {
        const int32_t ym = __builtin_amdgcn_readlane(Y, m);
        rank += (ym < Y || (ym == Y && m < lane)) ? 1 : 0;
    }
    int32_t *perm = scr, *stamp = scr + 64;
    __builtin_amdgcn_wave_barrier();
    if (act) perm[n - 1 - rank] = lane;
    __builtin_amdgcn_wave_barrier();
    const int wa = act ? perm[lane] : 0;
    const int32_t wX = __shfl(X, wa, 64), wY = __shfl(Y, wa, 64), wSP = __shfl(SP, wa, 64);
    int32_t F = 0, PJ = -1;
    double PR = 0.0;
    uint64_t in_out = 0, in_in = 0;
    int i0 = 0, st = 0, st_in = 0;
    for (int i = 0; i < n; ++i) {
        const int32_t xi = __builtin_amdgcn_readlane(X, i), yi = __builtin_amdgcn_readlane(Y, i);
        int32_t max_f = __builtin_amdgcn_readlane(SP, i), max_j = -1;
        if (i0 < i && __builtin_amdgcn_readlane(X, i0) != xi) {  // [i0, i) enter both trees
            const uint64_t mk = (i >= 64 ? ~0ull : (1ull << i) - 1) & ~((1ull << i0) - 1);
            in_out |= mk;
            if (P.max_dist_inner > 0) in_in |= mk;
            if (mk >> lane & 1) PR = prio(F, X, Y, c);
            i0 = i;
        }
        // window starts: x never decreases along the group, so the leaving entries are a
        // prefix of [st, i) (the tree-size cap is >= 64 on this path: never binding)
        {
            const uint64_t lv = __ballot(lane >= st && lane < i && (int64_t)(uint32_t)xi > (int64_t)(uint32_t)X + P.max_dist);
            const int st2 = st + __popcll(lv);
            in_out &= ~((st2 >= 64 ? ~0ull : (1ull << st2) - 1) & ~((1ull << st) - 1));
            st = st2;
        }
        if (P.max_dist_inner > 0) {
            const uint64_t lv =
                __ballot(lane >= st_in && lane < i && (int64_t)(uint32_t)xi > (int64_t)(uint32_t)X + P.max_dist_inner);
            const int s2 = st_in + __popcll(lv);
            in_in &= ~((s2 >= 64 ? ~0ull : (1ull << s2) - 1) & ~((1ull << st_in) - 1));
            st_in = s2;
        }
        // RMQ over (yi - max_dist, yi); the query's anchor 0 also at y == yi; ties -> larger index
        const int32_t ylo = yi - P.max_dist;
        const bool cand = (in_out >> lane & 1) && Y > ylo && (Y < yi || (Y == yi && qfirst && lane == 0));
        double bp = cand ? PR : 0.0;
        int32_t bj = cand ? lane : -1, dummy = 0;
        wave_argmin(bp, bj, dummy);
        bj = U(bj);
        if (bj >= 0) {
            int32_t exact, width;
            const int32_t fb = __builtin_amdgcn_readlane(F, bj);
            const int32_t sc = fb + comput_sc(xi, yi, __builtin_amdgcn_readlane(X, bj), __builtin_amdgcn_readlane(Y, bj),
                                              __builtin_amdgcn_readlane(SP, bj), P.pen_gap, P.pen_skip, &exact, &width);
            if (width <= P.bw && sc > max_f) max_f = sc, max_j = bj;
            bool walk = !exact && in_in != 0 && yi > 0;
#if HYMET_CHAIN_MIDSKIP
            // a candidate scores at most f_j + span_j (comput_sc <= the candidate's span), so
            // when no inner-tree entry reaches past max_f the walk changes nothing (its t[]
            // stamps only matter within this iteration) -- the wave kernel's max-deque test
            if (walk) {
                const int ub = __builtin_amdgcn_readlane(scan_max((in_in >> lane & 1) ? F + SP : INT32_MIN), 63);
                if (ub <= max_f) walk = false;
            }
#endif
            if (walk) {
                // inner walk: tree entries with y <= yi - 1 by (y, idx) descending, down to
                // yi - max_dist_inner -- in walk lanes, a prefix scan of the sequential loop
                const int32_t wF = __shfl(F, wa, 64), wPJ = __shfl(PJ, wa, 64);
                const bool inw = act && (in_in >> wa & 1) && wY <= yi - 1 && wY >= yi - P.max_dist_inner;
                int32_t ex2, w2;
                const int32_t sc2 = wF + comput_sc(xi, yi, wX, wY, wSP, P.pen_gap, P.pen_skip, &ex2, &w2);
                const bool valid = inw && w2 <= P.bw;
                // t[p[q]] = i by every valid candidate q: candidate j is stamped when an earlier
                // one (walk order) points to it
                stamp[lane] = 64;
                __builtin_amdgcn_wave_barrier();
                if (valid && wPJ >= 0) atomicMin(&stamp[wPJ], lane);
                __builtin_amdgcn_wave_barrier();
                const bool stamped = valid && stamp[wa] < lane;
                const int incl = scan_max(valid ? sc2 : INT32_MIN);
                const int excl = max(shr1(incl, INT32_MIN), max_f);
                const bool imp = valid && sc2 > excl;
                int a = imp ? -1 : (stamped ? 1 : 0);
                int bb = imp ? 0 : kNegInf;
                scan_maxplus(a, bb);
                const int sk = max(a, bb);
                const uint64_t mB = __ballot(valid && !imp && stamped && sk > P.max_chn_skip);
                const int lim = mB ? __ffsll((unsigned long long)mB) : 64;  // lanes < lim are reached
                const uint64_t mI = __ballot(imp && lane < lim);
                if (mI) {
                    const int Lh = 63 - __clzll((long long)mI);
                    max_f = __builtin_amdgcn_readlane(sc2, Lh);
                    max_j = __builtin_amdgcn_readlane(wa, Lh);
                }
            }
        }
        if (lane == i) F = max_f, PJ = max_j;
    }
    if (act) {
        P.f[g0 + lane] = F;
        P.p[g0 + lane] = PJ < 0 ? -1 : g0 + PJ;
        if (HYMET_CHAIN_TZERO) P.t_global[g0 + lane] = 0;  // the backtrack's marks start cleared
    }
    __builtin_amdgcn_wave_barrier();
}

#if HYMET_CHAIN_WPE > 0
#define HYMET_CHAIN_ATTR __attribute__((amdgpu_waves_per_eu(HYMET_CHAIN_WPE)))
#else
#define HYMET_CHAIN_ATTR
#endif
// kLongPass only names the instantiation (the long-join re-chain, bw_long) so that profiles
// separate the two passes; the code is the same.
template <int kLongPass>
__global__ __launch_bounds__(64) HYMET_CHAIN_ATTR void chain_groups_kernel(ChainParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    unsigned char *sp = smem;
    int4 *ring = reinterpret_cast<int4 *>(sp);
    sp += kRing * sizeof(int4);
    int4 *ssum = reinterpret_cast<int4 *>(sp);  // kSumInts int4 per block (staircase + meta)
    sp += kSumRing * kSumInts * sizeof(int4);
    int4 *hc = reinterpret_cast<int4 *>(sp);
    sp += 64 * sizeof(int4);
    int4 *hsuf = reinterpret_cast<int4 *>(sp);  // (pr lo, pr hi, j, y): argmin of [k, 64) of block hb
    sp += 64 * sizeof(int4);
    int4 *bdq = reinterpret_cast<int4 *>(sp);  // 2 per element: (pr lo, pr hi, idx, y), (x, f, pw, -)
    sp += kBdq * 2 * sizeof(int4);
    int2 *lst = reinterpret_cast<int2 *>(sp);
    sp += kInnerCap * sizeof(int2);
    int2 *idq = reinterpret_cast<int2 *>(sp);  // (idx, f + span)
    sp += kIdq * sizeof(int2);
    int32_t *xring = reinterpret_cast<int32_t *>(sp);  // x of anchor j at [j & (kXRing - 1)]
    sp += kXRing * sizeof(int32_t);
    int32_t *blx = reinterpret_cast<int32_t *>(sp);  // x of block b's last anchor at [b & (kBlx - 1)]
    const double c = 0.5 * (double)P.pen_gap;
    const int32_t n_work = P.work_end ? min(P.n_work, *P.work_end) : P.n_work;
    // work list dealt over kChainStripes counters on separate lines (stripe s: positions
    // s + kChainStripes t), as in backtrack_long_kernel: one returning atomic per group on a
    // single address serialises at its L2 channel
    int stripe = (int)(blockIdx.x % kChainStripes), exhausted = 0;
    for (;;) {
        int w = 0;
        if (lane == 0) w = atomicAdd(P.work_counter + stripe * kChainCtrPad, 1);
        w = __builtin_amdgcn_readfirstlane(w);
        w = stripe + kChainStripes * w;
        if (w >= n_work) {
            if (++exhausted == kChainStripes) break;
            stripe = stripe + 1 == kChainStripes ? 0 : stripe + 1;  // this stripe is done: help the next
            continue;
        }
        const int g = P.order[w];
        GTIME_START
        const int64_t g0 = P.g_start[g];
        const int32_t n = (int32_t)(P.g_start[g + 1] - g0);
        const bool qfirst = P.g_qfirst[g] != 0;
        if constexpr (kMidMax > 0 && !kLongPass) {
            if (n <= kMidMax && P.cap_rmq_size >= 64) {
                chain_mid_group(P, g0, n, qfirst, c, reinterpret_cast<int32_t *>(smem + kRing * sizeof(int4)));
                GTIME_STOP;
                continue;
            }
        }
        int4 *gsum = P.sum + ((g0 >> 6) + g) * kGSumInts;
        int32_t hb = -1;        // block held by the head cache
        bool hsuf_ok = false;   // hsuf holds the suffix argmins of block hb
        uint64_t hmask = ~0ull;  // lanes of block hb whose full entry is in hc (x always is)
        int32_t hlow = 0;        // hsuf is valid for the suffixes [k, 64), k >= hlow
        int32_t i = 0;
        CPROF_DECL
        // anchor jl (local) as seen at iteration i: ring [i - kRing, i), head cache, else HBM
        auto fetch = [&](int32_t jl) -> Ent {
            Ent e;
            int4 v;
            if (i - jl <= kRing) {
                v = ring[jl & kRingMask];
            } else if ((jl >> 6) == hb && (hmask >> (jl & 63) & 1)) {
                v = hc[jl & 63];
            } else {
                CCOUNT(0);
                const int32_t x = P.ax[g0 + jl];
                const uint64_t y = P.ay[g0 + jl];
#if HYMET_CHAIN_HNOP
                v = make_int4(x, (int32_t)y, ld_l2(P.f + g0 + jl), (int32_t)((uint32_t)(y >> 32 & 0xff) << 24));
#else
                const int64_t pp = ld_l2(P.p + g0 + jl);
                v = make_int4(x, (int32_t)y, ld_l2(P.f + g0 + jl),
                              (int32_t)((pp < 0 ? 0u : (uint32_t)(pp - g0 + 1)) | (uint32_t)(y >> 32 & 0xff) << 24));
#endif
            }
            e.x = v.x, e.y = v.y, e.f = v.z, e.pw = v.w;
            return e;
        };
        // the same with p (the inner walk): the ring, else HBM -- head-cache entries carry no p
        auto fetch_p = [&](int32_t jl) -> Ent {
#if HYMET_CHAIN_HNOP
            Ent e;
            int4 v;
            if (i - jl <= kRing) {
                v = ring[jl & kRingMask];
            } else {
                const int32_t x = P.ax[g0 + jl];
                const uint64_t y = P.ay[g0 + jl];
                const int64_t pp = ld_l2(P.p + g0 + jl);
                v = make_int4(x, (int32_t)y, ld_l2(P.f + g0 + jl),
                              (int32_t)((pp < 0 ? 0u : (uint32_t)(pp - g0 + 1)) | (uint32_t)(y >> 32 & 0xff) << 24));
            }
            e.x = v.x, e.y = v.y, e.f = v.z, e.pw = v.w;
            return e;
#else
            return fetch(jl);
#endif
        };
        // x of anchor jl (local) at iteration i, for the window-start probes: the x ring (last
        // kXRing anchors), the head cache, else a plain load of ax
        auto fetch_x = [&](int32_t jl) -> int32_t {
            if (i - jl <= kXRing) return xring[jl & (kXRing - 1)];
            if ((jl >> 6) == hb) return hc[jl & 63].x;
            return P.ax[g0 + jl];
        };
        auto fetch_y = [&](int32_t jl) -> int32_t {
            if (i - jl <= kRing) return ring[jl & kRingMask].y;
            if ((jl >> 6) == hb && (hmask >> (jl & 63) & 1)) return hc[jl & 63].y;
            return (int32_t)P.ay[g0 + jl];
        };
        int32_t i0 = 0, st = 0, st_in = 0;
        bool t_used = false;  // the overflow walk stamped t_global
        // head-cache prefetch (HYMET_CHAIN_HCPF: 1 both passes, 2 the long join only): when the
        // head cache takes block b, block b + 1's x, y, f are loaded into registers (p-less, as
        // every HBM entry fetch), so the next window-start block change does not wait on HBM
        constexpr bool kHcpf = HYMET_CHAIN_HCPF == 1 || (HYMET_CHAIN_HCPF == 2 && kLongPass);
        static_assert(!kHcpf || HYMET_CHAIN_HNOP, "the prefetched head entries carry no p");
        int32_t pfb = -1, pf_x = 0, pf_ylo = 0, pf_yhi = 0, pf_f = 0;  // block pfb's entries (lane l: entry l)
        auto hc_take = [&](int32_t b) -> Ent {  // entry (b << 6) + lane for the head cache
            if constexpr (!kHcpf) {
                return fetch((b << 6) + lane);
            } else {
                Ent e;
                if (b == pfb) {
                    e.x = pf_x, e.y = pf_ylo, e.f = pf_f;
                    e.pw = (int32_t)(((uint32_t)pf_yhi & 0xff) << 24);
                } else {
                    e = fetch((b << 6) + lane);
                }
                const int32_t jn = ((b + 1) << 6) + lane;
                if (((b + 1) << 6) + 63 < i0) {
                    const int32_t *ay32 = reinterpret_cast<const int32_t *>(P.ay + g0 + jn);
                    pf_x = P.ax[g0 + jn], pf_ylo = ay32[0], pf_yhi = ay32[1];
                    pf_f = ld_l2(P.f + g0 + jn);
                    pfb = b + 1;
                }
                return e;
            }
        };
        auto sum_at = [&](int32_t b, int k) -> int4 {  // word k of block b's summary
            if ((i0 >> 6) - b <= kSumRing) return ssum[(b & (kSumRing - 1)) * kSumInts + k];
            return ld_l2(gsum + (int64_t)b * kGSumInts + k);
        };
        // best (priority, index) over window entries [st, i0) with ylo < y < yq (quirk: y == yq
        // allowed for the query's anchor 0): per complete block the first staircase entry below
        // yq, entries of the partial head/tail blocks, rescans where a summary cannot decide
        auto window_best = [&](int32_t yq, int32_t ylo, bool quirk, double &bp, int32_t &bj) {
            const int32_t fb = (st + 63) >> 6, fe = i0 >> 6;
            auto in_q = [&](int32_t y, int32_t j) { return y > ylo && (y < yq || (quirk && y == yq && qfirst && j == 0)); };
            bp = 0.0, bj = -1;
            auto scan = [&](int32_t a, int32_t e) {  // entries [a, e), e - a <= 64
                const int32_t j = a + lane;
                if (j < e) {
                    const Ent en = fetch(j);
                    if (in_q(en.y, j)) {
                        const double pr = prio(en.f, en.x, en.y, c);
                        if (better(pr, j, bp, bj)) bp = pr, bj = j;
                    }
                }
            };
#if HYMET_CHAIN_HLEAN
            if (st < (fb << 6) && (st >> 6) == hb && hmask != ~0ull) {  // lean head cache: load it in full
                const Ent e = fetch((hb << 6) + lane);
                __builtin_amdgcn_wave_barrier();
                hc[lane] = make_int4(e.x, e.y, e.f, e.pw);
                __builtin_amdgcn_wave_barrier();
                hmask = ~0ull;
            }
#endif
            if (st < (fb << 6)) scan(st, min(fb << 6, i0));             // head
            if (fe >= fb && (fe << 6) < i0) scan(max(fe << 6, st), i0);  // tail
            for (int32_t base = fb; base < fe; base += 64) {
                const int32_t b = base + lane;
                bool rescan = false;
                if (b < fe) {
                    const int4 meta = sum_at(b, kStair);
                    if (quirk && qfirst && b == 0) {
                        rescan = true;  // the index-0 quirk admits y == yq
                    } else if (!(meta.y <= ylo || meta.x >= yq)) {
                        const int ns = meta.z & 255;
                        int k = 0;
                        int4 v = make_int4(0, 0, -1, 0);
                        for (; k < ns; ++k) {
                            v = sum_at(b, k);
                            if (v.w < yq) break;
                        }
                        if (k == ns) {
                            rescan = (meta.z & 256) != 0;  // truncated staircase
                        } else if (v.w > ylo) {
                            if (better(st_pr(v), v.z, bp, bj)) bp = st_pr(v), bj = v.z;
                        } else {
                            rescan = true;  // the best below yq lies at or below ylo
                        }
                    }
                }
                uint64_t m = __ballot(rescan);
                while (m) {
                    const int l = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    scan((base + l) << 6, ((base + l) << 6) + 64);
                }
            }
            int32_t dummy = 0;
            wave_argmin(bp, bj, dummy);
            bp = Ud(bp), bj = U(bj);
        };
        // inner list: ring-deque, logical k at lst[(lh + k) & (kInnerCap - 1)]; ends cached
        int ni = 0, lh = 0;
        int32_t lfy = 0, lfj = -1, lby = 0, lbj = -1;  // front / back keys
        bool overflow = false;
        auto L = [&](int k) -> int2 & { return lst[(lh + k) & (kInnerCap - 1)]; };
        auto reload_ends = [&]() {
            if (ni > 0) {
                const int2 a = UL2(L(0)), b = UL2(L(ni - 1));
                lfy = a.x, lfj = a.y, lby = b.x, lbj = b.y;
            }
        };
        // block deque [bh, bt) of complete blocks by their argmin, monotone (front = best)
        int bh = 0, bt = 0;
        bool bok = true;
        double bf_pr = 0.0, bb_pr = 0.0;
        int32_t bf_j = -1, bf_y = 0, bb_j = -1;
        int4 bf_e = make_int4(0, 0, 0, 0);  // front argmin entry (x, f, pw)
        // running argmin of the partial tail block [i0 & ~63, i0) (ignoring y)
        double t_pr = 0.0;
        int32_t t_j = -1, t_y = 0;
        // inner max-deque of f_j + span_j over [st_in, i0); front/back values cached
        int ih = 0, it = 0;
        bool iok = true;
        int32_t if_v = 0, ib_v = 0;
        __builtin_amdgcn_wave_barrier();
        // anchor chunks in registers, lane l holding anchor (chunk base + l): the current one
        // (cx, cy), the next (nx, ny) and the one after (nnx, nny).  Only x's low word is kept
        // (x >> 32 is the group's constant); y keeps the query span in bits 32..39.
        int32_t cx = 0, nx = 0, nnx = 0;
        uint64_t cy = 0, ny = 0, nny = 0;
        // unconditional loads (index clamped to the group): a `b < n ? load : 0` select made
        // the compiler land each prefetch in a temporary and wait for it (vmcnt) to copy it
        // into place, so the prefetch was synchronous.  Lanes past the group end hold copies of
        // its last anchor, which nothing reads (batches stop at the group end).
        auto ldx = [&](int32_t b) -> int32_t { return P.ax[g0 + min(b, n - 1)]; };
        auto ldy = [&](int32_t b) -> uint64_t { return P.ay[g0 + min(b, n - 1)]; };
        Ent prev{0, 0, 0, 0};  // anchor i-1
        // block b complete: staircase summary -- S1 = argmin, S(k+1) = argmin over y < y(Sk),
        // i.e. the entries better than every entry with y <= theirs, by y descending; the
        // best of (block, y < Y) is the first S with y < Y -- then the argmin joins the deque
        auto complete_block = [&](int32_t b) {
            AMARK(cb_begin);
            const int32_t jl = (b << 6) + lane;
            const Ent e = fetch(jl);
            const double pl = prio(e.f, e.x, e.y, c);
            bool rec = true;
            uint64_t recm;
            int rank = 0;  // records with larger y (records have distinct y)
            int32_t ymn = e.y, ymx = e.y;
            // y strictly increasing along the block (a colinear stretch): the entries with
            // y <= y_l are lanes [0, l], so l is a record iff it is the prefix best there
            // (ties -> the larger index, i.e. l itself: pl equals the inclusive prefix min),
            // its rank is the number of records in higher lanes, and the y range is lanes 0, 63
            const int32_t ynx = down1(e.y);
            if (__ballot(lane == 63 || e.y < ynx) == ~0ull) {
#if HYMET_CHAIN_CBFAST
#if HYMET_CHAIN_BMONO
                // priorities non-increasing along the block (a colinear chain): every lane is
                // its prefix's best, no scan needed
                const double plp = __hiloint2double(shr1(__double2hiint(pl), __double2hiint(pl)), shr1(__double2loint(pl), __double2loint(pl)));
                if (__ballot(!(plp < pl)) == ~0ull) rec = true;
                else
#endif
                rec = scan_min_d(pl) == pl;
                recm = __ballot(rec);
                rank = __popcll(lane == 63 ? 0ull : recm >> (lane + 1));
                ymn = rl(e.y, 0), ymx = rl(e.y, 63);
#else
                double bp = pl;
                int32_t bj = jl;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const double op = __shfl_up(bp, d, 64);
                    const int32_t oj = __shfl_up(bj, d, 64);
                    if (lane >= d && better(op, oj, bp, bj)) bp = op, bj = oj;
                }
                rec = bj == jl;
                recm = __ballot(rec);
                for (uint64_t m = recm; m;) {
                    const int k = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    rank += rl(e.y, k) > e.y;
                }
                wave_minmax(ymn, ymx);
#endif
            } else {
                for (int k = 0; k < 64; ++k) {
                    const int32_t yk = rl(e.y, k);
                    const double pk = rld(pl, k);
                    if (k != lane && yk <= e.y && better(pk, (b << 6) + k, pl, jl)) rec = false;
                }
                recm = __ballot(rec);
                for (uint64_t m = recm; m;) {
                    const int k = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1;
                    rank += rl(e.y, k) > e.y;
                }
                wave_minmax(ymn, ymx);
            }
            const int nrec = __popcll(recm);
            int32_t mw = 0;
#if HYMET_CHAIN_HLEAN
            // suffix records: lane l is one iff it beats every lane > l (ties -> larger index);
            // priorities non-increasing along the block leave lane 63 alone.  meta.w: lanes of
            // slots 1..3 (6 bits each), the slot count (bits 18..20) and the lowest lane whose
            // suffix the kept slots cover (bits 21..26)
            uint64_t srm = 1ull << 63;
            if (__ballot(lane == 63 || !(pl < down1d(pl))) != ~0ull) {
                double sp_ = pl;
                int32_t sj = jl, sy = e.y;
                suffix_argmin(sp_, sj, sy);
                srm = __ballot(sj == jl);
            }
            const int sslot = __popcll(lane == 63 ? 0ull : srm >> (lane + 1));  // records above this lane
            {
                uint64_t m = srm & ~(1ull << 63);
                int ns = 1;
                for (; m && ns < kSufRec; ++ns) {
                    const int l = 63 - __clzll((long long)m);
                    m &= ~(1ull << l);
                    mw |= l << (6 * (ns - 1));
                }
                mw |= ns << 18;
                if (m) mw |= (64 - __clzll((long long)m)) << 21;
            }
#endif
            const int4 meta = make_int4(ymn, ymx, min(nrec, kStair) | (nrec > kStair ? 256 : 0), mw);
            int4 *ls = ssum + (b & (kSumRing - 1)) * kSumInts;
            int4 *gs = gsum + (int64_t)b * kGSumInts;
            __builtin_amdgcn_wave_barrier();
            if (rec && rank < kStair) {
                ls[rank] = pack_st(pl, jl, e.y);
                gs[rank] = pack_st(pl, jl, e.y);
            }
#if HYMET_CHAIN_HLEAN
            if ((srm >> lane & 1) && sslot < kSufRec) gs[kSumInts + sslot] = make_int4(e.x, e.y, e.f, e.pw);
#endif
            if (lane == 0) ls[kStair] = meta, gs[kStair] = meta;
#if HYMET_CHAIN_BLX
            if (lane == 63) blx[b & (kBlx - 1)] = e.x;
#endif
            __builtin_amdgcn_wave_barrier();
            if (!bok) return;
            const int l0 = __ffsll((unsigned long long)__ballot(rec && rank == 0)) - 1;
            const double apr = rld(pl, l0);
            const int32_t aj = (b << 6) + l0, ay = rl(e.y, l0);
            while (bt > bh && better(apr, aj, bb_pr, bb_j)) {
                --bt;
                if (bt > bh) {
                    const int4 v = UL4(bdq[((bt - 1) & (kBdq - 1)) * 2]);
                    bb_pr = st_pr(v), bb_j = v.z;
                }
            }
            if (bt - bh >= kBdq) {
                bok = false;
                return;
            }
            const int4 ex = make_int4(rl(e.x, l0), rl(e.f, l0), rl(e.pw, l0), 0);
            if (lane == 0) {
                bdq[(bt & (kBdq - 1)) * 2] = pack_st(apr, aj, ay);
                bdq[(bt & (kBdq - 1)) * 2 + 1] = ex;
            }
            if (bt == bh) bf_pr = apr, bf_j = aj, bf_y = ay, bf_e = ex;
            bb_pr = apr, bb_j = aj;
            ++bt;
            AMARK(cb_end);
        };
        // entry j (now final) enters the window: inner list, inner max-deque, tail argmin
        auto insert_one = [&](int32_t j, const Ent ej_in) {
            AMARK(ins_begin);
            const Ent ej{UL(ej_in.x), UL(ej_in.y), UL(ej_in.f), UL(ej_in.pw)};
            if (P.max_dist_inner > 0) {
                if (!overflow && ni >= kInnerCap) overflow = true;
                if (!overflow) {
                    if (ni == 0 || key_less(lby, lbj, ej.y, j)) {  // append (colinear)
                        if (lane == 0) L(ni) = make_int2(ej.y, j);
                        if (ni == 0) lfy = ej.y, lfj = j;
                        lby = ej.y, lbj = j;
                        ni++;
                    } else {
                        // position among the last <= 64 entries (entries > key form a suffix)
                        const int m = min(ni, 64), base = ni - m;
                        bool gt = false;
                        if (lane < m) {
                            const int2 v = L(base + lane);
                            gt = key_less(ej.y, j, v.x, v.y);
                        }
                        const int ngt = __popcll(__ballot(gt));
                        int pos;
                        if (ngt < m || base == 0) {
                            pos = ni - ngt;
                        } else {
                            CCOUNT(1);
                            int cnt = 0;
                            for (int k = lane; k < ni; k += 64) cnt += key_less(L(k).x, L(k).y, ej.y, j);
                            cnt = wave_sum(cnt);
                            pos = cnt;
                        }
                        for (int top = ni - 1; top >= pos; top -= 64) {  // shift [pos, ni) right by one
                            const int k = top - lane;
                            int2 v;
                            if (k >= pos) v = L(k);
                            __builtin_amdgcn_wave_barrier();
                            if (k >= pos) L(k + 1) = v;
                            __builtin_amdgcn_wave_barrier();
                        }
                        if (lane == 0) L(pos) = make_int2(ej.y, j);
                        __builtin_amdgcn_wave_barrier();
                        ni++;
                        if (pos == 0) lfy = ej.y, lfj = j;
                    }
                }
                if (iok) {  // max-deque push of f_j + span_j
                    const int32_t v = ej.f + ej.sp();
                    while (it > ih && ib_v <= v) {
                        --it;
                        if (it > ih) ib_v = UL(idq[(it - 1) & (kIdq - 1)].y);
                    }
                    if (it - ih >= kIdq) {
                        iok = false;
                    } else {
                        if (lane == 0) idq[it & (kIdq - 1)] = make_int2(j, v);
                        if (it == ih) if_v = v;
                        ib_v = v;
                        ++it;
                    }
                }
            }
            // running argmin of the tail block (ties -> larger j)
            const double pr = prio(ej.f, ej.x, ej.y, c);
            if ((j & 63) == 0 || !(t_pr < pr)) t_pr = pr, t_j = j, t_y = ej.y;
            if ((j & 63) == 63) complete_block(j >> 6);
            AMARK(ins_end);
        };
        int32_t cb = -128;  // base of the chunk in cx/cy; nx/ny hold the next one
        // make chunk (ii >> 6) current.  Called at the end of each iteration for the next i,
        // ahead of that iteration's f / p stores: the rotation's copies wait (vmcnt, counted in
        // issue order) for the previous prefetch, and would otherwise wait for those stores too.
        auto advance = [&](int32_t ii) {
            if ((ii >> 6) == (cb >> 6) || ii >= n) return;
            // three chunks in registers: the batch reads chunk c+1, loaded a chunk earlier.
            // The rotation is unconditional (a jump first reloads the chunks it shifts in),
            // so the new loads can land in nnx / nny's own registers.
            if ((ii >> 6) != (cb >> 6) + 1) {
                const int32_t b = (ii & ~63) + lane;
                nx = ldx(b), ny = ldy(b), nnx = ldx(b + 64), nny = ldy(b + 64);
            }
            // the rotation as opaque moves ahead of the loads: as plain assignments they became
            // the merge's phi copies, placed after the loads -- which then had to land in
            // temporaries and be waited for (vmcnt) before the copy
            asm volatile("v_mov_b32 %0, %1" : "=v"(cx) : "v"(nx));
            asm volatile("v_mov_b64 %0, %1" : "=v"(cy) : "v"(ny));
            asm volatile("v_mov_b32 %0, %1" : "=v"(nx) : "v"(nnx));
            asm volatile("v_mov_b64 %0, %1" : "=v"(ny) : "v"(nny));
            cb = ii & ~63;
            nnx = ldx(cb + 128 + lane), nny = ldy(cb + 128 + lane);
        };
        // next batch attempt: back-off after short batches, doubling from kSpecGap0 (1: a lone
        // off-chain anchor fails its own batch, and the next anchor -- back on the chain, whose
        // predecessor B is the anchor before the off-chain one -- starts one right away)
        int32_t spec_next = 0, spec_gap = kSpecGap0;
        for (; i < n;) {
            i = U(i), i0 = U(i0), st = U(st), st_in = U(st_in);
            GCNT(x, 1);
            CCOUNT(23);
            CPROF(7);
            advance(i);
            const int32_t xi = rl(cx, i & 63);
            const int32_t yi = rl((int32_t)cy, i & 63);
            const int32_t span_i = rl((int32_t)(cy >> 32 & 0xff), i & 63);
            int32_t max_f = span_i;
            int32_t max_j = -1;
            // ---- 1. i0 advances: insert [i0, i) into the window structures
#if HYMET_CHAIN_DRAIN
            // x never decreases along a group: when anchor i-1 is beyond max_dist of anchor i,
            // every entry before i is, so both windows empty at once -- [i0, i) is not inserted
            // (it would leave again at step 2), st / st_in jump to i and the deques and the
            // inner list are cleared (and exact again).  Entries below st are never read through
            // the structures again: a block they complete is only ever a head block, scanned by
            // entry, and the tail argmin is used only while st <= the tail block's start.  First
            // pass only: on the long join (bw_long = 100 kbp) the branch measured slower.
            if (!kLongPass && st < i && (int64_t)(uint32_t)xi > (int64_t)(uint32_t)prev.x + P.max_dist) {
                i0 = st = st_in = i;
                bh = bt;
                bok = true;
                ni = 0, lh = 0;
                overflow = false;
                ih = it;
                iok = true;
            }
#endif
            if (i0 < i && prev.x != xi) {
                for (int32_t j = i0; j < i; ++j) insert_one(j, j == i - 1 ? prev : fetch(j));
                i0 = i;
            }
            CPROF(0);
            // ---- 2. outer window start: lane-parallel probe, one block at a time
            AMARK(st_begin);
#ifdef HYMET_CHAIN_PROF
            bool hchg = false;  // a head change earlier in this iteration
#endif
            // cache st's block in hc when it sits beyond the ring
            auto head_take = [&]() {
                if (st < i && (st >> 6) < (i0 >> 6) && i - st > kRing && (st >> 6) != hb) {
                    const int32_t hb2 = st >> 6;
#ifdef HYMET_CHAIN_PROF
                    CCOUNT(20);
                    if (hchg) CCOUNT(21);
                    hchg = true;
#endif
#if HYMET_CHAIN_HLEAN
                    // x of every entry and the block's suffix records (lanes 1..4: slots 0..3,
                    // lane 0: the summary's meta word); the suffix argmins come from the records
                    const int32_t xl = ldx((hb2 << 6) + lane);
                    const int4 *gw = gsum + (int64_t)hb2 * kGSumInts + kStair;
                    const int4 w = ld_l2(gw + min(lane, kSufRec));
                    const uint32_t mw = (uint32_t)rl(w.w, 0);
                    {
                        const int nr = mw >> 18 & 7;
                        int4 rv = make_int4(rl(w.x, 1), rl(w.y, 1), rl(w.z, 1), rl(w.w, 1));
                        int32_t rlane = 63;
                        uint64_t msk = 1ull << 63;
#pragma unroll
                        for (int s = 1; s < kSufRec; ++s) {
                            if (nr > s) {
                                const int ls = mw >> (6 * (s - 1)) & 63;
                                msk |= 1ull << ls;
                                if (ls >= lane) rv = make_int4(rl(w.x, 1 + s), rl(w.y, 1 + s), rl(w.z, 1 + s), rl(w.w, 1 + s)), rlane = ls;
                            }
                        }
                        const double rp = prio(rv.z, rv.x, rv.y, c);
                        __builtin_amdgcn_wave_barrier();
                        hc[lane] = rlane == lane ? rv : make_int4(xl, 0, 0, 0);
                        hsuf[lane] = pack_st(rp, (hb2 << 6) + rlane, rv.y);
                        __builtin_amdgcn_wave_barrier();
                        hb = hb2;
                        hmask = msk;
                        hlow = mw >> 21 & 63;  // hsuf holds the suffixes from lane hlow on
                        hsuf_ok = true;
                        return;
                    }
#endif
                    const Ent e = hc_take(hb2);
                    __builtin_amdgcn_wave_barrier();
                    hc[lane] = make_int4(e.x, e.y, e.f, e.pw);
                    __builtin_amdgcn_wave_barrier();
                    hb = hb2;
                    hmask = ~0ull;
                    hlow = 0;
                    hsuf_ok = false;
                }
            };
            for (;;) {
                if (st >= i) break;
#if HYMET_CHAIN_BLX
                // complete blocks the window start passes whole (their last anchor does, and x
                // never decreases) are skipped by that anchor's x, without loading them; only
                // the block the start stops in is cached
                while ((st & 63) == 0 && (st >> 6) < (i0 >> 6) && (i0 >> 6) - (st >> 6) <= kBlx) {
                    const int32_t xl = blx[(st >> 6) & (kBlx - 1)];
                    if (!((int64_t)(uint32_t)xi > (int64_t)(uint32_t)xl + P.max_dist || i0 - (st | 63) > P.cap_rmq_size)) break;
                    st += 64;
                }
                if (st >= i) break;
                head_take();
#endif
                const int32_t bend = min(i, ((st >> 6) + 1) << 6);
                const int32_t j = st + lane;
                bool adv = false;
                if (j < bend) adv = (int64_t)(uint32_t)xi > (int64_t)(uint32_t)fetch_x(j) + P.max_dist || i0 - j > P.cap_rmq_size;
                const uint64_t m = __ballot(adv);
                const int t = ~m ? __ffsll((unsigned long long)~m) - 1 : 64;  // lanes [0, t) advance
                st += min(t, bend - st);
                if (st < bend) break;
#if !HYMET_CHAIN_BLX
                head_take();
#endif
            }
            const int32_t fb = (st + 63) >> 6, fe = i0 >> 6;  // complete window blocks [fb, fe)
            while (bt > bh && (bf_j >> 6) < fb) {
                ++bh;
                if (bt > bh) {
                    const int4 v = UL4(bdq[(bh & (kBdq - 1)) * 2]);
                    bf_pr = st_pr(v), bf_j = v.z, bf_y = v.w;
                    bf_e = UL4(bdq[(bh & (kBdq - 1)) * 2 + 1]);
                }
            }
            if ((st & 63) && (st >> 6) < fe && ((st >> 6) != hb || !hsuf_ok || (st & 63) < hlow)) {
                // partial head block: cache it with its suffix argmins [lane, 64)
                CCOUNT(5);
                const int32_t b = st >> 6, j = (b << 6) + lane;
                const Ent e = fetch(j);
                double pr = prio(e.f, e.x, e.y, c);
                int32_t pj = j, py = e.y;
#if HYMET_CHAIN_MONO
                // priorities non-increasing along the block: every suffix's argmin is lane 63
                const double pnx = down1d(pr);
                if (__ballot(lane == 63 || !(pr < pnx)) == ~0ull) {
                    pr = rld(pr, 63), pj = (b << 6) + 63, py = rl(e.y, 63);
                } else
#endif
                    suffix_argmin(pr, pj, py);
                __builtin_amdgcn_wave_barrier();
                hc[lane] = make_int4(e.x, e.y, e.f, e.pw);
                hsuf[lane] = pack_st(pr, pj, py);
                __builtin_amdgcn_wave_barrier();
                hb = b;
                hmask = ~0ull;
                hlow = 0;
                hsuf_ok = true;
            }
            CPROF(1);
            // ---- 3. inner window start
            AMARK(stin_begin);
            if (P.max_dist_inner > 0) {
                for (;;) {
                    if (st_in >= i) break;
                    const int32_t j = st_in + lane;
                    bool adv = false;
                    if (j < i) adv = (int64_t)(uint32_t)xi > (int64_t)(uint32_t)fetch_x(j) + P.max_dist_inner || i0 - j > P.cap_rmq_size;
                    const uint64_t m = __ballot(adv);
                    const int t = ~m ? __ffsll((unsigned long long)~m) - 1 : 64;
                    if (t > 1 && !overflow && ni > 0) {
                        // several entries leave: stable compaction of the list keeps j >= st_in + t
                        const int32_t lim = st_in + t;
#if HYMET_CHAIN_IPOP
                        // the list holds exactly the entries [st_in, i0), so when its first nl
                        // entries all leave they are the nl leaving ones (colinear: lowest y and
                        // index together) and are popped from the front
                        const int nl = max(0, min(lim, i0) - st_in);
                        if (nl <= ni) {
                            const int2 v = L(min(lane, ni - 1));
                            if (__ballot(lane < nl && v.y >= lim) == 0ull) {
                                lh = (lh + nl) & (kInnerCap - 1);
                                ni -= nl;
                                if (ni > 0) {
                                    const int2 a = UL2(L(0));
                                    lfy = a.x, lfj = a.y;
                                }
                                st_in += t;
                                if (t < 64) break;
                                continue;
                            }
                        }
#endif
                        int kept = 0;
                        for (int base = 0; base < ni; base += 64) {
                            const int kk = base + lane;
                            int2 v = make_int2(0, 0);
                            if (kk < ni) v = L(kk);
                            const bool keep = kk < ni && v.y >= lim;
                            const uint64_t mk = __ballot(keep);
                            const int dst = kept + __popcll(mk & ((1ull << lane) - 1));
                            __builtin_amdgcn_wave_barrier();
                            if (keep) L(dst) = v;
                            __builtin_amdgcn_wave_barrier();
                            kept += __popcll(mk);
                        }
                        ni = kept;
                        reload_ends();
                        st_in += t;
                        if (t < 64) break;
                        continue;
                    }
                    const int32_t yj = lane < t && j < i0 ? fetch_y(j) : 0;  // keys of the leaving entries
                    for (int l = 0; l < t; ++l) {  // erase the passed entries from the inner list
                        const int32_t jj = st_in + l;
                        if (jj >= i0 || overflow) continue;
                        const int32_t y = rl(yj, l);
                        if (y == lfy && jj == lfj) {  // front (colinear)
                            lh = (lh + 1) & (kInnerCap - 1);
                            ni--;
                            if (ni > 0) {
                                const int2 a = UL2(L(0));
                                lfy = a.x, lfj = a.y;
                            }
                            continue;
                        }
                        // near the front: shift [0, pos) right by one and pop the front slot
                        bool eq = false;
                        if (lane < min(ni, 64)) {
                            const int2 v = L(lane);
                            eq = v.x == y && v.y == jj;
                        }
                        const uint64_t me = __ballot(eq);
                        if (me) {
                            const int pos = __ffsll((unsigned long long)me) - 1;
                            int2 v;
                            if (lane < pos) v = L(lane);
                            __builtin_amdgcn_wave_barrier();
                            if (lane < pos) L(lane + 1) = v;
                            __builtin_amdgcn_wave_barrier();
                            lh = (lh + 1) & (kInnerCap - 1);
                            ni--;
                            reload_ends();
                            continue;
                        }
                        CCOUNT(2);
                        int cnt = 0;
                        for (int k = lane; k < ni; k += 64) cnt += key_less(L(k).x, L(k).y, y, jj);
                        cnt = wave_sum(cnt);
                        for (int b = cnt; b < ni - 1; b += 64) {  // shift (cnt, ni) left by one
                            const int k = b + lane + 1;
                            int2 v;
                            if (k < ni) v = L(k);
                            __builtin_amdgcn_wave_barrier();
                            if (k < ni) L(k - 1) = v;
                            __builtin_amdgcn_wave_barrier();
                        }
                        ni--;
                        reload_ends();
                    }
                    st_in += t;
                    if (t < 64) break;
                }
                while (it > ih && UL(idq[ih & (kIdq - 1)].x) < st_in) {
                    ++ih;
                    if (it > ih) if_v = UL(idq[ih & (kIdq - 1)].y);
                }
            }
            CPROF(6);
            AMARK(stin_end);
            // ---- 3b. colinear batch: assume each of the next L anchors chains onto its
            // predecessor (max-plus scan for f), then verify, lane-parallel, every decision the
            // sequential DP would take: the predecessor is the window's best priority (it beats
            // the pre-batch window best B0 and every earlier batch entry, ignoring y) and lies
            // in the krmq range, its score passes bw, and the inner walk cannot improve max_f.
            // The verified prefix is committed in bulk; the first failing anchor runs below.
            // Attempts back off after short batches (non-colinear stretches).
#ifdef HYMET_CHAIN_PROF
            if (i0 != i) CCOUNT(9);                            // no attempt: same x as the previous anchor
            else if (i == 0 || st >= i0) CCOUNT(19);           // no attempt: empty window
            else if (i < spec_next) CCOUNT(22);                // no attempt: back-off
#endif
            if (i0 == i && i > 0 && st < i0 && i >= spec_next) {
                const bool walk_ok = P.max_dist_inner <= 0 || (iok && !overflow);
                int Lb = min(64, n - i);
                // the batch's inner-list keys go into one gap: before G, the first list key above
                // the first inserted key (entry i); all the tail [gpos, ni) shifts in one round
                int gpos = ni;
                int32_t gy = INT32_MAX, gj = INT32_MAX;
                if (P.max_dist_inner > 0) Lb = min(Lb, kInnerCap - ni);
                // B: the best pre-batch window entry with y <= Y, Y = y of the last batch anchor,
                // a superset of the krmq range of every batch anchor with y <= Y (the others are
                // not committed); the batch starts only if B is the predecessor of its first anchor
                double b0p = 0.0;
                int32_t b0j = -1;
                int32_t batch_y = INT32_MAX;  // B's y bound: every committed anchor must lie at or below it
#if HYMET_CHAIN_YPREFIX
                if (!kLongPass && walk_ok && Lb >= 2) {  // the long join's chained anchors rarely break y order
                    const int offy = (i - cb) + lane;
                    const int32_t ylo_ = __shfl((int32_t)cy, offy & 63, 64), yhi_ = __shfl((int32_t)ny, offy & 63, 64);
                    const int32_t yl = offy < 64 ? ylo_ : yhi_;
                    const int32_t yp = shr1(yl, INT32_MIN);
                    const uint64_t brk = __ballot(lane >= 1 && lane < Lb && !(yp < yl));
                    if (brk) Lb = __ffsll((unsigned long long)brk) - 1;
                }
#endif
                if (walk_ok && Lb >= 2) {
                    const int offl = (i - cb) + Lb - 1;
                    const int32_t ymax = (int32_t)(offl < 64 ? rl((int32_t)cy, offl) : rl((int32_t)ny, offl - 64));
                    batch_y = ymax;
#if HYMET_CHAIN_B0FAST
                    // the window's best ignoring y (head suffix, block deque front, tail argmin:
                    // the O(1) sources step 4 uses) is B when its y <= Y -- the colinear case;
                    // only otherwise scan the block summaries
                    bool cert = st <= (fe << 6);
                    double gp = 0.0;
                    int32_t gj = -1, gy = 0;
                    if (cert) {
                        if (st < (fb << 6)) {
                            const int4 v = UL4(hsuf[st & 63]);
                            gp = st_pr(v), gj = v.z, gy = v.w;
                        }
                        if (fb < fe) {
                            if (!bok) cert = false;
                            else if (better(bf_pr, bf_j, gp, gj)) gp = bf_pr, gj = bf_j, gy = bf_y;
                        }
                        if ((fe << 6) < i0 && better(t_pr, t_j, gp, gj)) gp = t_pr, gj = t_j, gy = t_y;
                    }
                    if (cert && gj >= 0 && gy <= ymax) b0p = gp, b0j = gj;
                    else
#endif
                    window_best(ymax == INT32_MAX ? ymax : ymax + 1, INT32_MIN, false, b0p, b0j);
                }
                CCOUNT(8);
                GCNT(y, 1);
                if (b0j != i - 1) CCOUNT(10);
                if (!walk_ok) CCOUNT(11);
#if HYMET_CHAIN_B0ANY
                // the batch's first anchor takes B as its predecessor (B is the best entry of its
                // krmq range whenever it lies in that range: checked with the others below), so a
                // batch also starts right after an anchor that chained elsewhere
                if (b0j >= 0 && walk_ok && Lb >= 2) {
                    const Ent e0 = b0j == i - 1 ? prev : fetch(b0j);
#else
                if (b0j == i - 1 && walk_ok && Lb >= 2) {
                    const Ent e0 = prev;
#endif
                    AMARK(batch_begin);
                    // anchors k = i + lane from the chunk registers (cx: [cb, cb+64), nx: next 64)
                    const int off = (i - cb) + lane;
                    const int32_t kx_lo = __shfl(cx, off & 63, 64), kx_hi = __shfl(nx, off & 63, 64);
                    const uint64_t ky_lo = __shfl(cy, off & 63, 64), ky_hi = __shfl(ny, off & 63, 64);
                    const bool inb = lane < Lb;
                    const int32_t kx = off < 64 ? kx_lo : kx_hi;
                    const uint64_t kyy = off < 64 ? ky_lo : ky_hi;
                    const int32_t ky = (int32_t)kyy, ksp = (int32_t)(kyy >> 32 & 0xff);
                    const int32_t px = shr1(kx, e0.x), py = shr1(ky, e0.y), psp = shr1(ksp, e0.sp());
                    int32_t ex = 1, wd = 0;
                    const int32_t s = comput_sc(kx, ky, px, py, psp, P.pen_gap, P.pen_skip, &ex, &wd);
                    // ky <= batch_y: B covers y <= Y, Y = the y of the batch's LAST anchor, which is a
                    // superset of anchor k's krmq range (y < ky) only while ky <= Y -- y rises along
                    // the committed prefix (py < ky), but an anchor past it may fall below Y
                    bool ok = inb && kx != px && (int64_t)(uint32_t)kx <= (int64_t)(uint32_t)px + P.max_dist &&
                              py > ky - P.max_dist && py < ky && ky <= batch_y && wd <= P.bw;
                    // f_k = max(span_k, f_{k-1} + s_k): maps f -> max(f + a, b), composed by scan
                    int a = s, bb = ksp;
                    scan_maxplus(a, bb);
                    const int32_t fk = max(e0.f + a, bb);
                    const int32_t fp = shr1(fk, e0.f);
                    const bool linked = fp + s > ksp;  // sc > max_f = span: predecessor k-1 (lane 0: B)
                    // priorities of batch entries; the candidate of lane l is entry l-1
                    const double pk = prio(fk, kx, ky, c);
                    const int vk = inb ? fk + ksp : INT32_MIN;
#if HYMET_CHAIN_BMONO
                    // a colinear batch: priorities fall and f + span rises along it, so each
                    // prefix min / max is the lane's own value and the two scans are skipped
                    // (lanes past the batch only feed lanes that fail `inb`)
                    const double pkp = __hiloint2double(shr1(__double2hiint(pk), __double2hiint(pk)), shr1(__double2loint(pk), __double2loint(pk)));
                    const bool bmono = __ballot(!inb || (!(pkp < pk) && vk >= shr1(vk, vk))) == ~0ull;
                    double ipm = pk;
                    int vmx = vk;
                    if (!bmono) ipm = scan_min_d(inb ? pk : 1e300), vmx = scan_max(vk);
                    const int vex = shr1(vmx, INT32_MIN);  // max over the entries before k
#else
                    const double ipm = scan_min_d(inb ? pk : 1e300);
                    const int vex = shr1(scan_max(vk), INT32_MIN);  // max over the entries before k
#endif
                    const bool best_here = pk == ipm && !(b0p < pk);  // beats B0 and earlier entries
                    // (cross-lane operations run with every lane active: DPP reads of an
                    // inactive lane return the fallback value)
                    const bool cand_ok = shr1(best_here ? 1 : 0, 1) != 0;
                    // inner walk: max(f_j + span_j) over the inner window must not exceed f_k
                    bool wok = true;
                    if (P.max_dist_inner > 0 && !ex && ky > 0) wok = max(vex, it > ih ? if_v : INT32_MIN) <= fk;
                    // inner-list keys (y, idx) of entries i.. strictly increase (py < ky); they must
                    // all fall into the gap of the list before G
                    bool gap_own = true;  // this lane's own entry falls into the gap
                    if (P.max_dist_inner > 0 && ni > 0) {
                        const int32_t e0y = rl(ky, 0);
                        if (!key_less(lby, lbj, e0y, i)) {
                            const int m = min(ni, 64), base = ni - m;
                            bool gt = false;
                            int2 v = make_int2(0, 0);
                            if (lane < m) {
                                v = L(base + lane);
                                gt = key_less(e0y, i, v.x, v.y);
                            }
                            const uint64_t mg = __ballot(gt);
                            const int ngt = __popcll(mg);
                            if (ngt == m && base > 0) {
                                gy = INT32_MIN;  // gap beyond the last 64 entries: no batch
                            } else {
                                gpos = ni - ngt;
                                const int lg = __ffsll((unsigned long long)mg) - 1;
                                gy = rl(v.x, lg), gj = rl(v.y, lg);
                            }
                        }
                        // entry k-1 (k = i + lane, lane >= 1) is inserted at anchor k
                        if (lane >= 1 && !key_less(py, i + lane - 1, gy, gj)) ok = false;
                        gap_own = key_less(ky, i + lane, gy, gj);
                    }
#ifdef HYMET_CHAIN_PROF
                    const bool ok_geom = ok;
#endif
                    ok = ok && cand_ok && wok;
                    const uint64_t bad = __ballot(!ok);
                    const int acc = bad ? __ffsll((unsigned long long)bad) - 1 : 64;
#ifdef HYMET_CHAIN_PROF
                    if (acc < Lb) {
                        const int fl = acc;
                        const bool g_ = rl(ok_geom ? 1 : 0, fl), c_ = rl(cand_ok ? 1 : 0, fl), w_ = rl(wok ? 1 : 0, fl);
                        const bool xs = rl(kx != px ? 1 : 0, fl), yr = rl((py > ky - P.max_dist && py < ky) ? 1 : 0, fl);
                        if (!xs) CCOUNT(12);
                        else if (!yr) CCOUNT(13);
                        else if (!g_) CCOUNT(14);
                        else if (!c_) CCOUNT(15);
                        else if (!w_) CCOUNT(16);
                        else CCOUNT(17);  // list gap
                    }
                    _pcnt[18] += acc;
#endif
                    if (acc < 4) {
                        spec_next = i + spec_gap;
                        spec_gap = min(spec_gap * 2, 64);
                    } else {
                        spec_gap = kSpecGap0;
                    }
                    AMARK(batch_verified);
                    if (acc > 0) {
#if HYMET_CHAIN_INSALL
                        // the anchor after the batch (lane acc, or the next chunk for a full batch):
                        // a different x lets the last committed entry enter the window now
                        bool ins_all = false;
                        if (i + acc < n) {
                            const int offn = (i - cb) + 64;
                            const int32_t xn = acc < 64 ? rl(kx, acc) : rl(nx, offn - 64);
                            ins_all = xn != rl(kx, acc - 1) && rl(gap_own ? 1 : 0, acc - 1) != 0;
                        }
#else
                        const bool ins_all = false;
#endif
                        // the next iteration's chunks first: nothing below reads the chunk
                        // registers, and the rotation then waits on no store of this commit
                        advance(i + acc);
                        // commit anchors [i, i + acc): f, p, ring; insert entries [i, i + acc - 1)
                        const int32_t k = i + lane;
                        const int32_t pk_local = linked ? (lane == 0 ? b0j : k - 1) : -1;
                        const int32_t pw = (int32_t)((uint32_t)(pk_local + 1) | (uint32_t)ksp << 24);
                        if (lane < acc) {
#if !HYMET_CHAIN_LATE_FP
                            P.f[g0 + k] = fk;
                            P.p[g0 + k] = pk_local < 0 ? -1 : g0 + pk_local;
                            if (HYMET_CHAIN_TZERO) P.t_global[g0 + k] = 0;
#endif
                            ring[k & kRingMask] = make_int4(kx, ky, fk, pw);
                            xring[k & (kXRing - 1)] = kx;
                        }
                        __builtin_amdgcn_wave_barrier();
                        CCOUNT(7);
                        GCNT(z, 1);
                        GCNT(w, acc);
                        const int nins = ins_all ? acc : acc - 1;
                        if (nins > 0) {
                            if (P.max_dist_inner > 0) {
                                // list: shift [gpos, ni) right by nins, batch keys into [gpos, gpos + nins)
                                if (gpos < ni) {  // (the ring index is always in bounds: read unconditionally)
                                    const int kk = gpos + lane;
                                    const int2 v = L(kk);
                                    __builtin_amdgcn_wave_barrier();
                                    if (kk < ni) L(kk + nins) = v;
                                }
                                {
                                    if (lane < nins) L(gpos + lane) = make_int2(ky, k);
                                    __builtin_amdgcn_wave_barrier();
                                }
                                if (gpos == 0) lfy = rl(ky, 0), lfj = i;
                                if (gpos == ni) lby = rl(ky, nins - 1), lbj = i + nins - 1;
                                ni += nins;
                                // max-deque: pop the back while <= the batch maximum, then append
                                // the batch's suffix records (values greater than all later ones)
                                const int v = fk + ksp;
                                int run = lane < nins ? v : INT32_MIN;
                                int sfx;
#if HYMET_CHAIN_MONO
                                // f + span increasing along the batch (colinear): the last entry
                                // is the only record and the maximum
                                const int vnx = down1(v);
                                if (__ballot(lane >= nins - 1 || v < vnx) == ~0ull) {
                                    run = rl(v, nins - 1);
                                    sfx = lane < nins - 1 ? run : INT32_MIN;
                                } else
#endif
                                {
                                    run = suffix_max(run);
                                    sfx = down1(run);
                                    if (lane == 63) sfx = INT32_MIN;
                                }
                                const int vmax = rl(run, 0);
                                while (it > ih && ib_v <= vmax) {
                                    --it;
                                    if (it > ih) ib_v = UL(idq[(it - 1) & (kIdq - 1)].y);
                                }
                                const bool recd = lane < nins && v > sfx;
                                const uint64_t rm = __ballot(recd);
                                const int nr = __popcll(rm);
                                if (it - ih + nr > kIdq) {
                                    iok = false;
                                } else {
                                    const int rank = __popcll(rm & ((1ull << lane) - 1));
                                    if (recd) idq[(it + rank) & (kIdq - 1)] = make_int2(k, v);
                                    __builtin_amdgcn_wave_barrier();
                                    if (it == ih) if_v = rl(v, __ffsll((unsigned long long)rm) - 1);
                                    ib_v = rl(v, 63 - __clzll((long long)rm));
                                    it += nr;
                                }
                            }
                            // tail-block argmin, and blocks completed by the insertions
                            const int32_t nb0 = i >> 6, nb1 = (i + nins) >> 6;
                            for (int32_t b = nb0; b < nb1; ++b) complete_block(b);
#if HYMET_CHAIN_MONO
                            // the last inserted entry is the batch's prefix minimum (priorities fall
                            // along a colinear chain): it is the argmin of any suffix of the batch,
                            // so the tail block's argmin is it (or the old tail's, no block completed)
                            const double pl_last = rld(pk, nins - 1);
                            if (((i + nins) & 63) == 0) {
                                t_pr = 0.0, t_j = -1, t_y = 0;  // the tail block is empty
                            } else if (rld(ipm, nins - 1) == pl_last) {
                                // the old tail [i & ~63, i) competes only if no block completed
                                if (nb1 > nb0 || (i & 63) == 0 || t_j < 0 || !(t_pr < pl_last))
                                    t_pr = pl_last, t_j = i + nins - 1, t_y = rl(ky, nins - 1);
                            } else
#endif
                            {
                                const int32_t tb = (i + nins) & ~63, j = tb + lane;
                                double tp = 0.0;
                                int32_t tj = -1, ty = 0;
                                if (j < i + nins) {
                                    const Ent e = fetch(j);
                                    tp = prio(e.f, e.x, e.y, c), tj = j, ty = e.y;
                                }
                                wave_argmin(tp, tj, ty);
                                t_pr = Ud(tp), t_j = U(tj), t_y = U(ty);
                            }
                            i0 = i + nins;
                        }
                        const int l = acc - 1;
#if HYMET_CHAIN_LATE_FP
                        // the batch's f / p stores go last: a vector-memory wait inside the commit
                        // (e.g. a spill reload) would otherwise wait for them too (vmcnt is in order)
                        if (lane < acc) {
                            P.f[g0 + k] = fk;
                            P.p[g0 + k] = pk_local < 0 ? -1 : g0 + pk_local;
                            if (HYMET_CHAIN_TZERO) P.t_global[g0 + k] = 0;
                        }
#endif
                        prev.x = rl(kx, l), prev.y = rl(ky, l), prev.f = rl(fk, l), prev.pw = rl(pw, l);
                        i += acc;
                        AMARK(batch_end);
                        continue;
                    }
                }
            }
            CPROF(2);
            // ---- 4. RMQ over the outer window [st, i0)
            double bp = 0.0;
            int32_t bj = -1;
            Ent eb;  // the winner's entry
            bool have_eb = false;
            const int32_t ylo = yi - P.max_dist;
            auto in_range = [&](int32_t y, int32_t j) { return y > ylo && (y < yi || (y == yi && qfirst && j == 0)); };
            if (st < i0) {
                // best of the whole window ignoring y: head suffix, best complete block, tail block
                bool cert = st <= (fe << 6);  // else the window lies inside the partial tail block
                int32_t wy = 0, src = -1;
                if (cert) {
                    if (st < (fb << 6)) {  // partial head block (complete, cached with suffix argmins)
                        const int4 v = UL4(hsuf[st & 63]);
                        bp = st_pr(v), bj = v.z, wy = v.w, src = 0;
                    }
                    if (fb < fe) {
                        if (!bok) cert = false;
                        else if (better(bf_pr, bf_j, bp, bj)) bp = bf_pr, bj = bf_j, wy = bf_y, src = 1;
                    }
                    if ((fe << 6) < i0 && better(t_pr, t_j, bp, bj)) bp = t_pr, bj = t_j, wy = t_y, src = 2;
                }
                if (cert && bj >= 0 && in_range(wy, bj)) {
                    if (src == 1) eb.x = bf_e.x, eb.y = bf_y, eb.f = bf_e.y, eb.pw = bf_e.z, have_eb = true;
                } else {
                    CCOUNT(3);
                    if (cert && bj >= 0) CCOUNT(6);
                    window_best(yi, ylo, true, bp, bj);
                }
            }
            CPROF(3);
            if (bj >= 0) {
                int32_t exact, width;
                if (!have_eb) eb = bj == i - 1 ? prev : fetch(bj);
                const int32_t sc = eb.f + comput_sc(xi, yi, eb.x, eb.y, eb.sp(), P.pen_gap, P.pen_skip, &exact, &width);
                if (width <= P.bw && sc > max_f) max_f = sc, max_j = bj;
                const int32_t n_inner = i0 > st_in ? i0 - st_in : 0;
                bool walk = !exact && n_inner > 0 && yi > 0 && P.max_dist_inner > 0;
                if (walk && iok && it > ih && if_v <= max_f) walk = false;  // no candidate can beat max_f
                CPROF(5);
                if (walk) {
                    CCOUNT(4);
                    const int32_t ylo_in = yi - P.max_dist_inner;
                    if (!overflow) {
                        // walk the list downwards from the last entry with y <= yi - 1
                        int cnt = 0;
                        for (int e = lane; e < ni; e += 64) cnt += L(e).x < yi;
                        cnt = wave_sum(cnt);
                        int nsk = 0;
                        for (int top = cnt - 1; top >= 0; top -= 64) {
                            const int e = top - lane;
                            const int nl = min(64, top + 1);
                            int32_t yj = 0, jl = -1, sc_l = 0, w_l = INT32_MAX, pj = -1;
                            if (e >= 0) {
                                const int2 v = L(e);
                                yj = v.x, jl = v.y;
                                const Ent ej = fetch_p(jl);
                                int32_t ex;
                                sc_l = ej.f + comput_sc(xi, yi, ej.x, ej.y, ej.sp(), P.pen_gap, P.pen_skip, &ex, &w_l);
                                pj = ej.p();
                            }
                            const uint64_t mA = __ballot(e >= 0 && yj < ylo_in);
                            const int LA = mA ? __ffsll((unsigned long long)mA) - 1 : nl;  // y-bound break
                            const bool valid = lane < LA && w_l <= P.bw;
                            // t[p[j]] = i marks (a mark always points later in walk order)
                            if (valid && pj >= st_in && pj < i0) P.t_global[g0 + pj] = i + 1;
                            t_used = true;
                            __builtin_amdgcn_s_waitcnt(0);  // the stamps are in L2 before any lane reads one
                            const bool stamped = valid && ld_l2(P.t_global + g0 + jl) == i + 1;
                            // running max_f before each candidate: exclusive prefix max
                            const int incl = scan_max(valid ? sc_l : INT32_MIN);
                            const int excl = max(shr1(incl, INT32_MIN), max_f);
                            const bool imp = valid && sc_l > excl;
                            // n_skip: improve -> max(s-1, 0); stamped -> s+1; as max-plus maps s -> max(s+a, b)
                            int a = imp ? -1 : (valid && stamped ? 1 : 0);
                            int bb = imp ? 0 : kNegInf;
                            scan_maxplus(a, bb);
                            const int s = max(nsk + a, bb);
                            const uint64_t mB = __ballot(valid && !imp && stamped && s > P.max_chn_skip);
                            const int LB = mB ? __ffsll((unsigned long long)mB) - 1 : 64;
                            const int lim = min(LA, LB + 1);  // candidates the sequential loop reaches
                            const uint64_t mI = __ballot(imp && lane < lim);
                            if (mI) {
                                const int Lh = 63 - __clzll((long long)mI);
                                max_f = rl(sc_l, Lh);
                                max_j = rl(jl, Lh);
                            }
                            if (mB || LA < nl) break;
                            nsk = rl(s, 63);
                            __builtin_amdgcn_wave_barrier();
                        }
                    } else {
                        // overflow path: next candidate = largest (y, idx) below the previous one
                        int n_skip = 0;
                        int32_t cy_ = yi, cj = INT32_MIN;
                        bool first = true;
                        for (;;) {
                            int32_t by = INT32_MIN, bjl = INT32_MIN;
                            for (int32_t j = st_in + lane; j < i0; j += 64) {
                                const int32_t yj = fetch(j).y;
                                const bool below = first ? (yj <= yi - 1) : key_less(yj, j, cy_, cj);
                                if (below && (bjl == INT32_MIN || key_less(by, bjl, yj, j))) by = yj, bjl = j;
                            }
                            auto take = [&](int32_t oy, int32_t oj) {
                                if (oj != INT32_MIN && (bjl == INT32_MIN || key_less(by, bjl, oy, oj))) by = oy, bjl = oj;
                            };
                            take(xstep<0>(by), xstep<0>(bjl));
                            take(xstep<1>(by), xstep<1>(bjl));
                            take(xstep<2>(by), xstep<2>(bjl));
                            take(xstep<3>(by), xstep<3>(bjl));
                            take(xstep<4>(by), xstep<4>(bjl));
                            take(xstep<5>(by), xstep<5>(bjl));
                            if (bjl == INT32_MIN) break;
                            first = false;
                            cy_ = by, cj = bjl;
                            if (by < ylo_in) break;
                            const Ent ej = fetch_p(bjl);
                            int32_t ex, wl;
                            const int32_t sl = ej.f + comput_sc(xi, yi, ej.x, ej.y, ej.sp(), P.pen_gap, P.pen_skip, &ex, &wl);
                            if (wl <= P.bw) {
                                if (sl > max_f) {
                                    max_f = sl, max_j = bjl;
                                    if (n_skip > 0) --n_skip;
                                } else if (ld_l2(P.t_global + g0 + bjl) == i + 1) {
                                    if (++n_skip > P.max_chn_skip) break;
                                }
                                // stamp i + 1 (t arrives zeroed); every lane writes: program order
                                if (ej.p() >= 0) P.t_global[g0 + ej.p()] = i + 1;
                                t_used = true;
                            }
                        }
                    }
                }
            }
            CPROF(4);
            advance(i + 1);
            // every lane stores the same values: later global loads by any lane see them.  t is
            // cleared as each anchor is decided (the backtrack's marks start at 0; the walk's
            // stamps only ever land on earlier anchors, and are cleared at the group's end)
            P.f[g0 + i] = max_f;
            P.p[g0 + i] = max_j < 0 ? -1 : g0 + max_j;
            if (HYMET_CHAIN_TZERO) P.t_global[g0 + i] = 0;
            prev.x = xi, prev.y = yi, prev.f = max_f, prev.pw = (int32_t)((uint32_t)(max_j + 1) | (uint32_t)span_i << 24);
            if (lane == 0) {
                ring[i & kRingMask] = make_int4(prev.x, prev.y, prev.f, prev.pw);
                xring[i & (kXRing - 1)] = prev.x;
            }
            __builtin_amdgcn_wave_barrier();
            ++i;
        }
        if (t_used) {  // hand the backtrack a zeroed t again
            __builtin_amdgcn_wave_barrier();
            for (int32_t j = lane; j < n; j += 64) P.t_global[g0 + j] = 0;
        }
        CPROF_FLUSH;
        GTIME_STOP;
    }
}

struct BacktrackParams {
    const int64_t *g_start;
    const int32_t *f;
    const int64_t *p;
    int32_t *t;                // zeroed by the caller
    const int32_t *z_cnt;      // per group: length of its (f, idx)-ascending z list
    const int32_t *z_idx;      // per group, from g_start[g]: anchor indices by (f, idx) ascending
    int32_t n_groups;
    int min_cnt, min_sc, max_drop;
    int64_t long_min;          // groups above this size go to backtrack_long_kernel
    unsigned long long *prof;  // HYMET_BT_PROF: long-kernel counters (nullptr = off)
    // outputs (per group region = its anchor range)
    int64_t *chain_ids;        // anchor ids of each chain, end -> start, packed in the group's range
    uint64_t *chain_u;         // score<<32 | count, packed at the group's range start
    int64_t *chain_first;      // offset in chain_ids of each chain
    int32_t *n_chains;         // per group
};

// mg_chain_backtrack, one thread per group.  The walk from a start anchor follows p[] once:
// its path is recorded in chain_ids (this thread's own scratch), so mg_chain_bk_end's t = 2
// marks and its reset walk are not needed (p[i] < i: a path never revisits itself), and the
// chain is path[0, best end), left in walk order (end -> start; chain_list / chain_copy read it
// reversed).  Path nodes are marked as the walk passes them and the few past the best end
// unmarked afterwards, so no pass re-reads the path.  t after the backtrack: 0 = free, 1 = used
// by a walk whose chain was dropped (score or count below the minimum), 2 = in a kept chain
// (the long join reads the 2s of its queries, mm_map.hip mark_count / mark_compact).
// Paths run mostly down consecutive anchors, so the walk keeps a
// window of kBtWin (p, f, t) triples below the current node, loaded together (one memory
// round trip per window instead of one per step); the z scan batches its t probes the same
// way.  Windows are refilled after every walk, since a walk's t marks make them stale.
constexpr int kBtWin = 8;

// Groups larger than kBtLong anchors (HYMET_BT_LONG overrides it, for tests) (a long contig against a close strain: tens of thousands
// of anchors, nearly all in one chain) would leave a single lane walking them while the rest
// of the grid idles.  They get a whole wave each (work list + atomic counter): the z scan
// probes 64 entries per step (ballot), and the walk - whose state is wave-uniform, kept in
// SGPRs via readfirstlane - refills a 64-node (p, f, t) window with one coalesced load and
// reads each step's node from it with readlane.  A fence after each walk and L2 loads of t
// make the walk's marks visible to the next probes.
// (C4: threshold 1024 -> 128 took mm_backtrack 623 -> 301 ms per step once the wave kernel
// stopped issuing agent-scope fences; round 5, 128 -> 64: 1,247 -> 1,239 ms per step, 256:
// 1,277 -- profiles/r05_bt_long/)
constexpr int64_t kBtLong = 64;
// The wave kernel's work counters (backtrack_long_kernel): kBtStripes of them, kBtCtrPad
// ints apart, each atomic taking kBtGrab positions of its stripe
#ifndef HYMET_BT_GRAB
#define HYMET_BT_GRAB 1
#endif
#ifndef HYMET_BT_STRIPES
#define HYMET_BT_STRIPES 8
#endif
constexpr int kBtGrab = HYMET_BT_GRAB, kBtStripes = HYMET_BT_STRIPES, kBtCtrPad = 64;
// The wave kernel's walk window covers kBtChunks * 64 entries per memory round trip.
// Measured on C4: 4 chunks are slower than 1 (mm_backtrack.long 549 -> 814 ms per step) --
// most walks are short (an off-path anchor walks into a marked chain after a step or two);
// one chunk widening to four after two reloads measured the same as one (round 4).
#ifndef HYMET_BT_CHUNKS
#define HYMET_BT_CHUNKS 1
#endif
constexpr int kBtChunks = HYMET_BT_CHUNKS;
#ifndef HYMET_BT_PROBE
#define HYMET_BT_PROBE 4
#endif
constexpr int kBtProbe = HYMET_BT_PROBE;
// Starts whose predecessor is already used are settled from the probe's prefetched t / f of
// that predecessor, without a walk (no window load, no mark re-read).
#ifndef HYMET_BT_TRIV
#define HYMET_BT_TRIV 1
#endif  // z probe block: kBtProbe * 64 entries

__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
    return (int64_t)((uint64_t)(uint32_t)uni((int32_t)(v >> 32)) << 32 | (uint32_t)uni((int32_t)v));
}
__device__ __forceinline__ int64_t rlane64(int64_t v, int l) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(v >> 32), l);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)v, l);
    return (int64_t)((uint64_t)hi << 32 | lo);
}

// order: the chaining work list (groups of >= min_cnt anchors by descending size); the
// wave kernel takes its prefix of groups larger than long_min, biggest first
__global__ void bt_long_count_kernel(const int64_t *g_start, const int32_t *order, int32_t n_work, int64_t long_min,
                                     int32_t *cnt) {
    int lo = 0, hi = n_work;  // first w with size(order[w]) <= long_min
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const int g = order[mid];
        if (g_start[g + 1] - g_start[g] > long_min) lo = mid + 1;
        else hi = mid;
    }
    cnt[0] = lo;
    for (int k = 1; k <= kBtStripes; k++) cnt[k * kBtCtrPad] = 0;  // the wave kernel's work counters
}

__global__ __launch_bounds__(64) void backtrack_long_kernel(BacktrackParams P, const int32_t *list, const int32_t *cnt,
                                                            int32_t *counter) {
    // No lane-divergent branch anywhere in the loops: the compiler may let lanes that skip
    // an `if (lane == 0)` region run ahead into the next iteration, where a readfirstlane /
    // readlane / ballot would then see a partial wave.  Single-address stores are executed
    // by every lane (same value, same address); the work counter goes through LDS with
    // barriers (one wave per workgroup, so they cost nothing but force convergence).
    __shared__ int32_t s_w;
    const int lane = threadIdx.x;
    const int32_t n_long = uni(ld_l2(cnt));
    // The work list is dealt over kBtStripes counters (stripe s: list positions s + kBtStripes t),
    // each on its own 256-byte line: a returning atomic per group on one counter address
    // serialised at its L2 channel (~10^5 groups per launch: mm_backtrack.long 232 ms/step).
    // A wave starts on stripe blockIdx % kBtStripes and moves on when it runs dry.
    int stripe = (int)(blockIdx.x % kBtStripes), exhausted = 0;
    int32_t w = 0, w_end = 0;  // stripe tickets [w, w_end) taken by this wave
    for (;;) {
        if (w >= w_end) {  // the next kBtGrab positions of this wave's stripe
            for (;;) {
                if (lane == 0) s_w = atomicAdd(counter + stripe * kBtCtrPad, kBtGrab);
                __syncthreads();
                w = uni(s_w);
                __syncthreads();
                w_end = w + kBtGrab;
                if (stripe + kBtStripes * w < n_long || ++exhausted == kBtStripes) break;
                stripe = stripe + 1 == kBtStripes ? 0 : stripe + 1;  // this stripe is done: help the next
            }
            if (exhausted == kBtStripes) break;
        }
        const int32_t wcur = stripe + kBtStripes * w++;
        if (wcur >= n_long) {
            w = w_end;  // the rest of this grab is past the list's end
            continue;
        }
        const int32_t g = uni(list[wcur]);
        const int64_t g0 = uni64(P.g_start[g]);
        const int64_t z0 = g0, z1 = g0 + uni(P.z_cnt[g]);
        int64_t wpos = g0;
        int nc = 0;
        int64_t k = z1 - 1;
        uint64_t c_probe = 0, c_walk = 0, c_step = 0, c_reload = 0, t_walk = 0, t_post = 0;
        const uint64_t t_g0 = P.prof ? clock64() : 0;
        // Probe block: kBtProbe * 64 z entries (z index, then t mark: two dependent loads),
        // kept across walks.  A walk only marks anchors that were unmarked before it (the few
        // it unmarks again were marked by itself), so a "marked" reading never goes stale:
        // after a walk only the marks that read unmarked are re-read, from the cached z
        // indices (one round trip instead of two).  (Re-reading just the next candidate after
        // each walk was 2.6x slower: walks mark the upcoming candidates, so most re-reads
        // failed one round trip at a time.)
        int64_t ptop = -1;  // the block covers z positions (ptop - 64 * kBtProbe, ptop]
        // z entries (f >= min_sc) not yet marked: every mark is counted as it is kept, so the
        // probes stop once none is left (after a group's main chain the remaining z entries
        // are all marked, and reading them back cost a few dependent round trips per block)
        int64_t zrem = z1 - z0;
        int32_t zc[kBtProbe], tv[kBtProbe], zfv[kBtProbe];
        int64_t zpv[kBtProbe];  // f and p of the entries that read unmarked: a walk's start
#if HYMET_BT_TRIV
        int32_t tqv[kBtProbe], fqv[kBtProbe];  // t and f of their predecessors (t as read at the probe)
#endif
        bool stale = false;
        while (k >= z0 && zrem > 0) {
            if (ptop < 0 || k <= ptop - 64 * kBtProbe) {
                c_probe++;
                ptop = k;
                stale = false;
#pragma unroll
                for (int c = 0; c < kBtProbe; c++) {
                    const int64_t kk = k - 64 * c - lane;
                    zc[c] = kk >= z0 ? P.z_idx[kk] : 0;
                }
#pragma unroll
                for (int c = 0; c < kBtProbe; c++) {
                    const int64_t kk = k - 64 * c - lane;
                    tv[c] = kk >= z0 ? ld_l2(P.t + zc[c]) : 1;
                }
#pragma unroll
                for (int c = 0; c < kBtProbe; c++) {  // (f and p are read-only here: never stale)
                    zfv[c] = tv[c] == 0 ? P.f[zc[c]] : 0;
                    zpv[c] = tv[c] == 0 ? P.p[zc[c]] : -1;
                }
#if HYMET_BT_TRIV
#pragma unroll
                for (int c = 0; c < kBtProbe; c++) {
                    const bool q = tv[c] == 0 && zpv[c] >= 0;
                    tqv[c] = q ? ld_l2(P.t + zpv[c]) : 0;
                    fqv[c] = q ? P.f[zpv[c]] : 0;
                }
#endif
            } else if (stale) {  // a walk since the probe: re-read the marks (z indices stay valid)
                stale = false;
#pragma unroll
                for (int c = 0; c < kBtProbe; c++) {
                    const int64_t kk = ptop - 64 * c - lane;
                    if (kk >= z0 && kk <= k && tv[c] == 0) tv[c] = ld_l2(P.t + zc[c]);
                }
            }
            const int d = (int)(ptop - k);  // entries above k in the block are done
            int hit = -1;
            int32_t zsel = 0, zfsel = 0;
            int64_t zpsel = -1;
#if HYMET_BT_TRIV
            int32_t tqsel = 0, fqsel = 0;
#endif
#pragma unroll
            for (int c = kBtProbe - 1; c >= 0; c--) {  // the nearest unmarked entry at or below k wins
                const uint64_t m = __ballot(tv[c] == 0 && 64 * c + lane >= d);
                if (m) {
                    const int h = __ffsll((unsigned long long)m) - 1;
                    hit = 64 * c + h;
                    zsel = __builtin_amdgcn_readlane(zc[c], h);
                    zfsel = __builtin_amdgcn_readlane(zfv[c], h);
                    zpsel = rlane64(zpv[c], h);
#if HYMET_BT_TRIV
                    tqsel = __builtin_amdgcn_readlane(tqv[c], h);
                    fqsel = __builtin_amdgcn_readlane(fqv[c], h);
#endif
                }
            }
            hit = uni(hit);
            if (hit < 0) {
                k = ptop - 64 * kBtProbe;
                continue;
            }
            const int64_t zi = (int64_t)uni(zsel);
            k = ptop - hit - 1;
            const int32_t zf = uni(zfsel);
#if HYMET_BT_TRIV
            // a start whose predecessor was already used (or that has none) walks one node: its
            // score z.x - f[p] (or z.x) decides whether it stays used, and a one-anchor path is
            // never a chain (min_cnt >= 2).  No other mark changes, so the block stays fresh.
            if (P.min_cnt >= 2 && (zpsel < 0 || uni(tqsel) != 0)) {
                const int32_t sv = zpsel < 0 ? zf : zf - uni(fqsel);
                if (sv > 0) P.t[zi] = 1, zrem--;  // every lane: same value, same address
                c_walk++;
                continue;
            }
#endif
            stale = true;
            int64_t *buf = P.chain_ids + wpos;
            buf[0] = zi;  // every lane: same value, same address
            P.t[zi] = 2;  // path nodes are marked as recorded; those past the best end are unmarked after
            int64_t len = 1, nv = 0;  // recorded path nodes; chain = path[0, nv)
            int64_t zc_len = 1, zc_nv = 0;  // z entries among path[0, len) and path[0, nv) (the start is one)
            int32_t max_s = 0;
            int64_t nxt = uni64(zpsel);
            int64_t whi = -1;  // window: chunk c, lane l holds anchor whi - 64c - l
            int64_t wpc[kBtChunks];
            int32_t wfc[kBtChunks], wtc[kBtChunks];
#pragma unroll
            for (int c = 0; c < kBtChunks; c++) wpc[c] = -1, wfc[c] = 0, wtc[c] = 1;
            c_walk++;
            const uint64_t t_w0 = P.prof ? clock64() : 0;
            // Each round evaluates a RUN of candidates at once: lanes o..R of the window, where
            // every node's predecessor is the next lane's node (p[j] == j - 1, the common case
            // along a colinear chain).  The sequential loop's decisions over the run -- running
            // max of s = zf - f (nv = path length at the last strict increase), the max_drop
            // break, the break on an already-used node (after that node's max update) -- are a
            // prefix max and two ballots.  A run ends at the window edge or where p jumps.
            for (;;) {
                c_step++;
                if (nxt < 0) {  // the path reached the start of its chain
                    if (zf > max_s) max_s = zf, nv = len, zc_nv = zc_len;
                    break;
                }
                if (nxt > whi || nxt <= whi - 64 * kBtChunks) {
                    c_reload++;
                    whi = nxt;
#pragma unroll
                    for (int c = 0; c < kBtChunks; c++) {
                        const int64_t jj = nxt - 64 * c - lane;
                        const bool ok = jj >= g0;
                        wpc[c] = ok ? P.p[jj] : -1;
                        wfc[c] = ok ? P.f[jj] : 0;
                        wtc[c] = ok ? ld_l2(P.t + jj) : 1;
                    }
                }
                const int d = (int)(whi - nxt);
                const int cc = d >> 6, o = d & 63;  // chunk of nxt, and its lane there
                int64_t wp = wpc[0];
                int32_t wf = wfc[0], wt = wtc[0];
#pragma unroll
                for (int c = 1; c < kBtChunks; c++)
                    if (cc == c) wp = wpc[c], wf = wfc[c], wt = wtc[c];
                const int64_t j = whi - 64 * cc - lane;
                const bool in = lane >= o;
                const uint64_t ms = __ballot(in && (lane == 63 || wp != j - 1 || j - 1 < g0));
                const int R = uni(__ffsll((unsigned long long)ms) - 1);
                const bool cand = in && lane <= R;
                const int32_t sv = cand ? zf - wf : INT32_MIN;
                const int32_t incl = scan_max(sv);
                const int32_t ex = max(max_s, shr1(incl, INT32_MIN));
                const bool upd = cand && sv > ex;
                const bool drop = cand && !upd && (int64_t)ex - sv > P.max_drop;
                const uint64_t mdrop = __ballot(drop);
                const uint64_t mb = mdrop | __ballot(cand && wt != 0);
                const uint64_t mupd = __ballot(upd);
                int last = R, ulim = R;  // lanes o..last recorded; updates up to lane ulim count
                const bool done = mb != 0;
                if (done) {
                    const int E = uni(__ffsll((unsigned long long)mb) - 1);
                    last = E - 1;
                    ulim = (mdrop >> E) & 1 ? E - 1 : E;
                }
                const uint64_t lim = ulim < 0 ? 0ull : ulim >= 63 ? ~0ull : (2ull << ulim) - 1;
                const uint64_t mu = mupd & lim;
                const uint64_t mz = __ballot(lane >= o && lane <= last && wf >= P.min_sc);  // recorded z entries
                if (mu) {
                    const int u = 63 - __clzll((long long)mu);
                    nv = len + (u - o);
                    zc_nv = zc_len + __popcll(mz & ((1ull << u) - 1));  // path[0, nv) ends at lane u - 1
                    max_s = __builtin_amdgcn_readlane(incl, u);  // = s_u: it beat every earlier value
                }
                if (lane >= o && lane <= last) {
                    buf[len + (lane - o)] = j;
                    P.t[j] = 2;  // the walk never re-reads a node it has passed (p[i] < i)
                }
                len += last - o + 1;
                zc_len += __popcll(mz);
                if (done) break;
                nxt = rlane64(wp, R);  // predecessor of the run's last node
            }
            const uint64_t t_w1 = P.prof ? clock64() : 0;
            t_walk += t_w1 - t_w0;
            // the chain is path[0, nv): unmark the few nodes past the best end.  The marks are
            // only read back by this wave (its probes and later walks, through L2), so the
            // ordering needed is workgroup scope -- its stores completed at L2 -- not an
            // agent-scope fence (an L2 writeback: ~8 us round trips once thousands of waves
            // issued them).
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            for (int64_t a = nv + lane; a < len; a += 64) P.t[ld_l2(buf + a)] = 0;
            zrem -= zc_nv;  // path[0, nv) stays marked (in a chain or used), the rest was cleared
            const int32_t sc = nv == 0 ? 0 : max_s;
            if (sc >= P.min_sc && nv > 0 && nv >= P.min_cnt) {
                P.chain_u[g0 + nc] = (uint64_t)(uint32_t)sc << 32 | (uint32_t)nv;  // every lane: same value
                P.chain_first[g0 + nc] = wpos;
                nc++;
                wpos += nv;
            } else {
                for (int64_t a = lane; a < nv; a += 64) P.t[ld_l2(buf + a)] = 1;  // used, but in no chain
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            if (P.prof) t_post += clock64() - t_w1;
        }
        P.n_chains[g] = nc;
        if (P.prof) {  // every lane adds, lane 0 the value (no divergent region)
            const uint64_t v[8] = {1, c_probe, c_walk, c_step, c_reload, t_walk, t_post, clock64() - t_g0};
            for (int q = 0; q < 8; q++) atomicAdd(P.prof + q, lane == 0 ? (unsigned long long)v[q] : 0ull);
        }
    }
}


__global__ __launch_bounds__(64) void backtrack_groups_kernel(BacktrackParams P) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= P.n_groups) return;
    const int64_t g0 = P.g_start[g];
    if (P.g_start[g + 1] - g0 > P.long_min) return;  // backtrack_long_kernel
    int64_t wpos = g0;  // next free slot in chain_ids
    int nc = 0;
    const int64_t z0 = g0, z1 = g0 + P.z_cnt[g];
    int64_t k = z1 - 1;
    while (k >= z0) {
        // next z entry (descending) whose anchor is unmarked
        int32_t zc[kBtWin], tc[kBtWin];
#pragma unroll
        for (int u = 0; u < kBtWin; u++) zc[u] = k - u >= z0 ? P.z_idx[k - u] : 0;
#pragma unroll
        for (int u = 0; u < kBtWin; u++) tc[u] = k - u >= z0 ? P.t[zc[u]] : 1;
        int hit = -1;
#pragma unroll
        for (int u = kBtWin - 1; u >= 0; u--)
            if (tc[u] == 0) hit = u;
        if (hit < 0) {
            k -= kBtWin;
            continue;
        }
        int64_t zi = 0;
#pragma unroll
        for (int u = 0; u < kBtWin; u++)
            if (u == hit) zi = zc[u];
        k -= hit + 1;
        const int32_t zf = P.f[zi];
        int64_t *buf = P.chain_ids + wpos;
        int64_t len = 0, nv = 0;
        int32_t max_s = 0;
        int64_t i = zi, nxt = P.p[zi];
        int64_t whi = -1;  // window covers anchors (whi - kBtWin, whi]
        int64_t wp[kBtWin];
        int32_t wf[kBtWin], wt[kBtWin];
        for (;;) {
            buf[len++] = i;
            P.t[i] = 2;  // no revisits: marking as we go cannot change this walk's reads
            int32_t fn = 0, tn = 1;
            int64_t pn = -1;
            if (nxt >= 0) {
                if (nxt > whi || nxt <= whi - kBtWin) {
                    whi = nxt;
#pragma unroll
                    for (int u = 0; u < kBtWin; u++) {
                        const bool ok = nxt - u >= g0;
                        wp[u] = ok ? P.p[nxt - u] : -1;
                        wf[u] = ok ? P.f[nxt - u] : 0;
                        wt[u] = ok ? P.t[nxt - u] : 1;
                    }
                }
                const int64_t o = whi - nxt;
#pragma unroll
                for (int u = 0; u < kBtWin; u++)
                    if (o == u) fn = wf[u], tn = wt[u], pn = wp[u];
            }
            const int32_t s = nxt < 0 ? zf : zf - fn;
            if (s > max_s) {
                max_s = s;
                nv = len;
            } else if (max_s - s > P.max_drop) {
                break;
            }
            if (nxt < 0 || tn != 0) break;
            i = nxt;
            nxt = pn;
        }
        const int32_t sc = nv == 0 ? 0 : max_s;  // zf - f[best end] (zf if the chain reaches -1)
        for (int64_t a = nv; a < len; a++) P.t[buf[a]] = 0;  // past the best end: stays unmarked
        if (sc >= P.min_sc && nv > 0 && nv >= P.min_cnt) {  // kept end -> start (readers reverse)
            P.chain_u[g0 + nc] = (uint64_t)(uint32_t)sc << 32 | (uint32_t)nv;
            P.chain_first[g0 + nc] = wpos;
            nc++;
            wpos += nv;
        } else {
            for (int64_t a = 0; a < nv; a++) P.t[buf[a]] = 1;  // used, but in no chain
        }
    }
    P.n_chains[g] = nc;
}

}  // namespace


// ---- small groups: one LANE per group of <= kSmall anchors
// A wave spends ~30 us of fixed latency on every group it takes (work-list atomic, group
// bounds, the chunk loads, f/p stores), which made groups of 3-16 anchors more than half of
// the kernel's wave time on C4 anchors.  Here 64 such groups run side by side, each lane
// replaying mg_lchain_rmq (lchain.c; oracle/mm_oracle.c chain_group) on its group with the
// group in registers: the window trees become bit masks and brute-force scans over <= 24
// entries, the inner walk a scan of the (y, idx) order.  Same decisions, same f/p.
// 24 anchors (225 VGPRs, two waves per SIMD) measured fastest on the real-anchor dumps: C4
// first pass 11.35 -> 10.7 ms, Zymo-backbone 20.3 -> 19.5 ms (16: 146 VGPRs but the wave
// kernel single-steps the 17-24-anchor groups at ~2.3 us per anchor; 32: 262 VGPRs, one
// wave per SIMD, 11.3 / 23.5 ms).  Packing span, predecessor and mark into one register
// brings 32 anchors to 227 VGPRs (two waves per SIMD), but measured no better in the bench:
// C4 first pass 374.5 -> 371.7 ms/step, Zymo 976 -> 986 (long join 299 -> 332).
#ifndef HYMET_CHAIN_SMALL
#define HYMET_CHAIN_SMALL 24
#endif
constexpr int kSmall = HYMET_CHAIN_SMALL;  // <= 32 (window sets are 32-bit masks)
// The long join's cut: its groups are chained anchors, which the wave kernel's colinear batches
// commit faster than the lane kernel replays them from 17 anchors up (Zymo-backbone long join
// 7.50 -> 7.03 ms per launch on the dump; C4 unchanged).  The first pass keeps kSmall: there
// the 17-24-anchor groups are repeat hits the lane kernel handles best.
#ifndef HYMET_CHAIN_SMALL_LONG
#define HYMET_CHAIN_SMALL_LONG 16
#endif
constexpr int kSmallLong = HYMET_CHAIN_SMALL_LONG < kSmall ? HYMET_CHAIN_SMALL_LONG : kSmall;

// first work item whose group has <= small_max anchors (the list is size-descending)
// (also zeroes the wave kernel's work counter)
__global__ void chain_small_split_kernel(const int64_t *g_start, const int32_t *order, int32_t n_work, int32_t *split,
                                         int32_t *counter, int small_max) {
    if (threadIdx.x != 0) return;
    for (int k = 0; k < kChainStripes; k++) counter[k * kChainCtrPad] = 0;
    int32_t lo = 0, hi = n_work;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        const int g = order[mid];
        if (g_start[g + 1] - g_start[g] <= small_max) hi = mid;
        else lo = mid + 1;
    }
    *split = lo;
}

// profiling only: anchors of the work items the wave kernel takes ([0, *split)) into cnt[0] and
// of those the lane kernel takes into cnt[1] (the bytes of the two profile scopes); a grid-stride
// pass over the work list, one pair of global atomics per block
__global__ __launch_bounds__(256) void chain_work_anchors_kernel(const int64_t *g_start, const int32_t *order,
                                                                  int32_t n_work, const int32_t *split, int64_t *cnt) {
    __shared__ unsigned long long sw, ss;
    if (threadIdx.x == 0) sw = 0, ss = 0;
    __syncthreads();
    const int32_t sp = *split;
    unsigned long long w = 0, s = 0;
    for (int32_t k = blockIdx.x * 256 + threadIdx.x; k < n_work; k += gridDim.x * 256) {
        const int g = order[k];
        const unsigned long long a = (unsigned long long)(g_start[g + 1] - g_start[g]);
        if (k < sp) w += a;
        else s += a;
    }
    for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o), s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(&sw, w), atomicAdd(&ss, s);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(reinterpret_cast<unsigned long long *>(cnt), sw);
        atomicAdd(reinterpret_cast<unsigned long long *>(cnt + 1), ss);
    }
}

__global__ __launch_bounds__(64) void chain_small_kernel(ChainParams P, const int32_t *split) {
    const int32_t w = *split + (int32_t)(blockIdx.x * 64 + threadIdx.x);
    if (w >= P.n_work) return;
    const int g = P.order[w];
    const int64_t g0 = P.g_start[g];
    const int n = (int)(P.g_start[g + 1] - g0);
    const bool qfirst = P.g_qfirst[g] != 0;
    const double c = 0.5 * (double)P.pen_gap;
    int32_t X[kSmall], Y[kSmall], SP[kSmall], F[kSmall], PJ[kSmall], T[kSmall];
    int8_t ord[kSmall];  // local indices by (y, idx) ascending
    for (int j = 0; j < n; ++j) {
        const uint64_t y = P.ay[g0 + j];
        X[j] = P.ax[g0 + j], Y[j] = (int32_t)y, SP[j] = (int32_t)(y >> 32 & 0xff);
        F[j] = 0, PJ[j] = -1, T[j] = -1;
        int k = j;  // insertion by (y, idx): later j is the larger idx, so ties stay behind
        while (k > 0 && Y[ord[k - 1]] > Y[j]) {
            ord[k] = ord[k - 1];
            --k;
        }
        ord[k] = (int8_t)j;
    }
    uint32_t in_out = 0, in_in = 0;
    int size_out = 0, size_in = 0, i0 = 0, st = 0, st_in = 0;
    for (int i = 0; i < n; ++i) {
        const int32_t xi = X[i], yi = Y[i];
        int32_t max_f = SP[i], max_j = -1;
        if (i0 < i && X[i0] != xi) {
            for (int j = i0; j < i; ++j) {
                in_out |= 1u << j, size_out++;
                if (P.max_dist_inner > 0) in_in |= 1u << j, size_in++;
            }
            i0 = i;
        }
        while (st < i && ((int64_t)(uint32_t)xi > (int64_t)(uint32_t)X[st] + P.max_dist || size_out > P.cap_rmq_size)) {
            if (st < i0) in_out &= ~(1u << st), size_out--;
            ++st;
        }
        if (P.max_dist_inner > 0)
            while (st_in < i &&
                   ((int64_t)(uint32_t)xi > (int64_t)(uint32_t)X[st_in] + P.max_dist_inner || size_in > P.cap_rmq_size)) {
                if (st_in < i0) in_in &= ~(1u << st_in), size_in--;
                ++st_in;
            }
        // RMQ over (yi - max_dist, yi) in (y, idx) order; the query's anchor 0 also at y == yi
        double bp = 0.0;
        int32_t bj = -1;
        const int32_t ylo = yi - P.max_dist;
        for (uint32_t m = in_out; m; m &= m - 1) {
            const int j = __ffs(m) - 1;
            const int32_t yj = Y[j];
            if (yj > ylo && (yj < yi || (yj == yi && qfirst && j == 0))) {
                const double pr = prio(F[j], X[j], yj, c);
                if (better(pr, j, bp, bj)) bp = pr, bj = j;
            }
        }
        if (bj >= 0) {
            int32_t exact, width;
            const int32_t sc = F[bj] + comput_sc(xi, yi, X[bj], Y[bj], SP[bj], P.pen_gap, P.pen_skip, &exact, &width);
            if (width <= P.bw && sc > max_f) max_f = sc, max_j = bj;
            if (!exact && size_in > 0 && yi > 0) {
                const int32_t ylo_in = yi - P.max_dist_inner;
                int r = n - 1;  // last (y, idx) with y < yi
                while (r >= 0 && Y[ord[r]] >= yi) --r;
                int n_skip = 0;
                for (; r >= 0; --r) {
                    const int jj = ord[r];
                    if (Y[jj] < ylo_in) break;
                    if (!(in_in >> jj & 1)) continue;
                    int32_t ex2, w2;
                    const int32_t sc2 = F[jj] + comput_sc(xi, yi, X[jj], Y[jj], SP[jj], P.pen_gap, P.pen_skip, &ex2, &w2);
                    if (w2 <= P.bw) {
                        if (sc2 > max_f) {
                            max_f = sc2, max_j = jj;
                            if (n_skip > 0) --n_skip;
                        } else if (T[jj] == i) {
                            if (++n_skip > P.max_chn_skip) break;
                        }
                        if (PJ[jj] >= 0) T[PJ[jj]] = i;
                    }
                }
            }
        }
        F[i] = max_f, PJ[i] = max_j;
        P.f[g0 + i] = max_f;
        P.p[g0 + i] = max_j < 0 ? -1 : g0 + max_j;
        if (HYMET_CHAIN_TZERO) P.t_global[g0 + i] = 0;
    }
}

// The chaining launches for a work list: the small-group split, the wave kernel on the
// groups above kSmall anchors, the lane kernel on the rest.  `split` is device scratch.
int launch_chain_raw(hipStream_t st, const ChainParams &P0, int64_t blocks, int32_t *split) {
    ChainParams P = P0;
    hipLaunchKernelGGL(chain_small_split_kernel, dim3(1), dim3(64), 0, st, P.g_start, P.order, P.n_work, split,
                       P.work_counter, P.max_dist > 10000 ? kSmallLong : kSmall);
    HY_CHECK_LAUNCH("chain_small_split_kernel");
    P.work_end = split;
    const bool long_pass = P.max_dist > 10000;
    if (long_pass) hipLaunchKernelGGL(chain_groups_kernel<1>, dim3((unsigned)blocks), dim3(64), kChainLds, st, P);
    else hipLaunchKernelGGL(chain_groups_kernel<0>, dim3((unsigned)blocks), dim3(64), kChainLds, st, P);
    HY_CHECK_LAUNCH("chain_groups_kernel");
    hipLaunchKernelGGL(chain_small_kernel, dim3((unsigned)cdiv(P.n_work, 64)), dim3(64), 0, st, P, (const int32_t *)split);
    HY_CHECK_LAUNCH("chain_small_kernel");
    return HYMET_OK;
}

int launch_chain(hymet_ctx *ctx, const int32_t *ax, const uint64_t *ay, const int64_t *g_start, const uint8_t *g_qfirst,
                 const int32_t *order, int32_t n_work, int32_t *f, int64_t *p, int32_t *t_global, int max_dist,
                 int max_dist_inner, int bw, int max_chn_skip, int cap_rmq_size, float pen_gap, float pen_skip,
                 int64_t n_anchors, int64_t n_groups) {
    if (n_work <= 0) return HYMET_OK;
    DevBuf cnt, sum, split;
    const size_t n_sum = (size_t)(n_anchors >> 6) + (size_t)n_groups + 2;
    HY_HIP(sum.alloc(16 * kGSumInts * n_sum, ctx->stream));
    HY_HIP(cnt.alloc(4 * (size_t)kChainCtrPad * kChainStripes, ctx->stream));  // the wave kernel's striped work counters
    HY_HIP(split.alloc(4, ctx->stream));
    if (max_dist < bw) max_dist = bw;
    if (max_dist_inner <= 0 || max_dist_inner >= max_dist) max_dist_inner = 0;
    ChainParams P{ax, ay, g_start, g_qfirst, order, n_work, cnt.as<int32_t>(), f, p, t_global, sum.as<int4>(), max_dist, max_dist_inner, bw, max_chn_skip, cap_rmq_size, pen_gap, pen_skip, nullptr};
    // one wave per block, as many resident per CU as registers and LDS allow
    int64_t blocks = n_work;
    int per_cu = 0;
    const bool long_pass = max_dist > 10000;
    auto kern = long_pass ? chain_groups_kernel<1> : chain_groups_kernel<0>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, kChainLds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 8;
    static const int waves_env = getenv("HYMET_CHAIN_WAVES") ? atoi(getenv("HYMET_CHAIN_WAVES")) : 0;  // A/B: resident waves per CU
    if (waves_env > 0 && waves_env < per_cu) per_cu = waves_env;
    const int64_t cap = (int64_t)ctx->n_cu * per_cu;
    if (blocks > cap) blocks = cap;
    // two profile scopes, one kernel each: the wave kernel (groups above kSmall anchors, the
    // mid-group path included) and the lane kernel; each scope's algorithmic bytes are 28 per
    // anchor it chains (x, y read; f, p written), counted on the device from the work list
    const int slot = long_pass ? 2 : 0;
    hipStream_t st = ctx->stream;
    {
        ProfScope _ps(ctx, long_pass ? "mm_chain_long" : "mm_chain", slot, 28.0);
        hipLaunchKernelGGL(chain_small_split_kernel, dim3(1), dim3(64), 0, st, P.g_start, P.order, P.n_work,
                           split.as<int32_t>(), P.work_counter, long_pass ? kSmallLong : kSmall);
        HY_CHECK_LAUNCH("chain_small_split_kernel");
        if (int64_t *pc = prof_dev_slot(ctx, slot)) {
            const unsigned wb = (unsigned)std::min<int64_t>(cdiv(P.n_work, 256), 1024);
            hipLaunchKernelGGL(chain_work_anchors_kernel, dim3(wb), dim3(256), 0, st, P.g_start, P.order, P.n_work,
                               (const int32_t *)split.as<int32_t>(), pc);
            HY_CHECK_LAUNCH("chain_work_anchors_kernel");
        }
        P.work_end = split.as<int32_t>();
        if (long_pass) hipLaunchKernelGGL(chain_groups_kernel<1>, dim3((unsigned)blocks), dim3(64), kChainLds, st, P);
        else hipLaunchKernelGGL(chain_groups_kernel<0>, dim3((unsigned)blocks), dim3(64), kChainLds, st, P);
        HY_CHECK_LAUNCH("chain_groups_kernel");
    }
    ProfScope _pl(ctx, long_pass ? "mm_chain_long_small" : "mm_chain_small", slot + 1, 28.0);
    hipLaunchKernelGGL(chain_small_kernel, dim3((unsigned)cdiv(P.n_work, 64)), dim3(64), 0, st, P, (const int32_t *)split.as<int32_t>());
    HY_CHECK_LAUNCH("chain_small_kernel");
    return HYMET_OK;
}

int launch_backtrack(hymet_ctx *ctx, const int64_t *g_start, const int32_t *f, const int64_t *p, int32_t *t,
                     const int32_t *z_cnt, const int32_t *z_idx, int32_t n_groups, const int32_t *order, int32_t n_work,
                     int min_cnt, int min_sc, int max_drop, int64_t *chain_ids, uint64_t *chain_u, int64_t *chain_first,
                     int32_t *n_chains, int64_t n_anchors) {
    if (n_groups <= 0) return HYMET_OK;
    // t arrives zeroed (the chaining kernels clear it anchor by anchor, nonwork_fp_kernel the
    // groups below min_cnt)
    const char *ev = getenv("HYMET_BT_LONG");
    const int64_t long_min = ev ? atoll(ev) : kBtLong;
    const bool prof = getenv("HYMET_BT_PROF") != nullptr;
    DevBuf pbuf;
    if (prof) {
        HY_HIP(pbuf.alloc(64, ctx->stream));
        HY_HIP(hipMemsetAsync(pbuf.p, 0, 64, ctx->stream));
    }
    BacktrackParams P{g_start,  f,         p,       t,           z_cnt,    z_idx, n_groups, min_cnt, min_sc, max_drop,
                      long_min, (unsigned long long *)pbuf.p, chain_ids, chain_u, chain_first, n_chains};
    DevBuf cnt;
    HY_HIP(cnt.alloc(4 * (size_t)kBtCtrPad * (kBtStripes + 1), ctx->stream));  // [0] long groups, then the stripe counters
    // z index + t probe + walked (p, f) + t mark + chain id write, per anchor
    ProfScope _ps(ctx, "mm_backtrack", 32.0 * (double)n_anchors);
    if (n_work > 0) {
        hipLaunchKernelGGL(bt_long_count_kernel, dim3(1), dim3(1), 0, ctx->stream, g_start, order, n_work, long_min,
                           cnt.as<int32_t>());
        HY_CHECK_LAUNCH("bt_long_count_kernel");
    }
    // (running the two kernels concurrently on two streams measured no faster: both are
    // throughput-bound)
    hipLaunchKernelGGL(backtrack_groups_kernel, dim3((unsigned)cdiv(n_groups, 64)), dim3(64), 0, ctx->stream, P);
    HY_CHECK_LAUNCH("backtrack_groups_kernel");
    if (n_work > 0) {
        ProfScope _pl(ctx, "mm_backtrack.long");  // the wave-per-group part of mm_backtrack
        // resident waves per CU for the wave kernel (HYMET_BT_WAVES overrides): 28 measured 4 %
        // slower than 16 on C4 under the single work counter; with the striped counters 24 (the
        // register limit) measured faster than 16, one-stream (112 vs 116 ms/step) and
        // two-stream (1,585 vs 1,594 ms per bench step)
        const char *ew = getenv("HYMET_BT_WAVES");
        const int per_cu = ew ? std::max(1, atoi(ew)) : 24;
        const int64_t nb = std::min<int64_t>(n_work, (int64_t)ctx->n_cu * per_cu);
        hipLaunchKernelGGL(backtrack_long_kernel, dim3((unsigned)nb), dim3(64), 0, ctx->stream, P, order,
                           cnt.as<int32_t>(), cnt.as<int32_t>() + kBtCtrPad);
        HY_CHECK_LAUNCH("backtrack_long_kernel");
    }
    if (prof) {
        unsigned long long h[8];
        HY_HIP(hipMemcpyAsync(h, pbuf.p, 64, hipMemcpyDeviceToHost, ctx->stream));
        HY_HIP(hipStreamSynchronize(ctx->stream));
        fprintf(stderr, "[bt_long] groups=%llu probes=%llu walks=%llu steps=%llu reloads=%llu cyc_walk=%.3g cyc_post=%.3g cyc_all=%.3g\n",
                h[0], h[1], h[2], h[3], h[4], (double)h[5], (double)h[6], (double)h[7]);
    }
    return HYMET_OK;
}

}  // namespace mm
}  // namespace hymet
