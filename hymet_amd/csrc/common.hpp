// Shared plumbing for libhymet_gpu.so: context, error reporting, launch helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <map>
#include <string>
#include <utility>
#include <vector>
#include "../../include/hymet_gpu.h"

struct hymet_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int n_cu = 256;
    // live per-kernel timing (hymet_prof_*): HIP events recorded on `stream` around launches
    bool prof = false;
    std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> ev;
    std::map<std::string, double> bytes;  // algorithmic bytes of the timed launches
    // algorithmic units counted on the device (e.g. the anchors a kernel took from a work list
    // the host never sees): scope -> (slot of prof_dev, bytes per unit); prof_dev[kProfSlots]
    // accumulates while profiling is on and is read by hymet_prof_query
    std::map<std::string, std::pair<int, double>> dev_bytes;
    int64_t *prof_dev = nullptr;
    // pinned staging for hymet_copy_to_host (two chunks, allocated on first use)
    void *stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    // mailbox: pinned, device-mapped, coherent host words that kernels store small results
    // into (scan totals, list counts, maxima) -- read on the host after a stream sync, with
    // no copy dispatch (hymet::mb_dev / mb_read)
    int64_t *mbox_h = nullptr;
    int64_t *mbox_d = nullptr;
    // device counters that kernels leave zeroed (hymet::mm::publish_counters), so counting
    // kernels need no memset before them
    int32_t *dctr = nullptr;
};

namespace hymet {
// RAII: records a start/stop event pair on the context stream around the enclosed launches
struct ProfScope {
    hymet_ctx *c;
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(hymet_ctx *ctx, const char *n, double alg_bytes = 0.0) : c(ctx), name(n) {
        if (c && c->prof && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess) {
            (void)hipEventRecord(a, c->stream);
            c->bytes[name] += alg_bytes;
        }
    }
    // bytes = per_unit x the units kernels add to prof_dev[slot] (prof_dev_slot) inside the scope
    ProfScope(hymet_ctx *ctx, const char *n, int slot, double per_unit) : ProfScope(ctx, n, 0.0) {
        if (c && c->prof) c->dev_bytes[name] = {slot, per_unit};
    }
    ~ProfScope() {
        if (c && c->prof && a && b) {
            (void)hipEventRecord(b, c->stream);
            c->ev[name].push_back({a, b});
        }
    }
};
constexpr int kProfSlots = 8;
// the device counter of slot k while profiling is on, else nullptr (kernels skip the count)
inline int64_t *prof_dev_slot(hymet_ctx *c, int k) { return c && c->prof && c->prof_dev ? c->prof_dev + k : nullptr; }
}  // namespace hymet

namespace hymet {
constexpr int kMbox = 64;  // mailbox words per context
// device address of mailbox word i (kernels store into it)
inline int64_t *mb_dev(hymet_ctx *c, int i) { return c->mbox_d + i; }
// host read of mailbox word i, after the stream has been synchronised
inline int64_t mb_read(const hymet_ctx *c, int i) { return __atomic_load_n(c->mbox_h + i, __ATOMIC_ACQUIRE); }
}  // namespace hymet

namespace hymet {
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
int hip_fail(hipError_t e, const char *what);
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
// Caching device allocator for kernel scratch, keyed by (device, stream, size class): a
// block released on a stream is reissued only to work queued behind it on the same stream.
// A request takes the best-fitting cached block of at most twice its size.  Cached bytes
// are capped (HYMET_SCRATCH_CAP_GB, default 160); hymet_scratch_trim frees them.
// (hipMalloc/hipFree and the stream-ordered pool cost 0.1-0.4 s per large block on this
// stack, at every mapping batch, hence the cache.)
hipError_t scratch_alloc(size_t bytes, hipStream_t stream, void **p, size_t *cls);
void set_oom_hook(void (*hook)(void *), void *user);
void scratch_free(void *p, hipStream_t stream, size_t cls);
}  // namespace hymet

#define HY_CHECK_LAUNCH(what)                                   \
    do {                                                        \
        hipError_t e_ = hipGetLastError();                      \
        if (e_ != hipSuccess) return hymet::hip_fail(e_, what); \
    } while (0)

#define HY_HIP(call)                                            \
    do {                                                        \
        hipError_t e_ = (call);                                 \
        if (e_ != hipSuccess) return hymet::hip_fail(e_, #call); \
    } while (0)

#define HY_ARG(cond, msg)                                                   \
    do {                                                                    \
        if (!(cond)) return hymet::fail(HYMET_E_ARG, std::string(msg));     \
    } while (0)
