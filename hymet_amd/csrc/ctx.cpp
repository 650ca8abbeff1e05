// Context lifetime and thread-local error strings for the C ABI (include/hymet_gpu.h).
#include "common.hpp"

#include <algorithm>
#include <thread>
#include <vector>

#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <cstdlib>
#include <vector>

namespace hymet {
static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char *what) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return HYMET_E_HIP;
}

static std::mutex g_cache_mu;
struct CacheKey {
    int dev;
    hipStream_t stream;
    size_t cls;
    bool operator<(const CacheKey &o) const {
        return std::tie(dev, stream, cls) < std::tie(o.dev, o.stream, o.cls);
    }
};
static std::map<CacheKey, std::vector<void *>> g_cache;  // free blocks
static size_t g_cached = 0;                                // bytes held in g_cache
static int64_t g_stats[3] = {0, 0, 0};  // hipMalloc calls (cache misses), OOM cache drops, frees over the cap
// Called when hipMalloc still fails after this allocator dropped its own cache: the host
// releases what another caching allocator in the process (torch's) holds unused.
static void (*g_oom_hook)(void *) = nullptr;
static void *g_oom_user = nullptr;

static size_t cache_cap() {
    static const size_t cap = [] {
        const char *e = getenv("HYMET_SCRATCH_CAP_GB");
        const double gb = e ? atof(e) : 160.0;
        return (size_t)(gb * 1073741824.0);
    }();
    return cap;
}

static size_t size_class(size_t b) {
    if (b <= 4096) return 4096;
    int e = 63 - __builtin_clzll((unsigned long long)b);
    const size_t q = ((size_t)1 << e) / 4;
    return (b + q - 1) / q * q;
}

// free every cached block of `dev` (all streams); caller holds g_cache_mu
static void drop_cached(int dev) {
    for (auto &kv : g_cache)
        if (kv.first.dev == dev) {
            for (void *q : kv.second) {
                (void)hipFree(q);
                g_cached -= kv.first.cls;
            }
            kv.second.clear();
        }
}

hipError_t scratch_alloc(size_t bytes, hipStream_t stream, void **p, size_t *cls) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    *cls = size_class(bytes);
    {
        // best fit among this stream's cached blocks of at most twice the request: batches
        // of varying sizes then reuse blocks instead of piling up one class per size
        std::lock_guard<std::mutex> lk(g_cache_mu);
        for (auto it = g_cache.lower_bound({dev, stream, *cls});
             it != g_cache.end() && it->first.dev == dev && it->first.stream == stream && it->first.cls <= 2 * *cls; ++it) {
            if (it->second.empty()) continue;
            *p = it->second.back();
            it->second.pop_back();
            *cls = it->first.cls;
            g_cached -= *cls;
            return hipSuccess;
        }
    }
    e = hipMalloc(p, *cls);
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        g_stats[0]++;
    }
    if (e == hipErrorOutOfMemory) {  // give the cached blocks of this device back and retry once
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        void (*hook)(void *) = nullptr;
        void *user = nullptr;
        {
            std::lock_guard<std::mutex> lk(g_cache_mu);
            g_stats[1]++;
            drop_cached(dev);
            e = hipMalloc(p, *cls);
            hook = g_oom_hook;
            user = g_oom_user;
        }
        if (e == hipErrorOutOfMemory && hook) {  // then the other pool's, outside our lock
            (void)hipGetLastError();
            hook(user);
            e = hipMalloc(p, *cls);
        }
        if (e != hipSuccess) (void)hipGetLastError();  // reported through the return value only:
                                                       // a stale error would fail torch's next check
    }
    return e;
}

void set_oom_hook(void (*hook)(void *), void *user) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_oom_hook = hook;
    g_oom_user = user;
}

void scratch_free(void *p, hipStream_t stream, size_t cls) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    if (g_cached + cls > cache_cap()) {  // over the cap: hand it back (hipFree waits for the device)
        g_stats[2]++;
        (void)hipFree(p);
        return;
    }
    g_cache[{dev, stream, cls}].push_back(p);
    g_cached += cls;
}

int scratch_trim(int dev, int64_t *freed) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    const size_t before = g_cached;
    drop_cached(dev);
    if (freed) *freed = (int64_t)(before - g_cached);
    return HYMET_OK;
}

int64_t scratch_cached() {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    return (int64_t)g_cached;
}

void scratch_stats(int64_t *out) {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (int k = 0; k < 3; k++) out[k] = g_stats[k];
}
}  // namespace hymet

extern "C" {

int hymet_version(void) { return 1; }

const char *hymet_last_error(void) { return hymet::g_err.c_str(); }

int hymet_init(int device, hymet_ctx **out) {
    HY_ARG(out != nullptr, "hymet_init: out is null");
    int n = 0;
    HY_HIP(hipGetDeviceCount(&n));
    HY_ARG(device >= 0 && device < n, "hymet_init: no such device");
    HY_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    HY_HIP(hipGetDeviceProperties(&prop, device));
    std::string arch = prop.gcnArchName;
    if (arch.rfind("gfx950", 0) != 0)
        return hymet::fail(HYMET_E_ARG, "hymet_init: device is " + arch + ", this build targets gfx950 (MI355X) only");
    hymet_ctx *c = new hymet_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount;
    HY_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
    if (hipHostMalloc((void **)&c->mbox_h, 8 * hymet::kMbox, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->mbox_d, c->mbox_h, 0) != hipSuccess) {
        hymet_destroy(c);
        return hymet::fail(HYMET_E_HIP, "hymet_init: mailbox allocation failed");
    }
    for (int i = 0; i < hymet::kMbox; i++) c->mbox_h[i] = 0;
    if (hipMalloc((void **)&c->prof_dev, 8 * hymet::kProfSlots) != hipSuccess ||
        hipMemset(c->prof_dev, 0, 8 * hymet::kProfSlots) != hipSuccess) {
        c->prof_dev = nullptr;  // device-counted profile bytes unavailable: reported as 0
    }
    if (hipMalloc((void **)&c->dctr, 4 * hymet::kMbox) != hipSuccess || hipMemset(c->dctr, 0, 4 * hymet::kMbox) != hipSuccess) {
        hymet_destroy(c);
        return hymet::fail(HYMET_E_HIP, "hymet_init: counter allocation failed");
    }
    *out = c;
    return HYMET_OK;
}

int hymet_destroy(hymet_ctx *ctx) {
    if (!ctx) return HYMET_OK;
    (void)hipSetDevice(ctx->device);
    for (int k = 0; k < 2; k++) {
        if (ctx->stage[k]) (void)hipHostFree(ctx->stage[k]);
        if (ctx->stage_ev[k]) (void)hipEventDestroy(ctx->stage_ev[k]);
    }
    if (ctx->mbox_h) (void)hipHostFree(ctx->mbox_h);
    if (ctx->dctr) (void)hipFree(ctx->dctr);
    if (ctx->prof_dev) (void)hipFree(ctx->prof_dev);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return HYMET_OK;
}

int hymet_set_stream(hymet_ctx *ctx, void *s) {
    HY_ARG(ctx != nullptr, "hymet_set_stream: null ctx");
    HY_HIP(hipSetDevice(ctx->device));
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    ctx->stream = (hipStream_t)s;
    ctx->own_stream = false;
    return HYMET_OK;
}

int hymet_prof_enable(hymet_ctx *ctx, int on) {
    HY_ARG(ctx != nullptr, "hymet_prof_enable: null ctx");
    ctx->prof = on != 0;
    return HYMET_OK;
}

int hymet_prof_reset(hymet_ctx *ctx) {
    HY_ARG(ctx != nullptr, "hymet_prof_reset: null ctx");
    HY_HIP(hipStreamSynchronize(ctx->stream));
    for (auto &kv : ctx->ev)
        for (auto &p : kv.second) {
            (void)hipEventDestroy(p.first);
            (void)hipEventDestroy(p.second);
        }
    ctx->ev.clear();
    ctx->bytes.clear();
    ctx->dev_bytes.clear();
    if (ctx->prof_dev) HY_HIP(hipMemsetAsync(ctx->prof_dev, 0, 8 * hymet::kProfSlots, ctx->stream));
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}

int hymet_prof_query(hymet_ctx *ctx, const char *name, double *total_ms, int64_t *count, double *alg_bytes) {
    HY_ARG(ctx && name && total_ms && count, "hymet_prof_query: null argument");
    HY_HIP(hipStreamSynchronize(ctx->stream));
    *total_ms = 0.0;
    *count = 0;
    if (alg_bytes) {
        *alg_bytes = ctx->bytes.count(name) ? ctx->bytes[name] : 0.0;
        auto db = ctx->dev_bytes.find(name);
        if (db != ctx->dev_bytes.end() && ctx->prof_dev) {
            int64_t units = 0;
            HY_HIP(hipMemcpy(&units, ctx->prof_dev + db->second.first, 8, hipMemcpyDeviceToHost));
            *alg_bytes += db->second.second * (double)units;
        }
    }
    auto it = ctx->ev.find(name);
    if (it == ctx->ev.end()) return HYMET_OK;
    for (auto &p : it->second) {
        float ms = 0.f;
        HY_HIP(hipEventElapsedTime(&ms, p.first, p.second));
        *total_ms += ms;
        (*count)++;
    }
    return HYMET_OK;
}

int hymet_prof_names(hymet_ctx *ctx, char *buf, int64_t cap) {
    HY_ARG(ctx && buf && cap > 0, "hymet_prof_names: null argument");
    std::string all;
    for (auto &kv : ctx->ev) all += kv.first + "\n";
    if ((int64_t)all.size() + 1 > cap) return hymet::fail(HYMET_E_CAPACITY, "hymet_prof_names: buffer too small");
    memcpy(buf, all.c_str(), all.size() + 1);
    return HYMET_OK;
}

int hymet_scratch_trim(hymet_ctx *ctx, int64_t *freed_bytes) {
    HY_ARG(ctx != nullptr, "hymet_scratch_trim: null ctx");
    HY_HIP(hipSetDevice(ctx->device));
    HY_HIP(hipDeviceSynchronize());  // cached blocks of every stream of the device go back
    return hymet::scratch_trim(ctx->device, freed_bytes);
}

int hymet_scratch_reserve(hymet_ctx *ctx, int64_t bytes) {
    HY_ARG(ctx && bytes > 0, "hymet_scratch_reserve: bad argument");
    HY_HIP(hipSetDevice(ctx->device));
    void *p = nullptr;
    size_t cls = 0;
    HY_HIP(hymet::scratch_alloc((size_t)bytes, ctx->stream, &p, &cls));
    hymet::scratch_free(p, ctx->stream, cls);
    return HYMET_OK;
}

int hymet_set_oom_hook(void (*hook)(void *user), void *user) {
    hymet::set_oom_hook(hook, user);
    return HYMET_OK;
}

int hymet_scratch_stats(hymet_ctx *ctx, int64_t *counts) {
    HY_ARG(ctx && counts, "hymet_scratch_stats: null argument");
    hymet::scratch_stats(counts);
    return HYMET_OK;
}

int hymet_scratch_cached(hymet_ctx *ctx, int64_t *bytes) {
    HY_ARG(ctx && bytes, "hymet_scratch_cached: null argument");
    *bytes = hymet::scratch_cached();
    return HYMET_OK;
}

int hymet_copy_to_host(hymet_ctx *ctx, void *dst, const void *src, int64_t n, int threads) {
    HY_ARG(ctx && (n == 0 || (dst && src)) && n >= 0, "hymet_copy_to_host: bad argument");
    if (n == 0) return HYMET_OK;
    // Pinned staging in 64 MiB chunks, double buffered: chunk k+1 crosses PCIe while host
    // threads copy chunk k into dst (their first touch of dst's fresh pages runs in parallel
    // too).  A pageable hipMemcpy does both steps on one thread (~7 GB/s).
    constexpr int64_t kChunk = 64ll << 20;
    threads = std::max(1, std::min(threads, 64));
    HY_HIP(hipSetDevice(ctx->device));
    for (int k = 0; k < 2; k++) {
        if (!ctx->stage[k]) HY_HIP(hipHostMalloc(&ctx->stage[k], kChunk, hipHostMallocDefault));
        if (!ctx->stage_ev[k]) HY_HIP(hipEventCreateWithFlags(&ctx->stage_ev[k], hipEventDisableTiming));
    }
    const int64_t nch = (n + kChunk - 1) / kChunk;
    auto issue = [&](int64_t c) -> hipError_t {
        const int64_t off = c * kChunk, len = std::min(kChunk, n - off);
        hipError_t e = hipMemcpyAsync(ctx->stage[c & 1], (const char *)src + off, (size_t)len, hipMemcpyDeviceToHost,
                                      ctx->stream);
        if (e == hipSuccess) e = hipEventRecord(ctx->stage_ev[c & 1], ctx->stream);
        return e;
    };
    HY_HIP(issue(0));
    for (int64_t c = 0; c < nch; c++) {
        HY_HIP(hipEventSynchronize(ctx->stage_ev[c & 1]));
        if (c + 1 < nch) HY_HIP(issue(c + 1));  // the other buffer: its previous copy-out is done
        const int64_t off = c * kChunk, len = std::min(kChunk, n - off);
        const char *from = (const char *)ctx->stage[c & 1];
        char *to = (char *)dst + off;
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) {
            const int64_t b = len * t / threads, e = len * (t + 1) / threads;
            if (b < e) th.emplace_back([=] { memcpy(to + b, from + b, (size_t)(e - b)); });
        }
        for (auto &x : th) x.join();
    }
    return HYMET_OK;
}

int hymet_copy_to_device(hymet_ctx *ctx, void *dst, const void *src, int64_t n, int threads) {
    HY_ARG(ctx && (n == 0 || (dst && src)) && n >= 0, "hymet_copy_to_device: bad argument");
    if (n == 0) return HYMET_OK;
    // The mirror of hymet_copy_to_host: host threads copy chunk k into a pinned stage while
    // chunk k-1 crosses PCIe from the other one (a pageable copy stages on one thread).
    // Returns once the last chunk has landed (the stages are reused by the next call).
    constexpr int64_t kChunk = 64ll << 20;
    threads = std::max(1, std::min(threads, 64));
    HY_HIP(hipSetDevice(ctx->device));
    for (int k = 0; k < 2; k++) {
        if (!ctx->stage[k]) HY_HIP(hipHostMalloc(&ctx->stage[k], kChunk, hipHostMallocDefault));
        if (!ctx->stage_ev[k]) HY_HIP(hipEventCreateWithFlags(&ctx->stage_ev[k], hipEventDisableTiming));
    }
    const int64_t nch = (n + kChunk - 1) / kChunk;
    bool pending[2] = {false, false};
    for (int64_t c = 0; c < nch; c++) {
        const int b = (int)(c & 1);
        if (pending[b]) HY_HIP(hipEventSynchronize(ctx->stage_ev[b]));  // its previous DMA has read it
        const int64_t off = c * kChunk, len = std::min(kChunk, n - off);
        char *to = (char *)ctx->stage[b];
        const char *from = (const char *)src + off;
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) {
            const int64_t lo = len * t / threads, hi = len * (t + 1) / threads;
            if (lo < hi) th.emplace_back([=] { memcpy(to + lo, from + lo, (size_t)(hi - lo)); });
        }
        for (auto &x : th) x.join();
        HY_HIP(hipMemcpyAsync((char *)dst + off, to, (size_t)len, hipMemcpyHostToDevice, ctx->stream));
        HY_HIP(hipEventRecord(ctx->stage_ev[b], ctx->stream));
        pending[b] = true;
    }
    for (int b = 0; b < 2; b++)
        if (pending[b]) HY_HIP(hipEventSynchronize(ctx->stage_ev[b]));
    return HYMET_OK;
}

int hymet_sync(hymet_ctx *ctx) {
    HY_ARG(ctx != nullptr, "hymet_sync: null ctx");
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}

}  // extern "C"
