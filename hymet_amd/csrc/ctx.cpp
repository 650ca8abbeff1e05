// Context lifetime and thread-local error strings for the C ABI (include/hymet_gpu.h).
#include "common.hpp"

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
    *out = c;
    return HYMET_OK;
}

int hymet_destroy(hymet_ctx *ctx) {
    if (!ctx) return HYMET_OK;
    (void)hipSetDevice(ctx->device);
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

int hymet_sync(hymet_ctx *ctx) {
    HY_ARG(ctx != nullptr, "hymet_sync: null ctx");
    HY_HIP(hipStreamSynchronize(ctx->stream));
    return HYMET_OK;
}

}  // extern "C"
