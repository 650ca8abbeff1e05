// Shared plumbing for libhymet_gpu.so: context, error reporting, launch helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "../../include/hymet_gpu.h"

struct hymet_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int n_cu = 256;
};

namespace hymet {
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
int hip_fail(hipError_t e, const char *what);
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
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
