// C-ABI housekeeping: version string and the per-thread last-error message.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace frcnn {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return FRCNN_EHIP;
    }
    return FRCNN_OK;
}

}  // namespace frcnn

extern "C" const char* frcnn_version(void) { return "frcnn_mi355x 0.1.0 gfx950"; }

extern "C" const char* frcnn_last_error(void) { return frcnn::g_err; }

// Streams restricted to a set of CUs (hipExtStreamCreateWithCUMask): lets the
// latency-bound proposal layer keep a few CUs of its own while the RoIPool of
// the previous step fills the rest, instead of waiting for whole CUs to drain.
extern "C" int frcnn_device_cu_count(int* out) {
    int dev = 0, n = 0;
    if (!out) {
        frcnn::set_error("frcnn_device_cu_count: null pointer");
        return FRCNN_EINVAL;
    }
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return frcnn::check_launch("frcnn_device_cu_count");
    *out = n;
    return FRCNN_OK;
}

extern "C" int frcnn_stream_create_cu_masked(const uint32_t* cu_mask, int n_words, void** stream) {
    if (!cu_mask || n_words <= 0 || !stream) {
        frcnn::set_error("frcnn_stream_create_cu_masked: bad argument");
        return FRCNN_EINVAL;
    }
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(n_words), cu_mask) != hipSuccess) {
        (void)hipGetLastError();
        frcnn::set_error("frcnn_stream_create_cu_masked: hipExtStreamCreateWithCUMask failed");
        return FRCNN_EHIP;
    }
    *stream = s;
    return FRCNN_OK;
}

extern "C" int frcnn_stream_destroy(void* stream) {
    if (stream && hipStreamDestroy(static_cast<hipStream_t>(stream)) != hipSuccess)
        return frcnn::check_launch("frcnn_stream_destroy");
    return FRCNN_OK;
}
