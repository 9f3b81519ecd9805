// C-ABI housekeeping: version string and the per-thread last-error message.
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
