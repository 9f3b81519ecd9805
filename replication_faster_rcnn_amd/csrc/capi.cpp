// C-ABI housekeeping: version string and the per-thread last-error message.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

static PathCfg g_path;

const PathCfg& path_cfg() { return g_path; }

int device_cu_count() {
    static int cus = 0;
    if (cus <= 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            cus = n;
        else
            cus = 256;
    }
    return cus;
}

}  // namespace frcnn

extern "C" const char* frcnn_version(void) { return "frcnn_mi355x 0.2.0 gfx950"; }

extern "C" int frcnn_set_path(const char* op, const char* path) {
    using namespace frcnn;
    if (!op || !path) {
        set_error("frcnn_set_path: null argument");
        return FRCNN_EINVAL;
    }
    auto is = [&](const char* a, const char* b) { return std::strcmp(a, b) == 0; };
    const bool aut = is(path, "auto");
    if (is(op, "roi_pool_fwd") && (aut || is(path, "wave") || is(path, "dense") || is(path, "generic"))) {
        g_path.roi_fwd = aut ? kPathAuto : is(path, "generic") ? kPathGeneric
                                       : is(path, "dense")     ? kPathDense
                                                               : kPathWave;
    } else if (is(op, "roi_pool_bwd") && (aut || is(path, "ring") || is(path, "plain"))) {
        g_path.roi_bwd = is(path, "plain") ? kPathPlain : kPathAuto;
    } else if (is(op, "propose") &&
               (aut || is(path, "hybrid") || is(path, "lazy") || is(path, "wide"))) {
        g_path.propose = aut ? kPathAuto : is(path, "hybrid") ? kPathHybrid
                                         : is(path, "lazy")   ? kPathLazy
                                                              : kPathWide;
    } else if (is(op, "roi_pool_split")) {
        char* end = nullptr;
        const long v = aut ? 0 : std::strtol(path, &end, 10);
        if (!aut && (end == path || *end != '\0' || v < 0 || v > 64)) {
            set_error("frcnn_set_path: roi_pool_split must be auto or 0..64, got '%s'", path);
            return FRCNN_EINVAL;
        }
        g_path.roi_split = static_cast<int>(v);
    } else if (is(op, "roi_pool_cg") && (aut || is(path, "4") || is(path, "8") || is(path, "16"))) {
        g_path.roi_cg = aut ? 0 : std::atoi(path);
    } else {
        set_error("frcnn_set_path: unknown op / path '%s' / '%s'", op, path);
        return FRCNN_EINVAL;
    }
    return FRCNN_OK;
}

extern "C" const char* frcnn_last_error(void) { return frcnn::g_err; }

// CU count of the current device, for callers sizing their own launches.
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
