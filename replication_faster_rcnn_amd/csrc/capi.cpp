// C-ABI housekeeping: version string and the per-thread last-error message.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <mutex>

#include "common.h"

namespace frcnn {

static thread_local char g_err[512] = "";
constexpr int kMaxDevices = 64;

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
    // per device (a process may drive several GPUs, one per thread)
    static std::atomic<int> cus[kMaxDevices] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        (void)hipGetLastError();
        return 256;
    }
    int n = cus[dev].load(std::memory_order_relaxed);
    if (n <= 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
            (void)hipGetLastError();
            n = 256;
        }
        cus[dev].store(n, std::memory_order_relaxed);
    }
    return n;
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
    if (is(op, "roi_pool_fwd") &&
        (aut || is(path, "wave") || is(path, "dense") || is(path, "generic"))) {
        g_path.roi_fwd = aut ? kPathAuto : is(path, "generic") ? kPathGeneric
                                       : is(path, "dense")     ? kPathDense
                                                               : kPathWave;
    } else if (is(op, "roi_pool_bwd") &&
               (aut || is(path, "ring") || is(path, "plain"))) {
        g_path.roi_bwd = aut ? kPathAuto : is(path, "plain") ? kPathPlain : kPathRing;
    } else if (is(op, "propose") &&
               (aut || is(path, "hybrid") || is(path, "lazy") || is(path, "wide"))) {
        g_path.propose = aut ? kPathAuto : is(path, "hybrid") ? kPathHybrid
                                         : is(path, "lazy")   ? kPathLazy
                                                              : kPathWide;
    } else if (is(op, "roi_pool_fwd_store") && (aut || is(path, "temporal") || is(path, "nt"))) {
        g_path.roi_store = is(path, "nt") ? 1 : 0;
    } else if (is(op, "sampler") && (aut || is(path, "walk") || is(path, "chip") || is(path, "chip_only") ||
                                     is(path, "chip_tight"))) {
        g_path.sampler = aut                   ? kPathAuto
                         : is(path, "walk")      ? kPathWalk
                         : is(path, "chip")      ? kPathChip
                         : is(path, "chip_only") ? kPathChipOnly
                                                 : kPathChipTight;
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

// ------------------------------------------------------ streams on CU subsets
// A stream whose kernels may only use the CUs set in `cu_mask` (bit i of word
// i/32 = CU i, hipExtStreamCreateWithCUMask numbering).  Used to run the
// latency-bound proposal chain on a few reserved CUs beside the RoIPool, which
// otherwise holds every CU's LDS for its whole run.
extern "C" int frcnn_stream_create(const uint32_t* cu_mask, int words, void** out) {
    if (!out || words < 0 || (words > 0 && !cu_mask)) {
        frcnn::set_error("frcnn_stream_create: bad arguments");
        return FRCNN_EINVAL;
    }
    hipStream_t s = nullptr;
    const hipError_t e = words > 0 ? hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(words), cu_mask)
                                   : hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) {
        frcnn::set_error("frcnn_stream_create: %s", hipGetErrorString(e));
        return FRCNN_EHIP;
    }
    *out = s;
    return FRCNN_OK;
}

namespace frcnn {
// CU counts of streams, keyed by (device, handle): a stream's CU mask is fixed
// at creation, and frcnn_stream_destroy evicts its entry, so a later stream
// that reuses the handle value is looked up afresh.
struct CuCache {
    std::mutex mu;
    hipStream_t s[16] = {};
    int dev[16] = {};
    int n[16] = {};
    int next = 0;
};
static CuCache g_cu_cache;

static void cu_cache_evict(hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_cu_cache.mu);
    for (int i = 0; i < 16; ++i)
        if (g_cu_cache.s[i] == st) g_cu_cache.s[i] = nullptr;
}
}  // namespace frcnn

extern "C" int frcnn_stream_destroy(void* stream) {
    if (!stream) return FRCNN_OK;
    frcnn::cu_cache_evict(frcnn::as_stream(stream));
    if (hipStreamDestroy(frcnn::as_stream(stream)) != hipSuccess)
        return frcnn::check_launch("frcnn_stream_destroy");
    return FRCNN_OK;
}

namespace frcnn {
// CUs a kernel launched on `s` may use: popcount of the stream's CU mask
// (every CU for the null stream and for unmasked streams).  Cached per stream
// handle: the mask is fixed at creation.
int stream_cu_count(hipStream_t s) {
    const int all = device_cu_count();
    if (!s) return all;
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lk(g_cu_cache.mu);
        for (int i = 0; i < 16; ++i)
            if (g_cu_cache.s[i] == s && g_cu_cache.dev[i] == dev) return g_cu_cache.n[i];
    }
    uint32_t m[32] = {};
    int n = all;
    if (hipExtStreamGetCUMask(s, 32, m) == hipSuccess) {
        int bits = 0;
        for (int i = 0; i < 32 && i * 32 < all; ++i) bits += __builtin_popcount(m[i]);
        if (bits > 0 && bits < all) n = bits;
    } else {
        (void)hipGetLastError();
    }
    std::lock_guard<std::mutex> lk(g_cu_cache.mu);
    const int i = g_cu_cache.next;
    g_cu_cache.s[i] = s;
    g_cu_cache.dev[i] = dev;
    g_cu_cache.n[i] = n;
    g_cu_cache.next = (i + 1) & 15;
    return n;
}
}  // namespace frcnn

extern "C" int frcnn_stream_cu_count(void* stream, int* out) {
    if (!out) {
        frcnn::set_error("frcnn_stream_cu_count: null pointer");
        return FRCNN_EINVAL;
    }
    *out = frcnn::stream_cu_count(frcnn::as_stream(stream));
    return FRCNN_OK;
}

// Diagnostic: where the workgroups of a launch ran.  out[2*b] = HW_ID
// (cu_id bits 11:8, sh_id 12, se_id 15:13), out[2*b+1] = XCC_ID of workgroup b.
__global__ void hw_id_probe_kernel(uint32_t* out, int spin) {
    if (threadIdx.x == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);  // hold the CU so blocks spread
}

extern "C" int frcnn_probe_hw_ids(uint32_t* out, int nblocks, int spin, void* stream) {
    if (!out || nblocks <= 0 || spin < 0 || spin > 4096) {
        frcnn::set_error("frcnn_probe_hw_ids: bad arguments");
        return FRCNN_EINVAL;
    }
    hipLaunchKernelGGL(hw_id_probe_kernel, dim3(nblocks), dim3(64), 0, frcnn::as_stream(stream), out, spin);
    return frcnn::check_launch("hw_id_probe_kernel");
}
