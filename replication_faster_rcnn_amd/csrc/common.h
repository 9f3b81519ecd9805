// Shared helpers for the gfx950 kernels and the C-ABI wrappers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/frcnn_capi.h"

namespace frcnn {

void set_error(const char* fmt, ...);

// Kernel-path selection (frcnn_set_path; process-global, default "auto").
// Read once per call as plain ints: no getenv on the launch path.
constexpr int kPathAuto = 0;
constexpr int kPathGeneric = 1;  // roi_pool_fwd: one workgroup per RoI
constexpr int kPathDense = 2;    // roi_pool_fwd: image tile, RoI bins packed per wave
constexpr int kPathWave = 3;     // roi_pool_fwd: image tile, one wave per RoI (RoIs grouped by image)
constexpr int kPathPlain = 1;    // roi_pool_bwd: the unpipelined plane-owner kernel
constexpr int kPathRing = 2;     // roi_pool_bwd: the RoI-at-a-time ring kernel (auto: leader kernel)
constexpr int kPathHybrid = 1;   // propose: fused per image + chip-wide first-chunk mask
constexpr int kPathLazy = 2;     // propose: fused per image, lazy NMS from the first chunk on
constexpr int kPathWide = 3;     // propose: chip-wide sort + bitmask NMS
constexpr int kPathWalk = 1;       // sampler: one workgroup walks the MT19937 stream
constexpr int kPathChip = 2;       // sampler: chip-wide segment tables, the walk as fallback (auto)
constexpr int kPathChipOnly = 3;   // sampler: chip-wide, no fallback launched (tests)
constexpr int kPathChipTight = 4;  // sampler: chip-wide with zero-margin domains (tests the fallback)
struct PathCfg {
    int roi_fwd = kPathAuto;
    int roi_bwd = kPathAuto;
    int propose = kPathAuto;
    int roi_split = 0;  // RoI shares per (image, channel group); 0 = auto
    int roi_cg = 0;     // channels per RoIPool workgroup (4 / 8 / 16); 0 = auto
    int sampler = kPathAuto;
    int roi_store = 0;  // RoIPool forward (wave kernel) output stores: 0 temporal (auto), 1 non-temporal
};
const PathCfg& path_cfg();

// CU count of the current device (cached after the first call).
int device_cu_count();
// CUs a launch on stream s may use (its CU mask; every CU if unmasked).
int stream_cu_count(hipStream_t s);

// Launch-and-check helper used by every C-ABI wrapper: returns FRCNN_EHIP
// with the HIP message when the last launch failed.
int check_launch(const char* what);

#define FRCNN_REQUIRE(cond, ...)                 \
    do {                                         \
        if (!(cond)) {                           \
            ::frcnn::set_error(__VA_ARGS__);     \
            return FRCNN_EINVAL;                 \
        }                                        \
    } while (0)

#define FRCNN_LAUNCH_CHECK(name)                         \
    do {                                                 \
        int _rc = ::frcnn::check_launch(name);           \
        if (_rc) return _rc;                             \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Bump allocator over the caller's workspace.  Every carve is 256-B aligned.
struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(void* p) : base(static_cast<char*>(p)) {}
    template <class T>
    T* take(size_t count) {
        off = align_up(off, 256);
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += count * sizeof(T);
        return p;
    }
    size_t used() const { return align_up(off, 256); }
};

// ------------------------------------------------------------ device helpers
constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
    uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Order-preserving map of an fp32 score to a u32 that sorts ASCENDING for
// DESCENDING scores (NaN first, like torch's descending sort).
__device__ __forceinline__ uint32_t desc_score_key(float s) {
    uint32_t u = __float_as_uint(s);
    uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    uint32_t k = ~asc;
    return k == 0xFFFFFFFFu ? 0xFFFFFFFEu : k;  // 0xFFFFFFFF is reserved for "invalid"
}

// torch.clamp(v, lo, hi) on fp32 with NaN propagation (nets/rpn.py:62-63).
__device__ __forceinline__ float clamp_nan(float v, float lo, float hi) {
    if (v != v) return v;
    float t = v < lo ? lo : v;
    return t > hi ? hi : t;
}

// Correctly rounded fp32 exp: fp64 exp, rounded once to fp32.  Never the
// hardware v_exp_f32 path (SURVEY.md §7 "Host-dependent exp").
__device__ __forceinline__ float exp_cr(float v) { return static_cast<float>(exp(static_cast<double>(v))); }

// utils/utils.py:57-72, fp32, every op separately rounded.
__device__ __forceinline__ float4 decode_box(float4 a, float4 d) {
    float ah = a.z - a.x;
    float aw = a.w - a.y;
    float acx = (a.z + a.x) * 0.5f;   // /2 == *0.5 exactly
    float acy = (a.y + a.w) * 0.5f;
    float x = d.x * ah;
    x = x + acx;
    float y = d.y * aw;
    y = y + acy;
    float h = exp_cr(d.z) * ah;
    float w = exp_cr(d.w) * aw;
    float hh = h * 0.5f, hw = w * 0.5f;
    return make_float4(x - hh, y - hw, x + hh, y + hw);
}

}  // namespace frcnn
