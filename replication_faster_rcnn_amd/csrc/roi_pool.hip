// RoI max-pooling forward / backward (nets/heads.py:42-48, torchvision
// roi_pool semantics) on gfx950.
//
// Forward: one 256-thread workgroup per RoI.  The RoI's PHxPW bin windows are
// computed once into LDS; each lane then produces 4 consecutive outputs
// ([c][ph][pw] order) and writes them as one float4 + one int4, so the two
// output streams -- which are the HBM roofline of this op -- are written
// fully coalesced.  Feature reads are window gathers served by L1/L2 (one
// image's feature map is a few MB).
//
// Backward: atomic-free, deterministic and bit-identical to the CPU kernel's
// summation order.  A workgroup owns CPW channel planes of one image; each
// wave accumulates one plane in LDS, walking that image's RoIs in ascending
// order.  Within one RoI the 64 lanes are the bins; two bins can hit the same
// pixel only if their windows overlap (mask precomputed per RoI), and such
// lanes apply their adds in rounds ordered by bin index, so every pixel sees
// exactly the CPU order n -> ph -> pw.  The finished planes are stored once
// (zero-fill of grad_in fused).
#include <cfloat>

#include "common.h"

namespace frcnn {

constexpr int kMaxBins = 1024;

// torchvision bin window (hs, he, ws, we) of bin (ph, pw) for RoI `roi`.
__device__ __forceinline__ int4 roi_bin(const float* roi, float ss, int H, int W, int PH, int PW,
                                        int ph, int pw) {
    int sw = static_cast<int>(roundf(roi[1] * ss));
    int sh = static_cast<int>(roundf(roi[2] * ss));
    int ew = static_cast<int>(roundf(roi[3] * ss));
    int eh = static_cast<int>(roundf(roi[4] * ss));
    int rw = ew - sw + 1;
    int rh = eh - sh + 1;
    rw = rw > 1 ? rw : 1;
    rh = rh > 1 ? rh : 1;
    float bh = static_cast<float>(rh) / static_cast<float>(PH);
    float bw = static_cast<float>(rw) / static_cast<float>(PW);
    int hs = static_cast<int>(floorf(static_cast<float>(ph) * bh)) + sh;
    int ws = static_cast<int>(floorf(static_cast<float>(pw) * bw)) + sw;
    int he = static_cast<int>(ceilf(static_cast<float>(ph + 1) * bh)) + sh;
    int we = static_cast<int>(ceilf(static_cast<float>(pw + 1) * bw)) + sw;
    hs = min(max(hs, 0), H);
    he = min(max(he, 0), H);
    ws = min(max(ws, 0), W);
    we = min(max(we, 0), W);
    return make_int4(hs, he, ws, we);
}

__device__ __forceinline__ void pool_window(const float* __restrict__ plane, int W, int4 g,
                                            float& mv, int& mi) {
    mv = (g.y <= g.x || g.w <= g.z) ? 0.0f : -FLT_MAX;
    mi = -1;
    for (int h = g.x; h < g.y; ++h) {
        const float* row = plane + h * W;
        for (int w = g.z; w < g.w; ++w) {
            float v = row[w];
            if (v > mv) {
                mv = v;
                mi = h * W + w;
            }
        }
    }
}

template <bool VEC>
__global__ __launch_bounds__(256) void roi_pool_fwd_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ rois, int N,
                                                           int C, int H, int W, int PH, int PW,
                                                           float ss, float* __restrict__ out,
                                                           int32_t* __restrict__ argmax) {
    __shared__ int4 bins[kMaxBins];
    const int r = blockIdx.x;
    const int tid = threadIdx.x;
    const int PHW = PH * PW;
    const float* roi = rois + static_cast<size_t>(r) * 5;
    for (int k = tid; k < PHW; k += 256) bins[k] = roi_bin(roi, ss, H, W, PH, PW, k / PW, k % PW);
    __syncthreads();
    const int b = static_cast<int>(roi[0]);
    const bool valid = b >= 0 && b < N;
    const size_t total = static_cast<size_t>(C) * PHW;
    float* o = out + static_cast<size_t>(r) * total;
    int32_t* am = argmax + static_cast<size_t>(r) * total;
    const size_t HW = static_cast<size_t>(H) * W;
    const float* xb = x + (valid ? static_cast<size_t>(b) * C * HW : 0);
    if (VEC) {
        for (size_t e0 = static_cast<size_t>(tid) * 4; e0 < total; e0 += 1024) {
            int c = static_cast<int>(e0 / PHW);
            int k = static_cast<int>(e0 - static_cast<size_t>(c) * PHW);
            float v[4];
            int m[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (valid) {
                    pool_window(xb + c * HW, W, bins[k], v[q], m[q]);
                } else {
                    v[q] = 0.0f;
                    m[q] = -1;
                }
                if (++k == PHW) {
                    k = 0;
                    ++c;
                }
            }
            *reinterpret_cast<float4*>(o + e0) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<int4*>(am + e0) = make_int4(m[0], m[1], m[2], m[3]);
        }
    } else {
        for (size_t e = tid; e < total; e += 256) {
            int c = static_cast<int>(e / PHW);
            int k = static_cast<int>(e - static_cast<size_t>(c) * PHW);
            float v = 0.0f;
            int m = -1;
            if (valid) pool_window(xb + c * HW, W, bins[k], v, m);
            o[e] = v;
            am[e] = m;
        }
    }
}

// nets/heads.py:42-47 (fp32 divide, then multiply) + [idx, box] pack.
__global__ __launch_bounds__(256) void roi_transform_kernel(const float* __restrict__ rois,
                                                            const float* __restrict__ inds,
                                                            int64_t R, float img_h, float img_w,
                                                            float fh, float fw,
                                                            float* __restrict__ boxes) {
    int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (r >= R) return;
    float4 v = reinterpret_cast<const float4*>(rois)[r];
    float* o = boxes + r * 5;
    o[0] = inds[r];
    o[1] = v.x / img_h * fh;
    o[2] = v.y / img_w * fw;
    o[3] = v.z / img_h * fh;
    o[4] = v.w / img_w * fw;
}

// ------------------------------------------------------------------ backward
// Per RoI and bin k: mask of the earlier bins of the same 64-bin chunk whose
// (non-empty) windows overlap bin k's -- the only bins that can share its
// argmax pixel.
__global__ __launch_bounds__(256) void roi_bwd_prep_kernel(const float* __restrict__ rois, int H,
                                                           int W, int PH, int PW, float ss,
                                                           uint64_t* __restrict__ cmask) {
    __shared__ int4 bins[kMaxBins];
    const int r = blockIdx.x;
    const int PHW = PH * PW;
    const float* roi = rois + static_cast<size_t>(r) * 5;
    for (int k = threadIdx.x; k < PHW; k += 256)
        bins[k] = roi_bin(roi, ss, H, W, PH, PW, k / PW, k % PW);
    __syncthreads();
    for (int k = threadIdx.x; k < PHW; k += 256) {
        int4 g = bins[k];
        uint64_t m = 0;
        bool ne = g.y > g.x && g.w > g.z;
        int k0 = k & ~63;
        for (int p = k0; ne && p < k; ++p) {
            int4 q = bins[p];
            bool ov = q.y > q.x && q.w > q.z && q.x < g.y && g.x < q.y && q.z < g.w && g.z < q.w;
            if (ov) m |= 1ull << (p - k0);
        }
        cmask[static_cast<size_t>(r) * PHW + k] = m;
    }
}

// Ordered per-image RoI lists: list[b][*] = RoIs with batch index b, ascending.
__global__ __launch_bounds__(1024) void roi_lists_kernel(const float* __restrict__ rois, int R,
                                                         int* __restrict__ list,
                                                         int* __restrict__ cnt) {
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    __shared__ int s_w[16];
    int base = 0;
    for (int r0 = 0; r0 < R; r0 += 1024) {
        int r = r0 + tid;
        bool m = r < R && static_cast<int>(rois[static_cast<size_t>(r) * 5]) == b;
        uint64_t bal = __ballot(m);
        if (lane == 0) s_w[wid] = __popcll(bal);
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            before += w < wid ? s_w[w] : 0;
            tot += s_w[w];
        }
        if (m) list[static_cast<size_t>(b) * R + base + before + __popcll(bal & lanemask_lt())] = r;
        base += tot;
        __syncthreads();
    }
    if (tid == 0) cnt[b] = base;
}

template <bool IN_LDS>
__global__ void roi_pool_bwd_kernel(const float* __restrict__ grad,
                                    const int32_t* __restrict__ argmax,
                                    const uint64_t* __restrict__ cmask,
                                    const int* __restrict__ list, const int* __restrict__ cnt,
                                    int R, int C, int HW, int PHW, int CPW,
                                    float* __restrict__ grad_in) {
    extern __shared__ __attribute__((aligned(16))) float planes[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b = blockIdx.y;
    const int c = blockIdx.x * CPW + wid;
    if (c >= C) return;  // whole wave; no workgroup barrier below
    float* gplane = grad_in + (static_cast<size_t>(b) * C + c) * HW;
    float* plane = IN_LDS ? planes + static_cast<size_t>(wid) * HW : gplane;
    for (int i = lane; i < HW; i += 64) {
        if (IN_LDS) plane[i] = 0.0f;
        else __hip_atomic_store(plane + i, 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!IN_LDS) __builtin_amdgcn_s_waitcnt(0);
    const int nr = cnt[b];
    const int* lst = list + static_cast<size_t>(b) * R;
    for (int t = 0; t < nr; ++t) {
        const int n = __builtin_amdgcn_readfirstlane(lst[t]);
        const size_t base = (static_cast<size_t>(n) * C + c) * PHW;
        for (int k0 = 0; k0 < PHW; k0 += 64) {
            const int k = k0 + lane;
            const bool act = k < PHW;
            const int am = act ? argmax[base + k] : -1;
            const float g = act ? grad[base + k] : 0.0f;
            uint64_t pend = (act && am != -1) ? cmask[static_cast<size_t>(n) * PHW + k] : 0ull;
            int depth = 0;
            while (__ballot(pend != 0)) {
                int p = pend ? __ffsll(static_cast<unsigned long long>(pend)) - 1 : lane;
                pend &= pend - 1;
                int amp = __shfl(am, p, 64);
                if (p != lane && amp == am) ++depth;
            }
            int dmax = (am != -1) ? depth : -1;
            for (int o = 32; o > 0; o >>= 1) dmax = max(dmax, __shfl_xor(dmax, o, 64));
            for (int d = 0; d <= dmax; ++d) {
                if (am != -1 && depth == d) {
                    if (IN_LDS) {
                        plane[am] += g;
                    } else {
                        float cur = __hip_atomic_load(plane + am, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(plane + am, cur + g, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                // Round boundary: this round's plane writes land before the next
                // round's reads (other lanes, same pixel).  Also a compiler barrier.
                if (IN_LDS) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                else __builtin_amdgcn_s_waitcnt(0);
            }
        }
    }
    if (IN_LDS) {
        if ((HW & 3) == 0) {
            const float4* s4 = reinterpret_cast<const float4*>(plane);
            float4* d4 = reinterpret_cast<float4*>(gplane);
            for (int i = lane; i < HW / 4; i += 64) d4[i] = s4[i];
        } else {
            for (int i = lane; i < HW; i += 64) gplane[i] = plane[i];
        }
    }
}

}  // namespace frcnn

using namespace frcnn;

extern "C" int frcnn_roi_transform(const float* rois, const float* roi_inds, int64_t R, float img_h,
                                   float img_w, int feat_h, int feat_w, float* boxes,
                                   void* stream) {
    FRCNN_REQUIRE(R >= 0, "frcnn_roi_transform: R < 0");
    if (R == 0) return FRCNN_OK;
    FRCNN_REQUIRE(rois && roi_inds && boxes, "frcnn_roi_transform: null pointer");
    hipLaunchKernelGGL(roi_transform_kernel, dim3(static_cast<unsigned>((R + 255) / 256)),
                       dim3(256), 0, as_stream(stream), rois, roi_inds, R, img_h, img_w,
                       static_cast<float>(feat_h), static_cast<float>(feat_w), boxes);
    FRCNN_LAUNCH_CHECK("roi_transform_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_roi_pool_fwd(const float* x, const float* rois, int64_t R, int N, int C,
                                  int H, int W, int PH, int PW, float spatial_scale, float* out,
                                  int32_t* argmax, void* stream) {
    FRCNN_REQUIRE(R >= 0 && N >= 0 && C >= 0 && H >= 0 && W >= 0, "frcnn_roi_pool_fwd: bad shape");
    FRCNN_REQUIRE(PH > 0 && PW > 0 && PH * PW <= kMaxBins,
                  "frcnn_roi_pool_fwd: output_size must have 1..%d bins", kMaxBins);
    FRCNN_REQUIRE(R <= 0x7fffffff, "frcnn_roi_pool_fwd: too many rois");
    if (R == 0 || C == 0) return FRCNN_OK;
    FRCNN_REQUIRE(x && rois && out && argmax, "frcnn_roi_pool_fwd: null pointer");
    const size_t total = static_cast<size_t>(C) * PH * PW;
    const bool vec = (total % 4 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                     (reinterpret_cast<uintptr_t>(argmax) % 16 == 0);
    hipStream_t st = as_stream(stream);
    if (vec)
        hipLaunchKernelGGL(roi_pool_fwd_kernel<true>, dim3(static_cast<unsigned>(R)), dim3(256), 0,
                           st, x, rois, N, C, H, W, PH, PW, spatial_scale, out, argmax);
    else
        hipLaunchKernelGGL(roi_pool_fwd_kernel<false>, dim3(static_cast<unsigned>(R)), dim3(256), 0,
                           st, x, rois, N, C, H, W, PH, PW, spatial_scale, out, argmax);
    FRCNN_LAUNCH_CHECK("roi_pool_fwd_kernel");
    return FRCNN_OK;
}

namespace {
struct BwdWs {
    uint64_t* cmask;
    int* list;
    int* cnt;
    size_t bytes;
};
BwdWs carve_bwd(void* ws, int64_t R, int N, int PH, int PW) {
    Carver c(ws);
    BwdWs w{};
    w.cmask = c.take<uint64_t>(static_cast<size_t>(R) * PH * PW);
    w.list = c.take<int>(static_cast<size_t>(N) * R);
    w.cnt = c.take<int>(N);
    w.bytes = c.used();
    return w;
}
constexpr size_t kPlaneBudget = 64 * 1024;  // LDS per workgroup for planes
}  // namespace

extern "C" size_t frcnn_roi_pool_bwd_workspace_size(int64_t R, int N, int PH, int PW) {
    if (R < 0 || N < 0 || PH <= 0 || PW <= 0) return 0;
    return carve_bwd(nullptr, R, N, PH, PW).bytes;
}

extern "C" int frcnn_roi_pool_bwd(const float* grad, const float* rois, const int32_t* argmax,
                                  int64_t R, int N, int C, int H, int W, int PH, int PW,
                                  float spatial_scale, float* grad_in, void* workspace,
                                  size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(R >= 0 && N >= 0 && C >= 0 && H >= 0 && W >= 0, "frcnn_roi_pool_bwd: bad shape");
    FRCNN_REQUIRE(PH > 0 && PW > 0 && PH * PW <= kMaxBins, "frcnn_roi_pool_bwd: bad output_size");
    FRCNN_REQUIRE(R <= 0x7fffffff, "frcnn_roi_pool_bwd: too many rois");
    hipStream_t st = as_stream(stream);
    const size_t HW = static_cast<size_t>(H) * W;
    if (N == 0 || C == 0 || HW == 0) return FRCNN_OK;
    FRCNN_REQUIRE(grad_in, "frcnn_roi_pool_bwd: null grad_in");
    if (R == 0) {
        if (hipMemsetAsync(grad_in, 0, sizeof(float) * N * C * HW, st) != hipSuccess)
            return check_launch("frcnn_roi_pool_bwd memset");
        return FRCNN_OK;
    }
    FRCNN_REQUIRE(grad && rois && argmax, "frcnn_roi_pool_bwd: null pointer");
    BwdWs w = carve_bwd(workspace, R, N, PH, PW);
    FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_roi_pool_bwd: workspace %zu < %zu",
                  ws_bytes, w.bytes);
    FRCNN_REQUIRE(N <= 65535, "frcnn_roi_pool_bwd: N > 65535");
    hipLaunchKernelGGL(roi_bwd_prep_kernel, dim3(static_cast<unsigned>(R)), dim3(256), 0, st, rois,
                       H, W, PH, PW, spatial_scale, w.cmask);
    FRCNN_LAUNCH_CHECK("roi_bwd_prep_kernel");
    hipLaunchKernelGGL(roi_lists_kernel, dim3(N), dim3(1024), 0, st, rois, static_cast<int>(R),
                       w.list, w.cnt);
    FRCNN_LAUNCH_CHECK("roi_lists_kernel");
    const size_t plane_bytes = HW * sizeof(float);
    const int PHW = PH * PW;
    if (plane_bytes <= kPlaneBudget) {
        int cpw = static_cast<int>(kPlaneBudget / plane_bytes);
        cpw = cpw > 16 ? 16 : cpw;
        cpw = cpw > C ? C : cpw;
        dim3 grid((C + cpw - 1) / cpw, N);
        hipLaunchKernelGGL(roi_pool_bwd_kernel<true>, grid, dim3(64 * cpw), cpw * plane_bytes, st,
                           grad, argmax, w.cmask, w.list, w.cnt, static_cast<int>(R), C,
                           static_cast<int>(HW), PHW, cpw, grad_in);
    } else {
        const int cpw = 4;
        dim3 grid((C + cpw - 1) / cpw, N);
        hipLaunchKernelGGL(roi_pool_bwd_kernel<false>, grid, dim3(64 * cpw), 0, st, grad, argmax,
                           w.cmask, w.list, w.cnt, static_cast<int>(R), C, static_cast<int>(HW),
                           PHW, cpw, grad_in);
    }
    FRCNN_LAUNCH_CHECK("roi_pool_bwd_kernel");
    return FRCNN_OK;
}
