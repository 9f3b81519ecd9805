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
#include <cmath>
#include <cstdlib>
#include <cstring>

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

// Image-tile forward: a workgroup owns CG channel planes of image b (staged in
// LDS with one coalesced pass over HBM) and produces every RoI of that image
// (its share `split` of them) for those channels.  Outputs of one RoI for the
// CG channels are CG*PH*PW contiguous floats, written 4 per lane (float4 +
// int4).  Bin geometry is recomputed per element from 4 RoI scalars in LDS.
struct RoiGeom {
    int sh, sw;
    float bh, bw;
};

__device__ __forceinline__ RoiGeom roi_geom(const float* roi, float ss, int PH, int PW) {
    int sw = static_cast<int>(roundf(roi[1] * ss));
    int sh = static_cast<int>(roundf(roi[2] * ss));
    int ew = static_cast<int>(roundf(roi[3] * ss));
    int eh = static_cast<int>(roundf(roi[4] * ss));
    int rw = ew - sw + 1;
    int rh = eh - sh + 1;
    rw = rw > 1 ? rw : 1;
    rh = rh > 1 ? rh : 1;
    RoiGeom g;
    g.sh = sh;
    g.sw = sw;
    g.bh = static_cast<float>(rh) / static_cast<float>(PH);
    g.bw = static_cast<float>(rw) / static_cast<float>(PW);
    return g;
}

__device__ __forceinline__ int4 geom_bin(const RoiGeom& g, int H, int W, int ph, int pw) {
    int hs = static_cast<int>(floorf(static_cast<float>(ph) * g.bh)) + g.sh;
    int ws = static_cast<int>(floorf(static_cast<float>(pw) * g.bw)) + g.sw;
    int he = static_cast<int>(ceilf(static_cast<float>(ph + 1) * g.bh)) + g.sh;
    int we = static_cast<int>(ceilf(static_cast<float>(pw + 1) * g.bw)) + g.sw;
    return make_int4(min(max(hs, 0), H), min(max(he, 0), H), min(max(ws, 0), W),
                     min(max(we, 0), W));
}

constexpr int kTileRois = 64;   // RoI geometry staged per batch
constexpr int kTileThreads = 512;

// Four bin windows scanned in lock-step (4 independent LDS chains per lane).
// Each window keeps torchvision's row-major scan with a strict '>' update, so
// the result (max, first index of the max) is exactly the CPU kernel's.
__device__ __forceinline__ void pool_window4(const float* const (&pl)[4], int W, const int4 (&g)[4],
                                             float (&mv)[4], int (&mi)[4]) {
    int hmax = 0, wmax = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        mv[q] = (g[q].y <= g[q].x || g[q].w <= g[q].z) ? 0.0f : -FLT_MAX;
        mi[q] = -1;
        hmax = max(hmax, g[q].y - g[q].x);
        wmax = max(wmax, g[q].w - g[q].z);
    }
    for (int dh = 0; dh < hmax; ++dh) {
        for (int dw = 0; dw < wmax; ++dw) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int h = g[q].x + dh, w = g[q].z + dw;
                if (h < g[q].y && w < g[q].w) {
                    const int ii = h * W + w;
                    const float v = pl[q][ii];
                    if (v > mv[q]) {
                        mv[q] = v;
                        mi[q] = ii;
                    }
                }
            }
        }
    }
}

__global__ __launch_bounds__(kTileThreads) void roi_pool_fwd_tile_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ list,
    const int* __restrict__ cnt, int R, int C, int H, int W, int PH, int PW, int CG, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
    extern __shared__ __attribute__((aligned(16))) float planes[];  // [CG][H*W]
    __shared__ RoiGeom geo[kTileRois];
    __shared__ int rid[kTileRois];
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x;
    const int HW = H * W;
    const int PHW = PH * PW;
    const int nr = cnt[b];
    const int split = gridDim.z;
    const int r_begin = static_cast<int>(static_cast<int64_t>(nr) * blockIdx.z / split);
    const int r_end = static_cast<int>(static_cast<int64_t>(nr) * (blockIdx.z + 1) / split);
    if (r_begin >= r_end) return;
    // stage the CG planes (contiguous in NCHW): float4 when aligned
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    const int nf = CG * HW;
    if ((nf & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(planes);
        for (int i = tid; i < nf / 4; i += kTileThreads) d4[i] = s4[i];
    } else {
        for (int i = tid; i < nf; i += kTileThreads) planes[i] = src[i];
    }
    const int per_roi = CG * PHW;  // multiple of 4 (CG % 4 == 0)
    const int* lst = list + static_cast<size_t>(b) * R;
    for (int t0 = r_begin; t0 < r_end; t0 += kTileRois) {
        const int nt = min(kTileRois, r_end - t0);
        __syncthreads();  // planes staged / previous batch's geometry consumed
        if (tid < nt) {
            int r = lst[t0 + tid];
            rid[tid] = r;
            geo[tid] = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
        }
        __syncthreads();
        const int total = nt * per_roi;
        for (int f0 = tid * 4; f0 < total; f0 += 4 * kTileThreads) {
            // f0..f0+3 lie in one RoI's contiguous run (per_roi % 4 == 0)
            const int t = f0 / per_roi;
            const int e = f0 - t * per_roi;
            int cl = e / PHW;
            int k = e - cl * PHW;
            const RoiGeom gm = geo[t];
            const float* pl[4];
            int4 g[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                g[q] = geom_bin(gm, H, W, k / PW, k % PW);
                pl[q] = planes + cl * HW;
                if (++k == PHW) {
                    k = 0;
                    ++cl;
                }
            }
            float v[4];
            int m[4];
            pool_window4(pl, W, g, v, m);
            const size_t o = static_cast<size_t>(rid[t]) * C * PHW + static_cast<size_t>(c0) * PHW + e;
            *reinterpret_cast<float4*>(out + o) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<int4*>(argmax + o) = make_int4(m[0], m[1], m[2], m[3]);
        }
    }
}

// Wave-per-RoI variant: lane = bin (PH*PW <= 64), each lane pools its bin
// window in CG channel planes at once -- one loop control, CG independent LDS
// chains (plane offsets are immediates).  A wave writes one RoI's CG channel
// rows: out[r][c0+q][0..PHW) are PHW consecutive floats per q.
template <int CG>
__global__ __launch_bounds__(kTileThreads) void roi_pool_fwd_wave_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ list,
    const int* __restrict__ cnt, int R, int C, int H, int W, int PH, int PW, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
    extern __shared__ __attribute__((aligned(16))) float planes[];  // [CG][H*W]
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int kWaves = kTileThreads / 64;
    const int HW = H * W;
    const int PHW = PH * PW;
    const int nr = cnt[b];
    const int split = gridDim.z;
    const int r_begin = static_cast<int>(static_cast<int64_t>(nr) * blockIdx.z / split);
    const int r_end = static_cast<int>(static_cast<int64_t>(nr) * (blockIdx.z + 1) / split);
    if (r_begin >= r_end) return;
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    const int nf = CG * HW;
    if ((nf & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
        float4* d4 = reinterpret_cast<float4*>(planes);
        for (int i = tid; i < nf / 4; i += kTileThreads) d4[i] = s4[i];
    } else {
        for (int i = tid; i < nf; i += kTileThreads) planes[i] = src[i];
    }
    __syncthreads();
    const int* lst = list + static_cast<size_t>(b) * R;
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    for (int t = r_begin + wid; t < r_end; t += kWaves) {
        const int r = __builtin_amdgcn_readfirstlane(lst[t]);
        const RoiGeom gm = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
        int4 g = geom_bin(gm, H, W, ph, pw);
        if (!act) g = make_int4(0, 0, 0, 0);
        const bool empty = g.y <= g.x || g.w <= g.z;
        float mv[CG];
        int mi[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            mv[q] = empty ? 0.0f : -FLT_MAX;
            mi[q] = -1;
        }
        for (int h = g.x; h < g.y; ++h) {
            const float* row = planes + h * W;
            for (int w = g.z; w < g.w; ++w) {
                const int ii = h * W + w;
#pragma unroll
                for (int q = 0; q < CG; ++q) {
                    const float v = row[q * HW + w];
                    if (v > mv[q]) {
                        mv[q] = v;
                        mi[q] = ii;
                    }
                }
            }
        }
        if (act) {
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
#pragma unroll
            for (int q = 0; q < CG; ++q) {
                out[o + static_cast<size_t>(q) * PHW] = mv[q];
                argmax[o + static_cast<size_t>(q) * PHW] = mi[q];
            }
        }
    }
}

// Pixel-major variant: the LDS tile is [H*W][8] (8 channels of one pixel are
// 32 contiguous bytes), so a lane reads its bin pixel for all 8 channels with
// two ds_read_b128 from a single address -- no per-channel address math.
// Count of RoIs with batch index < b0 and < b1 (block-wide), for RoIs grouped by
// non-decreasing batch index: image b's RoIs are then [count(<b), count(<b+1)).
template <int NT>
__device__ __forceinline__ int2 roi_range_sorted(const float* __restrict__ rois, int R, int b0,
                                                 int b1, int* red, int stride = 5) {
    int c0 = 0, c1 = 0;
    for (int r = threadIdx.x; r < R; r += NT) {
        const int rb = static_cast<int>(rois[static_cast<size_t>(r) * stride]);
        c0 += rb < b0;
        c1 += rb < b1;
    }
    for (int o = 32; o > 0; o >>= 1) {
        c0 += __shfl_xor(c0, o, 64);
        c1 += __shfl_xor(c1, o, 64);
    }
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[2 * wid] = c0;
        red[2 * wid + 1] = c1;
    }
    __syncthreads();
    int2 res = make_int2(0, 0);
    for (int w = 0; w < NT / 64; ++w) {
        res.x += red[2 * w];
        res.y += red[2 * w + 1];
    }
    return res;
}

// SORTED: RoIs grouped by non-decreasing batch index (no list kernel, no fill
// kernel: grid row y == N writes 0 / -1 for RoIs whose index is outside [0, N)).
template <int NT, bool SORTED>
__global__ __launch_bounds__(NT) void roi_pool_fwd_px8_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ list,
    const int* __restrict__ cnt, int* __restrict__ queue, int R, int C, int H, int W, int PH,
    int PW, float ss, float* __restrict__ out, int32_t* __restrict__ argmax) {
    constexpr int CG = 8;
    extern __shared__ __attribute__((aligned(16))) float4 tile4[];  // [H*W][2] float4
    __shared__ int s_red[2 * (NT / 64)];
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int HW = H * W;
    const int PHW = PH * PW;
    const int split = gridDim.z;
    int nr, rbase = 0;
    if (SORTED) {
        const int N = gridDim.y - 1;
        if (b == N) {  // out-of-range batch indices: [0, count(<0)) and [count(<N), R)
            const int2 rg = roi_range_sorted<NT>(rois, R, 0, N, s_red);
            const int n_lo = rg.x, n_hi = R - rg.y, tot = n_lo + n_hi;
            const int lo = static_cast<int>(static_cast<int64_t>(tot) * blockIdx.z / split);
            const int hi = static_cast<int>(static_cast<int64_t>(tot) * (blockIdx.z + 1) / split);
            for (int e = lo * CG * PHW + tid; e < hi * CG * PHW; e += NT) {
                const int t = e / (CG * PHW);
                const int rem = e - t * (CG * PHW);
                const int r = t < n_lo ? t : rg.y + (t - n_lo);
                const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + rem;
                out[o] = 0.0f;
                argmax[o] = -1;
            }
            return;
        }
        const int2 rg = roi_range_sorted<NT>(rois, R, b, b + 1, s_red);
        rbase = rg.x;
        nr = rg.y - rg.x;
    } else {
        nr = cnt[b];
    }
    const int r_begin = static_cast<int>(static_cast<int64_t>(nr) * blockIdx.z / split);
    const int r_end = static_cast<int>(static_cast<int64_t>(nr) * (blockIdx.z + 1) / split);
    if (r_begin >= r_end) return;
    // The waves pull this workgroup's RoIs from an LDS counter: RoI sizes vary
    // a lot, a static round-robin leaves a long tail.
    __shared__ int s_next;
    if (tid == 0) s_next = r_begin;
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    float* tile = reinterpret_cast<float*>(tile4);
    for (int i = tid; i < CG * HW; i += NT) {
        const int qq = i / HW, p = i - qq * HW;
        tile[p * CG + qq] = src[i];
    }
    __syncthreads();
    const int* lst = SORTED ? nullptr : list + static_cast<size_t>(b) * R;
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    int t = 0;
    if (lane == 0) t = atomicAdd(&s_next, 1);
    t = __builtin_amdgcn_readfirstlane(t);
    while (t < r_end) {
        int tn = 0;
        if (lane == 0) tn = atomicAdd(&s_next, 1);  // prefetch the next item
        const int r = SORTED ? rbase + t : __builtin_amdgcn_readfirstlane(lst[t]);
        const RoiGeom gm = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
        int4 g = geom_bin(gm, H, W, ph, pw);
        if (!act) g = make_int4(0, 0, 0, 0);
        const bool empty = g.y <= g.x || g.w <= g.z;
        float mv[CG];
        int mi[CG];
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            mv[c] = empty ? 0.0f : -FLT_MAX;
            mi[c] = -1;
        }
        for (int h = g.x; h < g.y; ++h) {
            int ii = h * W + g.z;
            const int iend = h * W + g.w;
            for (; ii < iend; ++ii) {
                const float4 lo = tile4[2 * ii];
                const float4 hi = tile4[2 * ii + 1];
                const float v[CG] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    if (v[c] > mv[c]) {
                        mv[c] = v[c];
                        mi[c] = ii;
                    }
                }
            }
        }
        if (act) {
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                out[o + static_cast<size_t>(c) * PHW] = mv[c];
                argmax[o + static_cast<size_t>(c) * PHW] = mi[c];
            }
        }
        t = __builtin_amdgcn_readfirstlane(tn);
    }
}

// Strict '>' update of 8 running (max, first index) pairs with one pixel.
__device__ __forceinline__ void take8(const float4& a, const float4& b, int ii, float (&mv)[8],
                                      int (&mi)[8]) {
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (v[c] > mv[c]) {
            mv[c] = v[c];
            mi[c] = ii;
        }
    }
}

// px8q: px8 for image-grouped RoIs with
//  * a split-plane LDS tile: lo[s] = channels 0-3, hi[s] = channels 4-7 of
//    pixel p in slot s = p ^ ((p >> 4) & 15) (an XOR swizzle inside each
//    aligned 16-pixel group; the tile is padded to a multiple of 16 pixels).
//    A ds_read_b128 serves 16 lanes per LDS cycle on 16-B bank groups
//    ((a/16) mod 16); bins of one bin row sit a bin width apart, which in the
//    32-B interleaved px8 tile collide every 8 pixels -- here only within a
//    16-pixel group, and the swizzle scatters strides that cross groups;
//  * staging one pixel (8 channels) per thread: 8 coalesced global loads, two
//    ds_write_b128 (px8's strided ds_write_b32 is 8-way bank-conflicted);
//  * a strided RoI share: workgroup z of `split` takes items z, z+split, ...
//    of its image (RoI sizes are uncorrelated with rank, so every share sees
//    the image's size mix);
//  * CG = 16 (when 16 channel planes fit the CU's LDS, one workgroup per CU):
//    the RoI geometry, the window walk and the per-pixel address are shared by
//    16 channels instead of 8 -- the scan is VALU-issue bound, and these are a
//    third of its instructions at CG = 8.  Planes of 4 channels each.
// HEAD: fused with the head's RoI transform (nets/heads.py:42-47): `rois` are
// the RPN / sampler boxes [R,4] in image pixels, `hd.inds` their image index
// [R]; the [idx, box] pack is formed in registers (the same fp32 divide-then-
// multiply as roi_transform_kernel) and, when hd.boxes is set, written out
// once (channel group 0) for the backward.
struct HeadArgs {
    const float* inds;
    float img_h, img_w, fh, fw;
    float* boxes;
};

template <int NT, int CG, int MODE = 0, bool HEAD = false, bool SWZ = true>  // MODE (tools only): 1 = no stores, 2 = no window scan
__global__ __launch_bounds__(NT) void roi_pool_fwd_px8q_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, int R, int C, int H, int W,
    int PH, int PW, float ss, float* __restrict__ out, int32_t* __restrict__ argmax, int geo_cap,
    HeadArgs hd = HeadArgs{}) {
    constexpr int NP = CG / 4;                                     // planes of 4 channels
    extern __shared__ __attribute__((aligned(16))) float4 q4[];  // plane k at q4 + k * HWs; geometry after
    __shared__ int s_red[2 * (NT / 64)];
    __shared__ int s_next;
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int HW = H * W;
    const int HWs = (HW + 15) & ~15;
    const int PHW = PH * PW;
    const int split = gridDim.z, z = blockIdx.z;
    const int N = gridDim.y - 1;
    if (b == N) {  // out-of-range batch indices: [0, count(<0)) and [count(<N), R)
        const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, 0, N, s_red, 1)
                             : roi_range_sorted<NT>(rois, R, 0, N, s_red);
        const int n_lo = rg.x, n_hi = R - rg.y, tot = n_lo + n_hi;
        const int lo = static_cast<int>(static_cast<int64_t>(tot) * z / split);
        const int hi = static_cast<int>(static_cast<int64_t>(tot) * (z + 1) / split);
        if (HEAD && hd.boxes && blockIdx.x == 0)
            for (int t = lo + tid; t < hi; t += NT) {
                const int r = t < n_lo ? t : rg.y + (t - n_lo);
                const float4 v = reinterpret_cast<const float4*>(rois)[r];
                float* o = hd.boxes + static_cast<size_t>(r) * 5;
                o[0] = hd.inds[r];
                o[1] = v.x / hd.img_h * hd.fh;
                o[2] = v.y / hd.img_w * hd.fw;
                o[3] = v.z / hd.img_h * hd.fh;
                o[4] = v.w / hd.img_w * hd.fw;
            }
        for (int e = lo * CG * PHW + tid; e < hi * CG * PHW; e += NT) {
            const int t = e / (CG * PHW);
            const int rem = e - t * (CG * PHW);
            const int r = t < n_lo ? t : rg.y + (t - n_lo);
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + rem;
            out[o] = 0.0f;
            argmax[o] = -1;
        }
        return;
    }
    const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, b, b + 1, s_red, 1)
                         : roi_range_sorted<NT>(rois, R, b, b + 1, s_red);
    const int rbase = rg.x, nr = rg.y - rg.x;
    if (z >= nr) return;
    const int nmine = (nr - z + split - 1) / split;  // items z, z+split, ...
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    for (int p = tid; p < HW; p += NT) {
        float v[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) v[q] = src[static_cast<size_t>(q) * HW + p];
        const int s = SWZ ? p ^ ((p >> 4) & 15) : p;
#pragma unroll
        for (int k = 0; k < NP; ++k)
            q4[k * HWs + s] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    // RoI geometry (sh, sw, bin_h, bin_w) of up to geo_cap items at a time, computed
    // once per workgroup instead of once per wave: the rounds and the IEEE divides
    // (and, for HEAD, the transform's) are a fifth of a small RoI's VALU work.
    int4* s_geo = reinterpret_cast<int4*>(q4 + NP * HWs);
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    for (int k0 = 0; k0 < nmine; k0 += geo_cap) {
        const int cn = min(geo_cap, nmine - k0);
        for (int i = tid; i < cn; i += NT) {
            const int r = rbase + z + (k0 + i) * split;
            RoiGeom gm;
            if (HEAD) {
                const float4 v = reinterpret_cast<const float4*>(rois)[r];
                const float bx[5] = {hd.inds[r], v.x / hd.img_h * hd.fh, v.y / hd.img_w * hd.fw,
                                     v.z / hd.img_h * hd.fh, v.w / hd.img_w * hd.fw};
                gm = roi_geom(bx, ss, PH, PW);
                if (hd.boxes && blockIdx.x == 0) {
                    float* o = hd.boxes + static_cast<size_t>(r) * 5;
#pragma unroll
                    for (int j = 0; j < 5; ++j) o[j] = bx[j];
                }
            } else {
                gm = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
            }
            s_geo[i] = make_int4(gm.sh, gm.sw, __float_as_int(gm.bh), __float_as_int(gm.bw));
        }
        if (tid == 0) s_next = 0;
        __syncthreads();
        int k = 0;
        if (lane == 0) k = atomicAdd(&s_next, 1);
        k = __builtin_amdgcn_readfirstlane(k);
        while (k < cn) {
            int kn = 0;
            if (lane == 0) kn = atomicAdd(&s_next, 1);  // prefetch the next item
            const int r = rbase + z + (k0 + k) * split;
            const int4 gq = s_geo[k];
            RoiGeom gm;
            gm.sh = gq.x;
            gm.sw = gq.y;
            gm.bh = __int_as_float(gq.z);
            gm.bw = __int_as_float(gq.w);
            int4 g = geom_bin(gm, H, W, ph, pw);
            if (!act) g = make_int4(0, 0, 0, 0);
            const bool empty = g.y <= g.x || g.w <= g.z;
            float mv[CG];
            int mi[CG];
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                mv[c] = empty ? 0.0f : -FLT_MAX;
                mi[c] = -1;
            }
            for (int h = g.x; h < (MODE == 2 ? g.x : g.y); ++h) {
                const int rb = h * W;
                for (int w = g.z; w < g.w; ++w) {
                    const int ii = rb + w;
                    const int s = SWZ ? ii ^ ((ii >> 4) & 15) : ii;
                    float4 v[NP];
#pragma unroll
                    for (int q = 0; q < NP; ++q) v[q] = q4[q * HWs + s];
#pragma unroll
                    for (int q = 0; q < NP; ++q) {
                        const float vv[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (vv[j] > mv[4 * q + j]) {  // torchvision's strict '>'
                                mv[4 * q + j] = vv[j];
                                mi[4 * q + j] = ii;
                            }
                        }
                    }
                }
            }
            if (act && (MODE != 1 || mv[0] == 1234.5f)) {
                const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    out[o + static_cast<size_t>(c) * PHW] = mv[c];
                    argmax[o + static_cast<size_t>(c) * PHW] = mi[c];
                }
            }
            k = __builtin_amdgcn_readfirstlane(kn);
        }
        __syncthreads();  // the chunk's geometry and s_next are reused
    }
}

__device__ __forceinline__ float nan_to_ninf(float v) { return v != v ? -INFINITY : v; }

// px8r: the px8q work split with fewer VALU per channel-pixel.
//  * Tile: two planes, lo[p] = channels 0-3, hi[p] = channels 4-7 of pixel p
//    (no swizzle: one address per pixel, stepped by 16 B; hi at a fixed
//    ds_read offset).  NaN is staged as -inf: neither ever passes the
//    reference's strict '>' against the -FLT_MAX start, so the result is the
//    same, and v_max3 never sees a NaN.
//  * Pixels are taken in row-major pairs (a, b) (b clamped to the row end: a
//    revisit of a is harmless).  Per channel: m' = max3(m, a, b); if m' > m the
//    max moved into the pair, to a if a == m' (a first), else to b.  That is
//    the strict-'>' first-max scan exactly (a tie with m never moves it), at
//    5 VALU per pair instead of 6; a shared pair of indices, one address.
//  * The kept value is m' from max3, which may differ from the first max in
//    the sign of a zero; the final value is re-read from the tile at the
//    argmax when it compares equal to 0.
__device__ __forceinline__ void take8_pair(const float4& a0, const float4& a1, const float4& b0,
                                           const float4& b1, int ia, int ib, float (&mv)[8],
                                           int (&mi)[8]) {
    const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float m2 = __builtin_fmaxf(__builtin_fmaxf(mv[c], a[c]), b[c]);
        const int ip = a[c] == m2 ? ia : ib;
        if (m2 > mv[c]) mi[c] = ip;
        mv[c] = m2;
    }
}

template <int NT, int MODE = 0>  // MODE (tools only): 1 = no stores
__global__ __launch_bounds__(NT) void roi_pool_fwd_px8r_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, int R, int C, int H, int W,
    int PH, int PW, float ss, float* __restrict__ out, int32_t* __restrict__ argmax) {
    constexpr int CG = 8;
    extern __shared__ __attribute__((aligned(16))) float4 r4[];  // lo[HW] then hi[HW]
    __shared__ int s_red[2 * (NT / 64)];
    __shared__ int s_next;
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int HW = H * W;
    const int PHW = PH * PW;
    const int split = gridDim.z, z = blockIdx.z;
    const int N = gridDim.y - 1;
    if (b == N) {  // out-of-range batch indices: [0, count(<0)) and [count(<N), R)
        const int2 rg = roi_range_sorted<NT>(rois, R, 0, N, s_red);
        const int n_lo = rg.x, n_hi = R - rg.y, tot = n_lo + n_hi;
        const int lo = static_cast<int>(static_cast<int64_t>(tot) * z / split);
        const int hi = static_cast<int>(static_cast<int64_t>(tot) * (z + 1) / split);
        for (int e = lo * CG * PHW + tid; e < hi * CG * PHW; e += NT) {
            const int t = e / (CG * PHW);
            const int rem = e - t * (CG * PHW);
            const int r = t < n_lo ? t : rg.y + (t - n_lo);
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + rem;
            out[o] = 0.0f;
            argmax[o] = -1;
        }
        return;
    }
    const int2 rg = roi_range_sorted<NT>(rois, R, b, b + 1, s_red);
    const int rbase = rg.x, nr = rg.y - rg.x;
    if (z >= nr) return;
    const int nmine = (nr - z + split - 1) / split;  // items z, z+split, ...
    if (tid == 0) s_next = 0;
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    for (int p = tid; p < HW; p += NT) {
        float v[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) v[q] = nan_to_ninf(src[static_cast<size_t>(q) * HW + p]);
        r4[p] = make_float4(v[0], v[1], v[2], v[3]);
        r4[HW + p] = make_float4(v[4], v[5], v[6], v[7]);
    }
    __syncthreads();
    const char* tb = reinterpret_cast<const char*>(r4);
    const int hoff = HW * 16;
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    int k = 0;
    if (lane == 0) k = atomicAdd(&s_next, 1);
    k = __builtin_amdgcn_readfirstlane(k);
    while (k < nmine) {
        int kn = 0;
        if (lane == 0) kn = atomicAdd(&s_next, 1);  // prefetch the next item
        const int r = rbase + z + k * split;
        const RoiGeom gm = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
        int4 g = geom_bin(gm, H, W, ph, pw);
        if (!act) g = make_int4(0, 0, 0, 0);
        const bool empty = g.y <= g.x || g.w <= g.z;
        float mv[CG];
        int mi[CG];
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            mv[c] = empty ? 0.0f : -FLT_MAX;
            mi[c] = -1;
        }
        const int wlast = g.w - 1;
        for (int h = g.x; h < g.y; ++h) {
            const int rb = h * W;
            for (int w = g.z; w < g.w; w += 2) {
                const int ia = rb + w, ib = rb + min(w + 1, wlast);
                const float4 a0 = *reinterpret_cast<const float4*>(tb + ia * 16);
                const float4 a1 = *reinterpret_cast<const float4*>(tb + hoff + ia * 16);
                const float4 b0 = *reinterpret_cast<const float4*>(tb + ib * 16);
                const float4 b1 = *reinterpret_cast<const float4*>(tb + hoff + ib * 16);
                take8_pair(a0, a1, b0, b1, ia, ib, mv, mi);
            }
        }
        if (act && (MODE != 1 || mv[0] == 1234.5f)) {
            const float* tf = reinterpret_cast<const float*>(r4);
#pragma unroll
            for (int c = 0; c < CG; ++c)  // exact bits of a zero maximum
                if (mv[c] == 0.0f && mi[c] >= 0) mv[c] = tf[(c < 4 ? 0 : 4 * HW) + 4 * mi[c] + (c & 3)];
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                out[o + static_cast<size_t>(c) * PHW] = mv[c];
                argmax[o + static_cast<size_t>(c) * PHW] = mi[c];
            }
        }
        k = __builtin_amdgcn_readfirstlane(kn);
    }
}

// ---------------------------------------------------- cost-balanced forward
// Work estimate of one RoI for the wave-per-RoI loop below: the wave's pixel
// loop runs (max bin-window height) x (max bin-window width) iterations --
// about floor(bin size) + 2 each way, at most the RoI's visible extent -- plus
// a fixed part (geometry, 2*CG stores).  A RoI with an out-of-range batch
// index, or entirely outside the map, only stores.
__device__ __forceinline__ int roi_cost_fast(const float* __restrict__ rois, int t, float ss, int N, int H,
                                             int W, int PH, int PW) {
    const float* roi = rois + static_cast<size_t>(t) * 5;
    const int b = static_cast<int>(roi[0]);
    const int sw = static_cast<int>(roundf(roi[1] * ss));
    const int sh = static_cast<int>(roundf(roi[2] * ss));
    const int ew = static_cast<int>(roundf(roi[3] * ss));
    const int eh = static_cast<int>(roundf(roi[4] * ss));
    if (b < 0 || b >= N) return 1;
    const int rw = max(ew - sw + 1, 1), rh = max(eh - sh + 1, 1);
    const int hv = min(sh + rh + 1, H) - max(sh, 0);
    const int wv = min(sw + rw + 1, W) - max(sw, 0);
    if (hv <= 0 || wv <= 0) return 1;
    const int mh = min(static_cast<int>(static_cast<float>(rh) * __frcp_rn(static_cast<float>(PH))) + 2, hv);
    const int mw = min(static_cast<int>(static_cast<float>(rw) * __frcp_rn(static_cast<float>(PW))) + 2, wv);
    return mh * mw + 6;
}

template <int NT>
__device__ __forceinline__ int block_min(int v, int64_t* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    int m = v;
    for (int w = 0; w < NT / 64; ++w) m = min(m, static_cast<int>(red[w]));
    return m;
}

// Cost-balanced forward for RoIs grouped by batch index (proposals;
// train.py's sample_rois), two launches:
//
// roi_partition_kernel (one workgroup): per-RoI cost (roi_cost_fast), prefix
// sum, and a cut of the RoI list into S contiguous segments of equal cost
// (RoI t goes to the 1/S slice holding its cost midpoint): seg_lo[0..S],
// plus, per segment, the positions where the batch index changes (up to
// kBalMaxRuns - 1 listed; the count is exact).
//
// roi_pool_fwd_bal_kernel, grid (S, C/8): workgroup (s, g) produces channels
// [8g, 8g+8) of segment s -- every workgroup of the (one resident round) grid
// gets the same work, so they end together; a split by RoI count waits for
// the workgroup that drew the largest RoIs.  It walks its segment in runs of
// equal batch index (usually one or two), stages that image's 8-channel tile
// into LDS as pixel-major [H*W][8], and its waves pull RoIs from an LDS
// counter: lane = bin, each lane scans its bin window once, 8 channel maxima
// from two ds_read_b128 per pixel, strict '>' in row-major order (the CPU
// kernel's first-max rule).  Runs split at every batch index change, so the
// result is exact for any RoI order (only slower when RoIs are not grouped).
constexpr int kBalMaxRuns = 32;
constexpr int kSegInfo = 1 + kBalMaxRuns;  // per segment: #changes, change positions
// tools-only timeline probe (variant "baldbg"): per workgroup, s_memrealtime
// (100 MHz) at entry / after the partition / after the first tile / exit
__device__ unsigned long long g_bal_dbg[8 * 8192];

template <int NT, int COST>
__global__ __launch_bounds__(NT) void roi_partition_kernel(const float* __restrict__ rois, int R, int N,
                                                           int H, int W, int PH, int PW, float ss, int S,
                                                           int* __restrict__ seg_lo,
                                                           int* __restrict__ seg_info) {
    constexpr int NWV = NT / 64;
    __shared__ int64_t s_red[NWV];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int q = tid; q < S; q += NT) seg_info[static_cast<size_t>(q) * kSegInfo] = 0;
    const int per_w = (R + NWV - 1) / NWV;
    const int wt0 = min(wid * per_w, R), wt1 = min(wt0 + per_w, R);
    auto cost = [&](int t) { return COST ? roi_cost_fast(rois, t, ss, N, H, W, PH, PW) : 1; };
    int64_t wsum = 0;
    for (int t = wt0 + lane; t < wt1; t += 64) wsum += cost(t);
    for (int o = 32; o > 0; o >>= 1) wsum += __shfl_xor(wsum, o, 64);
    if (lane == 0) s_red[wid] = wsum;
    __syncthreads();  // also orders the counter zeroing before the atomics below
    int64_t carry = 0, total = 0;
    for (int w = 0; w < NWV; ++w) {
        carry += w < wid ? s_red[w] : 0;
        total += s_red[w];
    }
    const double scale = static_cast<double>(S) / (2.0 * static_cast<double>(total));
    auto seg_at = [&](int64_t pre, int c) {
        const int st = static_cast<int>(static_cast<double>(2 * pre + c) * scale);
        return st < S - 1 ? st : S - 1;
    };
    // (segment, batch index) of the RoI before the current one
    int prev_seg = -1, prev_b = 0;
    if (wt0 > 0 && wt0 < wt1) {
        const int cp = cost(wt0 - 1);
        prev_seg = seg_at(carry - cp, cp);
        prev_b = static_cast<int>(rois[static_cast<size_t>(wt0 - 1) * 5]);
    }
    for (int base = wt0; base < wt1; base += 64) {
        const int t = base + lane;
        const bool in = t < wt1;
        const int c = in ? cost(t) : 0;
        const int bt = in ? static_cast<int>(rois[static_cast<size_t>(t) * 5]) : 0;
        int64_t inc = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        const int st = in ? seg_at(carry + inc - c, c) : S;
        int ps = __shfl_up(st, 1, 64), pb = __shfl_up(bt, 1, 64);
        if (lane == 0) {
            ps = prev_seg;
            pb = prev_b;
        }
        if (in) {
            for (int q = ps + 1; q <= st; ++q) seg_lo[q] = t;  // first RoI of segments (ps, st]
            if (t > 0 && st == ps && bt != pb) {               // batch change inside a segment
                const int k = atomicAdd(&seg_info[static_cast<size_t>(st) * kSegInfo], 1);
                if (k < kBalMaxRuns - 1) seg_info[static_cast<size_t>(st) * kSegInfo + 1 + k] = t;
            }
        }
        const int last = min(63, wt1 - 1 - base);  // last lane holding a RoI
        carry += __shfl(inc, last, 64);
        prev_seg = __shfl(st, last, 64);
        prev_b = __shfl(bt, last, 64);
    }
    // segments after the last RoI's are empty: the wave holding RoI R-1 closes them
    if (wt0 < wt1 && wt1 == R)
        for (int q = prev_seg + 1 + lane; q <= S; q += 64) seg_lo[q] = R;
}

// MODE (tools/ab_roi_pool.py diagnostics only): 0 = the op; 1 = no pooling
// (stores 0 / -1: staging + store floor); 2 = pooling, stores only if an
// impossible value shows up (compute floor)
template <int NT, bool DBG = false, int MODE = 0>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8, 8))) void roi_pool_fwd_bal_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ seg_lo,
    const int* __restrict__ seg_info, int N, int C, int H, int W, int PH, int PW, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
    constexpr int CG = 8;
    extern __shared__ __attribute__((aligned(16))) float4 tile4[];  // [H*W][2] float4
    __shared__ int64_t s_red[NT / 64];
    __shared__ int s_runs[kBalMaxRuns];
    __shared__ int s_next;
    const int seg = blockIdx.x;
    const int c0 = blockIdx.y * CG;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int HW = H * W;
    const int PHW = PH * PW;
    const unsigned wg = blockIdx.x + blockIdx.y * gridDim.x;
    if (DBG && tid == 0 && wg < 8192) {
        g_bal_dbg[wg * 8 + 0] = __builtin_amdgcn_s_memrealtime();
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        g_bal_dbg[wg * 8 + 5] = hw;
    }
    const int lo = seg_lo[seg], hi = seg_lo[seg + 1];
    const int* info = seg_info + static_cast<size_t>(seg) * kSegInfo;
    const int n_chg = info[0];
    const int n_runs = hi > lo ? n_chg + 1 : 0;
    const bool listed = n_runs <= kBalMaxRuns;
    if (listed && wid == 0 && n_runs > 1) {  // run starts: lo, then the sorted change positions
        int v = lane < n_chg ? info[1 + lane] : 0x7fffffff;
        for (int k = 2; k <= 64; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                const int o = __shfl_xor(v, j, 64);
                const bool up = (lane & k) == 0, low = (lane & j) == 0;
                v = (low == up) ? min(v, o) : max(v, o);
            }
        if (lane < n_chg) s_runs[1 + lane] = v;
    }
    if (tid == 0) s_runs[0] = lo;
    __syncthreads();
    if (DBG && tid == 0 && wg < 8192) {
        g_bal_dbg[wg * 8 + 1] = __builtin_amdgcn_s_memrealtime();
        g_bal_dbg[wg * 8 + 6] = (static_cast<unsigned long long>(hi - lo) << 32) | n_runs;
    }
    // 3. per run: stage the tile, pool every RoI of the run
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    int run = 0;
    int t_run = lo;
    while (t_run < hi) {
        const int b = static_cast<int>(rois[static_cast<size_t>(t_run) * 5]);
        int t_end;
        if (listed) {
            t_end = run + 1 < n_runs ? s_runs[run + 1] : hi;
            ++run;
        } else {
            int first = hi;
            for (int t = t_run + 1 + tid; t < hi; t += NT)
                if (static_cast<int>(rois[static_cast<size_t>(t) * 5]) != b) {
                    first = t;
                    break;
                }
            t_end = block_min<NT>(first, s_red);
        }
        const bool valid = b >= 0 && b < N;
        __syncthreads();  // the previous run's waves are done with the tile and s_next
        if (valid) {
            const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
            for (int p = tid; p < HW; p += NT) {
                float v[CG];
#pragma unroll
                for (int q = 0; q < CG; ++q) v[q] = src[static_cast<size_t>(q) * HW + p];
                tile4[2 * p] = make_float4(v[0], v[1], v[2], v[3]);
                tile4[2 * p + 1] = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
        if (tid == 0) s_next = t_run;
        __syncthreads();
        if (DBG && tid == 0 && wg < 8192 && run <= 1) g_bal_dbg[wg * 8 + 2] = __builtin_amdgcn_s_memrealtime();
        int t = 0;
        if (lane == 0) t = atomicAdd(&s_next, 1);
        t = __builtin_amdgcn_readfirstlane(t);
        while (t < t_end) {
            int tn = 0;
            if (lane == 0) tn = atomicAdd(&s_next, 1);  // prefetch the next item
            const size_t o = (static_cast<size_t>(t) * C + c0) * PHW + lane;
            float mv[CG];
            int mi[CG];
            if (valid && MODE != 1) {
                const RoiGeom gm = roi_geom(rois + static_cast<size_t>(t) * 5, ss, PH, PW);
                int4 g = geom_bin(gm, H, W, ph, pw);
                if (!act) g = make_int4(0, 0, 0, 0);
                const bool empty = g.y <= g.x || g.w <= g.z;
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    mv[c] = empty ? 0.0f : -FLT_MAX;
                    mi[c] = -1;
                }
                for (int h = g.x; h < g.y; ++h) {
                    int ii = h * W + g.z;
                    const int iend = h * W + g.w;
                    for (; ii < iend; ++ii) {
                        const float4 lo4 = tile4[2 * ii];
                        const float4 hi4 = tile4[2 * ii + 1];
                        const float v[CG] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
#pragma unroll
                        for (int c = 0; c < CG; ++c) {
                            if (v[c] > mv[c]) {
                                mv[c] = v[c];
                                mi[c] = ii;
                            }
                        }
                    }
                }
            } else {
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    mv[c] = 0.0f;
                    mi[c] = -1;
                }
            }
            if (act && (MODE != 2 || mv[0] == 1234.5f)) {
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    out[o + static_cast<size_t>(c) * PHW] = mv[c];
                    argmax[o + static_cast<size_t>(c) * PHW] = mi[c];
                }
            }
            t = __builtin_amdgcn_readfirstlane(tn);
        }
        t_run = t_end;
    }
    if (DBG) {
        __syncthreads();
        if (tid == 0 && wg < 8192) g_bal_dbg[wg * 8 + 3] = __builtin_amdgcn_s_memrealtime();
    }
}

// ------------------------------------------------ balanced forward, v2
// Same partition, runs and tile as roi_pool_fwd_bal_kernel; the per-RoI loop
// is wave-uniform: every lane walks the wave's largest bin window, (max bin
// height) x (max bin width), row-major over its own window with the row /
// column clamped to its last one.  A clamped step revisits a pixel the lane
// has already seen, which can never pass the strict '>' again, so each lane's
// (max, first index) is exactly its own row-major scan's; an empty bin reads
// the -inf pad pixel (index H*W).  Loop control is scalar (no exec-mask
// updates per pixel) and two pixels are in flight per step.
// SWAP: half the lanes of every ds_read_b128 lane group read a pixel's two
// 16-B slots in the other order, so lanes on pixels 8k apart hit different
// slots; such a lane's registers 0-3 hold channels 4-7 (a fixed per-lane
// permutation, undone by its store addresses).
// FIX: PH = PW = FIX at compile time (the reference's 7x7, nets/heads.py:8):
// constant lane -> bin map and immediate store offsets.
// XCD-aware order: workgroups go round-robin over the 8 XCDs by linear id
// (= blockIdx.x mod 8 when S % 8 == 0); each XCD gets a contiguous run of
// S/8 segments, so the workgroups staging the same image tile share an L2.
// MODE (diagnostics, tools/ab_roi_pool.py): 0 = the op; 2 = no stores;
// 3 = no stores and every lane reads lane 0's pixel (no bank conflicts).
__device__ __forceinline__ int wave_max_i32(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

template <int NT, int FIX, bool SWAP, int MODE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8, 8))) void roi_pool_fwd_bal2_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ seg_lo,
    const int* __restrict__ seg_info, int N, int C, int H, int W, int PH_, int PW_, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
    constexpr int CG = 8;
    extern __shared__ __attribute__((aligned(16))) float4 tile4[];  // [H*W + 1][2] float4
    __shared__ int64_t s_red[NT / 64];
    __shared__ int s_runs[kBalMaxRuns];
    __shared__ int s_next;
    const int PH = FIX ? FIX : PH_, PW = FIX ? FIX : PW_;
    const int S = gridDim.x;
    const int seg = (S % 8 == 0) ? static_cast<int>(blockIdx.x % 8) * (S / 8) + static_cast<int>(blockIdx.x / 8)
                                 : static_cast<int>(blockIdx.x);
    const int c0 = blockIdx.y * CG;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int HW = H * W;
    const int PHW = PH * PW;
    if (tid < 2) tile4[2 * HW + tid] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    const int lo = seg_lo[seg], hi = seg_lo[seg + 1];
    const int* info = seg_info + static_cast<size_t>(seg) * kSegInfo;
    const int n_chg = info[0];
    const int n_runs = hi > lo ? n_chg + 1 : 0;
    const bool listed = n_runs <= kBalMaxRuns;
    if (listed && wid == 0 && n_runs > 1) {  // run starts: lo, then the sorted change positions
        int v = lane < n_chg ? info[1 + lane] : 0x7fffffff;
        for (int k = 2; k <= 64; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                const int o = __shfl_xor(v, j, 64);
                const bool up = (lane & k) == 0, low = (lane & j) == 0;
                v = (low == up) ? min(v, o) : max(v, o);
            }
        if (lane < n_chg) s_runs[1 + lane] = v;
    }
    if (tid == 0) s_runs[0] = lo;
    __syncthreads();
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    const int swp = SWAP ? ((lane >> 2) & 1) : 0;
    const char* tb = reinterpret_cast<const char*>(tile4);
    const int offa = swp * 16;
    int run = 0;
    int t_run = lo;
    while (t_run < hi) {
        const int b = static_cast<int>(rois[static_cast<size_t>(t_run) * 5]);
        int t_end;
        if (listed) {
            t_end = run + 1 < n_runs ? s_runs[run + 1] : hi;
            ++run;
        } else {
            int first = hi;
            for (int t = t_run + 1 + tid; t < hi; t += NT)
                if (static_cast<int>(rois[static_cast<size_t>(t) * 5]) != b) {
                    first = t;
                    break;
                }
            t_end = block_min<NT>(first, s_red);
        }
        const bool valid = b >= 0 && b < N;
        __syncthreads();  // the previous run's waves are done with the tile and s_next
        if (valid) {
            const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
            for (int p = tid; p < HW; p += NT) {
                float v[CG];
#pragma unroll
                for (int q = 0; q < CG; ++q) v[q] = src[static_cast<size_t>(q) * HW + p];
                tile4[2 * p] = make_float4(v[0], v[1], v[2], v[3]);
                tile4[2 * p + 1] = make_float4(v[4], v[5], v[6], v[7]);
            }
        }
        if (tid == 0) s_next = t_run;
        __syncthreads();
        int t = 0;
        if (lane == 0) t = atomicAdd(&s_next, 1);
        t = __builtin_amdgcn_readfirstlane(t);
        while (t < t_end) {
            int tn = 0;
            if (lane == 0) tn = atomicAdd(&s_next, 1);  // prefetch the next item
            float mv[CG];
            int mi[CG];
            if (valid) {
                const RoiGeom gm = roi_geom(rois + static_cast<size_t>(t) * 5, ss, PH, PW);
                const int4 g = geom_bin(gm, H, W, ph, pw);
                const int hgt = g.y - g.x, wdt = g.w - g.z;
                const bool empty = hgt <= 0 || wdt <= 0;
                const bool live = act && !empty;
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    mv[c] = empty ? 0.0f : -FLT_MAX;
                    mi[c] = -1;
                }
                const int MH = wave_max_i32(live ? hgt : 0);
                const int MW = wave_max_i32(live ? wdt : 0);
                const int lastr = live ? hgt - 1 : 0, lastc = live ? wdt - 1 : 0;
                const int org = live ? g.x * W + g.z : HW;  // window origin; dead lanes: pad pixel
                const int rstep = live ? W : 0;
                const int tot = MH * MW;
                int dh = 0, dw = 0, rowi = org;
                for (int s = 0; s < tot; s += 2) {
                    if (dw == 0) rowi = org + min(dh, lastr) * rstep;
                    const int iiA = rowi + min(dw, lastc);
                    if (++dw == MW) {
                        dw = 0;
                        ++dh;
                    }
                    int iiB = iiA;  // past the end: a revisit of A
                    if (s + 1 < tot) {
                        if (dw == 0) rowi = org + min(dh, lastr) * rstep;
                        iiB = rowi + min(dw, lastc);
                        if (++dw == MW) {
                            dw = 0;
                            ++dh;
                        }
                    }
                    const int rA = MODE == 3 ? __builtin_amdgcn_readfirstlane(iiA) : iiA;
                    const int rB = MODE == 3 ? __builtin_amdgcn_readfirstlane(iiB) : iiB;
                    const int adA = rA * 32 + offa, adB = rB * 32 + offa;
                    const float4 a0 = *reinterpret_cast<const float4*>(tb + adA);
                    const float4 a1 = *reinterpret_cast<const float4*>(tb + (adA ^ 16));
                    const float4 b0 = *reinterpret_cast<const float4*>(tb + adB);
                    const float4 b1 = *reinterpret_cast<const float4*>(tb + (adB ^ 16));
                    take8(a0, a1, iiA, mv, mi);
                    take8(b0, b1, iiB, mv, mi);
                }
            } else {
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    mv[c] = 0.0f;
                    mi[c] = -1;
                }
            }
            if (act && (MODE == 0 || mv[0] == 1234.5f)) {
                // registers 0-3 / 4-7 hold channels 0-3 / 4-7, swapped when swp
                const size_t o = (static_cast<size_t>(t) * C + c0) * PHW + lane;
                const size_t qa = static_cast<size_t>(swp) * 4 * PHW;
                const size_t qb = static_cast<size_t>(4 - 4 * swp) * PHW;
                float* oa = out + o + qa;
                float* ob = out + o + qb;
                int32_t* ia = argmax + o + qa;
                int32_t* ib = argmax + o + qb;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    oa[c * PHW] = mv[c];
                    ob[c * PHW] = mv[4 + c];
                    ia[c * PHW] = mi[c];
                    ib[c * PHW] = mi[4 + c];
                }
            }
            t = __builtin_amdgcn_readfirstlane(tn);
        }
        t_run = t_end;
    }
}

// Flattened, software-pipelined pixel-major variant.  The LDS tile is
// [H*W+1][CG] (CG = 4 or 8 channels per pixel, one or two ds_read_b128); a lane
// walks its bin window as ONE loop over bin_h*bin_w pixels (row-major, so the
// strict-'>' first-max scan order is the reference's), loading pixel k+1
// before comparing pixel k.  Waves pull RoIs from an LDS counter.
template <int CG>
__global__ __launch_bounds__(kTileThreads) void roi_pool_fwd_pxf_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ list,
    const int* __restrict__ cnt, int R, int C, int H, int W, int PH, int PW, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
    constexpr int NV = CG / 4;  // float4 per pixel
    extern __shared__ __attribute__((aligned(16))) float4 tile4[];  // [H*W + 1][NV]
    __shared__ int s_next;
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int HW = H * W;
    const int PHW = PH * PW;
    const int nr = cnt[b];
    const int split = gridDim.z;
    const int r_begin = static_cast<int>(static_cast<int64_t>(nr) * blockIdx.z / split);
    const int r_end = static_cast<int>(static_cast<int64_t>(nr) * (blockIdx.z + 1) / split);
    if (r_begin >= r_end) return;
    if (tid == 0) s_next = r_begin;
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    float* tile = reinterpret_cast<float*>(tile4);
    for (int i = tid; i < CG * HW; i += kTileThreads) {
        const int qq = i / HW, p = i - qq * HW;
        tile[p * CG + qq] = src[i];
    }
    if (tid < CG) tile[HW * CG + tid] = 0.0f;  // pad pixel: the prefetch may touch it
    __syncthreads();
    const int* lst = list + static_cast<size_t>(b) * R;
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    int t = 0;
    if (lane == 0) t = atomicAdd(&s_next, 1);
    t = __builtin_amdgcn_readfirstlane(t);
    while (t < r_end) {
        int tn = 0;
        if (lane == 0) tn = atomicAdd(&s_next, 1);
        const int r = __builtin_amdgcn_readfirstlane(lst[t]);
        const RoiGeom gm = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
        int4 g = geom_bin(gm, H, W, ph, pw);
        if (!act) g = make_int4(0, 0, 0, 0);
        const int bwid = g.w - g.z;
        const int bhgt = g.y - g.x;
        const bool empty = bhgt <= 0 || bwid <= 0;
        const int n = empty ? 0 : bhgt * bwid;
        float mv[CG];
        int mi[CG];
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            mv[c] = empty ? 0.0f : -FLT_MAX;
            mi[c] = -1;
        }
        int ii = empty ? HW : g.x * W + g.z;  // HW = the pad pixel
        const int jump = W - bwid + 1;
        int col = 0;
        float4 cur[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) cur[v] = tile4[ii * NV + v];
        for (int k = 0; k < n; ++k) {
            const int here = ii;
            if (++col == bwid) {
                col = 0;
                ii += jump;
            } else {
                ++ii;
            }
            const int nx = ii < HW ? ii : HW;
            float4 nxt[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) nxt[v] = tile4[nx * NV + v];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const float vals[4] = {cur[v].x, cur[v].y, cur[v].z, cur[v].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (vals[e] > mv[4 * v + e]) {
                        mv[4 * v + e] = vals[e];
                        mi[4 * v + e] = here;
                    }
                }
            }
#pragma unroll
            for (int v = 0; v < NV; ++v) cur[v] = nxt[v];
        }
        if (act) {
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                out[o + static_cast<size_t>(c) * PHW] = mv[c];
                argmax[o + static_cast<size_t>(c) * PHW] = mi[c];
            }
        }
        t = __builtin_amdgcn_readfirstlane(tn);
    }
}

// Two-pass pixel-major variant (default).  The reference's strict-'>' scan
// selects the FIRST element (row-major) equal to the window maximum among the
// values > init (init = -FLT_MAX, or 0 for an empty bin).  So:
//   pass 1: per bin row, rowmax = max3-chain over pixel pairs (0.5 VALU per
//           channel-pixel); the running max keeps the FIRST row that raised it;
//   pass 2: in that row only, the first pixel equal to the max gives the index
//           and the output value (its exact bits, e.g. -0.0 vs +0.0).
// NaN never wins in the reference; it is staged into LDS as -inf, which never
// wins either.  A max not above init means "nothing selected": (init, -1).

__global__ __launch_bounds__(kTileThreads) void roi_pool_fwd_px8s_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ list,
    const int* __restrict__ cnt, int R, int C, int H, int W, int PH, int PW, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax) {
    constexpr int CG = 8;
    extern __shared__ __attribute__((aligned(16))) float4 tile4[];  // [H*W][2] float4
    const int b = blockIdx.y;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int kWaves = kTileThreads / 64;
    const int HW = H * W;
    const int PHW = PH * PW;
    const int nr = cnt[b];
    const int split = gridDim.z;
    const int r_begin = static_cast<int>(static_cast<int64_t>(nr) * blockIdx.z / split);
    const int r_end = static_cast<int>(static_cast<int64_t>(nr) * (blockIdx.z + 1) / split);
    if (r_begin >= r_end) return;
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    float* tile = reinterpret_cast<float*>(tile4);
    for (int i = tid; i < CG * HW; i += kTileThreads) {
        const int q = i / HW, p = i - q * HW;
        tile[p * CG + q] = nan_to_ninf(src[i]);
    }
    __syncthreads();
    const int* lst = list + static_cast<size_t>(b) * R;
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    for (int t = r_begin + wid; t < r_end; t += kWaves) {
        const int r = __builtin_amdgcn_readfirstlane(lst[t]);
        const RoiGeom gm = roi_geom(rois + static_cast<size_t>(r) * 5, ss, PH, PW);
        int4 g = geom_bin(gm, H, W, ph, pw);
        if (!act) g = make_int4(0, 0, 0, 0);
        const bool empty = g.y <= g.x || g.w <= g.z;
        const float init = empty ? 0.0f : -FLT_MAX;
        float mv[CG];
        int brow[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            mv[q] = init;
            brow[q] = -1;
        }
        const int wlast = g.w - 1;
        for (int h = g.x; h < g.y; ++h) {
            float rm[CG];
#pragma unroll
            for (int q = 0; q < CG; ++q) rm[q] = -INFINITY;
            const int rb = h * W;
            for (int w = g.z; w < g.w; w += 2) {
                const int i0 = rb + w;
                const int i1 = rb + min(w + 1, wlast);
                const float4 a0 = tile4[2 * i0], a1 = tile4[2 * i0 + 1];
                const float4 b0 = tile4[2 * i1], b1 = tile4[2 * i1 + 1];
                rm[0] = fmaxf(fmaxf(rm[0], a0.x), b0.x);
                rm[1] = fmaxf(fmaxf(rm[1], a0.y), b0.y);
                rm[2] = fmaxf(fmaxf(rm[2], a0.z), b0.z);
                rm[3] = fmaxf(fmaxf(rm[3], a0.w), b0.w);
                rm[4] = fmaxf(fmaxf(rm[4], a1.x), b1.x);
                rm[5] = fmaxf(fmaxf(rm[5], a1.y), b1.y);
                rm[6] = fmaxf(fmaxf(rm[6], a1.z), b1.z);
                rm[7] = fmaxf(fmaxf(rm[7], a1.w), b1.w);
            }
#pragma unroll
            for (int q = 0; q < CG; ++q) {
                if (rm[q] > mv[q]) {
                    mv[q] = rm[q];
                    brow[q] = h;
                }
            }
        }
        float ov[CG];
        int oi[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            ov[q] = init;
            oi[q] = -1;
            if (brow[q] >= 0) {
                const int rb = brow[q] * W;
                for (int w = wlast; w >= g.z; --w) {  // reverse scan: last hit = first in order
                    const float v = tile[(rb + w) * CG + q];
                    if (v == mv[q]) {
                        ov[q] = v;
                        oi[q] = rb + w;
                    }
                }
            }
        }
        if (act) {
            const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
#pragma unroll
            for (int q = 0; q < CG; ++q) {
                out[o + static_cast<size_t>(q) * PHW] = ov[q];
                argmax[o + static_cast<size_t>(q) * PHW] = oi[q];
            }
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
// With PH*PW <= 64 it also writes code[r][k]: which of bin k's earlier grid
// neighbours overlap it (1 left, 2 up, 4 up-left, 8 up-right) and, in bit 4,
// whether ANY bin of the RoI has an overlap outside that set (the RoI then
// takes the general mask walk in the ring kernel).
__global__ __launch_bounds__(256) void roi_bwd_prep_kernel(const float* __restrict__ rois, int H,
                                                           int W, int PH, int PW, float ss,
                                                           uint64_t* __restrict__ cmask,
                                                           uint8_t* __restrict__ code) {
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
    if (code == nullptr || PHW > 64) return;  // uniform
    const int k = threadIdx.x;
    uint32_t nb = 0;
    bool other = false;
    if (k < PHW) {
        const uint64_t m = cmask[static_cast<size_t>(r) * PHW + k];  // this thread's own write
        const int pw = k % PW;
        uint64_t known = 0;
        if (pw > 0) {
            known |= 1ull << (k - 1);
            nb |= (m >> (k - 1)) & 1u;
        }
        if (k >= PW) {
            known |= 1ull << (k - PW);
            nb |= ((m >> (k - PW)) & 1u) << 1;
            if (pw > 0) {
                known |= 1ull << (k - PW - 1);
                nb |= ((m >> (k - PW - 1)) & 1u) << 2;
            }
            if (pw < PW - 1) {
                known |= 1ull << (k - PW + 1);
                nb |= ((m >> (k - PW + 1)) & 1u) << 3;
            }
        }
        other = (m & ~known) != 0;
    }
    const int slow = __syncthreads_or(other);
    if (k < PHW) code[static_cast<size_t>(r) * PHW + k] = static_cast<uint8_t>(nb | (slow ? 16u : 0u));
}

// Ordered per-image RoI lists: list[b][*] = RoIs with batch index b, ascending.
// Block N (the extra one) collects the RoIs whose batch index is outside [0, N).
// Also zeroes the image's work-queue counters (`nq` per image) when given.
__global__ __launch_bounds__(1024) void roi_lists_kernel(const float* __restrict__ rois, int R,
                                                         int N, int* __restrict__ list,
                                                         int* __restrict__ cnt,
                                                         int* __restrict__ queue, int nq) {
    if (queue && blockIdx.x < N)
        for (int i = threadIdx.x; i < nq; i += 1024) queue[static_cast<size_t>(blockIdx.x) * nq + i] = 0;
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    __shared__ int s_w[16];
    int base = 0;
    for (int r0 = 0; r0 < R; r0 += 1024) {
        int r = r0 + tid;
        int rb = r < R ? static_cast<int>(rois[static_cast<size_t>(r) * 5]) : -1;
        bool m = r < R && (b < N ? rb == b : (rb < 0 || rb >= N));
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

// Same plane-owner backward for PH*PW <= 64 (one bin per lane, the 7x7 head),
// latency-hidden: a wave used to issue RoI t+1's argmax / grad / overlap-mask
// loads only after RoI t's LDS adds had retired, so every RoI paid a full HBM
// round trip (128 RoIs x ~2 us = the whole 288 us kernel at cfg5).  Here the
// loads of RoI t+D are issued before RoI t is applied (a D-deep register ring,
// slot index static after unrolling), and the RoI indices come from a 64-wide
// VGPR window read with v_readlane, so no vector load sits between the ring's
// loads in the in-order vmcnt queue.  Summation order per pixel is unchanged
// (RoIs ascending, bins ascending within a RoI): bit-identical results.
template <int D>
__global__ __launch_bounds__(1024) void roi_pool_bwd_pf_kernel(
    const float* __restrict__ grad, const int32_t* __restrict__ argmax,
    const uint64_t* __restrict__ cmask, const uint8_t* __restrict__ code,
    const int* __restrict__ list, const int* __restrict__ cnt,
    int R, int C, int HW, int PHW, int PW, int CPW, float* __restrict__ grad_in) {
    extern __shared__ __attribute__((aligned(16))) float planes[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b = blockIdx.y;
    const int c = blockIdx.x * CPW + wid;
    if (c >= C) return;  // whole wave; no workgroup barrier below
    float* gplane = grad_in + (static_cast<size_t>(b) * C + c) * HW;
    float* plane = planes + static_cast<size_t>(wid) * HW;
    for (int i = lane; i < HW; i += 64) plane[i] = 0.0f;
    const int nr = cnt[b];
    // Grid neighbours that come earlier in bin order: left, up-left, up,
    // up-right.  When every overlap of a RoI is among them (bins >= 1 pixel:
    // windows only share their floor/ceil border row / column), a bin's rank
    // among the bins with the same argmax pixel takes four fixed-lane reads
    // instead of a walk over its overlap mask.
    const int pw_i = lane % PW;
    const bool has_l = pw_i > 0, has_u = lane >= PW;
    const bool has_r = pw_i < PW - 1;
    const int n_l = has_l ? lane - 1 : lane, n_u = has_u ? lane - PW : lane;
    const int n_ul = (has_u && has_l) ? lane - PW - 1 : lane;
    const int n_ur = (has_u && has_r) ? lane - PW + 1 : lane;
    if (nr > 0) {
        const int* lst = list + static_cast<size_t>(b) * R;  // wave-uniform: scalar loads
        const bool act = lane < PHW;
        // Loads are unconditional (idle lanes re-read bin 0, RoIs past the end
        // re-read the last one): a conditional load makes the compiler wait
        // for the whole vmcnt queue at the branch join, which undoes the ring.
        const int kl = act ? lane : 0;
        int am_r[D];
        float g_r[D];
        uint32_t cd_r[D];
        uint64_t cm_r[D];  // full overlap mask, used only by RoIs flagged slow
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int n = lst[d < nr ? d : nr - 1];
            const size_t base = (static_cast<size_t>(n) * C + c) * PHW;
            am_r[d] = argmax[base + kl];
            g_r[d] = grad[base + kl];
            cd_r[d] = code[static_cast<size_t>(n) * PHW + kl];
            cm_r[d] = cmask[static_cast<size_t>(n) * PHW + kl];
            // keep the loop's issue order (slot by slot): the waitcnt pass then
            // merges identical queues at the loop header instead of draining
            asm volatile("" ::: "memory");
        }
        for (int t0 = 0; t0 < nr; t0 += D) {
            // RoI indices of this group's refills (scalar loads: lgkmcnt, not
            // in the vector-load queue)
            int nx[D];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int tn = t0 + D + d;
                nx[d] = lst[tn < nr ? tn : nr - 1];
            }
#pragma unroll
            for (int d = 0; d < D; ++d) {
                // no early exit for the tail: a break would give the loop a
                // second path into its header with another load order, and the
                // waitcnt pass would drain the queue there every group
                const bool live = t0 + d < nr;
                // Take slot d's values into fresh registers (asm copies the
                // compiler cannot coalesce away) so the refill lands in the
                // slot's own registers: no back-edge copy, no wait on it.
                int am;
                float g;
                uint32_t cd;
                asm volatile("v_mov_b32 %0, %1" : "=v"(am) : "v"(am_r[d]));
                asm volatile("v_mov_b32 %0, %1" : "=v"(g) : "v"(g_r[d]));
                asm volatile("v_mov_b32 %0, %1" : "=v"(cd) : "v"(cd_r[d]));
                uint32_t cm_lo, cm_hi;
                asm volatile("v_mov_b32 %0, %1" : "=v"(cm_lo) : "v"(static_cast<uint32_t>(cm_r[d])));
                asm volatile("v_mov_b32 %0, %1" : "=v"(cm_hi) : "v"(static_cast<uint32_t>(cm_r[d] >> 32)));
                if (!live || !act) am = -1;
                {  // refill this slot with RoI t + D before applying RoI t
                    const int n = nx[d];
                    const size_t base = (static_cast<size_t>(n) * C + c) * PHW;
                    am_r[d] = argmax[base + kl];
                    g_r[d] = grad[base + kl];
                    cd_r[d] = code[static_cast<size_t>(n) * PHW + kl];
                    cm_r[d] = cmask[static_cast<size_t>(n) * PHW + kl];
                }
                // depth = rank of this bin among the RoI's bins with the same
                // argmax pixel (those windows all contain the pixel, so they
                // overlap: candidates are the bits of the overlap mask)
                int depth = 0;
                if ((__builtin_amdgcn_readfirstlane(cd) & 16) == 0) {  // bin 0's code: the RoI flag
                    const int a_l = __builtin_amdgcn_ds_bpermute(n_l << 2, am);
                    const int a_u = __builtin_amdgcn_ds_bpermute(n_u << 2, am);
                    const int a_ul = __builtin_amdgcn_ds_bpermute(n_ul << 2, am);
                    const int a_ur = __builtin_amdgcn_ds_bpermute(n_ur << 2, am);
                    depth = ((cd & 1) && a_l == am) + ((cd & 2) && a_u == am) +
                            ((cd & 4) && a_ul == am) + ((cd & 8) && a_ur == am);
                } else {  // overlaps beyond the grid neighbours: walk the full mask
                    uint64_t pend = am != -1 ? ((static_cast<uint64_t>(cm_hi) << 32) | cm_lo) : 0ull;
                    while (__ballot(pend != 0)) {
                        const int p = pend ? __ffsll(static_cast<unsigned long long>(pend)) - 1 : lane;
                        pend &= pend - 1;
                        const int amp = __builtin_amdgcn_ds_bpermute(p << 2, am);
                        if (p != lane && amp == am) ++depth;
                    }
                }
                // apply in rank order; ranks are unique per pixel, so a round's
                // read-add-write touches distinct pixels.  LDS executes a wave's
                // instructions in issue order, so round r+1's reads see round
                // r's writes without a wait (the asm is only a compiler
                // barrier).  ds_add_f32 is exact too, but measured 1.4x slower.
                for (int r = 0;; ++r) {
                    if (am != -1 && depth == r) plane[am] += g;
                    asm volatile("" ::: "memory");
                    if (__ballot(am != -1 && depth > r) == 0) break;
                }
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((HW & 3) == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(plane);
        float4* d4 = reinterpret_cast<float4*>(gplane);
        for (int i = lane; i < HW / 4; i += 64) d4[i] = s4[i];
    } else {
        for (int i = lane; i < HW; i += 64) gplane[i] = plane[i];
    }
}

// Outputs of RoIs with an out-of-range batch index: 0 / -1 (torchvision: UB).
__global__ __launch_bounds__(256) void roi_pool_invalid_fill_kernel(const int* __restrict__ list,
                                                                    const int* __restrict__ cnt,
                                                                    int R, int N, size_t per_roi,
                                                                    float* __restrict__ out,
                                                                    int32_t* __restrict__ argmax) {
    const int n = cnt[N];
    for (int t = blockIdx.x; t < n; t += gridDim.x) {
        const size_t base = static_cast<size_t>(list[static_cast<size_t>(N) * R + t]) * per_roi;
        for (size_t e = threadIdx.x; e < per_roi; e += 256) {
            out[base + e] = 0.0f;
            argmax[base + e] = -1;
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

namespace {
struct FwdWs {
    int* list;
    int* cnt;
    int* queue;
    size_t bytes;
};
FwdWs carve_fwd(void* ws, int64_t R, int N, int C) {
    Carver c(ws);
    FwdWs w{};
    w.list = c.take<int>(static_cast<size_t>(N + 1) * R);
    w.cnt = c.take<int>(N + 1);
    w.queue = c.take<int>(static_cast<size_t>(N) * (C / 4 + 1));
    w.bytes = c.used();
    return w;
}
constexpr int kFwdCG = 4;                       // channels per image tile
constexpr size_t kFwdTileBudget = 96 * 1024;    // LDS for the CG planes
constexpr size_t kLdsPerCu = 160 * 1024;        // gfx950
constexpr size_t kBalStatic = 1024;             // static LDS of the balanced kernel (rounded up)
// default forward for image-grouped RoIs: px8q (px_plan: 16- or 8-channel
// swizzled planes, strided shares); 0 = px8 (count split), 2 = balanced v2
// are the A/B alternatives
constexpr int kSortedDefault = 1;

int device_cu_count();
// segments of the balanced forward: at most two resident workgroups per CU
int bal_max_segments() { return 2 * device_cu_count(); }
struct BalWs {
    int* seg_lo;
    int* seg_info;
    size_t bytes;
};
BalWs carve_bal(void* ws, int S) {
    Carver c(ws);
    BalWs w{};
    w.seg_lo = c.take<int>(static_cast<size_t>(S) + 1);
    w.seg_info = c.take<int>(static_cast<size_t>(S) * kSegInfo);
    w.bytes = c.used();
    return w;
}
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
// Launch plan of the image-tile forward (roi_pool_fwd_px8q_kernel) for RoIs
// grouped by image: CG = 16 channel planes when they fit the CU's LDS (one
// workgroup per CU), else 8 (two per CU when they fit).  Each workgroup gets
// the LDS left over for its RoI-geometry chunk; split = RoI shares per
// (image, channel group), sized so the grid fills every resident slot once.
struct PxPlan {
    int cg = 0, geo_cap = 0, split = 1, N = 0;
    size_t lds = 0;
};
PxPlan px_plan(int C, int N, int H, int W, int PH, int PW, int want_cg) {
    PxPlan pl;
    const size_t HW = static_cast<size_t>(H) * W;
    if (N <= 0 || HW == 0 || PH * PW > 64 || H > 65535 || W > 65535) return pl;
    constexpr size_t kReserve = 1024;  // static LDS + allocation rounding
    constexpr size_t kMinGeo = 64 * sizeof(int4);
    const size_t HWs = (HW + 15) & ~static_cast<size_t>(15);
    for (int cg : {16, 8}) {
        if ((want_cg && cg != want_cg) || C % cg != 0) continue;
        const size_t tile = static_cast<size_t>(cg / 4) * HWs * sizeof(float4);
        int per_cu = 0;
        if (2 * (tile + kMinGeo + kReserve) <= kLdsPerCu) per_cu = 2;
        else if (tile + kMinGeo + kReserve <= kLdsPerCu) per_cu = 1;
        if (!per_cu) continue;
        size_t geo = (kLdsPerCu / per_cu - kReserve - tile) / sizeof(int4);
        pl.geo_cap = static_cast<int>(geo > 512 ? 512 : geo);
        pl.cg = cg;
        pl.lds = tile + static_cast<size_t>(pl.geo_cap) * sizeof(int4);
        const int64_t wgs = static_cast<int64_t>(C / cg) * N;
        const int64_t target = static_cast<int64_t>(device_cu_count()) * per_cu;
        int64_t sp = (target + wgs - 1) / wgs;
        if (const char* e = getenv("FRCNN_ROIPOOL_SPLIT")) sp = std::atoi(e);  // A/B override
        pl.split = static_cast<int>(sp < 1 ? 1 : (sp > 64 ? 64 : sp));
        pl.N = N;
        return pl;
    }
    return pl;
}

int px_launch(const PxPlan& pl, int mode, const float* x, const float* rois, int64_t R, int C, int H,
              int W, int PH, int PW, float ss, float* out, int32_t* argmax, const HeadArgs& hd,
              hipStream_t st) {
    const dim3 grid(static_cast<unsigned>(C / pl.cg), static_cast<unsigned>(pl.N + 1),
                    static_cast<unsigned>(pl.split));
    const bool head = hd.inds != nullptr;
#define FRCNN_PX(CG, MD, HD)                                                                          \
    hipLaunchKernelGGL((roi_pool_fwd_px8q_kernel<1024, CG, MD, HD>), grid, dim3(1024), pl.lds, st, x, \
                       rois, static_cast<int>(R), C, H, W, PH, PW, ss, out, argmax, pl.geo_cap, hd)
    if (pl.cg == 16) {
        if (head) FRCNN_PX(16, 0, true);
        else if (mode == 3) hipLaunchKernelGGL((roi_pool_fwd_px8q_kernel<1024, 16, 0, false, false>), grid, dim3(1024),
                                               pl.lds, st, x, rois, static_cast<int>(R), C, H, W, PH, PW, ss, out,
                                               argmax, pl.geo_cap, hd);
        else if (mode == 1) FRCNN_PX(16, 1, false);
        else FRCNN_PX(16, 0, false);
    } else {
        if (head) FRCNN_PX(8, 0, true);
        else if (mode == 1) FRCNN_PX(8, 1, false);
        else if (mode == 2) FRCNN_PX(8, 2, false);
        else FRCNN_PX(8, 0, false);
    }
#undef FRCNN_PX
    FRCNN_LAUNCH_CHECK("roi_pool_fwd_px8q_kernel");
    return FRCNN_OK;
}
}  // namespace


extern "C" size_t frcnn_roi_pool_fwd_workspace_size(int64_t R, int N, int C) {
    if (R < 0 || N < 0 || C < 0) return 0;
    const size_t a = carve_fwd(nullptr, R, N, C).bytes;
    const size_t b = carve_bal(nullptr, bal_max_segments()).bytes;
    return a > b ? a : b;
}

extern "C" int frcnn_roi_pool_fwd(const float* x, const float* rois, int64_t R, int N, int C,
                                  int H, int W, int PH, int PW, float spatial_scale,
                                  int rois_sorted, float* out, int32_t* argmax, void* workspace,
                                  size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(R >= 0 && N >= 0 && C >= 0 && H >= 0 && W >= 0, "frcnn_roi_pool_fwd: bad shape");
    FRCNN_REQUIRE(PH > 0 && PW > 0 && PH * PW <= kMaxBins,
                  "frcnn_roi_pool_fwd: output_size must have 1..%d bins", kMaxBins);
    FRCNN_REQUIRE(R <= 0x7fffffff && N <= 65534, "frcnn_roi_pool_fwd: too many rois / images");
    if (R == 0 || C == 0) return FRCNN_OK;
    FRCNN_REQUIRE(x && rois && out && argmax, "frcnn_roi_pool_fwd: null pointer");
    hipStream_t st = as_stream(stream);
    const size_t HW = static_cast<size_t>(H) * W;
    const size_t tile_bytes = kFwdCG * HW * sizeof(float);
    const bool aligned = (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                         (reinterpret_cast<uintptr_t>(argmax) % 16 == 0);
    const char* var = getenv("FRCNN_ROIPOOL_VARIANT");  // A/B override (tests, tools/ab_roi_pool.py)
    auto is = [&](const char* v) { return var && std::strcmp(var, v) == 0; };
    const bool px8_ok = N > 0 && HW > 0 && C % 8 == 0 && 2 * tile_bytes <= kFwdTileBudget &&
                        PH * PW <= 64;
    const int64_t per_img = (R + (N > 0 ? N : 1) - 1) / (N > 0 ? N : 1);
    int64_t split8 = px8_ok ? (512 + static_cast<int64_t>(C / 8) * N - 1) / (static_cast<int64_t>(C / 8) * N) : 1;
    split8 = split8 < 1 ? 1 : (split8 > 64 ? 64 : split8);
    // default for RoIs grouped by image: one launch, cost-balanced over a
    // grid of exactly one resident round (2 x 1024-thread workgroups per CU
    // when two 8-channel tiles fit the CU's LDS)
    const size_t bal_lds = 2 * tile_bytes;
    const bool bal_ok = N > 0 && HW > 0 && C % 8 == 0 && PH * PW <= 64 &&
                        bal_lds + kBalStatic <= kLdsPerCu && R < (1 << 21) && C / 8 <= 65535;
    const bool bal2_var = is("bal2") || is("bal2ns") || is("bal2c") || is("bal2b");
    if (bal_ok && rois_sorted && (bal2_var || (kSortedDefault == 2 && !var))) {
        const int groups = C / 8;
        const size_t lds2 = bal_lds + 32;  // + the -inf pad pixel
        const int per_cu = kLdsPerCu / (lds2 + kBalStatic) >= 2 ? 2 : 1;
        int64_t S = static_cast<int64_t>(device_cu_count()) * per_cu / groups;
        S = S < 1 ? 1 : S;
        S = S > R ? R : S;
        S = S > bal_max_segments() ? bal_max_segments() : S;
        BalWs w = carve_bal(workspace, static_cast<int>(S));
        FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_roi_pool_fwd: workspace %zu < %zu",
                      ws_bytes, w.bytes);
        hipLaunchKernelGGL((roi_partition_kernel<1024, 1>), dim3(1), dim3(1024), 0, st, rois,
                           static_cast<int>(R), N, H, W, PH, PW, spatial_scale, static_cast<int>(S),
                           w.seg_lo, w.seg_info);
        FRCNN_LAUNCH_CHECK("roi_partition_kernel");
        const dim3 grid(static_cast<unsigned>(S), groups);
        const bool fix7 = PH == 7 && PW == 7;
#define FRCNN_BAL2(FX, SW, MD)                                                                         \
    hipLaunchKernelGGL((roi_pool_fwd_bal2_kernel<1024, FX, SW, MD>), grid, dim3(1024), lds2, st, x, rois, \
                       w.seg_lo, w.seg_info, N, C, H, W, PH, PW, spatial_scale, out, argmax)
        if (is("bal2ns")) {
            if (fix7) FRCNN_BAL2(7, false, 0); else FRCNN_BAL2(0, false, 0);
        } else if (is("bal2c")) {
            if (fix7) FRCNN_BAL2(7, true, 2); else FRCNN_BAL2(0, true, 2);
        } else if (is("bal2b")) {
            if (fix7) FRCNN_BAL2(7, true, 3); else FRCNN_BAL2(0, true, 3);
        } else {
            if (fix7) FRCNN_BAL2(7, true, 0); else FRCNN_BAL2(0, true, 0);
        }
#undef FRCNN_BAL2
        FRCNN_LAUNCH_CHECK("roi_pool_fwd_bal2_kernel");
        return FRCNN_OK;
    }
    if (bal_ok && rois_sorted && (is("bal") || is("balcnt") || is("baldbg") || is("balnc") || is("balns"))) {
        const int groups = C / 8;
        const int per_cu = kLdsPerCu / (bal_lds + kBalStatic) >= 2 ? 2 : 1;
        int64_t S = static_cast<int64_t>(device_cu_count()) * per_cu / groups;
        S = S < 1 ? 1 : S;
        S = S > R ? R : S;
        S = S > bal_max_segments() ? bal_max_segments() : S;
        BalWs w = carve_bal(workspace, static_cast<int>(S));
        FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_roi_pool_fwd: workspace %zu < %zu",
                      ws_bytes, w.bytes);
        if (is("balcnt"))
            hipLaunchKernelGGL((roi_partition_kernel<1024, 0>), dim3(1), dim3(1024), 0, st, rois,
                               static_cast<int>(R), N, H, W, PH, PW, spatial_scale, static_cast<int>(S),
                               w.seg_lo, w.seg_info);
        else
            hipLaunchKernelGGL((roi_partition_kernel<1024, 1>), dim3(1), dim3(1024), 0, st, rois,
                               static_cast<int>(R), N, H, W, PH, PW, spatial_scale, static_cast<int>(S),
                               w.seg_lo, w.seg_info);
        FRCNN_LAUNCH_CHECK("roi_partition_kernel");
        if (is("balnc") || is("balns"))
            hipLaunchKernelGGL((is("balnc") ? roi_pool_fwd_bal_kernel<1024, false, 1> : roi_pool_fwd_bal_kernel<1024, false, 2>),
                               dim3(static_cast<unsigned>(S), groups), dim3(1024), bal_lds, st, x, rois, w.seg_lo,
                               w.seg_info, N, C, H, W, PH, PW, spatial_scale, out, argmax);
        else if (is("baldbg"))
            hipLaunchKernelGGL((roi_pool_fwd_bal_kernel<1024, true>), dim3(static_cast<unsigned>(S), groups),
                               dim3(1024), bal_lds, st, x, rois, w.seg_lo, w.seg_info, N, C, H, W, PH, PW,
                               spatial_scale, out, argmax);
        else
            hipLaunchKernelGGL((roi_pool_fwd_bal_kernel<1024, false>), dim3(static_cast<unsigned>(S), groups),
                               dim3(1024), bal_lds, st, x, rois, w.seg_lo, w.seg_info, N, C, H, W, PH, PW,
                               spatial_scale, out, argmax);
        FRCNN_LAUNCH_CHECK("roi_pool_fwd_bal_kernel");
        return FRCNN_OK;
    }
    if (rois_sorted && (!var || is("px16") || is("px16S") || is("px16p") || is("px8q") || is("px8qS") ||
                        is("px8qC"))) {
        const PxPlan pl = px_plan(C, N, H, W, PH, PW, is("px8q") || is("px8qS") || is("px8qC") ? 8
                                                      : (is("px16") || is("px16S") || is("px16p")) ? 16 : 0);
        if (pl.cg) {
            const int mode = (is("px16S") || is("px8qS")) ? 1 : is("px8qC") ? 2 : is("px16p") ? 3 : 0;
            return px_launch(pl, mode, x, rois, R, C, H, W, PH, PW, spatial_scale, out, argmax, HeadArgs{}, st);
        }
    }
    if (px8_ok && rois_sorted && (is("px8r") || is("px8rS"))) {
        const size_t lds = 2 * HW * sizeof(float4);
        int64_t sp = split8;
        if (const char* s = getenv("FRCNN_ROIPOOL_SPLIT")) sp = std::atoi(s);
        sp = sp < 1 ? 1 : (sp > 64 ? 64 : sp);
        dim3 grid(C / 8, N + 1, static_cast<unsigned>(sp));
        if (is("px8rS"))  // timing probe: no stores
            hipLaunchKernelGGL((roi_pool_fwd_px8r_kernel<1024, 1>), grid, dim3(1024), lds, st, x, rois,
                               static_cast<int>(R), C, H, W, PH, PW, spatial_scale, out, argmax);
        else
            hipLaunchKernelGGL((roi_pool_fwd_px8r_kernel<1024>), grid, dim3(1024), lds, st, x, rois,
                               static_cast<int>(R), C, H, W, PH, PW, spatial_scale, out, argmax);
        FRCNN_LAUNCH_CHECK("roi_pool_fwd_px8r_kernel");
        return FRCNN_OK;
    }
    if (px8_ok && rois_sorted && (is("px8sorted") || (kSortedDefault == 0 && !var))) {
        dim3 grid(C / 8, N + 1, static_cast<unsigned>(split8));
        hipLaunchKernelGGL((roi_pool_fwd_px8_kernel<1024, true>), grid, dim3(1024), 2 * tile_bytes, st,
                           x, rois, nullptr, nullptr, nullptr, static_cast<int>(R), C, H, W, PH, PW,
                           spatial_scale, out, argmax);
        FRCNN_LAUNCH_CHECK("roi_pool_fwd_px8_kernel");
        return FRCNN_OK;
    }
    if (N > 0 && C % kFwdCG == 0 && HW > 0 && tile_bytes <= kFwdTileBudget && aligned) {
        FwdWs w = carve_fwd(workspace, R, N, C);
        FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_roi_pool_fwd: workspace %zu < %zu",
                      ws_bytes, w.bytes);
        hipLaunchKernelGGL(roi_lists_kernel, dim3(N + 1), dim3(1024), 0, st, rois,
                           static_cast<int>(R), N, w.list, w.cnt, w.queue, C / 4);
        FRCNN_LAUNCH_CHECK("roi_lists_kernel");
        const int groups = C / kFwdCG;
        int64_t split = (1024 + static_cast<int64_t>(groups) * N - 1) / (static_cast<int64_t>(groups) * N);
        int64_t cap = (per_img + 31) / 32;
        split = split < cap ? split : cap;
        split = split < 1 ? 1 : (split > 64 ? 64 : split);
        const size_t pad = 8 * sizeof(float);
        if (px8_ok && !(var && var[0] == 'w') && !is("tile") && !is("px8s") && !is("pxf8") &&
            !is("pxf4") && !is("px8")) {
            dim3 grid(C / 8, N, static_cast<unsigned>(split8));  // default (unsorted RoIs)
            hipLaunchKernelGGL((roi_pool_fwd_px8_kernel<1024, false>), grid, dim3(1024), 2 * tile_bytes,
                               st, x, rois, w.list, w.cnt, w.queue, static_cast<int>(R), C, H, W, PH,
                               PW, spatial_scale, out, argmax);
        } else if (px8_ok && is("px8")) {
            dim3 grid(C / 8, N, static_cast<unsigned>(split8));
            hipLaunchKernelGGL((roi_pool_fwd_px8_kernel<512, false>), grid, dim3(512), 2 * tile_bytes,
                               st, x, rois, w.list, w.cnt, w.queue, static_cast<int>(R), C, H, W, PH,
                               PW, spatial_scale, out, argmax);
        } else if (px8_ok && is("px8s")) {
            dim3 grid(C / 8, N, static_cast<unsigned>(split8));
            hipLaunchKernelGGL(roi_pool_fwd_px8s_kernel, grid, dim3(kTileThreads), 2 * tile_bytes, st,
                               x, rois, w.list, w.cnt, static_cast<int>(R), C, H, W, PH, PW,
                               spatial_scale, out, argmax);
        } else if (px8_ok && is("pxf8") && 2 * tile_bytes + pad <= kFwdTileBudget) {
            dim3 grid(C / 8, N, static_cast<unsigned>(split8));
            hipLaunchKernelGGL(roi_pool_fwd_pxf_kernel<8>, grid, dim3(kTileThreads), 2 * tile_bytes + pad,
                               st, x, rois, w.list, w.cnt, static_cast<int>(R), C, H, W, PH, PW,
                               spatial_scale, out, argmax);
        } else if (PH * PW <= 64 && is("pxf4")) {
            dim3 grid(groups, N, static_cast<unsigned>(split));
            hipLaunchKernelGGL(roi_pool_fwd_pxf_kernel<4>, grid, dim3(kTileThreads), tile_bytes + pad, st,
                               x, rois, w.list, w.cnt, static_cast<int>(R), C, H, W, PH, PW,
                               spatial_scale, out, argmax);
        } else if (PH * PW <= 64 && is("wave8") && C % 8 == 0 && 2 * tile_bytes <= kFwdTileBudget) {
            dim3 grid(C / 8, N, static_cast<unsigned>(split));
            hipLaunchKernelGGL(roi_pool_fwd_wave_kernel<8>, grid, dim3(kTileThreads), 2 * tile_bytes, st,
                               x, rois, w.list, w.cnt, static_cast<int>(R), C, H, W, PH, PW,
                               spatial_scale, out, argmax);
        } else if (PH * PW <= 64 && !is("tile")) {
            hipLaunchKernelGGL(roi_pool_fwd_wave_kernel<4>, dim3(groups, N, static_cast<unsigned>(split)),
                               dim3(kTileThreads), tile_bytes, st, x, rois, w.list, w.cnt,
                               static_cast<int>(R), C, H, W, PH, PW, spatial_scale, out, argmax);
        } else {
            hipLaunchKernelGGL(roi_pool_fwd_tile_kernel, dim3(groups, N, static_cast<unsigned>(split)),
                               dim3(kTileThreads), tile_bytes, st, x, rois, w.list, w.cnt,
                               static_cast<int>(R), C, H, W, PH, PW, kFwdCG, spatial_scale, out, argmax);
        }
        FRCNN_LAUNCH_CHECK("roi_pool_fwd (image tile)");
        hipLaunchKernelGGL(roi_pool_invalid_fill_kernel, dim3(64), dim3(256), 0, st, w.list, w.cnt,
                           static_cast<int>(R), N, static_cast<size_t>(C) * PH * PW, out, argmax);
        FRCNN_LAUNCH_CHECK("roi_pool_invalid_fill_kernel");
        return FRCNN_OK;
    }
    // generic path: one workgroup per RoI, gathers from L1/L2
    const size_t total = static_cast<size_t>(C) * PH * PW;
    if (total % 4 == 0 && aligned)
        hipLaunchKernelGGL(roi_pool_fwd_kernel<true>, dim3(static_cast<unsigned>(R)), dim3(256), 0,
                           st, x, rois, N, C, H, W, PH, PW, spatial_scale, out, argmax);
    else
        hipLaunchKernelGGL(roi_pool_fwd_kernel<false>, dim3(static_cast<unsigned>(R)), dim3(256), 0,
                           st, x, rois, N, C, H, W, PH, PW, spatial_scale, out, argmax);
    FRCNN_LAUNCH_CHECK("roi_pool_fwd_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_roi_pool_fwd_head(const float* x, const float* rois, const float* roi_inds,
                                       int64_t R, int N, int C, int H, int W, int PH, int PW,
                                       float img_h, float img_w, float spatial_scale,
                                       int rois_sorted, float* boxes, float* out, int32_t* argmax,
                                       void* workspace, size_t ws_bytes, void* stream) {
    FRCNN_REQUIRE(R >= 0 && N >= 0 && C >= 0 && H >= 0 && W >= 0, "frcnn_roi_pool_fwd_head: bad shape");
    FRCNN_REQUIRE(PH > 0 && PW > 0 && PH * PW <= kMaxBins,
                  "frcnn_roi_pool_fwd_head: output_size must have 1..%d bins", kMaxBins);
    FRCNN_REQUIRE(R <= 0x7fffffff && N <= 65534, "frcnn_roi_pool_fwd_head: too many rois / images");
    if (R == 0) return FRCNN_OK;
    FRCNN_REQUIRE(rois && roi_inds && boxes, "frcnn_roi_pool_fwd_head: null pointer");
    const char* var = getenv("FRCNN_ROIPOOL_VARIANT");
    const PxPlan pl = (rois_sorted && C > 0 && (!var || std::strcmp(var, "px8q") == 0 ||
                                               std::strcmp(var, "px16") == 0))
                          ? px_plan(C, N, H, W, PH, PW, !var ? 0 : (std::strcmp(var, "px8q") == 0 ? 8 : 16))
                          : PxPlan{};
    if (!pl.cg || reinterpret_cast<uintptr_t>(rois) % 16 != 0) {
        int rc = frcnn_roi_transform(rois, roi_inds, R, img_h, img_w, H, W, boxes, stream);
        if (rc != FRCNN_OK) return rc;
        if (C == 0) return FRCNN_OK;
        return frcnn_roi_pool_fwd(x, boxes, R, N, C, H, W, PH, PW, spatial_scale, rois_sorted, out,
                                  argmax, workspace, ws_bytes, stream);
    }
    FRCNN_REQUIRE(x && out && argmax, "frcnn_roi_pool_fwd_head: null pointer");
    const HeadArgs hd{roi_inds, img_h, img_w, static_cast<float>(H), static_cast<float>(W), boxes};
    return px_launch(pl, 0, x, rois, R, C, H, W, PH, PW, spatial_scale, out, argmax, hd, as_stream(stream));
}

namespace {
struct BwdWs {
    uint64_t* cmask;
    uint8_t* code;
    int* list;
    int* cnt;
    size_t bytes;
};
BwdWs carve_bwd(void* ws, int64_t R, int N, int PH, int PW) {
    Carver c(ws);
    BwdWs w{};
    w.cmask = c.take<uint64_t>(static_cast<size_t>(R) * PH * PW);
    w.code = c.take<uint8_t>(static_cast<size_t>(R) * PH * PW);
    w.list = c.take<int>(static_cast<size_t>(N + 1) * R);
    w.cnt = c.take<int>(N + 1);
    w.bytes = c.used();
    return w;
}
constexpr size_t kPlaneBudget = 64 * 1024;  // LDS per workgroup for planes
constexpr int kBwdRing = 8;                  // RoIs in flight per wave (pf kernel)
constexpr size_t kPlaneBudgetRing = 144 * 1024;  // ring kernel: one workgroup per CU
// A/B switch for tools (FRCNN_BWD_VARIANT=plain: the unpipelined kernel)
bool bwd_variant_is(const char* v) {
    const char* e = std::getenv("FRCNN_BWD_VARIANT");
    return e && std::strcmp(e, v) == 0;
}
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
                       H, W, PH, PW, spatial_scale, w.cmask, w.code);
    FRCNN_LAUNCH_CHECK("roi_bwd_prep_kernel");
    hipLaunchKernelGGL(roi_lists_kernel, dim3(N + 1), dim3(1024), 0, st, rois, static_cast<int>(R),
                       N, w.list, w.cnt, nullptr, 0);
    FRCNN_LAUNCH_CHECK("roi_lists_kernel");
    const size_t plane_bytes = HW * sizeof(float);
    const int PHW = PH * PW;
    const bool ring = PHW <= 64 && !bwd_variant_is("plain");
    if (ring && plane_bytes <= kPlaneBudgetRing) {
        // Every wave owns one (image, channel) plane and walks all of the
        // image's RoIs, so the work per wave is fixed: spread the N*C waves
        // evenly, one workgroup per CU (ceil(N*C / CUs) waves each) where the
        // LDS allows -- a 2:1 mix of busy and half-idle CUs cost 1.35x.
        const int64_t waves = static_cast<int64_t>(N) * C;
        int64_t cpw = (waves + device_cu_count() - 1) / device_cu_count();
        if (const char* e = std::getenv("FRCNN_BWD_CPW")) cpw = std::atoi(e);  // A/B override
        const int64_t lds_cap = static_cast<int64_t>(kPlaneBudgetRing / plane_bytes);
        cpw = cpw > 16 ? 16 : cpw;
        cpw = cpw > lds_cap ? lds_cap : cpw;
        cpw = cpw > C ? C : cpw;
        cpw = cpw < 1 ? 1 : cpw;
        const int icpw = static_cast<int>(cpw);
        dim3 grid((C + icpw - 1) / icpw, N);
        int ringd = kBwdRing;
        if (const char* e = std::getenv("FRCNN_BWD_RING")) ringd = std::atoi(e);  // A/B override
#define FRCNN_BWD_PF(DD)                                                                              \
    hipLaunchKernelGGL(roi_pool_bwd_pf_kernel<DD>, grid, dim3(64 * icpw), icpw * plane_bytes, st,    \
                       grad, argmax, w.cmask, w.code, w.list, w.cnt, static_cast<int>(R), C,         \
                       static_cast<int>(HW), PHW, PW, icpw, grad_in)
        if (ringd == 4) FRCNN_BWD_PF(4);
        else if (ringd == 16) FRCNN_BWD_PF(16);
        else FRCNN_BWD_PF(8);
#undef FRCNN_BWD_PF
    } else if (plane_bytes <= kPlaneBudget) {
        int cpw = static_cast<int>(kPlaneBudget / plane_bytes);
        cpw = cpw > 16 ? 16 : cpw;
        cpw = cpw > C ? C : cpw;
        dim3 grid((C + cpw - 1) / cpw, N);
        if (false)
            ;
        else
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

// tools-only (not part of the C-ABI): copy the "baldbg" timeline probe to host
extern "C" int frcnn_dbg_bal_stamps(unsigned long long* host, int n) {
    if (n > 8 * 8192) n = 8 * 8192;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bal_dbg), sizeof(unsigned long long) * n) == hipSuccess ? 0 : -2;
}
