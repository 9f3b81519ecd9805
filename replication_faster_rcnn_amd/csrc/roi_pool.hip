// RoI max-pooling forward / backward (nets/heads.py:42-48, torchvision
// roi_pool semantics) on gfx950.
//
// Forward, default ("dense"): a workgroup owns CG channel planes of one image,
// staged once into LDS, and a cost-balanced contiguous share of that image's
// RoIs.  The share's RoIs are ordered by window size and their PH*PW bins are
// packed densely into the 64 lanes of each wave (lane = bin of some RoI, so a
// 7x7 head uses 64/64 lanes instead of 49/64), each lane scanning its bin
// window for CG channels at once.  The per-channel update takes pixels in
// pairs: m' = max3(m, a, b), the index moves iff m' > m, to a if a == m' --
// torchvision's strict-'>' row-major first-max, exactly.
// Generic: one 256-thread workgroup per RoI (any output size, any layout).
//
// Backward: atomic-free, deterministic and bit-identical to the CPU kernel's
// summation order.  A wave owns one (image, channel) plane in LDS and walks
// that image's RoIs in ascending order; within one RoI the lanes are the bins;
// two bins can hit the same pixel only if their windows overlap (mask
// precomputed per RoI), and such lanes apply their adds in rounds ordered by
// bin index, so every pixel sees exactly the CPU order n -> ph -> pw.  The
// finished planes are stored once (zero-fill of grad_in fused).
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace frcnn {

constexpr int kMaxBins = 1024;
constexpr int kListPad = 16;  // entries past each image's RoI list (copies of its last entry)
__host__ __device__ constexpr int64_t list_stride(int64_t R) { return R + kListPad; }
constexpr size_t kLdsPerCu = 160 * 1024;  // gfx950

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

// Generic forward: one workgroup per RoI, window gathers served by L1/L2.
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

// RoI geometry shared by all bins: start (sh, sw) and bin size (bh, bw).
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

// Count of RoIs with batch index < b0 and < b1 (block-wide), for RoIs grouped by
// non-decreasing batch index: image b's RoIs are then [count(<b), count(<b+1)).
// `red` holds 2 ints per wave.
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
    __syncthreads();  // red is reused by the caller
    return res;
}

// The head's RoI transform + [idx, box] pack (nets/heads.py:42-47), fused into
// the forward: `rois` are then [R,4] image-pixel boxes, `inds` their image index.
struct HeadArgs {
    const float* inds;
    float img_h, img_w, fh, fw;
    float* boxes;  // [R,5] written once (channel group 0) for the backward
};

__device__ __forceinline__ void head_box(const float* __restrict__ rois, const HeadArgs& hd, int r,
                                         float (&bx)[5]) {
    const float4 v = reinterpret_cast<const float4*>(rois)[r];
    bx[0] = hd.inds[r];
    bx[1] = v.x / hd.img_h * hd.fh;  // fp32 divide, then multiply (nets/heads.py:43-44)
    bx[2] = v.y / hd.img_w * hd.fw;
    bx[3] = v.z / hd.img_h * hd.fh;
    bx[4] = v.w / hd.img_w * hd.fw;
}

// v_max3_f32 without the IEEE-mode canonicalisation the compiler adds around
// fmaxf on loaded values: the tile holds no NaN (staged as -inf), and the sign
// of a zero maximum is re-read from the tile after the scan.
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
    float d;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Window class of a RoI: (max bin height, max bin width), each capped at 15;
// the key orders the dense bin stream and the cost drives the balanced shares.
__device__ __forceinline__ int2 geom_class(const RoiGeom& g, int H, int W, int PH, int PW) {
    const int mh = min(min(static_cast<int>(ceilf(g.bh)) + 1, H), 15);
    const int mw = min(min(static_cast<int>(ceilf(g.bw)) + 1, W), 15);
    const int eh = g.sh + static_cast<int>(ceilf(g.bh * static_cast<float>(PH)));
    const int ew = g.sw + static_cast<int>(ceilf(g.bw * static_cast<float>(PW)));
    const bool outside = g.sh >= H || g.sw >= W || eh <= 0 || ew <= 0;
    const int key = outside ? 0 : mh * 16 + mw;
    const int cost = outside ? 2 : mh * ((mw + 1) >> 1) + 3;
    return make_int2(key, cost);
}

// ------------------------------------------------------------- dense forward
// Dynamic LDS (nothing static, the tile starts at offset 0):
//   tile  NP planes x HWs float4: plane q = channels 4q..4q+3, pixel p at [q*HWs + p]
//   geo   cap x int4 (sh, sw, bh bits, bw bits)   rid cap x int (RoI index)
//   ord   cap x int (item order)                  key cap x u8 (window class)
//   hist  256 x u32,  misc 64 x int
// Grid (C/CG, split, N [+1 when !LIST: RoIs with an out-of-range batch index]):
// the image index is slowest, so row N is dispatched after every real workgroup.
// LIST: RoIs in any order, per-image lists from roi_lists_kernel; else RoIs
// grouped by non-decreasing batch index (each workgroup finds its image's range).
constexpr int kDenseMisc = 64;
__host__ __device__ constexpr size_t dense_fixed_bytes() { return 256 * 4 + kDenseMisc * 4; }
__host__ __device__ constexpr size_t dense_item_bytes() { return 16 + 4 + 4 + 1; }

template <int NT, int CG, int FIX, bool HEAD, bool LIST>
__global__ __launch_bounds__(NT) void roi_pool_fwd_dense_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, const int* __restrict__ list,
    const int* __restrict__ cnt, int R, int C, int H, int W, int PH_, int PW_, float ss,
    float* __restrict__ out, int32_t* __restrict__ argmax, int cap, HeadArgs hd) {
    constexpr int NP = CG / 4;
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) float4 q4[];
    const int PH = FIX ? FIX : PH_, PW = FIX ? FIX : PW_;
    const int PHW = PH * PW;
    const int b = blockIdx.z;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int HW = H * W;
    const int HWs = (HW + 15) & ~15;
    const int split = gridDim.y, z = blockIdx.y;
    int4* s_geo = reinterpret_cast<int4*>(q4 + NP * HWs);
    int* s_rid = reinterpret_cast<int*>(s_geo + cap);
    int* s_ord = s_rid + cap;
    uint8_t* s_key = reinterpret_cast<uint8_t*>(s_ord + cap);
    unsigned* s_hist = reinterpret_cast<unsigned*>(s_key + ((cap + 15) & ~15));
    int* s_misc = reinterpret_cast<int*>(s_hist + 256);
    auto load_box = [&](int r, float (&bx)[5]) {
        if (HEAD) {
            head_box(rois, hd, r, bx);
        } else {
#pragma unroll
            for (int j = 0; j < 5; ++j) bx[j] = rois[static_cast<size_t>(r) * 5 + j];
        }
    };

    // ---- 0. the image's RoIs: [rbase, rbase + nr) or list[b][0, nr)
    int rbase = 0, nr;
    const int* lst = nullptr;
    if (LIST) {
        nr = cnt[b];
        lst = list + static_cast<size_t>(b) * list_stride(R);
    } else {
        const int N = gridDim.z - 1;
        if (b == N) {  // out-of-range batch indices: [0, count(<0)) and [count(<N), R)
            const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, 0, N, s_misc, 1)
                                 : roi_range_sorted<NT>(rois, R, 0, N, s_misc);
            const int n_lo = rg.x, n_hi = R - rg.y, tot = n_lo + n_hi;
            const int lo = static_cast<int>(static_cast<int64_t>(tot) * z / split);
            const int hi = static_cast<int>(static_cast<int64_t>(tot) * (z + 1) / split);
            if (HEAD && hd.boxes && blockIdx.x == 0)
                for (int t = lo + tid; t < hi; t += NT) {
                    const int r = t < n_lo ? t : rg.y + (t - n_lo);
                    float bx[5];
                    head_box(rois, hd, r, bx);
#pragma unroll
                    for (int j = 0; j < 5; ++j) hd.boxes[static_cast<size_t>(r) * 5 + j] = bx[j];
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
        const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, b, b + 1, s_misc, 1)
                             : roi_range_sorted<NT>(rois, R, b, b + 1, s_misc);
        rbase = rg.x;
        nr = rg.y - rg.x;
    }
    if (nr <= 0) return;
    auto roi_of = [&](int t) { return LIST ? lst[t] : rbase + t; };
    auto geom_of = [&](int r) {
        float bx[5];
        load_box(r, bx);
        return roi_geom(bx, ss, PH, PW);
    };

    // ---- 1. cost-balanced share [lo, hi) of the image's RoIs (contiguous, by
    // the cost midpoint of each RoI; every workgroup of the image computes the
    // same cut, so the shares tile [0, nr) exactly)
    int lo = 0, hi = nr;
    if (split > 1) {
        const int per = (nr + NT - 1) / NT;
        const int t0 = min(tid * per, nr), t1 = min(t0 + per, nr);
        int mine = 0;
        for (int t = t0; t < t1; ++t) mine += geom_class(geom_of(roi_of(t)), H, W, PH, PW).y;
        int incl = mine;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) s_misc[wid] = incl;
        if (tid == 0) {
            s_misc[32] = nr;
            s_misc[33] = 0;
        }
        __syncthreads();
        int64_t pre = incl - mine, total = 0;
        for (int w = 0; w < NW; ++w) {
            pre += w < wid ? s_misc[w] : 0;
            total += s_misc[w];
        }
        for (int t = t0; t < t1; ++t) {
            const int c = geom_class(geom_of(roi_of(t)), H, W, PH, PW).y;
            int s = static_cast<int>(((2 * pre + c) * split) / (2 * total));
            s = s < split - 1 ? s : split - 1;
            if (s == z) {
                atomicMin(&s_misc[32], t);
                atomicMax(&s_misc[33], t + 1);
            }
            pre += c;
        }
        __syncthreads();
        lo = s_misc[32];
        hi = s_misc[33];
        if (lo >= hi) return;  // uniform
    }

    // ---- 2. stage the CG planes (NaN -> -inf: never selected by the strict '>'
    // against the -FLT_MAX start, and max3 never sees a NaN)
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    for (int p = tid; p < HW; p += NT) {
        float v[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            const float e = src[static_cast<size_t>(q) * HW + p];
            v[q] = e != e ? -INFINITY : e;
        }
#pragma unroll
        for (int k = 0; k < NP; ++k)
            q4[k * HWs + p] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }

    const uint32_t plane_bytes = static_cast<uint32_t>(HWs) * 16u;
    const char* tb = reinterpret_cast<const char*>(q4);
    const uint32_t magic_phw = 0xFFFFFFFFu / static_cast<uint32_t>(PHW) + 1u;
    const uint32_t magic_pw = 0xFFFFFFFFu / static_cast<uint32_t>(PW) + 1u;
    // ---- 3. chunks of `cap` RoIs: geometry, order by window class, dense bins
    for (int k0 = lo; k0 < hi; k0 += cap) {
        const int cn = min(cap, hi - k0);
        for (int i = tid; i < 256; i += NT) s_hist[i] = 0;
        __syncthreads();  // tile staged / previous chunk done with geo, ord, hist
        for (int i = tid; i < cn; i += NT) {
            const int r = roi_of(k0 + i);
            float bx[5];
            load_box(r, bx);
            if (HEAD && hd.boxes && blockIdx.x == 0) {
#pragma unroll
                for (int j = 0; j < 5; ++j) hd.boxes[static_cast<size_t>(r) * 5 + j] = bx[j];
            }
            const RoiGeom gm = roi_geom(bx, ss, PH, PW);
            s_geo[i] = make_int4(gm.sh, gm.sw, __float_as_int(gm.bh), __float_as_int(gm.bw));
            s_rid[i] = r;
            const int key = geom_class(gm, H, W, PH, PW).x;
            s_key[i] = static_cast<uint8_t>(key);
            atomicAdd(&s_hist[255 - key], 1u);  // descending window class
        }
        __syncthreads();
        if (wid == 0) {  // exclusive scan of the 256 buckets, 4 per lane
            unsigned h[4], loc = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                h[j] = s_hist[4 * lane + j];
                loc += h[j];
            }
            unsigned incl = loc;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned v = __shfl_up(incl, o, 64);
                if (lane >= o) incl += v;
            }
            unsigned run = incl - loc;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s_hist[4 * lane + j] = run;
                run += h[j];
            }
        }
        if (tid == 0) s_misc[40] = 0;
        __syncthreads();
        for (int i = tid; i < cn; i += NT) s_ord[atomicAdd(&s_hist[255 - s_key[i]], 1u)] = i;
        __syncthreads();

        const int total = cn * PHW;
        int f0 = 0;
        if (lane == 0) f0 = atomicAdd(&s_misc[40], 64);
        f0 = __builtin_amdgcn_readfirstlane(f0);
        while (f0 < total) {
            int fn = 0;
            if (lane == 0) fn = atomicAdd(&s_misc[40], 64);  // prefetch the next chunk
            const int f = f0 + lane;
            const bool live = f < total;
            // (the magic reciprocal of 1 wraps to 0: divisors of 1 bypass it)
            const int t = FIX ? (live ? f / PHW : 0)
                              : (live ? (PHW == 1 ? f : static_cast<int>(__umulhi(static_cast<uint32_t>(f), magic_phw)))
                                      : 0);
            const int k = f - t * PHW;
            const int ph = FIX ? k / PW
                               : (PW == 1 ? k : static_cast<int>(__umulhi(static_cast<uint32_t>(k), magic_pw)));
            const int pw = k - ph * PW;
            const int item = s_ord[t];
            const int4 gq = s_geo[item];
            RoiGeom gm;
            gm.sh = gq.x;
            gm.sw = gq.y;
            gm.bh = __int_as_float(gq.z);
            gm.bw = __int_as_float(gq.w);
            int4 g = geom_bin(gm, H, W, ph, pw);
            if (!live) g = make_int4(0, 0, 0, 0);
            const bool empty = g.y <= g.x || g.w <= g.z;
            float mv[CG];
            int mi[CG];  // LDS byte offset of the max's pixel in plane 0 (-16: none)
#pragma unroll
            for (int c = 0; c < CG; ++c) {
                mv[c] = empty ? 0.0f : -FLT_MAX;
                mi[c] = -16;
            }
            // One pixel pair (a, b) in row-major order: per channel m' = max3(m, a, b);
            // the index moves iff m' > m, to a if a == m' (a comes first).  A pair
            // past the window's row end repeats its last pixel, which can never
            // pass the strict '>' again.  src -> dst are different registers; the
            // loop takes two pairs per trip (mv -> m2 -> mv), so the running
            // maxima need no copy back except after an odd pair at a row end.
            float m2[CG];
            auto pair = [&](const float (&src)[CG], float (&dst)[CG], int ia, int ib) {
                float4 va[NP], vb[NP];
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    va[q] = *static_cast<const float4*>(
                        __builtin_assume_aligned(tb + q * plane_bytes + ia, 16));
                    vb[q] = *static_cast<const float4*>(
                        __builtin_assume_aligned(tb + q * plane_bytes + ib, 16));
                }
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const float a4[4] = {va[q].x, va[q].y, va[q].z, va[q].w};
                    const float b4[4] = {vb[q].x, vb[q].y, vb[q].z, vb[q].w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int c = 4 * q + j;
                        const float m = max3_raw(src[c], a4[j], b4[j]);
                        const int ip = a4[j] == m ? ia : ib;
                        mi[c] = m > src[c] ? ip : mi[c];
                        dst[c] = m;
                    }
                }
            };
            const int wl = g.w - 1;
            for (int h = g.x; h < g.y; ++h) {
                const int rb = h * W;
                int w = g.z;
                for (; w + 2 < g.w; w += 4) {  // >= 3 pixels left: two pairs
                    pair(mv, m2, (rb + w) << 4, (rb + w + 1) << 4);
                    pair(m2, mv, (rb + w + 2) << 4, (rb + min(w + 3, wl)) << 4);
                }
                if (w < g.w) {  // 1 or 2 pixels left
                    pair(mv, m2, (rb + w) << 4, (rb + min(w + 1, wl)) << 4);
#pragma unroll
                    for (int c = 0; c < CG; ++c) mv[c] = m2[c];
                }
            }
            if (live) {
                const int r = s_rid[item];
                const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + k;
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    const int idx = mi[c] >> 4;
                    float v = mv[c];
                    if (v == 0.0f && idx >= 0)  // exact bits (sign) of a zero maximum
                        v = reinterpret_cast<const float*>(tb + (c >> 2) * plane_bytes)[idx * 4 + (c & 3)];
                    out[o + static_cast<size_t>(c) * PHW] = v;
                    argmax[o + static_cast<size_t>(c) * PHW] = idx;
                }
            }
            f0 = __builtin_amdgcn_readfirstlane(fn);
        }
    }
}

// Timeline probe of the wave-per-RoI forward (instrumented builds only,
// -DFRCNN_POOL_PROF, tools/probe_pool.py): per workgroup the realtime clock
// (100 MHz) at entry, after the RoI range, after the tile is staged, and the
// last wave's exit; plus the RoIs it pooled.
#ifdef FRCNN_POOL_PROF
constexpr int kPoolProfSlots = 8192;
__device__ unsigned long long g_pool_prof[kPoolProfSlots][4];
__device__ unsigned int g_pool_prof_rois[kPoolProfSlots];
#define PPROF_T(k)                                                                                  \
    do {                                                                                            \
        const unsigned long long _t = __builtin_amdgcn_s_memrealtime();                             \
        const unsigned _wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);         \
        if (_wg < kPoolProfSlots) {                                                                 \
            if ((k) == 3) {                                                                         \
                if ((threadIdx.x & 63) == 0) atomicMax(&g_pool_prof[_wg][3], _t);                   \
            } else if (threadIdx.x == 0) {                                                          \
                g_pool_prof[_wg][k] = _t;                                                           \
            }                                                                                       \
        }                                                                                           \
    } while (0)
#define PPROF_ROIS(n)                                                                               \
    do {                                                                                            \
        const unsigned _wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);         \
        if (_wg < kPoolProfSlots && threadIdx.x == 0) g_pool_prof_rois[_wg] = (n);                  \
    } while (0)
#else
#define PPROF_T(k) do {} while (0)
#define PPROF_ROIS(n) do {} while (0)
#endif

// Tile layout of the wave-per-RoI forward: NP 4-channel planes, plane q at
// byte q * PS, pixel p of a plane at byte 16 p (the tile starts at LDS address
// 0: the kernel has no static LDS).  PS is a multiple of 256 B, so lanes
// reading pixels p, p' collide only for p = p' mod 16 (a host-side model over
// the bench's RoIs: 1.78 LDS passes per b128 read vs 1.89 for the XOR-swizzled
// 16-pixel groups this replaced).  With PS a compile-time constant (KPS, the
// 7x7 head on maps of < kFixPx pixels) a pixel's NP reads take two addresses
// and immediate offsets, and the window walk steps one byte address: 3 VALU
// per pixel besides the 3 per channel, against 8 for the swizzled layout.
constexpr int kFixPx = 2400;  // pixels per plane (+ sentinel) at KPS = 38,400 B (38 x 63 + 1 fits)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f32x4 lds_f32x4;

// Pixel reads at LDS byte address a (planes 0, 1 from a, planes 2, 3 from a2 =
// a + 2 PS).  With a compile-time PS, a2 comes from an opaque add, else the
// compiler re-derives a + 2 PS and a + 3 PS from a (two adds instead of one).
template <int NP, int KPS>
__device__ __forceinline__ void tile_read(uint32_t a, uint32_t ps, f32x4 (&v)[NP]) {
    const uint32_t P = KPS ? static_cast<uint32_t>(KPS) : ps;
    uint32_t a2 = 0;
    if (NP > 2) {
        if (KPS) asm("v_add_u32_e32 %0, %1, %2" : "=v"(a2) : "i"(2 * KPS), "v"(a));
        else a2 = a + 2 * P;
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const uint32_t o = q < 2 ? a + q * P : a2 + (q - 2) * P;
        v[q] = *reinterpret_cast<lds_f32x4*>(static_cast<size_t>(o));
    }
}

// ------------------------------------------------- wave-per-RoI forward
// The default forward for RoIs grouped by image.  Grid (C/CG, split, N + 1):
// one 1024-thread workgroup owns CG channel planes of one image (staged once
// into LDS as plane-major 4-channel planes, see tile_read) and a strided
// share of that image's RoIs (items z, z+split, ...: RoI sizes are
// uncorrelated with rank, so every share sees the image's size mix).  One
// wave per RoI, lane = bin: each lane walks its window once and updates CG
// (max, first index) pairs with torchvision's strict '>' -- the RoI geometry,
// the window walk and the pixel address are shared by CG channels.  Waves pull
// RoIs from an LDS counter (RoI sizes vary 100x); the RoI geometry of a chunk
// of RoIs is computed once per workgroup into LDS.  Output: per channel, the
// 49 lanes write one contiguous 196-B run.
// HEAD: fused with the head's RoI transform (nets/heads.py:42-47): `rois` are
// the [R,4] image boxes, hd.inds their image index; the [idx, box] rows are
// formed in registers and (channel group 0) written to hd.boxes.  The image
// index is the slowest grid dimension, so the workgroups of row N (RoIs with a
// batch index outside [0, N): usually none, they exit at once) are dispatched
// after every real one instead of holding CUs between them.
// (Measured alternatives -- RoI bins packed 64 per wave, bins or rows sorted by
// window shape, RoIs in cost order, a byte window table -- are slower:
// DESIGN.md §3, profiles/r5_experiments.md.)
// FIX = PH = PW known at compile time (the 7x7 head): the 2 x CG output
// stores of a RoI take immediate offsets from one base address.
template <int NT, int CG, int FIX, bool HEAD, bool NTS = false, int KPS = 0>
__global__ __launch_bounds__(NT) void roi_pool_fwd_wave_kernel(
    const float* __restrict__ x, const float* __restrict__ rois, int R, int C, int H, int W, int PH_, int PW_,
    float ss, float* __restrict__ out, int32_t* __restrict__ argmax, int geo_cap, HeadArgs hd) {
    const int PH = FIX ? FIX : PH_, PW = FIX ? FIX : PW_;
    constexpr int NP = CG / 4;
    // tile (NP planes of PS bytes, from address 0), geometry chunk, reduction
    // scratch, work counter: all dynamic (no static LDS, so the tile is at 0)
    extern __shared__ __attribute__((aligned(16))) float4 q4[];
    char* const t = reinterpret_cast<char*>(q4);
    if ((size_t)(__attribute__((address_space(3))) float4*)q4 != 0) __builtin_trap();  // the argmax decode needs it
    const int b = blockIdx.z;
    const int c0 = blockIdx.x * CG;
    const int tid = threadIdx.x, lane = tid & 63;
    const int HW = H * W;
    const int HWs = (HW + 16) & ~15;  // + the zero sentinel pixel HW
    const uint32_t PS = KPS ? static_cast<uint32_t>(KPS) : static_cast<uint32_t>(HWs) * 16u;
    int4* s_geo = reinterpret_cast<int4*>(t + NP * PS);
    int* s_red = reinterpret_cast<int*>(s_geo + geo_cap);
    int* s_next = s_red + 2 * (NT / 64);
    const int PHW = PH * PW;
    const int split = gridDim.y, z = blockIdx.y;
    const int N = gridDim.z - 1;
    PPROF_T(0);
    if (b == N) {  // out-of-range batch indices: [0, count(<0)) and [count(<N), R)
        const int2 rg = HEAD ? roi_range_sorted<NT>(hd.inds, R, 0, N, s_red, 1)
                             : roi_range_sorted<NT>(rois, R, 0, N, s_red);
        const int n_lo = rg.x, tot = n_lo + (R - rg.y);
        const int lo = static_cast<int>(static_cast<int64_t>(tot) * z / split);
        const int hi = static_cast<int>(static_cast<int64_t>(tot) * (z + 1) / split);
        if (HEAD && hd.boxes && blockIdx.x == 0)
            for (int t = lo + tid; t < hi; t += NT) {
                const int r = t < n_lo ? t : rg.y + (t - n_lo);
                float bx[5];
                head_box(rois, hd, r, bx);
#pragma unroll
                for (int j = 0; j < 5; ++j) hd.boxes[static_cast<size_t>(r) * 5 + j] = bx[j];
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
    PPROF_T(1);
    if (z >= nr) return;
    const int nmine = (nr - z + split - 1) / split;  // items z, z+split, ...
    PPROF_ROIS(nmine);
    const float* src = x + (static_cast<size_t>(b) * C + c0) * HW;
    if (tid < NP) *reinterpret_cast<float4*>(t + tid * PS + HW * 16) = make_float4(0.f, 0.f, 0.f, 0.f);
    // Staged as max(v, -FLT_MAX) with NaN -> -FLT_MAX: no such value passes the
    // scan's strict '>' against a running maximum >= -FLT_MAX, and the window's
    // first pixel then starts the maximum as is (torchvision starts at -FLT_MAX).
    for (int p = tid; p < HW; p += NT) {
        float v[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            const float e = src[static_cast<size_t>(q) * HW + p];
            v[q] = e > -FLT_MAX ? e : -FLT_MAX;
        }
#pragma unroll
        for (int k = 0; k < NP; ++k)
            *reinterpret_cast<float4*>(t + k * PS + p * 16) = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    const int ph = lane / PW, pw = lane - (lane / PW) * PW;
    const bool act = lane < PHW;
    for (int k0 = 0; k0 < nmine; k0 += geo_cap) {
        const int cn = min(geo_cap, nmine - k0);
        for (int i = tid; i < cn; i += NT) {
            const int r = rbase + z + (k0 + i) * split;
            float bx[5];
            if (HEAD) {
                head_box(rois, hd, r, bx);
                if (hd.boxes && blockIdx.x == 0) {
#pragma unroll
                    for (int j = 0; j < 5; ++j) hd.boxes[static_cast<size_t>(r) * 5 + j] = bx[j];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 5; ++j) bx[j] = rois[static_cast<size_t>(r) * 5 + j];
            }
            const RoiGeom gm = roi_geom(bx, ss, PH, PW);
            s_geo[i] = make_int4(gm.sh, gm.sw, __float_as_int(gm.bh), __float_as_int(gm.bw));
        }
        if (tid == 0) *s_next = 0;
        __syncthreads();
        if (k0 == 0) PPROF_T(2);
        int k = 0;
        if (lane == 0) k = atomicAdd(s_next, 1);
        k = __builtin_amdgcn_readfirstlane(k);
        while (k < cn) {
            int kn = 0;
            if (lane == 0) kn = atomicAdd(s_next, 1);  // prefetch the next item
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
            // the window's first pixel starts the scan; an empty window reads the
            // zero sentinel pixel and keeps argmax -1.  The argmax is carried as
            // the pixel's byte address (16 p) and converted at the store.
            float mv[CG];
            int mi[CG];
            {
                const uint32_t a0 = static_cast<uint32_t>(empty ? HW : g.x * W + g.z) * 16u;
                const float thr = empty ? __int_as_float(0x7f800000) : -FLT_MAX;
                f32x4 v[NP];
                tile_read<NP, KPS>(a0, PS, v);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const float vv[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        mv[4 * q + j] = vv[j];
                        mi[4 * q + j] = vv[j] > thr ? static_cast<int>(a0) : -1;
                    }
                }
            }
            for (int h = g.x; h < g.y; ++h) {
                const uint32_t rb = static_cast<uint32_t>(h * W) * 16u;
                const uint32_t ae = rb + static_cast<uint32_t>(g.w) * 16u;
                uint32_t a = rb + static_cast<uint32_t>(h == g.x ? g.z + 1 : g.z) * 16u;
                for (; a < ae; a += 16) {
                    f32x4 v[NP];
                    tile_read<NP, KPS>(a, PS, v);
                    // all NP reads in flight before the first compare (else the compiler
                    // waits on each read in turn: NP LDS round trips per pixel)
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < NP; ++q) {
                        const float vv[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (vv[j] > mv[4 * q + j]) {  // torchvision's strict '>'
                                mv[4 * q + j] = vv[j];
                                mi[4 * q + j] = static_cast<int>(a);
                            }
                        }
                    }
                }
            }
            if (act) {
                const size_t o = (static_cast<size_t>(r) * C + c0) * PHW + lane;
                float* op = out + o;
                int32_t* ap = argmax + o;
                if constexpr (NTS) {  // (a template choice: a runtime branch gets its stores
                                      // merged with the temporal ones, hint dropped)
                    // non-temporal (frcnn_set_path("roi_pool_fwd_store", "nt")): the
                    // outputs then do not displace what concurrent kernels cache --
                    // the cfg2 pipeline gains 5 %, but alone every config loses and
                    // cfg1 / cfg3 / cfg4 lose 5-12 % (profiles/r4_experiments.md),
                    // and a real head reads the outputs next, so temporal is the default
#pragma unroll
                    for (int c = 0; c < CG; ++c) {
                        __builtin_nontemporal_store(mv[c], op + c * PHW);
                        __builtin_nontemporal_store(mi[c] >> 4, ap + c * PHW);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < CG; ++c) {
                        op[c * PHW] = mv[c];
                        ap[c * PHW] = mi[c] >> 4;
                    }
                }
            }
            k = __builtin_amdgcn_readfirstlane(kn);
        }
        __syncthreads();  // the chunk's geometry and s_next are reused
    }
    PPROF_T(3);
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

// Ordered per-image RoI lists: list[b][*] = RoIs with batch index b, ascending.
// Each image's list has room for kListPad entries past its RoIs.
// Block N (the extra one) collects the RoIs whose batch index is outside [0, N).
// `stride`: floats between consecutive batch indices (5 for [R,5] RoIs, 1 for
// the head's roi_inds).
// `code` (optional, the backward prep's per-bin codes): entries of RoIs whose
// bin 0 code has the "slow" bit (overlaps beyond the grid neighbours) get bit
// 31 set, so the leader backward learns a RoI's path from the scalar list load.
template <class Flag>
__device__ __forceinline__ void roi_lists_image(const float* __restrict__ rois, int R, int N, int b,
                                                int* __restrict__ list, int* __restrict__ cnt, int stride,
                                                Flag flag_of) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    __shared__ int s_w[16];
    __shared__ int s_last;
    int base = 0;
    for (int r0 = 0; r0 < R; r0 += 1024) {
        int r = r0 + tid;
        int rb = r < R ? static_cast<int>(rois[static_cast<size_t>(r) * stride]) : -1;
        bool m = r < R && (b < N ? rb == b : (rb < 0 || rb >= N));
        uint64_t bal = __ballot(m);
        if (lane == 0) s_w[wid] = __popcll(bal);
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            before += w < wid ? s_w[w] : 0;
            tot += s_w[w];
        }
        if (m) {
            const int flag = flag_of(r) ? static_cast<int>(0x80000000u) : 0;
            const int pos = base + before + __popcll(bal & lanemask_lt());
            list[static_cast<size_t>(b) * list_stride(R) + pos] = r | flag;
            if (pos == base + tot - 1) s_last = r | flag;
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) cnt[b] = base;
    // kListPad entries past the last one repeat it, so a reader may fetch whole
    // groups of entries past the image's count without bounds checks
    if (tid < kListPad) list[static_cast<size_t>(b) * list_stride(R) + base + tid] = base > 0 ? s_last : 0;
}

__global__ __launch_bounds__(1024) void roi_lists_kernel(const float* __restrict__ rois, int R,
                                                         int N, int* __restrict__ list,
                                                         int* __restrict__ cnt, int stride = 5,
                                                         const uint8_t* __restrict__ code = nullptr,
                                                         int PHW = 0) {
    roi_lists_image(rois, R, N, blockIdx.x, list, cnt, stride,
                    [&](int r) { return code && (code[static_cast<size_t>(r) * PHW] & 16); });
}

// Outputs of RoIs with an out-of-range batch index: 0 / -1 (torchvision: UB);
// with a head transform (hd.inds) also their [idx, box] rows.
__global__ __launch_bounds__(256) void roi_pool_invalid_fill_kernel(const int* __restrict__ list,
                                                                    const int* __restrict__ cnt,
                                                                    int R, int N, size_t per_roi,
                                                                    float* __restrict__ out,
                                                                    int32_t* __restrict__ argmax,
                                                                    const float* __restrict__ rois4 = nullptr,
                                                                    HeadArgs hd = HeadArgs{}) {
    const int n = cnt[N];
    for (int t = blockIdx.x; t < n; t += gridDim.x) {
        const int r = list[static_cast<size_t>(N) * list_stride(R) + t];
        const size_t base = static_cast<size_t>(r) * per_roi;
        if (hd.inds && threadIdx.x == 0) {
            float bx[5];
            head_box(rois4, hd, r, bx);
#pragma unroll
            for (int j = 0; j < 5; ++j) hd.boxes[static_cast<size_t>(r) * 5 + j] = bx[j];
        }
        for (size_t e = threadIdx.x; e < per_roi; e += 256) {
            out[base + e] = 0.0f;
            argmax[base + e] = -1;
        }
    }
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

// roi_bwd_prep_kernel for PH*PW <= 64 (same outputs): one wave per RoI, lane =
// bin.  Bin windows are separable (rows depend on ph only, columns on pw only),
// so a bin's overlap set is (rows overlapping its row) x (columns overlapping
// its column): PH + PW lane reads instead of a walk over every earlier bin.
__device__ __forceinline__ void roi_bwd_prep64_roi(const float* __restrict__ rois, int r, int H, int W, int PH,
                                                   int PW, float ss, uint64_t* __restrict__ cmask,
                                                   uint8_t* __restrict__ code) {
    const int lane = threadIdx.x & 63;
    const int PHW = PH * PW;
    const float* roi = rois + static_cast<size_t>(r) * 5;
    const int k = lane < PHW ? lane : 0;
    const int pw = k % PW;
    const int4 g = roi_bin(roi, ss, H, W, PH, PW, k / PW, pw);
    const bool ne = lane < PHW && g.y > g.x && g.w > g.z;
    uint64_t colbits = 0;  // columns q whose (non-empty) range overlaps this bin's
    for (int q = 0; q < PW; ++q) {
        const int qz = __shfl(g.z, q, 64), qw = __shfl(g.w, q, 64);  // bin (0, q)
        if (qw > qz && qz < g.w && g.z < qw) colbits |= 1ull << q;
    }
    uint64_t m = 0;
    for (int q = 0; q < PH; ++q) {
        const int qx = __shfl(g.x, q * PW, 64), qy = __shfl(g.y, q * PW, 64);  // bin (q, 0)
        if (qy > qx && qx < g.y && g.x < qy) m |= colbits << (q * PW);
    }
    m &= (1ull << lane) - 1;  // earlier bins only
    m = ne ? m : 0ull;
    uint32_t nb = 0;
    bool other = false;
    if (lane < PHW) {
        cmask[static_cast<size_t>(r) * PHW + lane] = m;
        uint64_t known = 0;
        if (pw > 0) {
            known |= 1ull << (lane - 1);
            nb |= (m >> (lane - 1)) & 1u;
        }
        if (lane >= PW) {
            known |= 1ull << (lane - PW);
            nb |= ((m >> (lane - PW)) & 1u) << 1;
            if (pw > 0) {
                known |= 1ull << (lane - PW - 1);
                nb |= ((m >> (lane - PW - 1)) & 1u) << 2;
            }
            if (pw < PW - 1) {
                known |= 1ull << (lane - PW + 1);
                nb |= ((m >> (lane - PW + 1)) & 1u) << 3;
            }
        }
        other = (m & ~known) != 0;
    }
    const bool slow = __ballot(other) != 0;
    if (lane < PHW) code[static_cast<size_t>(r) * PHW + lane] = static_cast<uint8_t>(nb | (slow ? 16u : 0u));
}

__global__ __launch_bounds__(256) void roi_bwd_prep64_kernel(const float* __restrict__ rois, int R,
                                                             int H, int W, int PH, int PW, float ss,
                                                             uint64_t* __restrict__ cmask,
                                                             uint8_t* __restrict__ code) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;  // whole wave
    roi_bwd_prep64_roi(rois, r, H, W, PH, PW, ss, cmask, code);
}

// Whether a RoI's bins can overlap beyond their grid neighbours: some bin row
// overlaps the row two below it, or some bin column the column two right of it
// (windows are separable and monotone).  A superset of the prep kernel's
// per-RoI "slow" flag (which also looks at emptiness), so a RoI it clears has
// only neighbour overlaps -- the leader backward's precondition; flagged RoIs
// take the exact ranked path either way.
__device__ __forceinline__ bool roi_far_overlap(const float* __restrict__ roi, float ss, int H, int W, int PH,
                                                int PW) {
    const RoiGeom g = roi_geom(roi, ss, PH, PW);
    bool far = false;
    for (int q = 0; q + 2 < PH; ++q) {
        const int4 a = geom_bin(g, H, W, q, 0), c = geom_bin(g, H, W, q + 2, 0);
        far |= a.y > c.x && a.y > a.x && c.y > c.x;
    }
    for (int q = 0; q + 2 < PW; ++q) {
        const int4 a = geom_bin(g, H, W, 0, q), c = geom_bin(g, H, W, 0, q + 2);
        far |= a.w > c.z && a.w > a.z && c.w > c.z;
    }
    return far;
}

// The leader backward's two preparations in one launch (PH*PW <= 64): workgroups
// [0, N] build the per-image RoI lists, their entries flagged from the RoI
// geometry (roi_far_overlap); the others compute the per-RoI overlap masks and
// codes (16 RoIs per workgroup, one wave each).  Independent, so one launch
// instead of two back to back.
__global__ __launch_bounds__(1024) void roi_bwd_prep_lists_kernel(const float* __restrict__ rois, int R, int N,
                                                                  int H, int W, int PH, int PW, float ss,
                                                                  uint64_t* __restrict__ cmask,
                                                                  uint8_t* __restrict__ code,
                                                                  int* __restrict__ list, int* __restrict__ cnt) {
    const int b = blockIdx.x;
    if (b <= N) {
        roi_lists_image(rois, R, N, b, list, cnt, 5, [&](int r) {
            return roi_far_overlap(rois + static_cast<size_t>(r) * 5, ss, H, W, PH, PW);
        });
        return;
    }
    const int r = (b - N - 1) * 16 + (threadIdx.x >> 6);
    if (r >= R) return;  // whole wave
    roi_bwd_prep64_roi(rois, r, H, W, PH, PW, ss, cmask, code);
}

// General plane-owner backward (any output size; planes in LDS or, when a
// plane does not fit, in grad_in itself with agent-scope load/store rounds).
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
    const int* lst = list + static_cast<size_t>(b) * list_stride(R);
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
// latency-hidden: the loads of RoI t+D are issued before RoI t is applied (a
// D-deep register ring, slot index static after unrolling), and the RoI
// indices come by scalar loads, so no vector load sits between the ring's loads
// in the in-order vmcnt queue.  Summation order per pixel is unchanged (RoIs
// ascending, bins ascending within a RoI): bit-identical results.
template <int D>
__global__ __launch_bounds__(1024) void roi_pool_bwd_pf_kernel(
    const float* __restrict__ grad, const int32_t* __restrict__ argmax,
    const uint64_t* __restrict__ cmask, const uint8_t* __restrict__ code,
    const int* __restrict__ list, const int* __restrict__ cnt,
    int R, int C, int HW, int PHW, int PW, int CPW, float* __restrict__ grad_in) {
    extern __shared__ __attribute__((aligned(16))) float planes[];
    const int lane = threadIdx.x & 63;
    // wave-uniform in an SGPR: the per-RoI grad / argmax bases are then scalar,
    // and each lane's load is base (SGPR) + its bin offset (VGPR, fixed)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
        const int* lst = list + static_cast<size_t>(b) * list_stride(R);  // wave-uniform: scalar loads
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
            const size_t nb = static_cast<size_t>(n) * PHW;
            am_r[d] = (argmax + base)[kl];
            g_r[d] = (grad + base)[kl];
            cd_r[d] = (code + nb)[kl];
            cm_r[d] = (cmask + nb)[kl];
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
                    const size_t nb = static_cast<size_t>(n) * PHW;
                    am_r[d] = (argmax + base)[kl];
                    g_r[d] = (grad + base)[kl];
                    cd_r[d] = (code + nb)[kl];
                    cm_r[d] = (cmask + nb)[kl];
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


// Phase timer of the leader backward (-DFRCNN_BWD_PROF, tools/probe_bwd_spans.py):
// per wave, the RoI count, start and end on the constant 100 MHz clock
// (s_memrealtime, the end after the plane write-out), the flagged RoIs, and the
// shader-clock cycles of their gathers.
#ifdef FRCNN_BWD_PROF
constexpr int kBwdProfWaves = 8192;
// columns: ring+exchange+apply cycles (0-2), RoIs (3), start (4), end (5), flagged
// RoIs (6), cycles in the flagged RoIs' gathers (7)
__device__ unsigned long long g_bwd_prof[kBwdProfWaves][8];
#define BPROF_T() __builtin_amdgcn_s_memtime()
#else
#define BPROF_T() 0ull
#endif
// Exchange row of the leader kernel (int2 (argmax, grad) entries): lane k at entry
// PW + 1 + k, linear in the lane, so that a wave's reads at any fixed lane offset
// are bank-conflict free (a layout with a pad entry per bin row, which would drop
// the grid-edge masks, spreads 32 lanes over > 256 B: 2-way conflicts, op 78 -> 88
// us at cfg5, profiles/r6_experiments.md).
constexpr int kBwdXRow = 80;

// Leader-gather plane-owner backward (PH*PW < 64, PW = 7), the default.
// A wave owns one (image, channel) plane in LDS and walks the image's RoIs in
// ascending order, lane = bin.  Bins that share an argmax pixel all contain it,
// so their windows overlap; when a RoI's overlaps are only between grid
// neighbours (its list entry unflagged) the bins of one pixel lie in a 2x2
// block.  The first of them in bin order (no earlier neighbour -- left, up-left,
// up, up-right -- with the same argmax) leads: it reads the pixel once, adds its
// own gradient and then those of its later neighbours with the same argmax
// (right or down-left, down, down-right: ascending bin order) and writes once.
// Every pixel so sees the CPU summation order n -> ph -> pw in one
// read-add-write per RoI.  Non-contributing neighbours add -0.0 (x + -0.0 == x
// for every plane value: sums started at +0.0 are never -0.0); non-leaders read
// and write a dummy word of their own past the plane.  The neighbours' (argmax,
// grad) pairs come through a per-wave LDS exchange row (one ds_write_b64, eight
// ds_read_b64 at immediate offsets).  A flagged RoI (tiny windows: bins share a
// pixel beyond their 2x2 block) gathers instead: every lane reads its pixel and
// adds the gradient of EVERY bin of the RoI with its argmax, in bin order, from
// broadcast reads of the row, so all bins of one pixel compute the same CPU-order
// sum and write the same word (round 6: 1,500 cycles per flagged RoI against
// ~3,200 for round 5's overlap-mask rank walk + ranked rounds, op 88.7 -> 78.3
// us at cfg5; profiles/r6_experiments.md).  D RoIs per step, two per exchange;
// each pair's read-add-writes go to the plane in RoI order behind the next
// pair's exchange (after it, when the pair holds a flagged RoI: its gather reads
// the row).  PHT = PH at compile time (the 7x7 head: the gather's reads all
// issued at once), or 0.
template <int D, int PWT, int PHT>
__global__ __launch_bounds__(1024) void roi_pool_bwd_lead_kernel(
    const float* __restrict__ grad, const int32_t* __restrict__ argmax,
    const int* __restrict__ list, const int* __restrict__ cnt,
    int R, int C, int HW, int HWs, int PH_, int CPW, float* __restrict__ grad_in) {
    extern __shared__ __attribute__((aligned(16))) float planes[];
    static_assert(PWT == 7, "exchange rows hold 7 bins and a pad");
    constexpr int PW = PWT;
    const int PH = PHT > 0 ? PHT : PH_;
    const int PHW = PH * PW;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // wave w of workgroup (x, y) takes image (y + w) mod N: every CU carries a mix of
    // the images, whose flagged-RoI gathers differ (the kernel is issue-bound; round 6:
    // 77.2-78.1 vs 78.5-79.3 µs op, span max 71.6 vs 74.3), each (image, channel) once
    const int b = static_cast<int>((blockIdx.y + static_cast<unsigned>(wid)) % gridDim.y);
    const int c = blockIdx.x * CPW + wid;
    if (c >= C) return;  // whole wave; no workgroup barrier below
#ifdef FRCNN_BWD_PROF
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long tq[2] = {0, 0};
#endif
    float* gplane = grad_in + (static_cast<size_t>(b) * C + c) * HW;
    // HWs >= HW + 64: word HW + lane is lane's dummy (a word per lane, so the
    // non-leaders' writes do not serialise on one bank)
    float* plane = planes + static_cast<size_t>(wid) * HWs;
    typedef __attribute__((address_space(3))) float lds_float;
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const i32x4 lds_i32x4;
    // this wave's two exchange rows: xbase = lane 0's entry in row 0, xrow = this lane's
    // entry minus PW + 1 entries (its up-left neighbour); a neighbour across the grid
    // edge is masked by the lane's has_* flags
    static_assert(64 + 2 * (PW + 1) <= kBwdXRow, "exchange row too short");
    const uint32_t xbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_float*)planes)) +
                           static_cast<uint32_t>(CPW * HWs * 4 + wid * 2 * kBwdXRow * 8 + (PW + 1) * 8);
    const uint32_t xrow = xbase + 8 * lane - 8 * (PW + 1);
    const bool act = lane < PHW;
    const int pw_i = lane % PW;
    const bool has_l = pw_i > 0, has_r = pw_i < PW - 1;
    const bool has_u = lane >= PW, has_d = lane + PW < PHW;
    const bool has_ul = has_u && has_l, has_ur = has_u && has_r;
    const bool has_dl = has_d && has_l, has_dr = has_d && has_r;
    for (int i = lane; i < HWs; i += 64) plane[i] = 0.0f;
    const int nr = cnt[b];
    if (nr > 0) {
        const int* lst = list + static_cast<size_t>(b) * list_stride(R);  // wave-uniform: scalar loads
        const uint32_t kl = act ? lane : 0;
        // the host guarantees R*C*PHW*4 < 2^31: byte offsets fit the descriptors
        const uint32_t gb = static_cast<uint32_t>(R) * C * PHW * 4;
        const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(grad), 0, gb, 0x00020000);
        const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(argmax), 0, gb, 0x00020000);
        const uint32_t cpb = static_cast<uint32_t>(c) * PHW * 4;
        const uint32_t rpb = static_cast<uint32_t>(C) * PHW * 4;
        int am_r[D], fl_r[D];
        float g_r[D];
        // list entries: RoI index | flag << 31 (roi_bwd_prep_lists_kernel);
        // the flag drops out of the byte offsets (index x an even stride, mod
        // 2^32).  Positions past the image's RoIs hold copies of its last entry
        // (kListPad of them: a raw buffer load's soffset is not range-checked,
        // so they must be real RoIs); those slots are dead (argmax -1).
        static_assert(2 * D <= kListPad, "ring refills read up to 2D entries past the count");
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int e = lst[d];
            fl_r[d] = e < 0;
            const uint32_t so = static_cast<uint32_t>(e) * rpb + cpb;
            am_r[d] = __builtin_amdgcn_raw_buffer_load_b32(rs_a, kl * 4, so, 0);
            g_r[d] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g, kl * 4, so, 0));
            asm volatile("" ::: "memory");
        }
        for (int t0 = 0; t0 < nr; t0 += D) {
            int nx[D];
#pragma unroll
            for (int d = 0; d < D; ++d) nx[d] = lst[t0 + D + d];
            int am[D], addr[D];
            float g[D], s1[D], s3[D], s4[D];
            bool slow[D];
            // take the slot's argmax / grad / flag, then refill it with RoI t + D
#pragma unroll
            for (int d = 0; d < D; ++d) {
                asm volatile("v_mov_b32 %0, %1" : "=v"(am[d]) : "v"(am_r[d]));
                asm volatile("v_mov_b32 %0, %1" : "=v"(g[d]) : "v"(g_r[d]));
                const bool live = t0 + d < nr;
                slow[d] = live && fl_r[d];
                am[d] = live ? am[d] : -1;
                am[d] = act ? am[d] : -2;
                const uint32_t so = static_cast<uint32_t>(nx[d]) * rpb + cpb;
                am_r[d] = __builtin_amdgcn_raw_buffer_load_b32(rs_a, kl * 4, so, 0);
                g_r[d] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_g, kl * 4, so, 0));
                fl_r[d] = nx[d] < 0;
            }
            // The exchange of slot pair k + 1 is issued before the read-add-writes of pair k
            // and waited for after them: LDS serves a wave in order, so its reads ride in the
            // shadow of the plane round trips.  The outputs are tied to the wait by "+v" operands.
            static_assert(D % 2 == 0, "slots are exchanged in pairs");
            auto lo = [](uint64_t q) { return static_cast<int>(static_cast<uint32_t>(q)); };
            auto hi = [](uint64_t q) { return __builtin_bit_cast(float, static_cast<uint32_t>(q >> 32)); };
            uint64_t q[2][8];
            auto x_issue = [&](int d0) {
                const uint64_t m0 = static_cast<uint32_t>(am[d0]) |
                                    (static_cast<uint64_t>(__builtin_bit_cast(uint32_t, g[d0])) << 32);
                const uint64_t m1 = static_cast<uint32_t>(am[d0 + 1]) |
                                    (static_cast<uint64_t>(__builtin_bit_cast(uint32_t, g[d0 + 1])) << 32);
                asm volatile(
                    "ds_write_b64 %16, %18 offset:%c20\n\t"
                    "ds_write_b64 %17, %19 offset:%c20\n\t"
                    "ds_read_b64 %0, %16 offset:%c21\n\t"
                    "ds_read_b64 %1, %16 offset:%c22\n\t"
                    "ds_read_b64 %2, %16\n\t"
                    "ds_read_b64 %3, %16 offset:%c23\n\t"
                    "ds_read_b64 %4, %16 offset:%c24\n\t"
                    "ds_read_b64 %5, %16 offset:%c25\n\t"
                    "ds_read_b64 %6, %16 offset:%c26\n\t"
                    "ds_read_b64 %7, %16 offset:%c27\n\t"
                    "ds_read_b64 %8, %17 offset:%c21\n\t"
                    "ds_read_b64 %9, %17 offset:%c22\n\t"
                    "ds_read_b64 %10, %17\n\t"
                    "ds_read_b64 %11, %17 offset:%c23\n\t"
                    "ds_read_b64 %12, %17 offset:%c24\n\t"
                    "ds_read_b64 %13, %17 offset:%c25\n\t"
                    "ds_read_b64 %14, %17 offset:%c26\n\t"
                    "ds_read_b64 %15, %17 offset:%c27"
                    : "=&v"(q[0][0]), "=&v"(q[0][1]), "=&v"(q[0][2]), "=&v"(q[0][3]), "=&v"(q[0][4]),
                      "=&v"(q[0][5]), "=&v"(q[0][6]), "=&v"(q[0][7]), "=&v"(q[1][0]), "=&v"(q[1][1]),
                      "=&v"(q[1][2]), "=&v"(q[1][3]), "=&v"(q[1][4]), "=&v"(q[1][5]), "=&v"(q[1][6]),
                      "=&v"(q[1][7])
                    : "v"(xrow), "v"(xrow + kBwdXRow * 8), "v"(m0), "v"(m1), "i"(8 * (PW + 1)),
                      "i"(8 * PW), "i"(8), "i"(16), "i"(8 * (PW + 2)), "i"(8 * (2 * PW)),
                      "i"(8 * (2 * PW + 1)), "i"(8 * (2 * PW + 2))
                    : "memory");
            };
            auto x_wait = [&]() {
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(q[0][0]), "+v"(q[0][1]), "+v"(q[0][2]), "+v"(q[0][3]), "+v"(q[0][4]),
                               "+v"(q[0][5]), "+v"(q[0][6]), "+v"(q[0][7]), "+v"(q[1][0]), "+v"(q[1][1]),
                               "+v"(q[1][2]), "+v"(q[1][3]), "+v"(q[1][4]), "+v"(q[1][5]), "+v"(q[1][6]),
                               "+v"(q[1][7])
                             :
                             : "memory");
            };
            auto apply = [&](int d) {
                float v = plane[addr[d]];
                v = v + g[d];
                v = v + s1[d];
                v = v + s3[d];
                v = v + s4[d];
                plane[addr[d]] = v;
                asm volatile("" ::: "memory");
            };
            // flagged RoI d, its pairs in exchange row e: every bin of the RoI, in bin order
            auto apply_gather = [&](int d, int e) {
#ifdef FRCNN_BWD_PROF
                const unsigned long long q0 = BPROF_T();
#endif
                const int a = am[d];
                const int ad = a >= 0 ? a : HW + lane;
                float v = plane[ad];
                const uint32_t row = xbase + e * kBwdXRow * 8;  // lane 0's entry (16-B aligned)
                // bins 2j, 2j + 1 per broadcast b128 read; entries past the RoI's bins are lanes
                // >= PHW (argmax -2): never a match.  (__builtin_bit_cast of a vector element .y /
                // .w read element 0 / 2 here -- a clang miscompile seen in the IR; __int_as_float
                // of [i] is right)
                auto pair_add = [&](i32x4 q4) {
                    v = v + (q4[0] == a ? __int_as_float(q4[1]) : -0.0f);
                    v = v + (q4[2] == a ? __int_as_float(q4[3]) : -0.0f);
                };
                auto pair_read = [&](int j) {
                    return *reinterpret_cast<lds_i32x4*>(static_cast<size_t>(row + 16 * j));
                };
                if constexpr (PHT > 0) {  // every read issued up front, the adds in bin order
                    constexpr int NQ = (PHT * PW + 1) / 2;
                    i32x4 qa[NQ];
#pragma unroll
                    for (int j = 0; j < NQ; ++j) qa[j] = pair_read(j);
#pragma unroll
                    for (int j = 0; j < NQ; ++j) pair_add(qa[j]);
                } else {
                    const int nq = (PHW + 1) >> 1;
                    for (int j0 = 0; j0 < nq; j0 += 4) {  // (reads up to entry 63 + 1: in the row)
                        i32x4 qa[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) qa[j] = pair_read(j0 + j);
#pragma unroll
                        for (int j = 0; j < 4; ++j) pair_add(qa[j]);
                    }
                }
                plane[ad] = v;
                asm volatile("" ::: "memory");
#ifdef FRCNN_BWD_PROF
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                tq[0] += 1;
                tq[1] += BPROF_T() - q0;
#endif
            };
            x_issue(0);
            x_wait();
#pragma unroll
            for (int d0 = 0; d0 < D; d0 += 2) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int d = d0 + e;
                    const int a = am[d];
                    // q[e]: left, up, up-left, up-right, right, down-left, down, down-right
                    const bool fol = static_cast<int>(has_l & (lo(q[e][0]) == a)) | (has_u & (lo(q[e][1]) == a)) |
                                     (has_ul & (lo(q[e][2]) == a)) | (has_ur & (lo(q[e][3]) == a));
                    const float t5 = (has_dl & (lo(q[e][5]) == a)) ? hi(q[e][5]) : -0.0f;
                    s1[d] = (has_r & (lo(q[e][4]) == a)) ? hi(q[e][4]) : t5;
                    s3[d] = (has_d & (lo(q[e][6]) == a)) ? hi(q[e][6]) : -0.0f;
                    s4[d] = (has_dr & (lo(q[e][7]) == a)) ? hi(q[e][7]) : -0.0f;
                    addr[d] = (a >= 0 && !fol) ? a : HW + lane;
                }
                if (!(slow[d0] | slow[d0 + 1])) {  // (wave-uniform)
                    if (d0 + 2 < D) x_issue(d0 + 2);
                    apply(d0);
                    apply(d0 + 1);
                } else {  // a flagged RoI reads its exchange row while it applies
                    if (slow[d0]) apply_gather(d0, 0);
                    else apply(d0);
                    if (slow[d0 + 1]) apply_gather(d0 + 1, 1);
                    else apply(d0 + 1);
                    if (d0 + 2 < D) x_issue(d0 + 2);
                }
                if (d0 + 2 < D) x_wait();
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
#ifdef FRCNN_BWD_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    const int gw = (blockIdx.y * gridDim.x + blockIdx.x) * CPW + wid;
    if (lane == 0 && gw < kBwdProfWaves) {
        g_bwd_prof[gw][3] = nr;
        g_bwd_prof[gw][4] = t_start;
        g_bwd_prof[gw][5] = t_end;
        g_bwd_prof[gw][6] = tq[0];
        g_bwd_prof[gw][7] = tq[1];
    }
#endif
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

#ifdef FRCNN_BWD_PROF
extern "C" int frcnn_debug_bwd_prof(unsigned long long* out, int reset) {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_prof), sizeof(g_bwd_prof));
    if (reset) {
        static unsigned long long z[kBwdProfWaves][8];
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_prof), z, sizeof(z));
    }
    return 0;
}
#endif
#ifdef FRCNN_POOL_PROF
extern "C" int frcnn_debug_pool_prof(unsigned long long* times, unsigned* rois, int reset) {
    (void)hipMemcpyFromSymbol(times, HIP_SYMBOL(g_pool_prof), sizeof(g_pool_prof));
    (void)hipMemcpyFromSymbol(rois, HIP_SYMBOL(g_pool_prof_rois), sizeof(g_pool_prof_rois));
    if (reset) {
        static unsigned long long zt[kPoolProfSlots][4];
        static unsigned zr[kPoolProfSlots];
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pool_prof), zt, sizeof(zt));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pool_prof_rois), zr, sizeof(zr));
    }
    return 0;
}
#endif

namespace {
struct FwdWs {
    int* list;
    int* cnt;
    size_t bytes;
};
FwdWs carve_fwd(void* ws, int64_t R, int N) {
    Carver c(ws);
    FwdWs w{};
    w.list = c.take<int>(static_cast<size_t>(N + 1) * list_stride(R));
    w.cnt = c.take<int>(N + 1);
    w.bytes = c.used();
    return w;
}

// Launch plan of the wave-per-RoI forward: CG = 16 channel planes when they
// fit the CU's LDS (one workgroup per CU), else 8 (two per CU when they fit),
// else 4.  Each workgroup gets the LDS left over for its RoI-geometry chunk;
// split = RoI shares per (image, channel group), sized so the grid fills every
// resident slot of the CUs the launch stream may use once.
struct PxPlan {
    int cg = 0, geo_cap = 0, split = 1;
    bool kps = false;  // plane stride = kFixPx pixels (compile time)
    size_t lds = 0;
};
constexpr size_t kWaveScratch = 256;  // the wave kernel's reduction scratch + work counter
constexpr size_t kGeoCap = 368;       // RoIs per geometry chunk (see px_plan)
PxPlan px_plan(int C, int N, int H, int W, int PH, int PW, hipStream_t st, size_t per_geo = sizeof(int4)) {
    PxPlan pl;
    const size_t HW = static_cast<size_t>(H) * W;
    const int PHW = PH * PW;
    if (N <= 0 || HW == 0 || PHW > 64 || H > 65535 || W > 65535) return pl;
    constexpr size_t kReserve = 1024;  // allocation rounding
    const size_t kMinGeo = 64 * per_geo;
    const size_t HWs = (HW + 16) & ~static_cast<size_t>(15);  // + the zero sentinel pixel
    auto fits = [&](size_t tile) {  // workgroups per CU for a tile of `tile` bytes (0: none)
        if (2 * (tile + kMinGeo + kWaveScratch + kReserve) <= kLdsPerCu) return 2;
        return tile + kMinGeo + kWaveScratch + kReserve <= kLdsPerCu ? 1 : 0;
    };
    for (int cg : {16, 8, 4}) {
        if (C % cg != 0) continue;
        if (path_cfg().roi_cg && cg != path_cfg().roi_cg) continue;  // A/B override
        const size_t tile_rt = static_cast<size_t>(cg / 4) * HWs * sizeof(float4);
        // The compile-time plane stride instantiates FIX = 7 (7x7 bins, not any 49-bin
        // shape), and its 153.6 KB tile holds the CU alone: take it only where the
        // run-time stride would also get one workgroup per CU.
        const bool kps = cg == 16 && PH == 7 && PW == 7 && HWs <= static_cast<size_t>(kFixPx) && fits(tile_rt) == 1;
        const size_t tile = kps ? static_cast<size_t>(cg / 4) * kFixPx * sizeof(float4) : tile_rt;
        const int per_cu = fits(tile);
        if (!per_cu) continue;
        const size_t geo = (kLdsPerCu / per_cu - kReserve - kWaveScratch - tile) / per_geo;
        // geometry chunk: at most kGeoCap RoIs, so that a 16-plane workgroup leaves
        // 4 KB of the CU's LDS to the proposal chain's IoU-tile kernel (3.3 KB)
        pl.geo_cap = static_cast<int>(geo > kGeoCap ? kGeoCap : geo);
        pl.cg = cg;
        pl.kps = kps;
        pl.lds = tile + static_cast<size_t>(pl.geo_cap) * per_geo + kWaveScratch;
        const int64_t wgs = static_cast<int64_t>(C / cg) * N;
        int64_t sp = (static_cast<int64_t>(stream_cu_count(st)) * per_cu + wgs - 1) / wgs;
        if (path_cfg().roi_split > 0) sp = path_cfg().roi_split;  // A/B override
        pl.split = static_cast<int>(sp < 1 ? 1 : (sp > 64 ? 64 : sp));
        return pl;
    }
    return pl;
}

template <bool HEAD>
int px_launch(const PxPlan& pl, const float* x, const float* rois, int64_t R, int N, int C, int H, int W,
              int PH, int PW, float ss, float* out, int32_t* argmax, const HeadArgs& hd, hipStream_t st) {
    const dim3 grid(static_cast<unsigned>(C / pl.cg), static_cast<unsigned>(pl.split), static_cast<unsigned>(N + 1));
    const bool fix7 = PH == 7 && PW == 7;
    FRCNN_REQUIRE(!pl.kps || fix7, "roi_pool_fwd: fixed-stride plan for a non-7x7 output");
#define FRCNN_PX(CG, FX, KP)                                                                                    \
    do {                                                                                                         \
        if (path_cfg().roi_store)                                                                                \
            hipLaunchKernelGGL((roi_pool_fwd_wave_kernel<1024, CG, FX, HEAD, true, KP>), grid, dim3(1024), pl.lds, \
                               st, x, rois, static_cast<int>(R), C, H, W, PH, PW, ss, out, argmax, pl.geo_cap, hd); \
        else                                                                                                     \
            hipLaunchKernelGGL((roi_pool_fwd_wave_kernel<1024, CG, FX, HEAD, false, KP>), grid, dim3(1024), pl.lds, \
                               st, x, rois, static_cast<int>(R), C, H, W, PH, PW, ss, out, argmax, pl.geo_cap, hd); \
    } while (0)
    if (pl.cg == 16) {
        if (pl.kps) FRCNN_PX(16, 7, kFixPx * 16);
        else if (fix7) FRCNN_PX(16, 7, 0);
        else FRCNN_PX(16, 0, 0);
    } else if (pl.cg == 8) {
        if (fix7) FRCNN_PX(8, 7, 0); else FRCNN_PX(8, 0, 0);
    } else {
        if (fix7) FRCNN_PX(4, 7, 0); else FRCNN_PX(4, 0, 0);
    }
#undef FRCNN_PX
    FRCNN_LAUNCH_CHECK("roi_pool_fwd_wave_kernel");
    return FRCNN_OK;
}

// Launch plan of the dense forward: CG = 16 channel planes when they fit the
// CU's LDS with room for a RoI chunk, else 8, else 4 (two workgroups per CU
// when two fit); cap = RoIs per geometry chunk from the LDS left over; split =
// cost-balanced RoI shares per (image, channel group), sized so the grid fills
// every resident slot once.
struct DensePlan {
    int cg = 0, cap = 0, split = 1;
    size_t lds = 0;
};
DensePlan dense_plan(int C, int N, int H, int W, int PHW) {
    DensePlan pl;
    const size_t HW = static_cast<size_t>(H) * W;
    if (N <= 0 || HW == 0 || PHW > 64 || H > 65535 || W > 65535) return pl;
    const size_t HWs = (HW + 15) & ~static_cast<size_t>(15);
    const size_t fixed = dense_fixed_bytes() + 64;  // + alignment slack
    constexpr size_t kMinItems = 64;
    for (int cg : {16, 8, 4}) {
        if (C % cg != 0) continue;
        if (path_cfg().roi_cg && cg != path_cfg().roi_cg) continue;  // A/B override
        const size_t tile = static_cast<size_t>(cg / 4) * HWs * sizeof(float4);
        const size_t need = tile + fixed + kMinItems * dense_item_bytes();
        if (HWs * 16 * (cg / 4) >= (1u << 31) || need > kLdsPerCu) continue;
        const int per_cu = 2 * need <= kLdsPerCu ? 2 : 1;
        size_t cap = (kLdsPerCu / per_cu - tile - fixed) / dense_item_bytes();
        cap = cap > 4096 ? 4096 : cap;
        pl.cg = cg;
        pl.cap = static_cast<int>(cap & ~static_cast<size_t>(15));
        pl.lds = tile + fixed + static_cast<size_t>(pl.cap) * dense_item_bytes();
        const int64_t wgs = static_cast<int64_t>(C / cg) * N;
        const int64_t target = static_cast<int64_t>(device_cu_count()) * per_cu;
        int64_t sp = (target + wgs - 1) / wgs;
        if (path_cfg().roi_split > 0) sp = path_cfg().roi_split;  // A/B override
        pl.split = static_cast<int>(sp < 1 ? 1 : (sp > 64 ? 64 : sp));
        return pl;
    }
    return pl;
}

template <bool HEAD, bool LIST>
int dense_launch(const DensePlan& pl, const float* x, const float* rois, const int* list, const int* cnt,
                 int64_t R, int N, int C, int H, int W, int PH, int PW, float ss, float* out,
                 int32_t* argmax, const HeadArgs& hd, hipStream_t st) {
    const dim3 grid(static_cast<unsigned>(C / pl.cg), static_cast<unsigned>(pl.split),
                    static_cast<unsigned>(LIST ? N : N + 1));
    const bool fix7 = PH == 7 && PW == 7;
#define FRCNN_DENSE(CG, FX)                                                                               \
    hipLaunchKernelGGL((roi_pool_fwd_dense_kernel<1024, CG, FX, HEAD, LIST>), grid, dim3(1024), pl.lds, st, \
                       x, rois, list, cnt, static_cast<int>(R), C, H, W, PH, PW, ss, out, argmax, pl.cap,  \
                       hd)
    if (pl.cg == 16) {
        if (fix7) FRCNN_DENSE(16, 7); else FRCNN_DENSE(16, 0);
    } else if (pl.cg == 8) {
        if (fix7) FRCNN_DENSE(8, 7); else FRCNN_DENSE(8, 0);
    } else {
        if (fix7) FRCNN_DENSE(4, 7); else FRCNN_DENSE(4, 0);
    }
#undef FRCNN_DENSE
    FRCNN_LAUNCH_CHECK("roi_pool_fwd_dense_kernel");
    return FRCNN_OK;
}
// One launch-plan choice for frcnn_roi_pool_fwd, frcnn_roi_pool_fwd_head and
// the kernel-name query, so the name a caller records is the kernel launched.
enum FwdKind { kFwdWave, kFwdDense, kFwdDenseList, kFwdGeneric };
struct FwdChoice {
    int kind = kFwdGeneric;
    PxPlan px;
    DensePlan dn;
};
FwdChoice choose_fwd(int N, int C, int H, int W, int PH, int PW, bool sorted, hipStream_t st) {
    FwdChoice ch;
    const int path = path_cfg().roi_fwd;
    const int PHW = PH * PW;
    if (sorted && C > 0) {
        if ((path == kPathAuto || path == kPathWave) &&
            (ch.px = px_plan(C, N, H, W, PH, PW, st)).cg) {
            ch.kind = kFwdWave;
            return ch;
        }
    }
    ch.px = PxPlan{};
    if (path != kPathGeneric && C > 0 && (ch.dn = dense_plan(C, N, H, W, PHW)).cg) {
        ch.kind = sorted ? kFwdDense : kFwdDenseList;
        return ch;
    }
    ch.kind = kFwdGeneric;
    return ch;
}

template <bool HEAD>
int fwd_tile_launch(const FwdChoice& ch, const float* x, const float* rois, int64_t R, int N, int C, int H, int W,
                    int PH, int PW, float ss, float* out, int32_t* argmax, const HeadArgs& hd, hipStream_t st) {
    switch (ch.kind) {
        case kFwdWave: return px_launch<HEAD>(ch.px, x, rois, R, N, C, H, W, PH, PW, ss, out, argmax, hd, st);
        default:
            return dense_launch<HEAD, false>(ch.dn, x, rois, nullptr, nullptr, R, N, C, H, W, PH, PW, ss, out,
                                             argmax, hd, st);
    }
}
}  // namespace

extern "C" size_t frcnn_roi_pool_fwd_workspace_size(int64_t R, int N, int C) {
    if (R < 0 || N < 0 || C < 0) return 0;
    return carve_fwd(nullptr, R, N).bytes;
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
    const FwdChoice ch = choose_fwd(N, C, H, W, PH, PW, rois_sorted != 0, st);
    if (ch.kind == kFwdDenseList) {  // any RoI order: per-image lists first
        FwdWs w = carve_fwd(workspace, R, N);
        FRCNN_REQUIRE(workspace && ws_bytes >= w.bytes, "frcnn_roi_pool_fwd: workspace %zu < %zu",
                      ws_bytes, w.bytes);
        hipLaunchKernelGGL(roi_lists_kernel, dim3(N + 1), dim3(1024), 0, st, rois, static_cast<int>(R), N,
                           w.list, w.cnt);
        FRCNN_LAUNCH_CHECK("roi_lists_kernel");
        int rc = dense_launch<false, true>(ch.dn, x, rois, w.list, w.cnt, R, N, C, H, W, PH, PW, spatial_scale,
                                           out, argmax, HeadArgs{}, st);
        if (rc) return rc;
        hipLaunchKernelGGL(roi_pool_invalid_fill_kernel, dim3(64), dim3(256), 0, st, w.list, w.cnt,
                           static_cast<int>(R), N, static_cast<size_t>(C) * PH * PW, out, argmax);
        FRCNN_LAUNCH_CHECK("roi_pool_invalid_fill_kernel");
        return FRCNN_OK;
    }
    if (ch.kind != kFwdGeneric)
        return fwd_tile_launch<false>(ch, x, rois, R, N, C, H, W, PH, PW, spatial_scale, out, argmax, HeadArgs{}, st);
    // generic path: one workgroup per RoI, gathers from L1/L2
    const size_t total = static_cast<size_t>(C) * PH * PW;
    const bool aligned = (reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                         (reinterpret_cast<uintptr_t>(argmax) % 16 == 0);
    if (total % 4 == 0 && aligned)
        hipLaunchKernelGGL(roi_pool_fwd_kernel<true>, dim3(static_cast<unsigned>(R)), dim3(256), 0,
                           st, x, rois, N, C, H, W, PH, PW, spatial_scale, out, argmax);
    else
        hipLaunchKernelGGL(roi_pool_fwd_kernel<false>, dim3(static_cast<unsigned>(R)), dim3(256), 0,
                           st, x, rois, N, C, H, W, PH, PW, spatial_scale, out, argmax);
    FRCNN_LAUNCH_CHECK("roi_pool_fwd_kernel");
    return FRCNN_OK;
}

// head != 0 names the launch of frcnn_roi_pool_fwd_head for 16-B aligned [R,4]
// rois (every torch allocation); unaligned rois take the transform + the
// head == 0 launch.
extern "C" int frcnn_roi_pool_fwd_kernel(int64_t R, int N, int C, int H, int W, int PH, int PW, int rois_sorted,
                                         int head, void* stream, char* name, size_t len) {
    FRCNN_REQUIRE(name && len > 0, "frcnn_roi_pool_fwd_kernel: null name");
    FRCNN_REQUIRE(R >= 0 && N >= 0 && C >= 0 && H >= 0 && W >= 0 && PH > 0 && PW > 0,
                  "frcnn_roi_pool_fwd_kernel: bad shape");
    const FwdChoice ch = choose_fwd(N, C, H, W, PH, PW, rois_sorted != 0, as_stream(stream));
    const int fx = PH == 7 && PW == 7 ? 7 : 0;
    // head == 2 (unaligned rois): frcnn_roi_pool_fwd_head transforms and then runs the
    // plain forward, like the dense-list / generic choices below
    const char* hb = head == 1 ? "true" : "false";
    int n = 0;
    switch (ch.kind) {
        case kFwdWave:
            if (ch.px.kps)  // kps implies the 7x7 head (px_plan)
                n = snprintf(name, len, "roi_pool_fwd_wave_kernel<1024, %d, %d, %s, %s, %d>", ch.px.cg, fx, hb,
                             path_cfg().roi_store ? "true" : "false", kFixPx * 16);
            else
                n = snprintf(name, len, "roi_pool_fwd_wave_kernel<1024, %d, %d, %s%s>", ch.px.cg, fx, hb,
                             path_cfg().roi_store ? ", true" : "");
            break;
        case kFwdDense:
            n = snprintf(name, len, "roi_pool_fwd_dense_kernel<1024, %d, %d, %s, false>", ch.dn.cg, fx, hb);
            break;
        case kFwdDenseList:
            n = snprintf(name, len, "roi_pool_fwd_dense_kernel<1024, %d, %d, false, true>", ch.dn.cg, fx);
            break;
        default:
            n = snprintf(name, len, "roi_pool_fwd_kernel<%s>",
                         (static_cast<size_t>(C) * PH * PW) % 4 == 0 ? "true" : "false");
    }
    return n < 0 ? FRCNN_EINVAL : FRCNN_OK;
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
    const bool aligned = reinterpret_cast<uintptr_t>(rois) % 16 == 0;
    const FwdChoice ch = choose_fwd(N, C, H, W, PH, PW, rois_sorted != 0, as_stream(stream));
    if (!aligned || ch.kind == kFwdDenseList || ch.kind == kFwdGeneric) {
        int rc = frcnn_roi_transform(rois, roi_inds, R, img_h, img_w, H, W, boxes, stream);
        if (rc != FRCNN_OK) return rc;
        if (C == 0) return FRCNN_OK;
        return frcnn_roi_pool_fwd(x, boxes, R, N, C, H, W, PH, PW, spatial_scale, rois_sorted, out,
                                  argmax, workspace, ws_bytes, stream);
    }
    // transform + pack inside the pool kernel
    FRCNN_REQUIRE(x && out && argmax, "frcnn_roi_pool_fwd_head: null pointer");
    const HeadArgs hd{roi_inds, img_h, img_w, static_cast<float>(H), static_cast<float>(W), boxes};
    return fwd_tile_launch<true>(ch, x, rois, R, N, C, H, W, PH, PW, spatial_scale, out, argmax, hd,
                                 as_stream(stream));
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
    w.list = c.take<int>(static_cast<size_t>(N + 1) * list_stride(R));
    w.cnt = c.take<int>(N + 1);
    w.bytes = c.used();
    return w;
}
constexpr size_t kPlaneBudget = 64 * 1024;       // LDS per workgroup for planes (plain kernel)
constexpr int kBwdRing = 8;                      // RoIs in flight per wave (ring kernel)
// RoIs per step of the leader kernel (4: 90.5-91.5 us for the cfg5 op vs 93.1-94.1 at 6,
// 140 at 8; -DFRCNN_BWD_LEAD_D for A/Bs)
#ifndef FRCNN_BWD_LEAD_D
#define FRCNN_BWD_LEAD_D 4
#endif
constexpr int kBwdLead = FRCNN_BWD_LEAD_D;                   // RoIs per step (leader kernel)
constexpr size_t kPlaneBudgetRing = 144 * 1024;  // ring kernel: one workgroup per CU
}  // namespace

extern "C" size_t frcnn_roi_pool_bwd_workspace_size(int64_t R, int N, int PH, int PW) {
    if (R < 0 || N < 0 || PH <= 0 || PW <= 0) return 0;
    return carve_bwd(nullptr, R, N, PH, PW).bytes;
}

namespace {
// Launch plan of the backward (shared by frcnn_roi_pool_bwd and the name query).
// Every wave owns one (image, channel) plane and walks all of the image's RoIs,
// so the work per wave is fixed: spread the N*C waves evenly, one workgroup per
// CU (ceil(N*C / CUs) waves each) where the LDS allows -- a 2:1 mix of busy and
// half-idle CUs cost 1.35x.
struct BwdPlan {
    bool ring = false, lead = false;
    int icpw = 1, HWs = 0;
    size_t lead_bytes = 0;
};
BwdPlan bwd_plan(int64_t R, int N, int C, int H, int W, int PH, int PW) {
    BwdPlan pl;
    const size_t HW = static_cast<size_t>(H) * W;
    const size_t plane_bytes = HW * sizeof(float);
    const int PHW = PH * PW;
    const int bp = path_cfg().roi_bwd;
    pl.ring = PHW <= 64 && bp != kPathPlain && plane_bytes <= kPlaneBudgetRing && plane_bytes > 0;
    if (pl.ring) {
        const int64_t waves = static_cast<int64_t>(N) * C;
        int64_t cpw = (waves + device_cu_count() - 1) / device_cu_count();
        const int64_t lds_cap = static_cast<int64_t>(kPlaneBudgetRing / plane_bytes);
        cpw = cpw > 16 ? 16 : cpw;
        cpw = cpw > lds_cap ? lds_cap : cpw;
        cpw = cpw > C ? C : cpw;
        cpw = cpw < 1 ? 1 : cpw;
        pl.icpw = static_cast<int>(cpw);
        const bool fits = static_cast<uint64_t>(R) * C * PHW * 4 < (1ull << 31);
        pl.HWs = static_cast<int>((HW + 64 + 3) & ~static_cast<size_t>(3));  // + dummy words
        pl.lead_bytes = static_cast<size_t>(pl.icpw) * (pl.HWs * sizeof(float) + 2 * kBwdXRow * 8);
        pl.lead = fits && bp == kPathAuto && PHW < 64 && PW == 7 && pl.lead_bytes <= kPlaneBudgetRing;
    }
    return pl;
}
}  // namespace

extern "C" int frcnn_roi_pool_bwd_kernel(int64_t R, int N, int C, int H, int W, int PH, int PW, char* name,
                                         size_t len) {
    FRCNN_REQUIRE(name && len > 0, "frcnn_roi_pool_bwd_kernel: null name");
    FRCNN_REQUIRE(R >= 0 && N >= 0 && C >= 0 && H >= 0 && W >= 0 && PH > 0 && PW > 0,
                  "frcnn_roi_pool_bwd_kernel: bad shape");
    const BwdPlan pl = bwd_plan(R, N, C, H, W, PH, PW);
    const size_t plane_bytes = static_cast<size_t>(H) * W * sizeof(float);
    int n;
    if (pl.lead)
        n = snprintf(name, len, "roi_pool_bwd_lead_kernel<%d, 7, %d>", kBwdLead, PH == 7 ? 7 : 0);
    else if (pl.ring)
        n = snprintf(name, len, "roi_pool_bwd_pf_kernel<%d>", kBwdRing);
    else
        n = snprintf(name, len, "roi_pool_bwd_kernel<%s>", plane_bytes <= kPlaneBudget ? "true" : "false");
    return n < 0 ? FRCNN_EINVAL : FRCNN_OK;
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
    const BwdPlan pl = bwd_plan(R, N, C, H, W, PH, PW);
    const int PHW = PH * PW;
    const size_t plane_bytes = HW * sizeof(float);
    const bool ring = pl.ring, lead = pl.lead;
    const int icpw = pl.icpw, HWs = pl.HWs;
    const size_t lead_bytes = pl.lead_bytes;
    if (lead) {  // lists only (entries flagged from the geometry): the flagged RoIs need no overlap masks
        const unsigned grid = static_cast<unsigned>(N + 1);
        hipLaunchKernelGGL(roi_bwd_prep_lists_kernel, dim3(grid), dim3(1024), 0, st, rois, static_cast<int>(R), N, H,
                           W, PH, PW, spatial_scale, w.cmask, w.code, w.list, w.cnt);
        FRCNN_LAUNCH_CHECK("roi_bwd_prep_lists_kernel");
    } else {
        if (PHW <= 64)
            hipLaunchKernelGGL(roi_bwd_prep64_kernel, dim3(static_cast<unsigned>((R + 3) / 4)), dim3(256), 0, st,
                               rois, static_cast<int>(R), H, W, PH, PW, spatial_scale, w.cmask, w.code);
        else
            hipLaunchKernelGGL(roi_bwd_prep_kernel, dim3(static_cast<unsigned>(R)), dim3(256), 0, st, rois,
                               H, W, PH, PW, spatial_scale, w.cmask, w.code);
        FRCNN_LAUNCH_CHECK("roi_bwd_prep_kernel");
        hipLaunchKernelGGL(roi_lists_kernel, dim3(N + 1), dim3(1024), 0, st, rois, static_cast<int>(R), N, w.list,
                           w.cnt, 5, nullptr, PHW);
        FRCNN_LAUNCH_CHECK("roi_lists_kernel");
    }
    if (ring) {
        dim3 grid((C + icpw - 1) / icpw, N);
        if (lead)
        {
            if (PH == 7)
                hipLaunchKernelGGL((roi_pool_bwd_lead_kernel<kBwdLead, 7, 7>), grid, dim3(64 * icpw), lead_bytes,
                                   st, grad, argmax, w.list, w.cnt, static_cast<int>(R), C, static_cast<int>(HW),
                                   HWs, PH, icpw, grad_in);
            else
                hipLaunchKernelGGL((roi_pool_bwd_lead_kernel<kBwdLead, 7, 0>), grid, dim3(64 * icpw), lead_bytes,
                                   st, grad, argmax, w.list, w.cnt, static_cast<int>(R), C, static_cast<int>(HW),
                                   HWs, PH, icpw, grad_in);
        }
        else
            hipLaunchKernelGGL(roi_pool_bwd_pf_kernel<kBwdRing>, grid, dim3(64 * icpw), icpw * plane_bytes, st,
                               grad, argmax, w.cmask, w.code, w.list, w.cnt, static_cast<int>(R), C,
                               static_cast<int>(HW), PHW, PW, icpw, grad_in);
    } else if (plane_bytes <= kPlaneBudget) {
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
