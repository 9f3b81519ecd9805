// RPN head epilogue (nets/rpn.py:117-124), SURVEY.md §8(f) row 1.
//
// The reference turns the two 1x1-conv outputs (NCHW) into the proposal
// layer's inputs with four separate passes: cls.permute(0,2,3,1).contiguous(),
// F.softmax(dim=-1), [:, :, 1].contiguous() and reg.permute(0,2,3,1).contiguous().
// Here ONE launch reads each conv output once and writes all three tensors:
//   cls_nhwc [N, A, 2]  (= the reference's cls before its final view-permute)
//   fg       [N, A]     (softmax of channel pair (2k, 2k+1), element 1)
//   reg_nhwc [N, A, 4]  (the proposal layer's deltas, and the loss's reg)
// with A = H*W*K and row (y*W + x)*K + k.
//
// HBM-bound transpose: a workgroup owns a 64-pixel strip of one image.  Reads
// are channel-major (64 consecutive pixels of one channel = one 256 B run per
// wave), staged through LDS, and the NHWC outputs are written as contiguous
// runs (the strip's rows of every output tensor are adjacent in memory), so
// both sides are fully coalesced.  Algorithmic bytes per image:
// 6K*H*W*4 read + 7K*H*W*4 written.
#include "common.h"

namespace frcnn {

constexpr int kEpiPix = 64;      // pixels per workgroup strip
constexpr int kEpiThreads = 256;

// torch CPU softmax over a last dim of 2 (ATen _vec_softmax_lastdim): m = max,
// e_i = exp(x_i - m), s = e_0 + e_1, out_i = e_i * (1 / s).  Every op is fp32
// and separately rounded (library built with -ffp-contract=off); exp is the
// correctly rounded one (torch's vectorised exp is host-dependent in its last
// bits, like the decode's).
__device__ __forceinline__ float fg_softmax(float a, float b) {
    float m = fmaxf(a, b);
    float ea = exp_cr(a - m);
    float eb = exp_cr(b - m);
    float inv = 1.0f / (ea + eb);
    return eb * inv;
}

__global__ __launch_bounds__(kEpiThreads) void rpn_head_epilogue_kernel(
    const float* __restrict__ cls, const float* __restrict__ reg, int K, int HW,
    float* __restrict__ cls_nhwc, float* __restrict__ fg, float* __restrict__ reg_nhwc) {
    extern __shared__ float epi_lds[];
    const int n = blockIdx.y;
    const int p0 = blockIdx.x * kEpiPix;
    const int cnt = min(kEpiPix, HW - p0);
    const int C2 = 2 * K, C4 = 4 * K;
    float* lc = epi_lds;                 // [kEpiPix][2K]
    float* lr = epi_lds + kEpiPix * C2;  // [kEpiPix][4K]
    const float* cn = cls + static_cast<int64_t>(n) * C2 * HW + p0;
    const float* rn = reg + static_cast<int64_t>(n) * C4 * HW + p0;

    for (int i = threadIdx.x; i < kEpiPix * C2; i += kEpiThreads) {
        int c = i / kEpiPix, p = i % kEpiPix;
        if (p < cnt) lc[p * C2 + c] = cn[static_cast<int64_t>(c) * HW + p];
    }
    for (int i = threadIdx.x; i < kEpiPix * C4; i += kEpiThreads) {
        int c = i / kEpiPix, p = i % kEpiPix;
        if (p < cnt) lr[p * C4 + c] = rn[static_cast<int64_t>(c) * HW + p];
    }
    __syncthreads();

    const int64_t row0 = static_cast<int64_t>(n) * HW + p0;  // first pixel of the strip
    float* oc = cls_nhwc + row0 * C2;
    for (int i = threadIdx.x; i < cnt * C2; i += kEpiThreads) oc[i] = lc[i];
    float* of = fg + row0 * K;
    for (int i = threadIdx.x; i < cnt * K; i += kEpiThreads) {
        int p = i / K, k = i - p * K;
        of[i] = fg_softmax(lc[p * C2 + 2 * k], lc[p * C2 + 2 * k + 1]);
    }
    float* orr = reg_nhwc + row0 * C4;
    for (int i = threadIdx.x; i < cnt * C4; i += kEpiThreads) orr[i] = lr[i];
}

}  // namespace frcnn

using namespace frcnn;

extern "C" int frcnn_rpn_head_epilogue(const float* cls, const float* reg, int N, int K,
                                       int feat_h, int feat_w, float* cls_nhwc, float* fg,
                                       float* reg_nhwc, void* stream) {
    FRCNN_REQUIRE(N >= 0 && K > 0 && K <= 32 && feat_h >= 0 && feat_w >= 0,
                  "frcnn_rpn_head_epilogue: bad shape (need N >= 0, 1 <= K <= 32)");
    const int64_t hw = static_cast<int64_t>(feat_h) * feat_w;
    if (N == 0 || hw == 0) return FRCNN_OK;
    FRCNN_REQUIRE(hw <= (int64_t(1) << 30) && N <= 65535, "frcnn_rpn_head_epilogue: too large");
    FRCNN_REQUIRE(cls && reg && cls_nhwc && fg && reg_nhwc, "frcnn_rpn_head_epilogue: null pointer");
    const int HW = static_cast<int>(hw);
    const size_t lds = static_cast<size_t>(kEpiPix) * 6 * K * sizeof(float);  // <= 48 KB
    dim3 grid(static_cast<unsigned>((HW + kEpiPix - 1) / kEpiPix), static_cast<unsigned>(N));
    hipLaunchKernelGGL(rpn_head_epilogue_kernel, grid, dim3(kEpiThreads), lds, as_stream(stream),
                       cls, reg, K, HW, cls_nhwc, fg, reg_nhwc);
    FRCNN_LAUNCH_CHECK("rpn_head_epilogue_kernel");
    return FRCNN_OK;
}
