// Anchor generation and box decode (utils/anchors.py, utils/utils.py:47-73).
//
// HBM-bound elementwise work: one float4 per lane in and out, 256-thread
// blocks, no LDS.  Arithmetic order matches the reference op by op (the
// library is compiled with -ffp-contract=off, so no FMA contraction).
#include "common.h"

namespace frcnn {

struct AnchorCfg {
    double ratios[16];
    double scales[16];
    int n_ratios;
    int n_scales;
    double base_size;
};

// utils/anchors.py:17-29: h = base*scale*sqrt(r), w = base*scale*sqrt(1/r) in
// fp64, rows r*n_scales+s = fp32([-h/2, -w/2, h/2, w/2]).
__global__ void anchor_base_kernel(AnchorCfg cfg, float4* __restrict__ out) {
    int t = threadIdx.x;
    if (t >= cfg.n_ratios * cfg.n_scales) return;
    int r = t / cfg.n_scales, s = t % cfg.n_scales;
    double side = cfg.base_size * cfg.scales[s];
    double h = side * sqrt(cfg.ratios[r]);
    double w = side * sqrt(1.0 / cfg.ratios[r]);
    out[t] = make_float4(static_cast<float>(-(h / 2)), static_cast<float>(-(w / 2)),
                         static_cast<float>(h / 2), static_cast<float>(w / 2));
}

// utils/anchors.py:46-59: row ((y*W)+x)*K+k = base[k] + [s*x, s*y, s*x, s*y]
// (x = WIDTH index into columns 0 and 2).  fp32 + exact integer = one rounding.
__global__ __launch_bounds__(256) void generate_anchors_kernel(const float4* __restrict__ base,
                                                               int K, int stride, int W,
                                                               int64_t total,
                                                               float4* __restrict__ out) {
    int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int k = static_cast<int>(i % K);
    int64_t cell = i / K;
    int x = static_cast<int>(cell % W);
    int y = static_cast<int>(cell / W);
    float sx = static_cast<float>(stride * x);
    float sy = static_cast<float>(stride * y);
    float4 b = base[k];
    out[i] = make_float4(b.x + sx, b.y + sy, b.z + sx, b.w + sy);
}

__global__ __launch_bounds__(256) void reg2bbox_kernel(const float4* __restrict__ anchors,
                                                       const float4* __restrict__ reg,
                                                       int64_t n, float4* __restrict__ out) {
    int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = decode_box(anchors[i], reg[i]);
}

}  // namespace frcnn

using namespace frcnn;

extern "C" int frcnn_anchor_base(const double* ratios, int n_ratios, const double* scales,
                                 int n_scales, double base_size, float* out_base, void* stream) {
    FRCNN_REQUIRE(ratios && scales && out_base, "frcnn_anchor_base: null pointer");
    FRCNN_REQUIRE(n_ratios > 0 && n_ratios <= 16 && n_scales > 0 && n_scales <= 16,
                  "frcnn_anchor_base: 1..16 ratios and scales supported");
    AnchorCfg cfg{};
    for (int i = 0; i < n_ratios; ++i) cfg.ratios[i] = ratios[i];
    for (int i = 0; i < n_scales; ++i) cfg.scales[i] = scales[i];
    cfg.n_ratios = n_ratios;
    cfg.n_scales = n_scales;
    cfg.base_size = base_size;
    hipLaunchKernelGGL(anchor_base_kernel, dim3(1), dim3(256), 0, as_stream(stream), cfg,
                       reinterpret_cast<float4*>(out_base));
    FRCNN_LAUNCH_CHECK("anchor_base_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_generate_anchors(const float* anchor_base, int K, int feat_stride, int width,
                                      int height, float* out, void* stream) {
    FRCNN_REQUIRE(anchor_base && out, "frcnn_generate_anchors: null pointer");
    FRCNN_REQUIRE(K > 0 && width >= 0 && height >= 0, "frcnn_generate_anchors: bad shape");
    int64_t total = static_cast<int64_t>(K) * width * height;
    if (total == 0) return FRCNN_OK;
    unsigned blocks = static_cast<unsigned>((total + 255) / 256);
    hipLaunchKernelGGL(generate_anchors_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(anchor_base), K, feat_stride, width, total,
                       reinterpret_cast<float4*>(out));
    FRCNN_LAUNCH_CHECK("generate_anchors_kernel");
    return FRCNN_OK;
}

extern "C" int frcnn_reg2bbox(const float* anchors, const float* reg, int64_t n, float* out,
                              void* stream) {
    FRCNN_REQUIRE(n >= 0, "frcnn_reg2bbox: n < 0");
    if (n == 0) return FRCNN_OK;
    FRCNN_REQUIRE(anchors && reg && out, "frcnn_reg2bbox: null pointer");
    unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(reg2bbox_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const float4*>(anchors),
                       reinterpret_cast<const float4*>(reg), n, reinterpret_cast<float4*>(out));
    FRCNN_LAUNCH_CHECK("reg2bbox_kernel");
    return FRCNN_OK;
}
