/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the two third-party CPU kernels that the reference
 * hot path calls but does not vendor (torchvision is absent from
 * /root/reference and from this image):
 *
 *   torchvision.ops.nms         called at nets/rpn.py:75
 *   torchvision.ops.roi_pool    called at nets/heads.py:48 (forward), and its
 *                               autograd backward reached from train.py:126
 *
 * The semantics follow torchvision's published CPU kernels
 * (csrc/ops/cpu/nms_kernel.cpp, csrc/ops/cpu/roi_pool_kernel.cpp) as spelled
 * out in SURVEY.md Appendix A.3/A.4.  torchvision's version is unpinned (no
 * requirements file in the reference), so these two ops are "parity
 * unpinned" against torchvision itself; the golden fixtures pin this
 * restatement as it is driven by the genuine reference Python code.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product path never links or calls it.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off: every fp32 op is a
 * separately rounded IEEE op, as in the x86-64 torchvision build).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Stable descending order of scores (torch sort(stable=true, descending=true)).
 * NaN sorts first in torch's descending order; we follow that. */
static int gt_desc(float a, float b) {
    int an = isnan(a), bn = isnan(b);
    if (an || bn) return an && !bn;
    return a > b;
}

static void merge_sort_desc(int64_t* idx, int64_t* tmp, const float* s, int64_t n) {
    /* bottom-up stable merge sort of idx by s descending */
    for (int64_t w = 1; w < n; w <<= 1) {
        for (int64_t lo = 0; lo < n; lo += 2 * w) {
            int64_t mid = lo + w < n ? lo + w : n;
            int64_t hi = lo + 2 * w < n ? lo + 2 * w : n;
            int64_t i = lo, j = mid, k = lo;
            while (i < mid && j < hi) {
                /* take right only if strictly "greater" => stable */
                if (gt_desc(s[idx[j]], s[idx[i]])) tmp[k++] = idx[j++];
                else tmp[k++] = idx[i++];
            }
            while (i < mid) tmp[k++] = idx[i++];
            while (j < hi) tmp[k++] = idx[j++];
        }
        memcpy(idx, tmp, (size_t)n * sizeof(int64_t));
    }
}

/* Greedy NMS.  boxes [n,4] (x1,y1,x2,y2), scores [n].
 * Writes kept indices (into the original array) to keep[], returns count. */
int64_t oracle_nms_f32(const float* boxes, const float* scores, int64_t n,
                       double iou_threshold, int64_t* keep) {
    if (n <= 0) return 0;
    int64_t* order = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* tmp = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    float* areas = (float*)malloc((size_t)n * sizeof(float));
    unsigned char* sup = (unsigned char*)calloc((size_t)n, 1);
    for (int64_t i = 0; i < n; ++i) {
        order[i] = i;
        const float* b = boxes + 4 * i;
        float dx = b[2] - b[0];
        float dy = b[3] - b[1];
        areas[i] = dx * dy;
    }
    merge_sort_desc(order, tmp, scores, n);
    int64_t nk = 0;
    for (int64_t oi = 0; oi < n; ++oi) {
        int64_t i = order[oi];
        if (sup[i]) continue;
        keep[nk++] = i;
        const float* bi = boxes + 4 * i;
        float ix1 = bi[0], iy1 = bi[1], ix2 = bi[2], iy2 = bi[3];
        float iarea = areas[i];
        for (int64_t oj = oi + 1; oj < n; ++oj) {
            int64_t j = order[oj];
            if (sup[j]) continue;
            const float* bj = boxes + 4 * j;
            float xx1 = ix1 < bj[0] ? bj[0] : ix1;   /* std::max(a,b) = a<b ? b : a */
            float yy1 = iy1 < bj[1] ? bj[1] : iy1;
            float xx2 = bj[2] < ix2 ? bj[2] : ix2;   /* std::min(a,b) = b<a ? b : a */
            float yy2 = bj[3] < iy2 ? bj[3] : iy2;
            float w = xx2 - xx1;
            float h = yy2 - yy1;
            w = 0.0f < w ? w : 0.0f;
            h = 0.0f < h ? h : 0.0f;
            float inter = w * h;
            float uni = iarea + areas[j];
            uni = uni - inter;
            float ovr = inter / uni;
            if ((double)ovr > iou_threshold) sup[j] = 1;
        }
    }
    free(order); free(tmp); free(areas); free(sup);
    return nk;
}

/* torchvision bin geometry for one RoI (App. A.4). */
static void roi_bins(const float* roi, float ss, int H, int W, int PH, int PW,
                     int ph, int pw, int* hs, int* he, int* ws, int* we) {
    int sw = (int)roundf(roi[1] * ss);
    int sh = (int)roundf(roi[2] * ss);
    int ew = (int)roundf(roi[3] * ss);
    int eh = (int)roundf(roi[4] * ss);
    int rw = ew - sw + 1; if (rw < 1) rw = 1;
    int rh = eh - sh + 1; if (rh < 1) rh = 1;
    float bh = (float)rh / (float)PH;
    float bw = (float)rw / (float)PW;
    int h0 = (int)floorf((float)ph * bh);
    int w0 = (int)floorf((float)pw * bw);
    int h1 = (int)ceilf((float)(ph + 1) * bh);
    int w1 = (int)ceilf((float)(pw + 1) * bw);
    h0 += sh; h1 += sh; w0 += sw; w1 += sw;
    h0 = h0 < 0 ? 0 : (h0 > H ? H : h0);
    h1 = h1 < 0 ? 0 : (h1 > H ? H : h1);
    w0 = w0 < 0 ? 0 : (w0 > W ? W : w0);
    w1 = w1 < 0 ? 0 : (w1 > W ? W : w1);
    *hs = h0; *he = h1; *ws = w0; *we = w1;
}

/* RoIPool forward.  x [N,C,H,W], rois [R,5] (b, x1, y1, x2, y2),
 * out / argmax [R,C,PH,PW]. */
void oracle_roi_pool_fwd_f32(const float* x, const float* rois, int64_t R, int C,
                             int H, int W, int PH, int PW, float ss,
                             float* out, int32_t* argmax) {
    for (int64_t n = 0; n < R; ++n) {
        const float* roi = rois + 5 * n;
        int b = (int)roi[0];
        for (int ph = 0; ph < PH; ++ph) {
            for (int pw = 0; pw < PW; ++pw) {
                int hs, he, ws, we;
                roi_bins(roi, ss, H, W, PH, PW, ph, pw, &hs, &he, &ws, &we);
                int empty = (he <= hs) || (we <= ws);
                for (int c = 0; c < C; ++c) {
                    float mv = empty ? 0.0f : -FLT_MAX;
                    int mi = -1;
                    const float* plane = x + ((int64_t)b * C + c) * (int64_t)H * W;
                    for (int h = hs; h < he; ++h)
                        for (int w = ws; w < we; ++w) {
                            int ii = h * W + w;
                            if (plane[ii] > mv) { mv = plane[ii]; mi = ii; }
                        }
                    int64_t o = ((n * C + c) * PH + ph) * PW + pw;
                    out[o] = mv;
                    argmax[o] = mi;
                }
            }
        }
    }
}

/* RoIPool backward: grad_in [N,C,H,W] zeroed, then for n, c, ph, pw in order
 * grad_in[b, c, argmax] += grad[n, c, ph, pw]. */
void oracle_roi_pool_bwd_f32(const float* grad, const float* rois, const int32_t* argmax,
                             int64_t R, int N, int C, int H, int W, int PH, int PW,
                             float* grad_in) {
    memset(grad_in, 0, sizeof(float) * (size_t)N * C * H * W);
    for (int64_t n = 0; n < R; ++n) {
        int b = (int)rois[5 * n];
        for (int c = 0; c < C; ++c) {
            float* plane = grad_in + ((int64_t)b * C + c) * (int64_t)H * W;
            const int64_t base = (n * C + c) * (int64_t)PH * PW;
            for (int k = 0; k < PH * PW; ++k) {
                int am = argmax[base + k];
                if (am != -1) plane[am] += grad[base + k];
            }
        }
    }
}
