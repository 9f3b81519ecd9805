/*
 * frcnn_capi.h -- C-ABI of the MI355X-native region-proposal + RoI hot path.
 *
 * This is the drop-in boundary.  Every entry point:
 *   - is extern "C", takes plain pointers / sizes, no torch types;
 *   - takes caller-owned DEVICE buffers (unless a parameter says "host");
 *   - is stream-ordered and asynchronous on `stream` (a hipStream_t, passed
 *     as void*; NULL = the default stream), never synchronises, never
 *     allocates (workspace comes from the caller, sized by the matching
 *     *_workspace_size() query), so a sequence of calls can be captured in a
 *     hipGraph;
 *   - returns 0 on success or a negative FRCNN_E* code, never throws across
 *     the ABI; frcnn_last_error() returns a message for the calling thread.
 *
 * Each function cites the reference interface it replaces (file:line in
 * juniorliu95/replication_faster_rcnn, or the torchvision op the reference
 * calls at that line).  Numerics: see DESIGN.md "Parity contract".
 */
#ifndef FRCNN_CAPI_H_
#define FRCNN_CAPI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRCNN_OK 0
#define FRCNN_EINVAL (-1)     /* bad shape / argument */
#define FRCNN_EHIP (-2)       /* HIP runtime error (launch failure) */
#define FRCNN_EWORKSPACE (-3) /* workspace too small */

const char* frcnn_version(void);
const char* frcnn_last_error(void);

/* Runtime helpers (no reference counterpart: the reference runs one image at
 * a time on the host).  CU count of the current device (sizes the grids). */
int frcnn_device_cu_count(int* out);

/* Streams on a CU subset (hipExtStreamCreateWithCUMask: bit i of word i/32 =
 * CU i; words = 0 -> an ordinary non-blocking stream).  The proposal chain is
 * latency bound on a few workgroups while the RoIPool forward holds every CU's
 * LDS for its whole run; giving each its own CUs lets them overlap.  The
 * RoIPool forward sizes its RoI shares to the CUs of the stream it is launched on.
 * frcnn_stream_cu_count: CUs a launch on `stream` may use.
 * frcnn_probe_hw_ids: diagnostic -- out[2b] = HW_ID, out[2b+1] = XCC_ID of
 * workgroup b of an nblocks launch (spin: s_sleep rounds that keep it resident). */
int frcnn_stream_create(const uint32_t* cu_mask, int words, void** out);
int frcnn_stream_destroy(void* stream);
int frcnn_stream_cu_count(void* stream, int* out);
int frcnn_probe_hw_ids(uint32_t* out, int nblocks, int spin, void* stream);

/* Kernel-path selection, process-global (tests and A/B tools; the default
 * "auto" is what every caller should use).  op / path:
 *   "roi_pool_fwd"   : "auto" | "wave" (plane-major image tile in LDS, compare-and-select scan,
 *                      one wave per RoI; RoIs grouped by image; the auto choice) | "dense" (image
 *                      tile, bins packed 64 per wave; any RoI order) | "generic" (one
 *                      workgroup per RoI)
 *   "roi_pool_bwd"   : "auto" (leader-gather plane owner for 7-wide outputs, else ring) | "ring" (latency-hidden plane owner) | "plain"
 *   "propose"        : "auto" | "hybrid" | "lazy" (fused per image) | "wide" (chip-wide bitmask)
 *   "roi_pool_split" : "auto" | "1".."64" (RoI shares per image and channel group)
 *   "roi_pool_cg"    : "auto" | "4" | "8" | "16" (channels per RoIPool forward workgroup)
 *   "roi_pool_fwd_store": "auto" = "temporal" | "nt" (the wave forward's output stores
 *                      non-temporal: better beside concurrent kernels at cfg2, worse alone)
 *   "sampler"        : "auto" = "chip" (the stream cut into 1024-word segments, each one's
 *                      map of entering to leaving step count tabulated chip-wide and
 *                      chained; the walk below runs instead when a step count leaves
 *                      its planned range, or for > 128 images) | "walk" (one workgroup
 *                      walks the MT19937 stream) | "chip_only" (no walk behind it) |
 *                      "chip_tight" (zero-margin ranges: exercises the walk behind it);
 *                      the target creators' _draw / _sample entry points
 * All paths give bit-identical results.  Not thread-safe against calls in
 * flight on other threads; set it before launching. */
int frcnn_set_path(const char* op, const char* path);

/* ---------------------------------------------------------------- anchors */

/* utils/anchors.py:5 generate_anchor_base(base_size, ratios, anchor_scales).
 * ratios / scales are HOST arrays (n_ratios*n_scales <= 64).  out_base: device
 * fp32 [n_ratios*n_scales, 4], row r*n_scales+s. */
int frcnn_anchor_base(const double* ratios, int n_ratios, const double* scales, int n_scales,
                      double base_size, float* out_base, void* stream);

/* utils/anchors.py:33 generate_anchors(anchor_base, feat_stride, width, height).
 * anchor_base fp32 [K,4]; out fp32 [height*width*K, 4]. */
int frcnn_generate_anchors(const float* anchor_base, int K, int feat_stride, int width,
                           int height, float* out, void* stream);

/* utils/utils.py:47 reg2bbox(anchors, reg): fp32 [n,4] x [n,4] -> [n,4]. */
int frcnn_reg2bbox(const float* anchors, const float* reg, int64_t n, float* out, void* stream);

/* nets/rpn.py:117-124 RPN head epilogue, one launch instead of the reference's
 * permute/contiguous/softmax/slice chain:
 *   cls fp32 [N, 2K, H, W] (self.cls conv output), reg fp32 [N, 4K, H, W]
 *   -> cls_nhwc fp32 [N, A, 2]  = cls.permute(0,2,3,1).contiguous().view(N,-1,2)  (:117-118)
 *      fg       fp32 [N, A]     = F.softmax(cls_nhwc, -1)[:, :, 1]              (:119)
 *      reg_nhwc fp32 [N, A, 4]  = reg.permute(0,2,3,1).contiguous().view(N,-1,4)  (:123-124)
 * A = H*W*K, 1 <= K <= 32.  fg feeds frcnn_propose's scores, reg_nhwc its deltas. */
int frcnn_rpn_head_epilogue(const float* cls, const float* reg, int N, int K, int feat_h,
                            int feat_w, float* cls_nhwc, float* fg, float* reg_nhwc,
                            void* stream);

/* ------------------------------------------------------------- proposals */

/* Parameters of the batched proposal layer (nets/rpn.py:22-45 kwargs). */
typedef struct frcnn_propose_params {
    int N;            /* images in the batch */
    int A;            /* anchors per image */
    int K;            /* anchors per location (used when anchors == NULL) */
    int feat_h;       /* feature map height   (used when anchors == NULL) */
    int feat_w;       /* feature map width    (used when anchors == NULL) */
    int feat_stride;  /* 16                   (used when anchors == NULL) */
    float img_h;      /* clamp bound of box columns 0,2 (nets/rpn.py:62) */
    float img_w;      /* clamp bound of box columns 1,3 (nets/rpn.py:63) */
    float min_size;   /* nets/rpn.py:27,65 */
    int pre_nms;      /* nets/rpn.py:39-43 */
    int post_nms;     /* nets/rpn.py:40-43 */
    double iou_threshold; /* nets/rpn.py:44 */
} frcnn_propose_params;

size_t frcnn_propose_workspace_size(const frcnn_propose_params* p);

/* nets/rpn.py:47-79 region_proposal.__call__, batched over N images
 * (replaces the per-image loop nets/rpn.py:131-136).
 *   scores  fp32 [N, A]     fg softmax (nets/rpn.py:119)
 *   deltas  fp32 [N, A, 4]  RPN reg    (nets/rpn.py:124)
 *   anchors fp32 [A, 4] or NULL; if NULL, anchors are generated in-kernel from
 *           anchor_base fp32 [K,4] on the feat_h x feat_w grid (A = feat_h*feat_w*K)
 * Outputs (padded to post_nms):
 *   out_rois  fp32 [N, post_nms, 4]   rows >= out_count[n] are zero
 *   out_idx   int32 [N, post_nms]     anchor index of each roi, -1 padding
 *   out_count int32 [N]               min(post_nms, #kept by NMS) */
int frcnn_propose(const frcnn_propose_params* p, const float* scores, const float* deltas,
                  const float* anchors, const float* anchor_base, float* out_rois,
                  int32_t* out_idx, int32_t* out_count, void* workspace, size_t ws_bytes,
                  void* stream);

/* torchvision.ops.nms(boxes, scores, iou_threshold) as called at nets/rpn.py:75.
 *   boxes fp32 [n,4] (x1,y1,x2,y2), scores fp32 [n]
 *   keep int64 [n]: kept indices in descending-score order; *count (device
 *   int32) = number kept. */
size_t frcnn_nms_workspace_size(int64_t n);
int frcnn_nms(const float* boxes, const float* scores, int64_t n, double iou_threshold,
              int64_t* keep, int32_t* count, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- RoIPool */

/* nets/heads.py:42-47: image-space rois fp32 [R,4] + roi_inds fp32 [R] ->
 * boxes fp32 [R,5] = [idx, r0/img_h*feat_h, r1/img_w*feat_w, r2/img_h*feat_h,
 * r3/img_w*feat_w]. */
int frcnn_roi_transform(const float* rois, const float* roi_inds, int64_t R, float img_h,
                        float img_w, int feat_h, int feat_w, float* boxes, void* stream);

/* torchvision.ops.roi_pool forward (nets/heads.py:48):
 *   x fp32 [N,C,H,W], rois fp32 [R,5] -> out fp32 [R,C,PH,PW],
 *   argmax int32 [R,C,PH,PW] (h*W+w within the plane, -1 for empty bins).
 * RoIs whose batch index is outside [0,N) produce 0 / -1.
 * rois_sorted != 0 PROMISES the RoIs are grouped by non-decreasing batch
 * index (true for proposals and for train.py's sample_rois_ind): one launch,
 * each workgroup finds its image's RoI range itself.  rois_sorted == 0 works
 * for any order (a list kernel groups them first).
 * The workspace (frcnn_roi_pool_fwd_workspace_size bytes) is always required. */
size_t frcnn_roi_pool_fwd_workspace_size(int64_t R, int N, int C);
int frcnn_roi_pool_fwd(const float* x, const float* rois, int64_t R, int N, int C, int H, int W,
                       int PH, int PW, float spatial_scale, int rois_sorted, float* out,
                       int32_t* argmax, void* workspace, size_t ws_bytes, void* stream);

/* ResnetHead.forward's RoI transform + pack + roi_pool (nets/heads.py:42-48)
 * in one call: rois fp32 [R,4] in image pixels (RPN output / sample_rois),
 * roi_inds fp32 [R] -> boxes fp32 [R,5] exactly as frcnn_roi_transform, and
 * out / argmax exactly as frcnn_roi_pool_fwd on those boxes.  With
 * rois_sorted != 0 (same promise as above) the transform runs inside the pool
 * kernel (one launch); otherwise the two calls run back to back.  boxes is
 * always written (the backward needs it).  Workspace: frcnn_roi_pool_fwd_
 * workspace_size(R, N, C). */
int frcnn_roi_pool_fwd_head(const float* x, const float* rois, const float* roi_inds, int64_t R,
                            int N, int C, int H, int W, int PH, int PW, float img_h, float img_w,
                            float spatial_scale, int rois_sorted, float* boxes, float* out,
                            int32_t* argmax, void* workspace, size_t ws_bytes, void* stream);

/* The kernel frcnn_roi_pool_fwd_head (head == 1: 16-B aligned rois; head == 2:
 * an unaligned rois pointer, which the head entry point handles as transform +
 * the plain forward) or frcnn_roi_pool_fwd (head == 0) launches for this shape on
 * `stream` under the current frcnn_set_path choices, as its template name (e.g.
 * "roi_pool_fwd_wave_kernel<1024, 16, 7, true, false, 38400>"), NUL-terminated in name[len]:
 * the label bench.py and the rocprofv3 records key the dominant kernel on. */
int frcnn_roi_pool_fwd_kernel(int64_t R, int N, int C, int H, int W, int PH, int PW, int rois_sorted,
                              int head, void* stream, char* name, size_t len);

/* torchvision _roi_pool_backward (autograd of nets/heads.py:48, reached from
 * train.py:126):  grad_in fp32 [N,C,H,W] = 0, then for n, c, ph, pw in order
 * grad_in[b(n), c, argmax] += grad[n, c, ph, pw].  Deterministic, atomic-free,
 * same summation order as the CPU kernel. */
size_t frcnn_roi_pool_bwd_workspace_size(int64_t R, int N, int PH, int PW);
int frcnn_roi_pool_bwd(const float* grad, const float* rois, const int32_t* argmax, int64_t R,
                       int N, int C, int H, int W, int PH, int PW, float spatial_scale,
                       float* grad_in, void* workspace, size_t ws_bytes, void* stream);
/* The RoIPool backward kernel frcnn_roi_pool_bwd launches for this shape under
 * the current frcnn_set_path choice (e.g. "roi_pool_bwd_lead_kernel<4, 7, 7>"),
 * NUL-terminated in name[len] (bench.py's label for it; the per-image lists
 * launch before it is not named). */
int frcnn_roi_pool_bwd_kernel(int64_t R, int N, int C, int H, int W, int PH, int PW, char* name, size_t len);

/* --------------------------------------------------------- target creators */

/* utils/utils.py:102 bbox_iou(bbox_a, bbox_b) -> [na, nb], with numpy's dtype
 * promotion: a, b each fp32 or fp64 (flag); out fp32 if both fp32, else fp64. */
int frcnn_bbox_iou(const void* a, int a_is_f64, int64_t na, const void* b, int b_is_f64,
                   int64_t nb, void* out, void* stream);

/* utils/utils.py:75 bbox2reg(anchors, bbox) -> fp64 [n, 4] (anchor statistics in
 * the anchors' dtype, box statistics in the boxes' dtype, as numpy does). */
int frcnn_bbox2reg(const void* anchors, int a_is_f64, const void* bbox, int b_is_f64, int64_t n,
                   double* out, void* stream);

/* utils/utils.py:122-204 AnchorTargetCreator.__call__, batched over N images in
 * the order of train.py:71-79.
 *   anchors fp32 [A,4]; boxes fp64 [N,G,4] + labels fp64 [N,G] (rows with label
 *   -1 are padding, train.py:74-76; G <= 256)
 *   rng_state u32 [625] = numpy legacy MT19937 key[624] + pos, updated in place
 *   exactly as the reference's np.random.choice calls would; NULL = no sampling
 *   (labels before the disable step, no RNG use)
 * Outputs: reg fp64 [N,A,4] (zeros for an image without gt), label int32 [N,A],
 * optional argmax int32 [N,A] (after the gt override, utils/utils.py:171-172) and
 * max_iou fp64 [N,A]. */
size_t frcnn_anchor_target_workspace_size(int N, int A, int G);
int frcnn_anchor_target(int N, int A, int G, const float* anchors, const double* boxes,
                        const double* labels, int n_sample, double pos_iou_thresh,
                        double neg_iou_thresh, double pos_ratio, uint32_t* rng_state,
                        double* reg, int32_t* label, int32_t* argmax, double* max_iou,
                        void* workspace, size_t ws_bytes, void* stream);

/* frcnn_anchor_target in two halves on one workspace (frcnn_anchor_target =
 * prepare + sample on the same stream):
 *   prepare: gt compaction, anchor x gt IoU, labels and the ordered positive /
 *            negative lists (utils/utils.py:146-188) -- no RNG, so a training
 *            loop can run it ahead, on another stream, beside the previous
 *            step's draws;
 *   sample:  the np.random.choice draws on rng_state (utils/utils.py:190-202)
 *            and the regression targets; runs after prepare on the same
 *            workspace (order the streams with an event). */
int frcnn_anchor_target_prepare(int N, int A, int G, const float* anchors, const double* boxes,
                                const double* labels, double pos_iou_thresh, double neg_iou_thresh,
                                void* workspace, size_t ws_bytes, void* stream);
int frcnn_anchor_target_sample(int N, int A, int G, const float* anchors, int n_sample, double pos_ratio,
                               uint32_t* rng_state, double* reg, int32_t* label, int32_t* argmax,
                               double* max_iou, void* workspace, size_t ws_bytes, void* stream);
/* frcnn_anchor_target_sample in two steps on the same workspace (same arguments):
 * _draw the np.random.choice calls of utils/utils.py:190-202 (the RNG stream's only
 * kernel), _finish the final labels and bbox2reg targets of utils/utils.py:146-150,
 * 203-204 (any stream, after _draw: order the streams with an event). */
int frcnn_anchor_target_draw(int N, int A, int G, int n_sample, double pos_ratio, uint32_t* rng_state,
                             void* workspace, size_t ws_bytes, void* stream);
int frcnn_anchor_target_finish(int N, int A, int G, const float* anchors, double* reg, int32_t* label,
                               int32_t* argmax, double* max_iou, void* workspace, size_t ws_bytes,
                               void* stream);
/* The chip-wide draws' plan of the last _draw on this workspace (synchronous; a
 * diagnostic, no reference counterpart): out[9] = fail (0: the segment tables held;
 * 1: plan over the workspace's capacity; 2: a step count left its planned range --
 * the walk did the draws), calls with >= 1 step, steps, segments, groups, state
 * blocks, start pos, widest range, missed group (-1).  Returns 1 when the
 * workspace has no chip-wide part (> 128 images: the walk only). */
int frcnn_anchor_target_draw_status(int N, int A, int G, const void* workspace, size_t ws_bytes, int* out);

/* utils/utils.py:207-276 ProposalTargetCreator.__call__, batched over N images in
 * the order of train.py:91-104.
 *   rois fp32 [N,Rp,4] with rcount int32 [N] valid rows per image; boxes/labels as
 *   for frcnn_anchor_target; reg_mean / reg_std: HOST fp64 [4] (the fp32 values of
 *   utils/utils.py:272 widened); rng_state as above (required).
 * Outputs (padded to n_sample): sample_roi fp64 [N,n_sample,4], gt_roi_reg fp64
 * [N,n_sample,4], gt_roi_label fp64 [N,n_sample], sample_count int32 [N]. */
size_t frcnn_proposal_target_workspace_size(int N, int Rp, int G, int n_sample);
int frcnn_proposal_target(int N, int Rp, const float* rois, const int32_t* rcount, int G,
                          const double* boxes, const double* labels, int n_sample,
                          double pos_ratio, double pos_iou_thresh, double neg_iou_thresh_high,
                          double neg_iou_thresh_low, const double* reg_mean,
                          const double* reg_std, uint32_t* rng_state, double* sample_roi,
                          double* gt_roi_reg, double* gt_roi_label, int32_t* sample_count,
                          void* workspace, size_t ws_bytes, void* stream);
/* frcnn_proposal_target in two halves on one workspace (same arguments):
 *   _prepare: utils/utils.py:221-246 (gt concat, IoU, argmax, fg / bg lists) --
 *             no RNG, so it can run on the proposals' stream, off the draws' stream;
 *   _sample:  utils/utils.py:248-276 (the np.random.choice draws on rng_state,
 *             sample order, regression targets); runs after prepare on the same
 *             workspace (order the streams with an event). */
int frcnn_proposal_target_prepare(int N, int Rp, const float* rois, const int32_t* rcount, int G,
                                  const double* boxes, const double* labels, int n_sample,
                                  double pos_iou_thresh, double neg_iou_thresh_high,
                                  double neg_iou_thresh_low, void* workspace, size_t ws_bytes,
                                  void* stream);
int frcnn_proposal_target_sample(int N, int Rp, int G, int n_sample, double pos_ratio,
                                 const double* reg_mean, const double* reg_std, uint32_t* rng_state,
                                 double* sample_roi, double* gt_roi_reg, double* gt_roi_label,
                                 int32_t* sample_count, void* workspace, size_t ws_bytes, void* stream);
/* frcnn_proposal_target_sample in two steps on the same workspace: _draw the
 * np.random.choice calls of utils/utils.py:248-258 (sample order, sample_count),
 * _finish sample_roi / gt_roi_reg / gt_roi_label of utils/utils.py:260-276 (any
 * stream, after _draw). */
int frcnn_proposal_target_draw(int N, int Rp, int G, int n_sample, double pos_ratio, uint32_t* rng_state,
                               int32_t* sample_count, void* workspace, size_t ws_bytes, void* stream);
int frcnn_proposal_target_finish(int N, int Rp, int G, int n_sample, const double* reg_mean,
                                 const double* reg_std, const int32_t* sample_count, double* sample_roi,
                                 double* gt_roi_reg, double* gt_roi_label, void* workspace, size_t ws_bytes,
                                 void* stream);
/* frcnn_anchor_target_draw then frcnn_proposal_target_draw on one RNG stream, as
 * one pass (the order of train.py:71 / :91: every AnchorTarget draw, then every
 * ProposalTarget draw, for the same N images): both prepares must have run on
 * their workspaces (same arguments as the two _draw calls; the pass uses the
 * anchor workspace's chip-wide part, frcnn_anchor_target_draw_status reads it).
 * Bit-identical to the two calls in sequence. */
int frcnn_target_draws(int N, int A, int G_at, int n_sample_at, double pos_ratio_at, void* at_workspace,
                       size_t at_bytes, int Rp, int G_pt, int n_sample_pt, double pos_ratio_pt, void* pt_workspace,
                       size_t pt_bytes, int32_t* sample_count, uint32_t* rng_state, void* stream);
/* As frcnn_anchor_target_draw_status, for the last frcnn_proposal_target_draw. */
int frcnn_proposal_target_draw_status(int N, int Rp, int G, int n_sample, const void* workspace, size_t ws_bytes,
                                      int* out);

#ifdef __cplusplus
}
#endif

#endif /* FRCNN_CAPI_H_ */
