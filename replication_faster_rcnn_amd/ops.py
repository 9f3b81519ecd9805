"""torchvision-surface ops the reference calls, on the HIP path.

* ``nms(boxes, scores, iou_threshold)`` -- ``torchvision.ops.nms`` as called at
  nets/rpn.py:75 (imported nets/rpn.py:4, utils/utils.py:4).
* ``roi_pool(input, boxes, output_size, spatial_scale)`` -- ``torchvision.ops.
  roi_pool`` as called at nets/heads.py:48, with an autograd backward (the
  reference reaches torchvision's ``_roi_pool_backward`` from
  ``total_loss.backward()`` at train.py:126).
* ``propose(...)`` -- the batched proposal layer (nets/rpn.py:47-79 over all
  images at once, replacing the per-image loop nets/rpn.py:131-136).

Inputs may live on the CPU (reference style); they are moved to the current
HIP device, and results are returned on the input's device.  Errors follow
torchvision's ``TORCH_CHECK`` -> ``RuntimeError`` convention.
"""
from __future__ import annotations

from typing import List, Tuple, Union

import torch

from . import _lib


def _to_dev(t: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    # the device-resident fast path: already on the device the kernels launch on
    if t.is_cuda and t.dtype == dtype and t.is_contiguous() and t.device.index == _lib._cur_device():
        return t
    return t.to(device=_lib.device(), dtype=dtype).contiguous()


# ----------------------------------------------------------------------- nms
def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float) -> torch.Tensor:
    """torchvision.ops.nms: int64 indices of kept boxes, by decreasing score."""
    lib = _lib.load()
    if boxes.dim() != 2 or boxes.size(1) != 4:
        raise RuntimeError(f"boxes should have 2 dimensions with 4 columns, got {tuple(boxes.shape)}")
    if scores.dim() != 1 or scores.size(0) != boxes.size(0):
        raise RuntimeError("boxes and scores should have the same number of elements in dim 0")
    out_dev = boxes.device
    b = _to_dev(boxes)
    s = _to_dev(scores)
    n = b.size(0)
    keep = torch.empty(max(n, 1), dtype=torch.int64, device=b.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=b.device)
    ws = _lib.workspace(lib.frcnn_nms_workspace_size(n), b.device)
    _lib.check(lib.frcnn_nms(_lib.ptr(b), _lib.ptr(s), n, float(iou_threshold), _lib.ptr(keep),
                             _lib.ptr(cnt), _lib.ptr(ws), ws.numel(), _lib.stream_ptr()), "nms")
    k = int(cnt.item())
    return keep[:k].to(out_dev)


# ------------------------------------------------------------------ roi_pool
def _roi_pool_fwd(x: torch.Tensor, rois: torch.Tensor, ph: int, pw: int, ss: float,
                  rois_sorted: bool = False):
    lib = _lib.load()
    N, C, H, W = x.shape
    R = rois.size(0)
    out = torch.empty((R, C, ph, pw), dtype=torch.float32, device=x.device)
    am = torch.empty((R, C, ph, pw), dtype=torch.int32, device=x.device)
    ws = _lib.cached_workspace("roi_pool_fwd", lib.frcnn_roi_pool_fwd_workspace_size(R, N, C), x.device)
    _lib.check(lib.frcnn_roi_pool_fwd(_lib.ptr(x), _lib.ptr(rois), R, N, C, H, W, ph, pw, float(ss),
                                      int(bool(rois_sorted)), _lib.ptr(out), _lib.ptr(am),
                                      _lib.ptr(ws), ws.numel(), _lib.stream_ptr()), "roi_pool forward")
    return out, am


def _sorted_by_image(boxes) -> bool:
    """Host-side check when the RoIs live on the host (the reference's case);
    device RoIs are treated as unsorted unless the caller says otherwise."""
    if isinstance(boxes, torch.Tensor) and boxes.is_cuda:
        return False
    b = (boxes.detach() if isinstance(boxes, torch.Tensor) else torch.as_tensor(boxes))[:, 0]
    bi = b.to(torch.int64)
    return bool((bi[1:] >= bi[:-1]).all()) if bi.numel() > 1 else True


def _roi_pool_bwd(grad: torch.Tensor, rois: torch.Tensor, am: torch.Tensor, shape, ss: float):
    lib = _lib.load()
    N, C, H, W = shape
    R, _, ph, pw = grad.shape
    gi = torch.empty((N, C, H, W), dtype=torch.float32, device=grad.device)
    ws = _lib.cached_workspace("roi_pool_bwd", lib.frcnn_roi_pool_bwd_workspace_size(R, N, ph, pw),
                               grad.device)
    _lib.check(lib.frcnn_roi_pool_bwd(_lib.ptr(grad), _lib.ptr(rois), _lib.ptr(am), R, N, C, H, W,
                                      ph, pw, float(ss), _lib.ptr(gi), _lib.ptr(ws), ws.numel(),
                                      _lib.stream_ptr()), "roi_pool backward")
    return gi


class _RoIPoolFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rois, ph, pw, ss, rois_sorted=False):
        out, am = _roi_pool_fwd(x, rois, ph, pw, ss, rois_sorted)
        ctx.save_for_backward(rois, am)
        ctx.meta = (tuple(x.shape), ss)
        ctx.mark_non_differentiable(am)
        return out, am

    @staticmethod
    def backward(ctx, grad_out, _grad_am):
        rois, am = ctx.saved_tensors
        shape, ss = ctx.meta
        gi = _roi_pool_bwd(grad_out.contiguous().float(), rois, am, shape, ss)
        return gi, None, None, None, None, None


def _roi_pool_head_fwd(x, rois, roi_inds, ph, pw, img_h, img_w, ss, rois_sorted, outs=None):
    lib = _lib.load()
    N, C, H, W = x.shape
    R = rois.size(0)
    if outs is None:
        boxes = torch.empty((R, 5), dtype=torch.float32, device=x.device)
        out = torch.empty((R, C, ph, pw), dtype=torch.float32, device=x.device)
        am = torch.empty((R, C, ph, pw), dtype=torch.int32, device=x.device)
    else:  # caller-owned (out, argmax, boxes): no allocation on the issue path
        out, am, boxes = outs
        if (tuple(out.shape) != (R, C, ph, pw) or tuple(am.shape) != (R, C, ph, pw)
                or tuple(boxes.shape) != (R, 5) or out.dtype != torch.float32
                or am.dtype != torch.int32 or boxes.dtype != torch.float32):
            raise RuntimeError("roi_pool_head: out buffers must be fp32 [R,C,ph,pw], int32 [R,C,ph,pw], "
                               "fp32 [R,5]")
    ws = _lib.cached_workspace("roi_pool_fwd", lib.frcnn_roi_pool_fwd_workspace_size(R, N, C), x.device)
    _lib.check(lib.frcnn_roi_pool_fwd_head(
        _lib.ptr(x), _lib.ptr(rois), _lib.ptr(roi_inds), R, N, C, H, W, ph, pw, float(img_h),
        float(img_w), float(ss), int(bool(rois_sorted)), _lib.ptr(boxes), _lib.ptr(out),
        _lib.ptr(am), _lib.ptr(ws), ws.numel(), _lib.stream_ptr()), "roi_pool_head forward")
    return out, am, boxes


class _RoIPoolHeadFunction(torch.autograd.Function):
    """nets/heads.py:42-48 (RoI transform + pack + roi_pool) as one op; the
    backward is roi_pool's, on the [R,5] boxes the forward wrote."""

    @staticmethod
    def forward(ctx, x, rois, roi_inds, ph, pw, img_h, img_w, ss, rois_sorted):
        out, am, boxes = _roi_pool_head_fwd(x, rois, roi_inds, ph, pw, img_h, img_w, ss, rois_sorted)
        ctx.save_for_backward(boxes, am)
        ctx.meta = (tuple(x.shape), ss)
        ctx.mark_non_differentiable(am, boxes)
        return out, am, boxes

    @staticmethod
    def backward(ctx, grad_out, _grad_am, _grad_boxes):
        boxes, am = ctx.saved_tensors
        shape, ss = ctx.meta
        gi = _roi_pool_bwd(grad_out.contiguous().float(), boxes, am, shape, ss)
        return gi, None, None, None, None, None, None, None, None


def roi_pool_head(input: torch.Tensor, rois: torch.Tensor, roi_inds: torch.Tensor, output_size,
                  img_h, img_w, spatial_scale: float = 1.0, rois_sorted: bool = False, out=None):
    """ResnetHead's RoI transform + ``[idx, box]`` pack + roi_pool
    (nets/heads.py:42-48) in one call on device tensors: rois fp32 [R,4] in
    image pixels, roi_inds [R] -> (out [R,C,ph,pw], argmax int32, boxes [R,5]).
    ``rois_sorted`` promises RoIs grouped by non-decreasing image index (RPN
    proposals, train.py's sample_rois): then the transform runs inside the
    pool kernel.  ``out`` = caller-owned (out, argmax, boxes) buffers
    (inference only)."""
    if input.dim() != 4:
        raise RuntimeError("input must be [N, C, H, W]")
    if rois.dim() != 2 or rois.size(1) != 4 or roi_inds.dim() != 1 or roi_inds.size(0) != rois.size(0):
        raise RuntimeError(f"rois must be [R, 4] and roi_inds [R]; got {tuple(rois.shape)}, "
                           f"{tuple(roi_inds.shape)}")
    ph, pw = (output_size, output_size) if isinstance(output_size, int) else tuple(output_size)
    x = _to_dev(input)
    args = (x, _to_dev(rois), _to_dev(roi_inds), int(ph), int(pw), float(img_h), float(img_w),
            float(spatial_scale), bool(rois_sorted))
    if not (torch.is_grad_enabled() and x.requires_grad):  # inference: no autograd node
        return _roi_pool_head_fwd(*args, outs=out)
    if out is not None:
        raise RuntimeError("roi_pool_head: out= is for inference (no autograd)")
    return _RoIPoolHeadFunction.apply(*args)


def _boxes_to_rois(boxes: Union[torch.Tensor, List[torch.Tensor]]) -> torch.Tensor:
    if isinstance(boxes, (list, tuple)):  # torchvision's List[Tensor[L,4]] form
        parts = [torch.cat([torch.full((b.size(0), 1), i, dtype=b.dtype, device=b.device), b], 1)
                 for i, b in enumerate(boxes)]
        boxes = torch.cat(parts, 0) if parts else torch.zeros((0, 5))
    if boxes.dim() != 2 or boxes.size(1) != 5:
        raise RuntimeError(f"boxes must be [K, 5] (batch_idx, x1, y1, x2, y2); got {tuple(boxes.shape)}")
    return boxes


def roi_pool_with_argmax(input: torch.Tensor, boxes, output_size, spatial_scale: float = 1.0,
                         rois_sorted=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """roi_pool returning (out, argmax int32) -- the torch.ops.torchvision.roi_pool pair.
    ``rois_sorted``: RoIs grouped by non-decreasing batch index (None = check
    host-resident RoIs, assume unsorted for device RoIs)."""
    if input.dim() != 4:
        raise RuntimeError("input must be [N, C, H, W]")
    ph, pw = (output_size, output_size) if isinstance(output_size, int) else tuple(output_size)
    out_dev = input.device
    x = _to_dev(input)  # differentiable move, so CPU leaf tensors get their grad
    b = _boxes_to_rois(boxes)
    if rois_sorted is None:
        rois_sorted = _sorted_by_image(b)
    rois = _to_dev(b)
    out, am = _RoIPoolFunction.apply(x.contiguous(), rois, int(ph), int(pw), float(spatial_scale),
                                     bool(rois_sorted))
    return out.to(out_dev), am.to(out_dev)


def roi_pool(input: torch.Tensor, boxes, output_size, spatial_scale: float = 1.0,
             rois_sorted=None) -> torch.Tensor:
    """torchvision.ops.roi_pool (nets/heads.py:48)."""
    return roi_pool_with_argmax(input, boxes, output_size, spatial_scale, rois_sorted)[0]


# ------------------------------------------------------------------ proposals
_params_cache = {}  # launch-parameter block + workspace size per layer shape (built once)


def propose(scores: torch.Tensor, deltas: torch.Tensor, *, img_w: float, img_h: float,
            pre_nms: int, post_nms: int, nms_thresh: float = 0.7, min_size: float = 16,
            anchors: torch.Tensor = None, anchor_base: torch.Tensor = None, feat_h: int = 0,
            feat_w: int = 0, feat_stride: int = 16, out=None, workspace=None):
    """Batched proposal layer on device tensors.

    scores fp32 [N, A], deltas fp32 [N, A, 4]; either explicit ``anchors``
    [A, 4] or ``anchor_base`` [K, 4] + the feature grid (anchors generated in
    the decode kernel).  Returns padded (rois [N, post, 4], anchor_idx int32
    [N, post], count int32 [N]) -- no host synchronisation.
    """
    lib = _lib.load()
    dev = scores.device
    N, A = scores.shape
    K = 0 if anchors is None and anchor_base is None else (anchor_base.size(0) if anchors is None else 0)
    key = (N, A, K, feat_h, feat_w, feat_stride, float(img_h), float(img_w), float(min_size),
           int(pre_nms), int(post_nms), float(nms_thresh))
    cached = _params_cache.get(key)
    if cached is None:
        if anchors is None and K * feat_h * feat_w != A:
            raise RuntimeError(f"A={A} != feat_h*feat_w*K={feat_h}*{feat_w}*{K}")
        p = _lib.ProposeParams()
        p.N, p.A = N, A
        p.K, p.feat_h, p.feat_w, p.feat_stride = K, feat_h, feat_w, feat_stride
        p.img_h, p.img_w, p.min_size = float(img_h), float(img_w), float(min_size)
        p.pre_nms, p.post_nms, p.iou_threshold = int(pre_nms), int(post_nms), float(nms_thresh)
        cached = (p, int(lib.frcnn_propose_workspace_size(p)))
        _params_cache[key] = cached
    p, need = cached
    if out is None:
        rois = torch.empty((N, post_nms, 4), dtype=torch.float32, device=dev)
        idx = torch.empty((N, post_nms), dtype=torch.int32, device=dev)
        cnt = torch.empty((N,), dtype=torch.int32, device=dev)
    else:  # caller-owned outputs (static buffers of a captured HIP graph)
        rois, idx, cnt = out
        if (tuple(rois.shape) != (N, post_nms, 4) or tuple(idx.shape) != (N, post_nms)
                or tuple(cnt.shape) != (N,) or rois.dtype != torch.float32
                or idx.dtype != torch.int32 or cnt.dtype != torch.int32):
            raise RuntimeError("propose: out buffers must be fp32 [N,post,4], int32 [N,post], int32 [N]")
    ws = workspace if workspace is not None else _lib.cached_workspace("propose", need, dev)
    if ws.numel() < need:
        raise RuntimeError(f"propose: workspace of {ws.numel()} B < {need} B")
    _lib.check(lib.frcnn_propose(p, _lib.ptr(scores), _lib.ptr(deltas), _lib.ptr(anchors),
                                 _lib.ptr(anchor_base), _lib.ptr(rois), _lib.ptr(idx),
                                 _lib.ptr(cnt), _lib.ptr(ws), ws.numel(), _lib.stream_ptr()),
               "propose")
    return rois, idx, cnt


# ------------------------------------------------------------- RPN epilogue
class _RPNHeadEpilogueFunction(torch.autograd.Function):
    """nets/rpn.py:117-124 as one launch.  The backward of the two permutes is
    the inverse permute (plain tensor ops); the fg scores feed only the
    (non-differentiable) proposal layer, as in the reference."""

    @staticmethod
    def forward(ctx, cls, reg, K):
        lib = _lib.load()
        N, C2, H, W = cls.shape
        if C2 != 2 * K or tuple(reg.shape) != (N, 4 * K, H, W):
            raise RuntimeError(f"rpn_head_epilogue: cls {tuple(cls.shape)} / reg {tuple(reg.shape)} "
                               f"do not match K={K}")
        A = H * W * K
        cls_nhwc = torch.empty((N, A, 2), dtype=torch.float32, device=cls.device)
        fg = torch.empty((N, A), dtype=torch.float32, device=cls.device)
        reg_nhwc = torch.empty((N, A, 4), dtype=torch.float32, device=cls.device)
        _lib.check(lib.frcnn_rpn_head_epilogue(_lib.ptr(cls), _lib.ptr(reg), N, K, H, W,
                                               _lib.ptr(cls_nhwc), _lib.ptr(fg), _lib.ptr(reg_nhwc),
                                               _lib.stream_ptr()), "rpn_head_epilogue")
        ctx.meta = (N, K, H, W)
        ctx.mark_non_differentiable(fg)
        return cls_nhwc, fg, reg_nhwc

    @staticmethod
    def backward(ctx, g_cls, _g_fg, g_reg):
        N, K, H, W = ctx.meta
        gc = gr = None
        if g_cls is not None:
            gc = g_cls.reshape(N, H, W, 2 * K).permute(0, 3, 1, 2).contiguous()
        if g_reg is not None:
            gr = g_reg.reshape(N, H, W, 4 * K).permute(0, 3, 1, 2).contiguous()
        return gc, gr, None


def rpn_head_epilogue(cls: torch.Tensor, reg: torch.Tensor, K: int):
    """nets/rpn.py:117-124: conv outputs cls [N,2K,H,W], reg [N,4K,H,W] (device,
    fp32) -> (cls_nhwc [N,A,2], fg [N,A], reg_nhwc [N,A,4]), A = H*W*K.
    ``cls_nhwc.permute(0, 2, 1)`` is the reference's returned ``cls``; ``fg`` is
    its ``cls_fg_softmax``; ``reg_nhwc`` its ``reg``."""
    if cls.dim() != 4 or reg.dim() != 4:
        raise RuntimeError("rpn_head_epilogue: cls and reg must be NCHW")
    return _RPNHeadEpilogueFunction.apply(cls.float().contiguous(), reg.float().contiguous(), int(K))


def roi_transform(rois: torch.Tensor, roi_inds: torch.Tensor, img_h, img_w, feat_h: int,
                  feat_w: int) -> torch.Tensor:
    """nets/heads.py:42-47 on device: [R,4] image rois + [R] inds -> [R,5]."""
    lib = _lib.load()
    R = rois.size(0)
    out = torch.empty((R, 5), dtype=torch.float32, device=rois.device)
    _lib.check(lib.frcnn_roi_transform(_lib.ptr(rois), _lib.ptr(roi_inds), R, float(img_h),
                                       float(img_w), int(feat_h), int(feat_w), _lib.ptr(out),
                                       _lib.stream_ptr()), "roi_transform")
    return out
