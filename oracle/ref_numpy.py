"""ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

numpy restatement of the reference hot path.  Every function cites the
reference file:line it follows.  Arithmetic types follow the reference
exactly (fp32 where the reference computes in fp32 torch/numpy, fp64 where it
computes in fp64 numpy), with one documented deviation:

* ``exp`` in the box decode is correctly rounded (fp64 exp, then rounded to
  fp32).  The reference calls torch CPU ``exp`` (MKL VML), whose last bit
  depends on the host ISA path (SURVEY.md §7 "Host-dependent exp"), so decoded
  boxes are held to the 1e-5 relative contract and kept indices bit-exact.
* ``argsort`` of the proposal scores is stable (ties by ascending post-filter
  position).  The reference's torch CPU argsort is unstable under ties; parity
  inputs are tie-free.

The two torchvision kernels are restated in C (oracle/tv_ops.c) and loaded
here through ctypes.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _tvops():
    """Load (building on first use) the C restatement of torchvision's ops."""
    global _LIB
    if _LIB is None:
        so = os.path.join(_HERE, "libtvops.so")
        src = os.path.join(_HERE, "tv_ops.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(so)
        P = ctypes.c_void_p
        lib.oracle_nms_f32.argtypes = [P, P, ctypes.c_int64, ctypes.c_double, P]
        lib.oracle_nms_f32.restype = ctypes.c_int64
        lib.oracle_roi_pool_fwd_f32.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_float, P, P]
        lib.oracle_roi_pool_fwd_f32.restype = None
        lib.oracle_roi_pool_bwd_f32.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, P]
        lib.oracle_roi_pool_bwd_f32.restype = None
        _LIB = lib
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------
# anchors: utils/anchors.py
# --------------------------------------------------------------------------
def generate_anchor_base(base_size=16, ratios=(0.5, 1.0, 2.0), anchor_scales=(8, 16, 32)):
    """utils/anchors.py:5-31.  Row ``r*len(scales)+s``; sides in fp64, stored fp32."""
    r = np.asarray(ratios, dtype=np.float64)
    s = np.asarray(anchor_scales)
    side = base_size * s                              # python int * int (exact)
    h = side[None, :] * np.sqrt(r)[:, None]           # utils/anchors.py:23
    w = side[None, :] * np.sqrt(1.0 / r)[:, None]     # utils/anchors.py:24
    out = np.stack([-h / 2, -w / 2, h / 2, w / 2], axis=-1).reshape(-1, 4)
    return out.astype(np.float32)


def generate_anchors(anchor_base, feat_stride, width, height):
    """utils/anchors.py:33-61.  Row ``(y*W + x)*K + k``; the WIDTH offset goes
    into columns 0 and 2 (utils/anchors.py:51-52)."""
    xs = np.arange(0, feat_stride * width, feat_stride)
    ys = np.arange(0, feat_stride * height, feat_stride)
    gx, gy = np.meshgrid(xs, ys)
    shift = np.stack([gx.ravel(), gy.ravel(), gx.ravel(), gy.ravel()], axis=1)
    # fp32 base + int64 shift -> fp64 (exact) -> fp32: one rounding
    out = anchor_base[None, :, :].astype(np.float64) + shift[:, None, :]
    return out.reshape(-1, 4).astype(np.float32)


# --------------------------------------------------------------------------
# box utilities: utils/utils.py
# --------------------------------------------------------------------------
def exp_cr(v):
    """Correctly rounded fp32 exp (see module docstring)."""
    return np.exp(np.asarray(v, dtype=np.float64)).astype(np.float32)


def reg2bbox(anchors, reg):
    """utils/utils.py:47-73 in fp32, each op separately rounded."""
    a = np.asarray(anchors, dtype=np.float32)
    r = np.asarray(reg, dtype=np.float32)
    two = np.float32(2)
    half = np.float32(0.5)
    ah = a[:, 2] - a[:, 0]
    aw = a[:, 3] - a[:, 1]
    acx = (a[:, 2] + a[:, 0]) / two
    acy = (a[:, 1] + a[:, 3]) / two
    x = r[:, 0] * ah
    x = x + acx
    y = r[:, 1] * aw
    y = y + acy
    h = exp_cr(r[:, 2]) * ah
    w = exp_cr(r[:, 3]) * aw
    hh = h * half
    hw = w * half
    return np.stack([x - hh, y - hw, x + hh, y + hw], axis=1).astype(np.float32)


def rpn_head_epilogue(cls, reg):
    """nets/rpn.py:117-124: cls fp32 [N,2K,H,W], reg fp32 [N,4K,H,W] ->
    (cls_nhwc [N,A,2], fg [N,A], reg_nhwc [N,A,4]).  The softmax follows torch's
    CPU last-dim kernel (ATen _vec_softmax_lastdim): m = max, e = exp(x - m),
    out = e * (1 / (e0 + e1)), each op fp32; exp correctly rounded (see module
    docstring -- torch's vectorised exp is host-dependent in its last bits)."""
    cls = np.asarray(cls, dtype=np.float32)
    reg = np.asarray(reg, dtype=np.float32)
    n = cls.shape[0]
    c = np.ascontiguousarray(cls.transpose(0, 2, 3, 1)).reshape(n, -1, 2)   # :118
    r = np.ascontiguousarray(reg.transpose(0, 2, 3, 1)).reshape(n, -1, 4)   # :124
    m = np.maximum(c[:, :, 0], c[:, :, 1])
    e0 = exp_cr(c[:, :, 0] - m)
    e1 = exp_cr(c[:, :, 1] - m)
    inv = np.float32(1) / (e0 + e1)
    return c, (e1 * inv).astype(np.float32), r                                # :119-120


def bbox2reg(anchors, bbox):
    """utils/utils.py:75-100.  Anchor statistics in the anchors' dtype, box
    statistics in the boxes' dtype, output fp64."""
    ah = anchors[:, 2] - anchors[:, 0]
    aw = anchors[:, 3] - anchors[:, 1]
    acx = (anchors[:, 2] + anchors[:, 0]) / 2
    acy = (anchors[:, 1] + anchors[:, 3]) / 2
    bh = bbox[:, 2] - bbox[:, 0]
    bw = bbox[:, 3] - bbox[:, 1]
    bcx = (bbox[:, 2] + bbox[:, 0]) / 2
    bcy = (bbox[:, 1] + bbox[:, 3]) / 2
    out = np.zeros(bbox.shape)
    out[:, 0] = (bcx - acx) / ah
    out[:, 1] = (bcy - acy) / aw
    out[:, 2] = np.log(bh / ah)
    out[:, 3] = np.log(bw / aw)
    return out


def bbox_iou(a, b):
    """utils/utils.py:102-119: pairwise IoU with numpy dtype promotion."""
    if a.shape[1] != 4 or b.shape[1] != 4:
        raise IndexError
    tl = np.maximum(a[:, None, :2], b[:, :2])
    br = np.minimum(a[:, None, 2:], b[:, 2:])
    d = br - tl
    inter = (d[..., 0] * d[..., 1]) * (tl < br).all(axis=2)
    da = a[:, 2:] - a[:, :2]
    db = b[:, 2:] - b[:, :2]
    area_a = da[:, 0] * da[:, 1]
    area_b = db[:, 0] * db[:, 1]
    return inter / (area_a[:, None] + area_b - inter)


# --------------------------------------------------------------------------
# torchvision ops (C restatement)
# --------------------------------------------------------------------------
def nms(boxes, scores, iou_threshold):
    """torchvision.ops.nms semantics."""
    b = np.ascontiguousarray(boxes, dtype=np.float32)
    s = np.ascontiguousarray(scores, dtype=np.float32)
    n = b.shape[0]
    keep = np.empty(max(n, 1), dtype=np.int64)
    k = _tvops().oracle_nms_f32(_ptr(b), _ptr(s), n, float(iou_threshold), _ptr(keep))
    return keep[:k].copy()


def roi_pool_forward(x, rois, output_size, spatial_scale=1.0):
    """torchvision roi_pool forward (App. A.4) -> (out, argmax int32)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    rois = np.ascontiguousarray(rois, dtype=np.float32)
    ph, pw = (output_size, output_size) if np.isscalar(output_size) else output_size
    N, C, H, W = x.shape
    R = rois.shape[0]
    out = np.empty((R, C, ph, pw), np.float32)
    am = np.empty((R, C, ph, pw), np.int32)
    _tvops().oracle_roi_pool_fwd_f32(_ptr(x), _ptr(rois), R, C, H, W, ph, pw,
                                     float(spatial_scale), _ptr(out), _ptr(am))
    return out, am


def roi_pool_backward(grad, rois, argmax, input_shape):
    """torchvision _roi_pool_backward (App. A.4), CPU summation order."""
    grad = np.ascontiguousarray(grad, dtype=np.float32)
    rois = np.ascontiguousarray(rois, dtype=np.float32)
    argmax = np.ascontiguousarray(argmax, dtype=np.int32)
    N, C, H, W = input_shape
    R, _, ph, pw = grad.shape
    gi = np.empty((N, C, H, W), np.float32)
    _tvops().oracle_roi_pool_bwd_f32(_ptr(grad), _ptr(rois), _ptr(argmax), R, N, C, H, W,
                                     ph, pw, _ptr(gi))
    return gi


# --------------------------------------------------------------------------
# proposal layer: nets/rpn.py:47-79
# --------------------------------------------------------------------------
def propose_one(anchors, scores, reg, img_w, img_h, pre_nms, post_nms,
                nms_thresh=0.7, min_size=16):
    """nets/rpn.py:58-77 for ONE image.  Returns (rois fp32 [k,4],
    anchor indices int64 [k]) where ``rois == reg2bbox(...)[idx]`` clamped."""
    bbox = reg2bbox(anchors, reg)
    bbox[:, [0, 2]] = np.clip(bbox[:, [0, 2]], np.float32(0), np.float32(img_h))  # :62
    bbox[:, [1, 3]] = np.clip(bbox[:, [1, 3]], np.float32(0), np.float32(img_w))  # :63
    m = (bbox[:, 2] - bbox[:, 0] >= min_size) & (bbox[:, 3] - bbox[:, 1] >= min_size)
    sel = np.nonzero(m)[0]                                                          # :65
    s = np.asarray(scores, dtype=np.float32)[sel]
    rank = np.argsort(-s, kind="stable")[:pre_nms]                                  # :71-72
    cand = bbox[sel][rank]
    keep = nms(cand, s[rank], nms_thresh)[:post_nms]                                # :75-77
    idx = sel[rank][keep]
    return cand[keep].copy(), idx.astype(np.int64)


def roi_transform(rois, roi_inds, img_h, img_w, feat_h, feat_w):
    """nets/heads.py:42-47: image-space RoIs -> ``[idx, r0, r1, r2, r3]`` on the
    feature map, fp32 divide-then-multiply."""
    r = np.asarray(rois, dtype=np.float32)
    fr = np.zeros(r.shape, np.float32)
    fr[:, [0, 2]] = r[:, [0, 2]] / np.float32(img_h) * np.float32(feat_h)
    fr[:, [1, 3]] = r[:, [1, 3]] / np.float32(img_w) * np.float32(feat_w)
    return np.concatenate([np.asarray(roi_inds, np.float32)[:, None], fr], axis=1)


# --------------------------------------------------------------------------
# target creators: utils/utils.py:122-276 (global numpy RNG, like the reference)
# --------------------------------------------------------------------------
def anchor_target(bbox, anchor, n_sample=256, pos_iou_thresh=0.7, neg_iou_thresh=0.3,
                  pos_ratio=0.5, return_internals=False):
    """AnchorTargetCreator.__call__ (utils/utils.py:137-204)."""
    ious = bbox_iou(anchor, bbox)
    A = len(anchor)
    if len(bbox) == 0:                                            # :162-163
        argmax_ious = np.zeros(A, np.int32)
        max_ious = np.zeros(A)
        gt_argmax = np.zeros(0)
    else:
        argmax_ious = ious.argmax(axis=1)                         # :165
        max_ious = ious.max(axis=1)                               # :167
        gt_argmax = ious.argmax(axis=0)                           # :169
        for i in range(len(gt_argmax)):                           # :171-172 (later gt wins)
            argmax_ious[gt_argmax[i]] = i
    label = np.full(A, -1, dtype=np.int32)                        # :178-179
    label[max_ious < neg_iou_thresh] = 0                          # :183
    label[max_ious >= pos_iou_thresh] = 1                         # :185
    if len(gt_argmax) > 0:
        label[gt_argmax] = 1                                      # :187-188
    n_pos = int(pos_ratio * n_sample)                             # :190
    pos_index = np.where(label == 1)[0]
    if len(pos_index) > n_pos:                                    # :193-195
        dis = np.random.choice(pos_index, size=(len(pos_index) - n_pos), replace=False)
        label[dis] = -1
    n_neg = n_sample - np.sum(label == 1)                         # :198
    neg_index = np.where(label == 0)[0]
    if len(neg_index) > n_neg:                                    # :200-202
        dis = np.random.choice(neg_index, size=(len(neg_index) - n_neg), replace=False)
        label[dis] = -1
    if (label > 0).any():                                         # :146-150
        reg = bbox2reg(anchor, bbox[argmax_ious])
    else:
        reg = np.zeros_like(anchor)
    if return_internals:
        return reg, label, argmax_ious, max_ious
    return reg, label


def proposal_target(roi, bbox, label, n_sample=128, pos_ratio=0.5, pos_iou_thresh=0.5,
                    neg_iou_thresh_high=0.5, neg_iou_thresh_low=0.0,
                    reg_normalize_mean=(0., 0., 0., 0.), reg_normalize_std=(0.1, 0.1, 0.2, 0.2)):
    """ProposalTargetCreator.__call__ (utils/utils.py:216-276).  ``roi`` fp32."""
    pos_per_image = np.round(n_sample * pos_ratio)                 # :211
    roi = np.concatenate((np.asarray(roi, np.float32), bbox), axis=0)   # :230
    iou = bbox_iou(roi, bbox)
    if len(bbox) == 0:
        gt_assignment = np.zeros(len(roi), np.int32)
        max_iou = np.zeros(len(roi))
        gt_roi_label = np.zeros(len(roi))
    else:
        gt_assignment = iou.argmax(axis=1)
        max_iou = iou.max(axis=1)
        gt_roi_label = label[gt_assignment]
    pos_index = np.where(max_iou >= pos_iou_thresh)[0]             # :248
    n_pos = int(min(pos_per_image, pos_index.size))
    if pos_index.size > 0:
        pos_index = np.random.choice(pos_index, size=n_pos, replace=False)
    neg_index = np.where((max_iou < neg_iou_thresh_high) & (max_iou >= neg_iou_thresh_low))[0]
    n_neg = int(min(n_sample - n_pos, neg_index.size))
    if neg_index.size > 0:
        neg_index = np.random.choice(neg_index, size=n_neg, replace=False)
    keep = np.append(pos_index, neg_index)                        # :265 permutation order
    sample_roi = roi[keep]
    if len(bbox) == 0:
        return sample_roi, np.zeros_like(sample_roi), gt_roi_label[keep]
    gt_roi_reg = bbox2reg(sample_roi, bbox[gt_assignment[keep]])
    gt_roi_reg = ((gt_roi_reg - np.array(reg_normalize_mean, np.float32))
                  / np.array(reg_normalize_std, np.float32))
    gt_roi_label = gt_roi_label[keep]
    gt_roi_label[n_pos:] = 0
    return sample_roi, gt_roi_reg, gt_roi_label
