"""Box utilities and target creators (utils/utils.py) on the HIP path.

Module constants and signatures mirror utils/utils.py:6-21 and :47-276.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

# rpn (utils/utils.py:6-12)
nms_thresh = 0.7
n_train_pre_nms = 12000
n_train_post_nms = 600
n_test_pre_nms = 3000
n_test_post_nms = 300
min_size = 16

# VOC dataset (utils/utils.py:15-21)
PASCAL_VOC_CLASSES = ['__background__',
                      'aeroplane', 'bicycle', 'bird', 'boat',
                      'bottle', 'bus', 'car', 'cat', 'chair',
                      'cow', 'diningtable', 'dog', 'horse',
                      'motorbike', 'person', 'pottedplant',
                      'sheep', 'sofa', 'train', 'tvmonitor']
PASCAL_VOC_NUM_CLASSES = 20 + 1


def reg2bbox(anchors, reg):
    """utils/utils.py:47-73: [dx, dy, dh, dw] deltas -> boxes (fp32).

    Tensor in, tensor out on the input's device (the reference returns a CPU
    tensor for CPU inputs); computed by ``reg2bbox_kernel``."""
    lib = _lib.load()
    out_dev = reg.device if isinstance(reg, torch.Tensor) else torch.device("cpu")
    dev = _lib.device()
    a = torch.as_tensor(anchors).to(device=dev, dtype=torch.float32).contiguous()
    r = torch.as_tensor(reg).to(device=dev, dtype=torch.float32).contiguous()
    if a.shape != r.shape or a.dim() != 2 or a.size(1) != 4:
        raise RuntimeError(f"reg2bbox: anchors {tuple(a.shape)} and reg {tuple(r.shape)} must be [n, 4]")
    out = torch.empty_like(r)
    _lib.check(lib.frcnn_reg2bbox(_lib.ptr(a), _lib.ptr(r), a.size(0), _lib.ptr(out),
                                  _lib.stream_ptr()), "reg2bbox")
    return out.to(out_dev)


# ------------------------------------------------------------ numpy RNG bridge
def rng_state_to_device(dev):
    """numpy's GLOBAL legacy MT19937 state (the one the reference's
    np.random.choice calls consume) -> u32 [625] device tensor (key + pos)."""
    st = np.random.get_state()
    if st[0] != "MT19937":
        raise RuntimeError("numpy global RNG is not MT19937")
    buf = np.empty(625, np.uint32)
    buf[:624] = st[1]
    buf[624] = st[2]
    return torch.from_numpy(buf.view(np.int32)).to(dev), st


def rng_state_from_device(t, st):
    buf = t.cpu().numpy().view(np.uint32)
    np.random.set_state(("MT19937", buf[:624].copy(), int(buf[624]), st[3], st[4]))


def _np_dtype_of(x):
    return x.dtype if isinstance(x, np.ndarray) else np.dtype(str(x.dtype).replace("torch.", ""))


def _as_dev(x, f64, dev):
    t = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
    return t.to(device=dev, dtype=torch.float64 if f64 else torch.float32).contiguous()


def bbox_iou(bbox_a, bbox_b):
    """utils/utils.py:102-119 -> numpy [Na, Nb] (fp32 if both inputs are fp32,
    else fp64, as numpy promotes); raises IndexError like the reference."""
    lib = _lib.load()
    a = np.asarray(bbox_a) if not isinstance(bbox_a, torch.Tensor) else bbox_a
    b = np.asarray(bbox_b) if not isinstance(bbox_b, torch.Tensor) else bbox_b
    if a.shape[1] != 4 or b.shape[1] != 4:
        print(bbox_a, bbox_b)
        raise IndexError
    a64 = _np_dtype_of(a) != np.float32
    b64 = _np_dtype_of(b) != np.float32
    dev = _lib.device()
    ta, tb = _as_dev(a, a64, dev), _as_dev(b, b64, dev)
    out = torch.empty((ta.size(0), tb.size(0)), device=dev,
                      dtype=torch.float64 if (a64 or b64) else torch.float32)
    _lib.check(lib.frcnn_bbox_iou(_lib.ptr(ta), int(a64), ta.size(0), _lib.ptr(tb), int(b64),
                                  tb.size(0), _lib.ptr(out), _lib.stream_ptr()), "bbox_iou")
    return out.cpu().numpy()


def bbox2reg(anchors, bbox):
    """utils/utils.py:75-100 -> numpy fp64 [n, 4]."""
    lib = _lib.load()
    a64 = _np_dtype_of(anchors) != np.float32
    b64 = _np_dtype_of(bbox) != np.float32
    dev = _lib.device()
    ta, tb = _as_dev(anchors, a64, dev), _as_dev(bbox, b64, dev)
    out = torch.empty((tb.size(0), 4), device=dev, dtype=torch.float64)
    _lib.check(lib.frcnn_bbox2reg(_lib.ptr(ta), int(a64), _lib.ptr(tb), int(b64), tb.size(0),
                                  _lib.ptr(out), _lib.stream_ptr()), "bbox2reg")
    return out.cpu().numpy()


class AnchorTargetCreator(object):
    """utils/utils.py:122-204; __call__(bbox, anchor) -> (reg, label) with the
    reference's types (fp64 reg / int32 label, fp32 zeros without gt) and the
    same consumption of numpy's global RNG."""

    def __init__(self, n_sample=256, pos_iou_thresh=0.7, neg_iou_thresh=0.3, pos_ratio=0.5):
        self.n_sample = n_sample
        self.pos_iou_thresh = pos_iou_thresh
        self.neg_iou_thresh = neg_iou_thresh
        self.pos_ratio = pos_ratio

    def __call__(self, bbox, anchor, return_internals=False):
        from . import targets
        bb = np.asarray(bbox, np.float64).reshape(1, -1, 4)
        lab = np.zeros(bb.shape[:2])
        reg, label, argmax, max_iou = targets.anchor_targets(
            bb, lab, anchor, n_sample=self.n_sample, pos_iou_thresh=self.pos_iou_thresh,
            neg_iou_thresh=self.neg_iou_thresh, pos_ratio=self.pos_ratio, internals=True)
        label = label[0].cpu().numpy()
        if bb.shape[1] == 0:
            reg_np = np.zeros_like(np.asarray(anchor, np.float32))
        else:
            reg_np = reg[0].cpu().numpy()
        if return_internals:
            return reg_np, label, argmax[0].cpu().numpy(), max_iou[0].cpu().numpy()
        return reg_np, label


class ProposalTargetCreator(object):
    """utils/utils.py:207-276; __call__(roi, bbox, label, mean, std) ->
    (sample_roi, gt_roi_reg, gt_roi_label), fp64 numpy, rows in the
    reference's (permutation) order."""

    def __init__(self, n_sample=128, pos_ratio=0.5, pos_iou_thresh=0.5, neg_iou_thresh_high=0.5,
                 neg_iou_thresh_low=0):
        self.n_sample = n_sample
        self.pos_ratio = pos_ratio
        self.pos_roi_per_image = np.round(self.n_sample * self.pos_ratio)
        self.pos_iou_thresh = pos_iou_thresh
        self.neg_iou_thresh_high = neg_iou_thresh_high
        self.neg_iou_thresh_low = neg_iou_thresh_low

    def __call__(self, roi, bbox, label, reg_normalize_mean=(0., 0., 0., 0.),
                 reg_normalize_std=(0.1, 0.1, 0.2, 0.2)):
        from . import targets
        r = torch.as_tensor(roi).detach().to(_lib.device(), torch.float32).reshape(1, -1, 4)
        bb = np.asarray(bbox, np.float64).reshape(1, -1, 4)
        lab = np.asarray(label, np.float64).reshape(1, -1)
        if bb.shape[1] and (lab == -1).any():
            raise ValueError("label -1 marks padding; pass only the valid gt rows")
        cnt = torch.tensor([r.size(1)], dtype=torch.int32, device=r.device)
        s_roi, s_reg, s_lab, s_cnt = targets.proposal_targets(
            r, cnt, bb, lab, n_sample=self.n_sample, pos_ratio=self.pos_ratio,
            pos_iou_thresh=self.pos_iou_thresh, neg_iou_thresh_high=self.neg_iou_thresh_high,
            neg_iou_thresh_low=self.neg_iou_thresh_low, reg_normalize_mean=reg_normalize_mean,
            reg_normalize_std=reg_normalize_std)
        k = int(s_cnt[0])
        return (s_roi[0, :k].cpu().numpy(), s_reg[0, :k].cpu().numpy(),
                s_lab[0, :k].cpu().numpy())
