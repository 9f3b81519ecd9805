"""Region proposal network (nets/rpn.py) on the HIP path.

``region_proposal`` and ``RPN`` keep the reference constructor arguments,
call signatures and return types (nets/rpn.py:20-138).  The proposal layer is
the batched HIP pipeline (``ops.propose``): the per-image Python loop of
nets/rpn.py:131-136 becomes one launch sequence over the whole batch, with
anchors generated inside the decode kernel.  The conv outputs' permutes and
the fg softmax are one HIP launch (``ops.rpn_head_epilogue``); the 3x3/1x1
convolutions stay plain PyTorch (not the target).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib, ops
from .anchors import generate_anchor_base, generate_anchor_base_device, generate_anchors
from .utils import (n_test_post_nms, n_test_pre_nms, n_train_post_nms, n_train_pre_nms,
                    nms_thresh)


def normal_init(m, mean, stddev, truncated=False):
    """nets/rpn.py:11-17."""
    if truncated:
        m.weight.data.normal_().fmod_(2).mul_(stddev).add_(mean)
    else:
        m.weight.data.normal_(mean, stddev)
        m.bias.data.zero_()


class region_proposal(nn.Module):
    """nets/rpn.py:20-79: decode -> clamp -> min-size filter -> top pre_nms ->
    NMS -> top post_nms, for one image."""

    def __init__(self, mode, nms_thresh=nms_thresh, n_train_pre_nms=n_train_pre_nms,
                 n_train_post_nms=n_train_post_nms, n_test_pre_nms=n_test_pre_nms,
                 n_test_post_nms=n_test_post_nms, min_size=16):
        super().__init__()
        self.mode = mode
        self.pre_nms = n_train_pre_nms
        self.post_nms = n_train_post_nms
        if mode == 'test':
            self.pre_nms = n_test_pre_nms
            self.post_nms = n_test_post_nms
        self.nms_threshold = nms_thresh
        self.min_size = min_size

    def __call__(self, anchors, cls_fg_softmax, reg, img_w, img_h):
        """anchors [A,4] (numpy or tensor), cls_fg_softmax [A], reg [A,4] ->
        rois fp32 [<=post_nms, 4] on the device of ``reg``."""
        dev = _lib.device()
        out_dev = reg.device if isinstance(reg, torch.Tensor) else torch.device("cpu")
        a = torch.as_tensor(np.asarray(anchors, np.float32)) if not isinstance(anchors, torch.Tensor) \
            else anchors
        a = a.to(device=dev, dtype=torch.float32).contiguous()
        s = torch.as_tensor(cls_fg_softmax).to(device=dev, dtype=torch.float32).reshape(1, -1)
        r = torch.as_tensor(reg).to(device=dev, dtype=torch.float32).reshape(1, -1, 4).contiguous()
        rois, _, cnt = ops.propose(s.contiguous(), r, img_w=img_w, img_h=img_h,
                                   pre_nms=self.pre_nms, post_nms=self.post_nms,
                                   nms_thresh=self.nms_threshold, min_size=self.min_size,
                                   anchors=a)
        return rois[0, :int(cnt[0])].to(out_dev)


class RPN(nn.Module):
    """nets/rpn.py:82-138."""

    def __init__(self, in_channels=256, mid_channels=256, ratios=[0.5, 1., 2.],
                 anchor_scales=[8, 16, 32], feat_stride=16, mode="training",
                 anchors_as_numpy=True):
        super().__init__()
        self.base_anchor = generate_anchor_base(ratios=ratios, anchor_scales=anchor_scales)
        self._ratios, self._scales = list(ratios), list(anchor_scales)
        self.K = self.base_anchor.shape[0]
        self.feat_stride = feat_stride
        self.proposal_layer = region_proposal(mode)
        self.anchors_as_numpy = anchors_as_numpy
        self.conv1 = nn.Conv2d(in_channels, mid_channels, kernel_size=3, stride=1, padding=1)
        self.cls = nn.Conv2d(mid_channels, self.K * 2, kernel_size=1, stride=1, padding=0)
        self.reg = nn.Conv2d(mid_channels, self.K * 4, kernel_size=1, stride=1, padding=0)
        normal_init(self.conv1, 0, 0.01)
        normal_init(self.cls, 0, 0.01)
        normal_init(self.reg, 0, 0.01)
        self._base_dev = None

    def forward(self, x, img_width, img_height):
        """-> (cls [N,2,A], reg [N,A,4], rois [sum R,4], roi_inds fp32 [sum R], anchors [A,4])."""
        n_img, _, conv_h, conv_w = x.shape
        x = F.relu(self.conv1(x))
        # nets/rpn.py:117-124: permute/contiguous/softmax/slice in ONE launch
        # (ops.rpn_head_epilogue); results return to x's device like the reference's
        dev = _lib.device()
        cls_nhwc, cls_fg_softmax, reg = ops.rpn_head_epilogue(
            self.cls(x).to(dev), self.reg(x).to(dev), self.K)
        cls = cls_nhwc.to(x.device).permute(0, 2, 1)

        if self._base_dev is None:
            self._base_dev = generate_anchor_base_device(ratios=self._ratios,
                                                         anchor_scales=self._scales)
        pl = self.proposal_layer
        rois_p, _, cnt = ops.propose(
            cls_fg_softmax, reg.detach(), img_w=img_width, img_h=img_height,
            pre_nms=pl.pre_nms, post_nms=pl.post_nms, nms_thresh=pl.nms_threshold,
            min_size=pl.min_size, anchor_base=self._base_dev, feat_h=conv_h, feat_w=conv_w,
            feat_stride=self.feat_stride)
        # padded per-image form (the batched samplers take it as is) + fg scores
        self.rois_padded, self.rois_count, self.fg_scores = rois_p, cnt, cls_fg_softmax.detach()
        counts = cnt.tolist()  # the one host sync: the output length is data-dependent
        rois = torch.cat([rois_p[i, :c] for i, c in enumerate(counts)], 0).to(x.device)
        roi_inds = torch.cat([torch.full((c,), float(i)) for i, c in enumerate(counts)], 0)
        roi_inds = roi_inds.to(x.device)
        anchors = generate_anchors(self._base_dev, self.feat_stride, conv_w, conv_h)
        if self.anchors_as_numpy:
            anchors = anchors.cpu().numpy()
        self.anchors = anchors
        return cls, reg.to(x.device), rois, roi_inds, anchors
