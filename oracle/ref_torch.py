"""ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference's own CPU path for the proposal layer and the head's RoIPool,
restated in torch CPU ops exactly as the reference issues them, for the timed
host baseline of bench.py (``cpu_baseline``).  torchvision's ``nms`` and
``roi_pool`` are absent here, so the C restatement of their
CPU kernels (oracle/tv_ops.c, single-threaded like torchvision's own CPU
kernels) stands in; every other op is the torch op the reference calls, run on
all the host threads torch is given.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ref_numpy as orc


def reg2bbox(anchors: torch.Tensor, reg: torch.Tensor) -> torch.Tensor:
    """utils/utils.py:47-73 (torch CPU ops, as written there)."""
    anchor_h = anchors[:, 2] - anchors[:, 0]
    anchor_w = anchors[:, 3] - anchors[:, 1]
    anchor_cx = (anchors[:, 2] + anchors[:, 0]) / 2
    anchor_cy = (anchors[:, 1] + anchors[:, 3]) / 2
    x = reg[:, 0] * anchor_h + anchor_cx
    y = reg[:, 1] * anchor_w + anchor_cy
    h = torch.exp(reg[:, 2]) * anchor_h
    w = torch.exp(reg[:, 3]) * anchor_w
    bbox = torch.zeros(reg.shape)
    bbox[:, 0] = x - h * .5
    bbox[:, 1] = y - w * .5
    bbox[:, 2] = x + h * .5
    bbox[:, 3] = y + w * .5
    return bbox


def _nms(bbox: torch.Tensor, scores: torch.Tensor, thr: float) -> torch.Tensor:
    return torch.from_numpy(orc.nms(bbox.numpy(), scores.numpy(), thr))


def region_proposal(anchors: np.ndarray, cls_fg_softmax: torch.Tensor, reg: torch.Tensor, img_w, img_h,
                    pre_nms, post_nms, nms_threshold=0.7, min_size=16) -> torch.Tensor:
    """nets/rpn.py:58-77 for one image."""
    anchors = torch.from_numpy(anchors)
    bbox = reg2bbox(anchors, reg)
    bbox[:, [0, 2]] = torch.clamp(bbox[:, [0, 2]], min=0, max=img_h)
    bbox[:, [1, 3]] = torch.clamp(bbox[:, [1, 3]], min=0, max=img_w)
    select_scale = torch.where((bbox[:, 2] - bbox[:, 0] >= min_size) &
                               (bbox[:, 3] - bbox[:, 1] >= min_size))[0]
    bbox = bbox[select_scale, :]
    cls_fg_softmax = cls_fg_softmax[select_scale]
    rank = torch.argsort(cls_fg_softmax, descending=True)
    rank = rank[:pre_nms]
    cls_fg_softmax = cls_fg_softmax[rank]
    bbox = bbox[rank, :]
    nms_ind = _nms(bbox, cls_fg_softmax, nms_threshold)
    roi = bbox[nms_ind]
    return roi[:post_nms]


def head_roi_pool(x: torch.Tensor, rois: torch.Tensor, roi_inds: torch.Tensor, img_h, img_w,
                  roi_size=7, spatial_scale=1.0):
    """nets/heads.py:40-48: RoI transform, [idx, box] pack, roi_pool -> (out, argmax)."""
    feature_rois = torch.zeros(rois.shape)
    feature_rois[:, [0, 2]] = rois[:, [0, 2]] / img_h * x.shape[2]
    feature_rois[:, [1, 3]] = rois[:, [1, 3]] / img_w * x.shape[3]
    boxes = torch.cat([roi_inds[:, None], feature_rois], dim=-1)
    out, am = orc.roi_pool_forward(x.numpy(), boxes.numpy(), roi_size, spatial_scale)
    return torch.from_numpy(out), torch.from_numpy(am), boxes
