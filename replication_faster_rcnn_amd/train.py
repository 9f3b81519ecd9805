"""Training-step harness around the HIP hot path (train.py:13-127).

``Trainer.train_step`` mirrors ``trainer.train_step`` (train.py:59-127) from the
backbone features on: RPN (nets/rpn.py) -> anchor targets for every image ->
RPN losses -> proposal targets for every image -> head (RoI transform + pack +
RoIPool, nets/heads.py:42-48) -> label gather -> losses -> backward.  The two
per-image Python loops (train.py:71-79 and :91-104) are one batched HIP call
each (``targets.anchor_targets`` / ``targets.proposal_targets``), consuming
numpy's global RNG in the reference's order (all images' anchor targets, then
all images' proposal targets), and every tensor stays on the device: the
sampled RoIs go to the head without the reference's numpy round trip.  The
losses are plain PyTorch (train.py:29-57, :81-83, :114-121); the backbone,
the RPN convolutions and the head FCs are not the target.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib, targets


def fast_rcnn_loc_loss(pred_loc, gt_loc, gt_label, sigma=1):
    """train.py:29-57: smooth-L1 over the rows with label > 0, divided by
    max(#positives, 1)."""
    pos = gt_label > 0
    pred_loc = pred_loc[pos]
    gt_loc = gt_loc[pos]
    sigma_squared = sigma ** 2
    diff = (pred_loc - gt_loc).abs()
    loss = torch.where(diff < (1. / sigma_squared), 0.5 * sigma_squared * diff ** 2,
                       diff - 0.5 / sigma_squared).sum()
    num_pos = pos.sum().float()
    return loss / torch.max(num_pos, torch.ones_like(num_pos))


class Trainer:
    """train.py:13-27 without the data loader / backbone construction: takes
    the RPN and head modules (``rpn.RPN``, ``heads.ResnetHead``)."""

    def __init__(self, rpn, head, n_sample=(256, 128), optimizer=None):
        self.rpn = rpn
        self.head = head
        self.n_sample = list(n_sample)
        self.optimizer = optimizer
        self.last = {}

    def train_step(self, features, img_h, img_w, boxes, labels):
        """features [N,C,H,W] (backbone output, device), boxes [N,G,4] fp64
        ``[ymin,xmin,ymax,xmax]`` with -1 padding rows, labels [N,G] (-1 = pad).
        Returns the five losses (train.py:123)."""
        if self.optimizer is not None:
            self.optimizer.zero_grad()
        dev = _lib.device()
        N = features.shape[0]
        cls, reg, rois, roi_inds, anchors = self.rpn(features, img_w, img_h)
        a = anchors if isinstance(anchors, torch.Tensor) else torch.from_numpy(np.asarray(anchors))
        # train.py:67-79: anchor targets of every image (one batched call)
        reg_t, lab = targets.anchor_targets(boxes, labels, a.to(dev), n_sample=self.n_sample[0])
        reg_targets_rpn = reg_t.float()           # torch.zeros(...) fp32 buffer, :68,78
        cls_labels_rpn = lab.float()              # :69,79
        rpn_reg_loss = fast_rcnn_loc_loss(reg, reg_targets_rpn, cls_labels_rpn)
        rpn_cls_loss = F.cross_entropy(cls, cls_labels_rpn.long(), ignore_index=-1)
        # train.py:85-104: proposal targets of every image, on device
        s_roi, s_reg, s_lab, s_cnt = targets.proposal_targets(
            self.rpn.rois_padded, self.rpn.rois_count, boxes, labels, n_sample=self.n_sample[1])
        S = self.n_sample[1]
        cnt = s_cnt.cpu()
        if bool((cnt != S).any()):  # train.py:102 assigns into an [N, 128, 4] buffer
            raise RuntimeError(f"proposal targets: expected {S} samples per image, got {cnt.tolist()}")
        sample_rois = s_roi.float().contiguous().view(-1, 4)                      # :86,102,107
        sample_rois_ind = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(S)
        reg_targets_classifier = s_reg.float()                                     # :89,103
        cls_labels_classifier = s_lab.float()                                      # :90,104
        cls_output, reg_output = self.head(features, sample_rois, sample_rois_ind, img_h, img_w,
                                           rois_sorted=True)  # grouped by construction
        # train.py:112-117: gather the regression of each sample's class
        reg_ind = cls_labels_classifier.detach().unsqueeze(-1).long() * 4
        reg_ind = torch.cat([reg_ind, reg_ind + 1, reg_ind + 2, reg_ind + 3], dim=-1)
        reg_output = torch.gather(reg_output, dim=-1, index=reg_ind)
        reg_loss = fast_rcnn_loc_loss(reg_output, reg_targets_classifier, cls_labels_classifier)
        cls_loss = F.cross_entropy(cls_output, cls_labels_classifier.long(), ignore_index=-1)
        total_loss = rpn_cls_loss + rpn_reg_loss + cls_loss + reg_loss
        total_loss.backward()
        if self.optimizer is not None:
            self.optimizer.step()
        self.last = dict(cls=cls, reg=reg, rpn_labels=lab, rpn_reg_targets=reg_t, sample_rois=s_roi,
                         sample_reg=s_reg, sample_labels=s_lab, cls_output=cls_output,
                         reg_output=reg_output)
        return dict(total=total_loss.detach(), rpn_cls=rpn_cls_loss.detach(),
                    rpn_reg=rpn_reg_loss.detach(), cls=cls_loss.detach(), reg=reg_loss.detach())
