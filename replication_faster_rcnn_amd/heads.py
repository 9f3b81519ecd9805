"""Second-stage head (nets/heads.py) on the HIP path.

``ResnetHead.forward`` keeps the reference signature (nets/heads.py:27).  The
RoI transform + ``[idx, box]`` pack (nets/heads.py:42-47) and RoIPool forward
(nets/heads.py:48) are one HIP launch (``ops.roi_pool_head``) when the RoIs
are grouped by image, with roi_pool's HIP backward; the classifier (layer4 +
avgpool) and the two FCs stay plain PyTorch (not the target).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib, ops


class ResnetHead(nn.Module):
    def __init__(self, classifier, roi_size=7, spatial_scale=1, n_classes=21):
        super().__init__()
        self.classifier = classifier
        self.reg = nn.Linear(in_features=512, out_features=n_classes * 4)
        self.cls = nn.Linear(in_features=512, out_features=n_classes)
        self.roi_size = roi_size
        self.spatial_scale = spatial_scale

    def forward(self, x, rois, roi_inds, img_h, img_w, rois_sorted=None):
        """-> (cls [N, n_classes, n_sample], reg [N, n_sample, n_classes*4]).

        ``rois_sorted`` (extension): True promises RoIs grouped by non-decreasing
        image index, as RPN.forward (nets/rpn.py:129-136) and train.py's sampler
        loop (:91-108) produce them -- the one-launch path.  None checks: on the
        host for host-resident indices (the reference's case, no device sync),
        with one device->host sync for device-resident ones."""
        N = x.shape[0]
        dev = _lib.device()
        if rois_sorted is None:
            bi = torch.as_tensor(roi_inds).detach().to(torch.int64)  # host tensors: no sync
            rois_sorted = bool((bi[1:] >= bi[:-1]).all()) if bi.numel() > 1 else True
        r = torch.as_tensor(rois).detach().to(dev, torch.float32).contiguous()
        ri = torch.as_tensor(roi_inds).detach().to(dev, torch.float32).contiguous()
        out_dev = x.device
        cropped = ops.roi_pool_head(x, r, ri, (self.roi_size, self.roi_size), img_h, img_w,
                                    self.spatial_scale, rois_sorted=bool(rois_sorted))[0].to(out_dev)
        fc6 = self.classifier(cropped)
        fc6 = fc6.view(fc6.shape[0], -1)
        reg = self.reg(fc6)
        cls = self.cls(fc6)
        reg = reg.view(N, -1, reg.shape[-1])
        cls = cls.view(N, -1, cls.shape[-1])
        return cls.permute(0, 2, 1), reg
