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
