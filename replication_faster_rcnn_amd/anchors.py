"""Anchors (utils/anchors.py) on the HIP path.

Same signatures and numpy-in / numpy-out behaviour as the reference; the
arithmetic runs in the ``anchor_base_kernel`` / ``generate_anchors_kernel``
HIP kernels (the batched proposal path never materialises anchors: its
decode kernel generates them in registers).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def generate_anchor_base(base_size=16, ratios=[0.5, 1., 2.], anchor_scales=[8, 16, 32]):
    """utils/anchors.py:5-31 -> np.float32 [len(ratios)*len(scales), 4]."""
    base = generate_anchor_base_device(base_size, ratios, anchor_scales)
    return base.cpu().numpy()


def generate_anchor_base_device(base_size=16, ratios=(0.5, 1., 2.), anchor_scales=(8, 16, 32)):
    lib = _lib.load()
    r = np.ascontiguousarray(ratios, dtype=np.float64)
    s = np.ascontiguousarray(anchor_scales, dtype=np.float64)
    out = torch.empty((len(r) * len(s), 4), dtype=torch.float32, device=_lib.device())
    _lib.check(lib.frcnn_anchor_base(r.ctypes.data, len(r), s.ctypes.data, len(s), float(base_size),
                                     _lib.ptr(out), _lib.stream_ptr()), "generate_anchor_base")
    return out


def generate_anchors(anchor_base, feat_stride, width, height):
    """utils/anchors.py:33-61 -> np.float32 [height*width*K, 4] (numpy in,
    numpy out); a device tensor in gives a device tensor out."""
    on_dev = isinstance(anchor_base, torch.Tensor) and anchor_base.is_cuda
    base = torch.as_tensor(np.asarray(anchor_base, np.float32)) if not on_dev else anchor_base
    out = generate_anchors_device(base, feat_stride, width, height)
    return out if on_dev else out.cpu().numpy()


def generate_anchors_device(anchor_base: torch.Tensor, feat_stride: int, width: int, height: int):
    lib = _lib.load()
    base = anchor_base.to(device=_lib.device(), dtype=torch.float32).contiguous()
    K = base.size(0)
    out = torch.empty((int(height) * int(width) * K, 4), dtype=torch.float32, device=base.device)
    _lib.check(lib.frcnn_generate_anchors(_lib.ptr(base), K, int(feat_stride), int(width),
                                          int(height), _lib.ptr(out), _lib.stream_ptr()),
               "generate_anchors")
    return out
