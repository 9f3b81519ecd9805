"""Batched target assignment on the HIP path (train.py:67-108 without the
per-image Python loops).

``anchor_targets`` = AnchorTargetCreator over all images, ``proposal_targets``
= ProposalTargetCreator over all images.  Both consume numpy's GLOBAL legacy
RNG exactly like the reference's per-image loops do (all images in order),
by shipping the MT19937 state to the device and back (one round trip per
call -- the only host synchronisation).  A caller that owns a device-resident
RNG stream (``rng=``: int32 [625] from ``utils.rng_state_to_device``) skips the
round trip: the state advances in place on the device, sync-free.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .utils import rng_state_from_device, rng_state_to_device


def _gt(boxes, labels, dev):
    b = torch.as_tensor(np.asarray(boxes, np.float64)) if not isinstance(boxes, torch.Tensor) else boxes
    l = torch.as_tensor(np.asarray(labels, np.float64)) if not isinstance(labels, torch.Tensor) else labels
    b = b.to(dev, torch.float64).contiguous()
    l = l.to(dev, torch.float64).contiguous()
    if b.dim() != 3 or b.size(-1) != 4 or l.shape != b.shape[:2]:
        raise RuntimeError(f"boxes must be [N,G,4] and labels [N,G]; got {tuple(b.shape)}, {tuple(l.shape)}")
    return b, l


def anchor_targets(boxes, labels, anchors, n_sample=256, pos_iou_thresh=0.7, neg_iou_thresh=0.3,
                   pos_ratio=0.5, sample=True, internals=False, rng=None):
    """boxes [N,G,4] fp64 (label -1 rows = padding), labels [N,G], anchors [A,4]
    -> reg fp64 [N,A,4], label int32 [N,A] (device tensors)."""
    lib = _lib.load()
    dev = _lib.device()
    b, l = _gt(boxes, labels, dev)
    a = (anchors if isinstance(anchors, torch.Tensor) else torch.as_tensor(np.asarray(anchors, np.float32)))
    a = a.to(dev, torch.float32).contiguous()
    N, G = b.shape[:2]
    A = a.size(0)
    reg = torch.empty((N, A, 4), dtype=torch.float64, device=dev)
    lab = torch.empty((N, A), dtype=torch.int32, device=dev)
    am = torch.empty((N, A), dtype=torch.int32, device=dev) if internals else None
    mx = torch.empty((N, A), dtype=torch.float64, device=dev) if internals else None
    ws = _lib.cached_workspace("anchor_target", lib.frcnn_anchor_target_workspace_size(N, A, G), dev)
    own = rng is None
    if own:
        rng, st = rng_state_to_device(dev) if sample else (None, None)
    elif not sample:
        rng = None
    _lib.check(lib.frcnn_anchor_target(N, A, G, _lib.ptr(a), _lib.ptr(b), _lib.ptr(l), int(n_sample),
                                       float(pos_iou_thresh), float(neg_iou_thresh),
                                       float(pos_ratio), _lib.ptr(rng), _lib.ptr(reg),
                                       _lib.ptr(lab), _lib.ptr(am), _lib.ptr(mx), _lib.ptr(ws),
                                       ws.numel(), _lib.stream_ptr()), "anchor_target")
    if sample and own:
        rng_state_from_device(rng, st)
    if internals:
        return reg, lab, am, mx
    return reg, lab


class AnchorTargetPlan:
    """The RNG-free half of AnchorTargetCreator (anchor_targets_prepare): the
    gt, IoU, labels and candidate lists in a workspace, ready for the draws."""

    def __init__(self, N, A, G, anchors, boxes, labels, ws):
        self.N, self.A, self.G = N, A, G
        self.anchors, self.boxes, self.labels, self.ws = anchors, boxes, labels, ws


def anchor_targets_workspace(N, A, G, device=None):
    """A workspace for anchor_targets_prepare / _sample (caller-owned, so a
    training loop can double-buffer plans across streams)."""
    lib = _lib.load()
    return torch.empty(max(int(lib.frcnn_anchor_target_workspace_size(N, A, G)), 1), dtype=torch.uint8,
                       device=device if device is not None else _lib.device())


def anchor_targets_prepare(boxes, labels, anchors, pos_iou_thresh=0.7, neg_iou_thresh=0.3, workspace=None):
    """First half of ``anchor_targets`` (utils/utils.py:146-188: IoU, labels,
    candidate lists) on the current stream; uses no RNG, so it can run ahead of
    the previous step's draws on another stream."""
    lib = _lib.load()
    dev = _lib.device()
    b, l = _gt(boxes, labels, dev)
    a = (anchors if isinstance(anchors, torch.Tensor) else torch.as_tensor(np.asarray(anchors, np.float32)))
    a = a.to(dev, torch.float32).contiguous()
    N, G = b.shape[:2]
    A = a.size(0)
    ws = workspace if workspace is not None else anchor_targets_workspace(N, A, G, dev)
    _lib.check(lib.frcnn_anchor_target_prepare(N, A, G, _lib.ptr(a), _lib.ptr(b), _lib.ptr(l),
                                               float(pos_iou_thresh), float(neg_iou_thresh), _lib.ptr(ws),
                                               ws.numel(), _lib.stream_ptr()), "anchor_target_prepare")
    return AnchorTargetPlan(N, A, G, a, b, l, ws)


def anchor_targets_sample(plan, n_sample=256, pos_ratio=0.5, rng=None, out=None):
    """Second half of ``anchor_targets``: the np.random.choice draws (numpy's
    global RNG, or the device stream ``rng``) and the regression targets, on the
    current stream, after ``plan``'s prepare (order the streams with an event).
    ``out`` = caller-owned (reg fp64 [N,A,4], label int32 [N,A])."""
    lib = _lib.load()
    dev = plan.ws.device
    N, A, G = plan.N, plan.A, plan.G
    if out is None:
        reg = torch.empty((N, A, 4), dtype=torch.float64, device=dev)
        lab = torch.empty((N, A), dtype=torch.int32, device=dev)
    else:
        reg, lab = out
    own = rng is None
    if own:
        rng, st = rng_state_to_device(dev)
    _lib.check(lib.frcnn_anchor_target_sample(N, A, G, _lib.ptr(plan.anchors), int(n_sample), float(pos_ratio),
                                              _lib.ptr(rng), _lib.ptr(reg), _lib.ptr(lab), None, None,
                                              _lib.ptr(plan.ws), plan.ws.numel(), _lib.stream_ptr()),
               "anchor_target_sample")
    if own:
        rng_state_from_device(rng, st)
    return reg, lab


def anchor_targets_draw(plan, n_sample=256, pos_ratio=0.5, rng=None):
    """The draws of ``anchor_targets_sample`` alone (utils/utils.py:190-202), on
    the current stream; ``anchor_targets_finish`` then writes the targets on any
    stream ordered after it."""
    lib = _lib.load()
    dev = plan.ws.device
    own = rng is None
    if own:
        rng, st = rng_state_to_device(dev)
    _lib.check(lib.frcnn_anchor_target_draw(plan.N, plan.A, plan.G, int(n_sample), float(pos_ratio), _lib.ptr(rng),
                                            _lib.ptr(plan.ws), plan.ws.numel(), _lib.stream_ptr()),
               "anchor_target_draw")
    if own:
        rng_state_from_device(rng, st)


_STATUS_KEYS = ("fail", "walks", "steps", "segments", "groups", "blocks", "pos", "widest", "missed_group")


def _draw_status(rc, buf):
    if rc == 1:
        return None  # no chip-wide part (> 128 images)
    _lib.check(rc, "draw_status")
    return dict(zip(_STATUS_KEYS, list(buf)))


def anchor_targets_draw_status(plan):
    """The chip-wide draws' plan of the last draw on ``plan`` (synchronous
    diagnostic): fail 0 = the segment tables held; None = walk-only workspace."""
    import ctypes
    buf = (ctypes.c_int * 9)()
    rc = _lib.load().frcnn_anchor_target_draw_status(plan.N, plan.A, plan.G, _lib.ptr(plan.ws), plan.ws.numel(), buf)
    return _draw_status(rc, buf)


def anchor_targets_finish(plan, out=None):
    """Final labels and regression targets after ``anchor_targets_draw``
    (utils/utils.py:146-150,203-204); ``out`` = caller-owned (reg, label)."""
    lib = _lib.load()
    dev = plan.ws.device
    N, A = plan.N, plan.A
    if out is None:
        out = (torch.empty((N, A, 4), dtype=torch.float64, device=dev),
               torch.empty((N, A), dtype=torch.int32, device=dev))
    reg, lab = out
    _lib.check(lib.frcnn_anchor_target_finish(N, A, plan.G, _lib.ptr(plan.anchors), _lib.ptr(reg), _lib.ptr(lab),
                                              None, None, _lib.ptr(plan.ws), plan.ws.numel(), _lib.stream_ptr()),
               "anchor_target_finish")
    return reg, lab


def proposal_targets(rois, rcount, boxes, labels, n_sample=128, pos_ratio=0.5, pos_iou_thresh=0.5,
                     neg_iou_thresh_high=0.5, neg_iou_thresh_low=0.0,
                     reg_normalize_mean=(0., 0., 0., 0.), reg_normalize_std=(0.1, 0.1, 0.2, 0.2),
                     rng=None):
    """rois fp32 [N,Rp,4] + rcount int32 [N] -> (sample_roi fp64 [N,S,4],
    gt_roi_reg fp64 [N,S,4], gt_roi_label fp64 [N,S], count int32 [N])."""
    lib = _lib.load()
    dev = _lib.device()
    b, l = _gt(boxes, labels, dev)
    r = rois.to(dev, torch.float32).contiguous()
    c = rcount.to(dev, torch.int32).contiguous()
    N, G = b.shape[:2]
    Rp = r.size(1)
    s_roi = torch.empty((N, n_sample, 4), dtype=torch.float64, device=dev)
    s_reg = torch.empty((N, n_sample, 4), dtype=torch.float64, device=dev)
    s_lab = torch.empty((N, n_sample), dtype=torch.float64, device=dev)
    s_cnt = torch.empty((N,), dtype=torch.int32, device=dev)
    # utils/utils.py:272 subtracts / divides np.float32 arrays
    mean = np.asarray(reg_normalize_mean, np.float32).astype(np.float64)
    std = np.asarray(reg_normalize_std, np.float32).astype(np.float64)
    ws = _lib.cached_workspace("proposal_target",
                                lib.frcnn_proposal_target_workspace_size(N, Rp, G, n_sample), dev)
    own = rng is None
    if own:
        rng, st = rng_state_to_device(dev)
    _lib.check(lib.frcnn_proposal_target(N, Rp, _lib.ptr(r), _lib.ptr(c), G, _lib.ptr(b), _lib.ptr(l),
                                         int(n_sample), float(pos_ratio), float(pos_iou_thresh),
                                         float(neg_iou_thresh_high), float(neg_iou_thresh_low),
                                         mean.ctypes.data, std.ctypes.data, _lib.ptr(rng),
                                         _lib.ptr(s_roi), _lib.ptr(s_reg), _lib.ptr(s_lab),
                                         _lib.ptr(s_cnt), _lib.ptr(ws), ws.numel(),
                                         _lib.stream_ptr()), "proposal_target")
    if own:
        rng_state_from_device(rng, st)
    return s_roi, s_reg, s_lab, s_cnt


class ProposalTargetPlan:
    """The RNG-free half of ProposalTargetCreator (proposal_targets_prepare):
    gt concat, IoU, argmax and the fg / bg lists in a workspace, ready for the draws."""

    def __init__(self, N, Rp, G, n_sample, ws):
        self.N, self.Rp, self.G, self.n_sample, self.ws = N, Rp, G, n_sample, ws


def proposal_targets_workspace(N, Rp, G, n_sample=128, device=None):
    """A workspace for proposal_targets_prepare / _sample (caller-owned, so a
    training loop can double-buffer plans across streams)."""
    lib = _lib.load()
    return torch.empty(max(int(lib.frcnn_proposal_target_workspace_size(N, Rp, G, n_sample)), 1),
                       dtype=torch.uint8, device=device if device is not None else _lib.device())


def proposal_targets_prepare(rois, rcount, boxes, labels, n_sample=128, pos_iou_thresh=0.5,
                             neg_iou_thresh_high=0.5, neg_iou_thresh_low=0.0, workspace=None):
    """First half of ``proposal_targets`` (utils/utils.py:221-246) on the current
    stream; uses no RNG, so it can run on the proposals' stream, off the draws'."""
    lib = _lib.load()
    dev = _lib.device()
    b, l = _gt(boxes, labels, dev)
    r = rois.to(dev, torch.float32).contiguous()
    c = rcount.to(dev, torch.int32).contiguous()
    N, G = b.shape[:2]
    Rp = r.size(1)
    ws = workspace if workspace is not None else proposal_targets_workspace(N, Rp, G, n_sample, dev)
    _lib.check(lib.frcnn_proposal_target_prepare(N, Rp, _lib.ptr(r), _lib.ptr(c), G, _lib.ptr(b), _lib.ptr(l),
                                                 int(n_sample), float(pos_iou_thresh), float(neg_iou_thresh_high),
                                                 float(neg_iou_thresh_low), _lib.ptr(ws), ws.numel(),
                                                 _lib.stream_ptr()), "proposal_target_prepare")
    return ProposalTargetPlan(N, Rp, G, int(n_sample), ws)


def proposal_targets_sample(plan, pos_ratio=0.5, reg_normalize_mean=(0., 0., 0., 0.),
                            reg_normalize_std=(0.1, 0.1, 0.2, 0.2), rng=None, out=None):
    """Second half of ``proposal_targets`` (utils/utils.py:248-276): the draws
    (numpy's global RNG, or the device stream ``rng``), sample order and
    regression targets, on the current stream after ``plan``'s prepare (order
    the streams with an event).  ``out`` = caller-owned (sample_roi, gt_roi_reg,
    gt_roi_label, count) as ``proposal_targets`` returns them."""
    lib = _lib.load()
    dev = plan.ws.device
    N, S = plan.N, plan.n_sample
    if out is None:
        out = (torch.empty((N, S, 4), dtype=torch.float64, device=dev),
               torch.empty((N, S, 4), dtype=torch.float64, device=dev),
               torch.empty((N, S), dtype=torch.float64, device=dev),
               torch.empty((N,), dtype=torch.int32, device=dev))
    s_roi, s_reg, s_lab, s_cnt = out
    mean = np.asarray(reg_normalize_mean, np.float32).astype(np.float64)  # utils/utils.py:272
    std = np.asarray(reg_normalize_std, np.float32).astype(np.float64)
    own = rng is None
    if own:
        rng, st = rng_state_to_device(dev)
    _lib.check(lib.frcnn_proposal_target_sample(N, plan.Rp, plan.G, S, float(pos_ratio), mean.ctypes.data,
                                                std.ctypes.data, _lib.ptr(rng), _lib.ptr(s_roi), _lib.ptr(s_reg),
                                                _lib.ptr(s_lab), _lib.ptr(s_cnt), _lib.ptr(plan.ws),
                                                plan.ws.numel(), _lib.stream_ptr()), "proposal_target_sample")
    if own:
        rng_state_from_device(rng, st)
    return s_roi, s_reg, s_lab, s_cnt


def proposal_targets_draw(plan, pos_ratio=0.5, rng=None, count=None):
    """The draws of ``proposal_targets_sample`` alone (utils/utils.py:248-258:
    sample order and per-image counts), on the current stream; returns the
    count tensor (int32 [N], ``count`` if given)."""
    lib = _lib.load()
    dev = plan.ws.device
    if count is None:
        count = torch.empty((plan.N,), dtype=torch.int32, device=dev)
    own = rng is None
    if own:
        rng, st = rng_state_to_device(dev)
    _lib.check(lib.frcnn_proposal_target_draw(plan.N, plan.Rp, plan.G, plan.n_sample, float(pos_ratio),
                                              _lib.ptr(rng), _lib.ptr(count), _lib.ptr(plan.ws), plan.ws.numel(),
                                              _lib.stream_ptr()), "proposal_target_draw")
    if own:
        rng_state_from_device(rng, st)
    return count


def target_draws(at_plan, pt_plan, rng, count=None, n_sample_at=256, pos_ratio_at=0.5, pos_ratio_pt=0.5):
    """``anchor_targets_draw(at_plan)`` then ``proposal_targets_draw(pt_plan)`` on the
    device stream ``rng`` as one pass (train.py:71 / :91: every AnchorTarget draw
    before any ProposalTarget one; bit-identical to the two calls); both plans'
    prepares must be ordered before it.  Returns the ProposalTarget count tensor."""
    lib = _lib.load()
    assert at_plan.N == pt_plan.N, "one batch of images"
    if count is None:
        count = torch.empty((pt_plan.N,), dtype=torch.int32, device=pt_plan.ws.device)
    _lib.check(lib.frcnn_target_draws(at_plan.N, at_plan.A, at_plan.G, int(n_sample_at), float(pos_ratio_at),
                                      _lib.ptr(at_plan.ws), at_plan.ws.numel(), pt_plan.Rp, pt_plan.G,
                                      pt_plan.n_sample, float(pos_ratio_pt), _lib.ptr(pt_plan.ws), pt_plan.ws.numel(),
                                      _lib.ptr(count), _lib.ptr(rng), _lib.stream_ptr()), "target_draws")
    return count


def proposal_targets_draw_status(plan):
    """As ``anchor_targets_draw_status`` for the last proposal-target draw."""
    import ctypes
    buf = (ctypes.c_int * 9)()
    rc = _lib.load().frcnn_proposal_target_draw_status(plan.N, plan.Rp, plan.G, plan.n_sample, _lib.ptr(plan.ws),
                                                       plan.ws.numel(), buf)
    return _draw_status(rc, buf)


def proposal_targets_finish(plan, count, reg_normalize_mean=(0., 0., 0., 0.),
                            reg_normalize_std=(0.1, 0.1, 0.2, 0.2), out=None):
    """sample_roi / gt_roi_reg / gt_roi_label after ``proposal_targets_draw``
    (utils/utils.py:260-276), on any stream ordered after it; ``out`` =
    caller-owned (sample_roi, gt_roi_reg, gt_roi_label)."""
    lib = _lib.load()
    dev = plan.ws.device
    N, S = plan.N, plan.n_sample
    if out is None:
        out = (torch.empty((N, S, 4), dtype=torch.float64, device=dev),
               torch.empty((N, S, 4), dtype=torch.float64, device=dev),
               torch.empty((N, S), dtype=torch.float64, device=dev))
    s_roi, s_reg, s_lab = out
    mean = np.asarray(reg_normalize_mean, np.float32).astype(np.float64)  # utils/utils.py:272
    std = np.asarray(reg_normalize_std, np.float32).astype(np.float64)
    _lib.check(lib.frcnn_proposal_target_finish(N, plan.Rp, plan.G, S, mean.ctypes.data, std.ctypes.data,
                                                _lib.ptr(count), _lib.ptr(s_roi), _lib.ptr(s_reg), _lib.ptr(s_lab),
                                                _lib.ptr(plan.ws), plan.ws.numel(), _lib.stream_ptr()),
               "proposal_target_finish")
    return s_roi, s_reg, s_lab
