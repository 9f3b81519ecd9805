"""The training-step harness (train.py:59-127) on the HIP path against the
oracle: everything downstream of the RPN convolutions -- proposals, anchor and
proposal targets (with numpy's global RNG), the sampled RoIs fed to the head,
the label gather and the five losses -- plus the backward reaching the
features through RoIPool."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import synth
from replication_faster_rcnn_amd.heads import ResnetHead
from replication_faster_rcnn_amd.rpn import RPN
from replication_faster_rcnn_amd.train import Trainer, fast_rcnn_loc_loss

pytestmark = pytest.mark.gpu


def _loc_loss_ref(pred, gt, lab):  # train.py:29-57 on the host
    pos = lab > 0
    d = (pred[pos] - gt[pos]).abs()
    loss = torch.where(d < 1.0, 0.5 * d ** 2, d - 0.5).sum()
    return loss / max(float(pos.sum()), 1.0)


def test_train_step_vs_oracle(rng_guard):
    torch.manual_seed(3)
    N, C, img = 2, 256, 600
    rpn = RPN(mode="training").cuda()
    classifier = nn.Sequential(nn.Conv2d(C, 512, 1), nn.AdaptiveAvgPool2d(1)).cuda()
    head = ResnetHead(classifier).cuda()
    x = torch.from_numpy(np.stack([synth.features(C, 38, 38, 9, i) for i in range(N)])).cuda()
    x.requires_grad_(True)
    bl = [synth.gt_boxes(img, img, 32, 9, i, n_valid=[32, 11][i]) for i in range(N)]
    boxes = np.stack([b for b, _ in bl])
    labels = np.stack([l for _, l in bl])
    tr = Trainer(rpn, head)
    np.random.seed(123)
    losses = tr.train_step(x, img, img, boxes, labels)
    st_after = np.random.get_state()
    assert all(torch.isfinite(v) for v in losses.values())
    assert x.grad is not None and torch.isfinite(x.grad).all() and x.grad.abs().sum() > 0
    L = tr.last
    # oracle, from the same RPN outputs (fg scores and deltas of the step)
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, 38, 38)
    fg = rpn.fg_scores.cpu().numpy()
    dl = L["reg"].detach().cpu().numpy()
    rois = [orc.propose_one(anchors, fg[i], dl[i], img, img, 12000, 600)[0] for i in range(N)]
    np.random.seed(123)
    at = []
    for i in range(N):
        v = labels[i] != -1
        at.append(orc.anchor_target(boxes[i, v], anchors))
    pt = []
    for i in range(N):
        v = labels[i] != -1
        pt.append(orc.proposal_target(rois[i], boxes[i, v], labels[i][v]))
    assert np.array_equal(np.random.get_state()[1], st_after[1]) and np.random.get_state()[2] == st_after[2]
    for i in range(N):
        assert np.array_equal(L["rpn_labels"][i].cpu().numpy(), at[i][1])
        np.testing.assert_allclose(L["rpn_reg_targets"][i].cpu().numpy(), at[i][0], rtol=1e-12, atol=0)
        assert np.array_equal(L["sample_rois"][i].cpu().numpy(), pt[i][0])
        assert np.array_equal(L["sample_labels"][i].cpu().numpy(), pt[i][2])
        np.testing.assert_allclose(L["sample_reg"][i].cpu().numpy(), pt[i][1], rtol=1e-12, atol=1e-15)
    # the five losses, recomputed on the host from the oracle's targets
    cls = L["cls"].detach().cpu()
    reg = L["reg"].detach().cpu()
    lab_rpn = torch.from_numpy(np.stack([a[1] for a in at])).float()
    reg_rpn = torch.from_numpy(np.stack([a[0] for a in at])).float()
    lab_cls = torch.from_numpy(np.stack([p[2] for p in pt])).float()
    reg_cls = torch.from_numpy(np.stack([p[1] for p in pt])).float()
    ro = L["reg_output"].detach().cpu()
    co = L["cls_output"].detach().cpu()
    ref = {"rpn_reg": _loc_loss_ref(reg, reg_rpn, lab_rpn),
           "rpn_cls": F.cross_entropy(cls, lab_rpn.long(), ignore_index=-1),
           "reg": _loc_loss_ref(ro, reg_cls, lab_cls),
           "cls": F.cross_entropy(co, lab_cls.long(), ignore_index=-1)}
    for k, v in ref.items():
        np.testing.assert_allclose(float(losses[k]), float(v), rtol=1e-5, atol=1e-7)
    # the head pooled exactly the sampled RoIs: its input boxes are the oracle's
    srois = np.concatenate([p[0] for p in pt]).astype(np.float32)
    inds = np.repeat(np.arange(N), 128).astype(np.float32)
    ob = orc.roi_transform(srois, inds, img, img, 38, 38)
    oo, _ = orc.roi_pool_forward(x.detach().cpu().numpy(), ob, 7)
    from replication_faster_rcnn_amd import ops
    out, _, boxes_dev = ops.roi_pool_head(x.detach(), torch.from_numpy(srois).cuda(),
                                          torch.from_numpy(inds).cuda(), 7, img, img, rois_sorted=True)
    assert np.array_equal(boxes_dev.cpu().numpy(), ob)
    assert np.array_equal(out.cpu().numpy(), oo)


def test_fast_rcnn_loc_loss_matches_reference_formula():
    r = torch.Generator().manual_seed(0)
    pred = torch.randn(50, 4, generator=r) * 2
    gt = torch.randn(50, 4, generator=r)
    lab = torch.randint(-1, 3, (50,), generator=r).float()
    np.testing.assert_allclose(float(fast_rcnn_loc_loss(pred.cuda(), gt.cuda(), lab.cuda())),
                               float(_loc_loss_ref(pred, gt, lab)), rtol=1e-6)
    none = torch.zeros(50)
    assert float(fast_rcnn_loc_loss(pred.cuda(), gt.cuda(), none.cuda())) == 0.0
