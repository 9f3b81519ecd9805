"""The drop-in modules (RPN, region_proposal, ResnetHead) against the oracle,
called exactly the way train.py:59-127 calls the reference ones."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import ops, synth
from replication_faster_rcnn_amd.heads import ResnetHead
from replication_faster_rcnn_amd.rpn import RPN, region_proposal

pytestmark = pytest.mark.gpu


def test_region_proposal_module_cpu_in_cpu_out():
    """nets/rpn.py:132 call: numpy anchors, CPU tensors -> CPU tensor."""
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, 30, 20)
    A = len(anchors)
    sc = torch.from_numpy(synth.rpn_scores(A, 4, 0))
    de = torch.from_numpy(synth.rpn_deltas(A, 4, 0))
    layer = region_proposal("train")
    roi = layer(anchors, sc, de, 480, 320)
    assert roi.device.type == "cpu" and roi.dtype == torch.float32
    orois, _ = orc.propose_one(anchors, sc.numpy(), de.numpy(), 480, 320, 12000, 600)
    assert np.array_equal(roi.numpy(), orois)
    test_layer = region_proposal("test")
    assert (test_layer.pre_nms, test_layer.post_nms) == (3000, 300)


@pytest.mark.parametrize("device", ["cpu", "cuda"])
def test_rpn_forward_matches_oracle(device):
    torch.manual_seed(0)
    rpn = RPN(mode="training").to(device)
    x = torch.from_numpy(np.stack([synth.features(256, 38, 38, 6, i) for i in range(2)])).to(device)
    cls, reg, rois, roi_inds, anchors = rpn(x, 600, 600)
    assert cls.shape == (2, 2, 38 * 38 * 9) and reg.shape == (2, 38 * 38 * 9, 4)
    assert isinstance(anchors, np.ndarray) and anchors.shape == (38 * 38 * 9, 4)
    assert rois.device.type == device and roi_inds.dtype == torch.float32
    # the proposal layer ran on the epilogue kernel's fg (oracle-exact); torch's
    # own softmax of the returned cls agrees to 1e-6 (host exp bits)
    fg = rpn.fg_scores.cpu().numpy()
    fg_t = torch.softmax(cls.permute(0, 2, 1), -1)[:, :, 1].detach().cpu().numpy()
    np.testing.assert_allclose(fg, fg_t, rtol=1e-6, atol=1e-30)
    off = 0
    for i in range(2):
        orois, _ = orc.propose_one(anchors, fg[i], reg[i].detach().cpu().numpy(), 600, 600,
                                   12000, 600)
        k = len(orois)
        assert np.array_equal(rois[off:off + k].cpu().numpy(), orois)
        assert (roi_inds[off:off + k] == i).all()
        off += k
    assert off == rois.shape[0]


def test_resnet_head_forward_backward():
    torch.manual_seed(1)
    C = 16
    classifier = nn.Sequential(nn.Conv2d(C, 512, 1), nn.AdaptiveAvgPool2d(1)).cuda()
    head = ResnetHead(classifier).cuda()
    x = torch.from_numpy(np.stack([synth.features(C, 38, 63, 8, i) for i in range(2)])).cuda()
    x.requires_grad_(True)
    rois = torch.tensor([[0, 0, 600, 1000], [100, 200, 300, 500], [10, 10, 50, 70],
                         [200, 300, 590, 990]] * 2, dtype=torch.float32)
    inds = torch.tensor([0, 0, 0, 0, 1, 1, 1, 1], dtype=torch.float32)
    cls, reg = head(x, rois, inds, 600, 1000)
    assert cls.shape == (2, 21, 4) and reg.shape == (2, 4, 84)
    (cls.sum() + reg.sum()).backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    # pooled features equal the oracle's
    from replication_faster_rcnn_amd import ops
    boxes = orc.roi_transform(rois.numpy(), inds.numpy(), 600, 1000, 38, 63)
    out = ops.roi_pool(x.detach(), torch.from_numpy(boxes).cuda(), 7)
    oo, _ = orc.roi_pool_forward(x.detach().cpu().numpy(), boxes, 7)
    assert np.array_equal(out.cpu().numpy(), oo)


@pytest.mark.parametrize("N,K,H,W", [(8, 9, 38, 63), (1, 15, 50, 84), (3, 9, 5, 7), (2, 4, 1, 1)])
def test_rpn_head_epilogue_vs_oracle(N, K, H, W):
    """nets/rpn.py:117-124 in one launch: permuted cls / reg bit-exact, fg
    bit-exact vs the oracle restatement (ragged strips: H*W not a multiple of 64)."""
    g = torch.Generator().manual_seed(N * 100 + K)
    cls = torch.randn(N, 2 * K, H, W, generator=g) * 4
    reg = torch.randn(N, 4 * K, H, W, generator=g)
    # special pairs: equal logits, large gaps (exp underflow), +-inf, NaN
    flat = cls.view(N, K, 2, H * W)
    flat[0, 0, 1, 0] = flat[0, 0, 0, 0]
    flat[0, 0, 0, -1], flat[0, 0, 1, -1] = 100.0, -100.0
    if K > 1:
        flat[0, 1, 0, 0], flat[0, 1, 1, 0] = -float("inf"), 2.0
        flat[0, 1, 0, -1] = float("nan")
    c, fg, r = ops.rpn_head_epilogue(cls.cuda(), reg.cuda(), K)
    oc, ofg, orr = orc.rpn_head_epilogue(cls.numpy(), reg.numpy())
    assert np.array_equal(c.cpu().numpy(), oc, equal_nan=True)
    assert np.array_equal(r.cpu().numpy(), orr)
    assert np.array_equal(fg.cpu().numpy(), ofg, equal_nan=True)


def test_rpn_head_epilogue_backward():
    """The permutes' gradients equal torch autograd of the reference chain."""
    K, H, W = 9, 6, 10
    cls = torch.randn(2, 2 * K, H, W, device="cuda", requires_grad=True)
    reg = torch.randn(2, 4 * K, H, W, device="cuda", requires_grad=True)
    c, fg, r = ops.rpn_head_epilogue(cls, reg, K)
    assert not fg.requires_grad
    gc, gr = torch.randn_like(c), torch.randn_like(r)
    (c * gc).sum().add((r * gr).sum()).backward()
    cls2 = cls.detach().clone().requires_grad_(True)
    reg2 = reg.detach().clone().requires_grad_(True)
    c2 = cls2.permute(0, 2, 3, 1).contiguous().view(2, -1, 2)
    r2 = reg2.permute(0, 2, 3, 1).contiguous().view(2, -1, 4)
    (c2 * gc).sum().add((r2 * gr).sum()).backward()
    assert torch.equal(cls.grad, cls2.grad) and torch.equal(reg.grad, reg2.grad)


def test_rpn_head_epilogue_bad_shape():
    with pytest.raises(RuntimeError):
        ops.rpn_head_epilogue(torch.zeros(1, 18, 4, 4, device="cuda"),
                              torch.zeros(1, 35, 4, 4, device="cuda"), 9)
