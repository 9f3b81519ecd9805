"""Pin the oracle (CPU restatement) against fixtures the genuine reference
produced (tests/golden/make_golden.py).  CPU only."""
import hashlib

import numpy as np
import torch
import pytest

from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import synth


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_anchor_base_and_grid(golden):
    g = golden("anchors.npz")
    for tag, scales in [("k9", (8, 16, 32)), ("k15", (2, 4, 8, 16, 32))]:
        base = orc.generate_anchor_base(anchor_scales=scales)
        assert base.dtype == np.float32
        assert np.array_equal(base, g[f"base_{tag}"])
        for (w, h) in [(10, 10), (63, 38), (38, 38), (84, 50), (7, 3)]:
            a = orc.generate_anchors(base, 16, w, h)
            assert sha(a) == str(g[f"sha_{tag}_{w}x{h}"]), (tag, w, h)
    a10 = orc.generate_anchors(orc.generate_anchor_base(), 10, 10, 10)
    assert np.array_equal(a10, g["anchors_main_10"])


def test_bbox_iou_known_answer(golden):
    g = golden("anchors.npz")
    out = orc.bbox_iou(g["iou_main_a"], g["iou_main_b"])
    assert np.array_equal(out, g["iou_main_out"])
    # value printed by utils/utils.py:280-284
    np.testing.assert_allclose(out, [[1 / 7, 0, 1], [0, 1 / 3, 0], [0, 0, 0], [0.4, 0, 0]],
                               rtol=1e-6)


def test_reg2bbox_vs_reference(golden):
    g = golden("reg2bbox.npz")
    out = orc.reg2bbox(g["anchors"], g["reg"])
    ref = g["out"]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(out), fin)
    np.testing.assert_allclose(out[fin], ref[fin], rtol=1e-5, atol=1e-3)
    # the only allowed difference is the last bit of MKL's exp
    assert np.mean(out[fin] == ref[fin]) > 0.9


@pytest.mark.parametrize("case", [0, 1, 2])
def test_proposal_small_vs_reference(golden, case):
    g = golden(f"proposal_small{case}.npz")
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, int(g["feat_w"]), int(g["feat_h"]))
    rois, idx = orc.propose_one(anchors, g["scores"], g["deltas"], int(g["img_w"]),
                                int(g["img_h"]), int(g["pre"]), int(g["post"]))
    assert np.array_equal(idx, g["idx"])
    np.testing.assert_allclose(rois, g["rois"], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("key", ["cfg2_img0", "cfg2_img1", "cfg5_img0"])
def test_proposal_full_vs_reference(golden, key):
    g = golden("proposal_full.npz")
    cfg, img = key.split("_img")
    c = synth.CONFIGS[cfg]
    base = orc.generate_anchor_base(anchor_scales=c["scales"])
    anchors = orc.generate_anchors(base, 16, c["feat_w"], c["feat_h"])
    A = len(anchors)
    sc = synth.rpn_scores(A, 0, int(img))
    de = synth.rpn_deltas(A, 0, int(img))
    rois, idx = orc.propose_one(anchors, sc, de, c["img_w"], c["img_h"], c["pre_nms"],
                                c["post_nms"])
    assert np.array_equal(idx, g[f"{key}_idx"])
    np.testing.assert_allclose(rois, g[f"{key}_rois"], rtol=1e-5, atol=1e-4)


def test_nms_fixtures(golden):
    g = golden("nms.npz")
    names = sorted({k.rsplit("_", 1)[0] for k in g if k.endswith("_keep")})
    assert len(names) >= 6
    for n in names:
        keep = orc.nms(g[f"{n}_boxes"], g[f"{n}_scores"], float(g[f"{n}_thr"]))
        assert np.array_equal(keep, g[f"{n}_keep"]), n


def test_roi_transform_and_pool(golden):
    g = golden("roi_pool.npz")
    x = g["x"]
    boxes = orc.roi_transform(g["rois_img"], g["roi_inds"], int(g["img_h"]), int(g["img_w"]),
                              x.shape[2], x.shape[3])
    assert np.array_equal(boxes, g["boxes"])
    out, am = orc.roi_pool_forward(x, boxes, 7, 1.0)
    assert np.array_equal(out, g["out"]) and np.array_equal(am, g["argmax"])
    gi = orc.roi_pool_backward(g["grad"], boxes, am, x.shape)
    assert np.array_equal(gi, g["grad_in"])
    # bins past H clip to empty (transposed RoIs) -> argmax -1
    assert (am == -1).any()


@pytest.mark.parametrize("tag", ["small", "train"])
def test_targets_vs_reference(golden, tag):
    g = golden(f"targets_{tag}.npz")
    anchors, boxes, labels = g["anchors"], g["boxes"], g["labels"]
    n_img = boxes.shape[0]
    st = ("MT19937", g["rng_key_in"], int(g["rng_pos_in"]), 0, 0.0)
    saved = np.random.get_state()
    try:
        np.random.set_state(st)
        for i in range(n_img):
            v = labels[i] != -1
            reg, lab, am, mx = orc.anchor_target(boxes[i, v], anchors, return_internals=True)
            assert np.array_equal(lab, g[f"at{i}_label"])
            assert np.array_equal(np.asarray(am), g[f"at{i}_argmax"])
            assert sha(np.asarray(mx, np.float64)) == str(g[f"at{i}_maxiou_sha"])
            assert sha(reg) == str(g[f"at{i}_reg_sha"])
            assert np.random.get_state()[2] == int(g[f"at{i}_rng_pos"])
            assert sha(np.random.get_state()[1]) == str(g[f"at{i}_rng_key_sha"])
        for i in range(n_img):
            v = labels[i] != -1
            s_roi, s_reg, s_lab = orc.proposal_target(g[f"roi{i}"], boxes[i, v], labels[i][v])
            assert np.array_equal(s_roi, g[f"pt{i}_roi"])
            assert np.array_equal(s_reg, g[f"pt{i}_reg"])
            assert np.array_equal(s_lab, g[f"pt{i}_label"])
            assert np.random.get_state()[2] == int(g[f"pt{i}_rng_pos"])
        assert np.array_equal(np.random.get_state()[1], g["rng_key_out"])
    finally:
        np.random.set_state(saved)


@pytest.mark.parametrize("K,H,W", [(9, 38, 38), (15, 7, 11)])
def test_rpn_head_epilogue_oracle_vs_torch(K, H, W):
    """Pins oracle.rpn_head_epilogue against the genuine torch ops the reference
    runs at nets/rpn.py:117-124: permutes exact, fg softmax within 2 ulp-scale
    relative error (torch's CPU exp is host-dependent in its last bits)."""
    g = torch.Generator().manual_seed(K)
    cls = torch.randn(2, 2 * K, H, W, generator=g) * 3
    reg = torch.randn(2, 4 * K, H, W, generator=g)
    c_t = cls.permute(0, 2, 3, 1).contiguous().view(2, -1, 2)
    fg_t = torch.nn.functional.softmax(c_t, dim=-1)[:, :, 1].contiguous().view(2, -1)
    r_t = reg.permute(0, 2, 3, 1).contiguous().view(2, -1, 4)
    c, fg, r = orc.rpn_head_epilogue(cls.numpy(), reg.numpy())
    assert np.array_equal(c, c_t.numpy()) and np.array_equal(r, r_t.numpy())
    np.testing.assert_allclose(fg, fg_t.numpy(), rtol=1e-6, atol=1e-30)
