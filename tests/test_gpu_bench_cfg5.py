"""The benched cfg5 training step (BASELINE configs[4], bench.py
train_step_fn) exactly as the bench runs it -- three HIP streams, two
alternating target workspaces, numpy's MT19937 stream kept on the device, the
target creators split into prepare / draw / finish on different streams across
consecutive steps -- at the full shape (16 x 256 x 38 x 38 features, 600
proposals and 128 samples per image, R = 2048), for three consecutive steps,
against the oracle's per-image loop of train.py:67-126 in the reference's
order (all anchor targets, then all proposal targets, per step): anchor labels
and regression targets, sampled RoIs / labels / regression targets, the pooled
features and argmax, the RoIPool gradient, and the RNG state after every step."""
import types

import numpy as np
import pytest
import torch

import bench
from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import anchors as A, synth

pytestmark = pytest.mark.gpu


def test_benched_cfg5_steps_vs_oracle(rng_guard):
    dev = torch.device("cuda", 0)
    cfg = "cfg5"
    N, S, steps = 16, 128, 4  # (4 steps: the 3 rotating target workspaces wrap once)
    c, sets, _ = bench.make_input_sets(cfg, range(N), dev, 2)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    args = types.SimpleNamespace(streams=2, rng_waits="front", target_bufs=3)
    ev = {"fwd": [], "bwd": [], "draw": [], "i": 0, "pairs": []}
    step = bench.train_step_fn(args, c, sets, base, 0, ev)   # seeds numpy's global RNG with 0
    st0 = np.random.get_state()
    got = []
    for _ in range(steps):
        step(False)
        torch.cuda.synchronize()
        s = step.state
        got.append({k: s[k].cpu().numpy() for k in ("lab", "reg_t", "s_roi", "s_reg", "s_lab", "pooled",
                                                     "am", "bx", "gi", "s_cnt")})
        got[-1]["rng"] = step.fixed["rng"].cpu().numpy().view(np.uint32).copy()
    fx = step.fixed
    boxes, labels = fx["boxes"].cpu().numpy(), fx["labels"].cpu().numpy()
    grad = fx["grad"].cpu().numpy()
    anchors = orc.generate_anchors(orc.generate_anchor_base(anchor_scales=c["scales"]), 16, c["feat_w"],
                                   c["feat_h"])
    host = [[t.cpu().numpy() for t in st] for st in sets]
    np.random.set_state(st0)
    inds = np.repeat(np.arange(N), S).astype(np.float32)
    for k in range(steps):
        sc, de, x = host[k % len(host)]
        g = got[k]
        rois = [orc.propose_one(anchors, sc[i], de[i], c["img_w"], c["img_h"], c["pre_nms"], c["post_nms"])[0]
                for i in range(N)]
        valid = [labels[i] != -1 for i in range(N)]
        at = [orc.anchor_target(boxes[i][valid[i]], anchors) for i in range(N)]           # train.py:71-79
        pt = [orc.proposal_target(rois[i], boxes[i][valid[i]], labels[i][valid[i]]) for i in range(N)]  # :91-104
        st = np.random.get_state()
        assert np.array_equal(g["rng"][:624], st[1]) and int(g["rng"][624]) == st[2], f"RNG state, step {k}"
        assert (g["s_cnt"] == S).all()
        for i in range(N):
            assert np.array_equal(g["lab"][i], at[i][1]), (k, i)
            np.testing.assert_allclose(g["reg_t"][i], at[i][0], rtol=1e-12, atol=0)
            assert np.array_equal(g["s_roi"][i], pt[i][0]), (k, i)
            assert np.array_equal(g["s_lab"][i], pt[i][2]), (k, i)
            np.testing.assert_allclose(g["s_reg"][i], pt[i][1], rtol=1e-12, atol=1e-15)
        srois = np.concatenate([p[0] for p in pt]).astype(np.float32)                      # train.py:107
        ob = orc.roi_transform(srois, inds, c["img_h"], c["img_w"], c["feat_h"], c["feat_w"])
        assert np.array_equal(g["bx"], ob)
        oo, oa = orc.roi_pool_forward(x, ob, 7)
        assert np.array_equal(g["am"], oa), k
        assert np.array_equal(g["pooled"].view(np.uint32), oo.view(np.uint32)), k
        ogi = orc.roi_pool_backward(grad, ob, oa, x.shape)
        assert np.array_equal(g["gi"].view(np.uint32), ogi.view(np.uint32)), k
