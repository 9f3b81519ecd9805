"""The benched cfg2 inference step (BASELINE configs[1], bench.py
inference_step_fn) exactly as the driver times it: the default arguments of
bench.py (four step streams, each step's proposals and its transform + pack +
RoIPool back to back on its stream, consecutive steps overlapping on different
streams, every output buffer preallocated per stream and reused every fourth
step), three input sets cycled, twelve steps issued with no host
synchronisation between them, so every stream's proposal and pooled buffers are
rewritten three times while the neighbouring streams' steps run beside them.
Afterwards stream j holds step 8 + j's outputs: its rois, anchor indices,
counts, packed boxes, pooled features and argmax are compared bit for bit with
the oracle's nets/rpn.py:58-77 per image -> nets/heads.py:42-47 -> torchvision
roi_pool for that step's input set."""
import sys

import numpy as np
import pytest
import torch

import bench
from oracle import ref_numpy as orc
from replication_faster_rcnn_amd import anchors as A, synth

pytestmark = pytest.mark.gpu


def test_benched_cfg2_steps_vs_oracle(monkeypatch):
    dev = torch.device("cuda", 0)
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse()  # the driver's defaults
    assert args.streams == 2 and args.pool_on == "prop" and args.prop_streams == 4
    cfg, n_sets, steps = "cfg2", 3, 12
    c = synth.CONFIGS[cfg]
    N, post, H, W = c["batch"], c["post_nms"], c["feat_h"], c["feat_w"]
    c, sets, _ = bench.make_input_sets(cfg, range(N), dev, n_sets)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    ev = {"fwd": [], "bwd": [], "draw": [], "i": 0, "pairs": []}
    step = bench.inference_step_fn(args, c, sets, base, 1, N, None, ev)
    nps = len(step.prop_out)
    assert nps == 4 and len(step.pool_outs) == 4
    for _ in range(steps):
        step(False)
    torch.cuda.synchronize()
    anchors = orc.generate_anchors(orc.generate_anchor_base(anchor_scales=c["scales"]), 16, W, H)
    inds = np.repeat(np.arange(N), post).astype(np.float32)
    for j in range(nps):
        k = steps - nps + j                      # the last step that ran on stream j
        sc, de, x = (t.cpu().numpy() for t in sets[k % n_sets])
        rois, idx, cnt = (t.cpu().numpy() for t in step.prop_out[j])
        out, am, boxes = (t.cpu().numpy() for t in step.pool_outs[j])
        o_rois = np.zeros((N, post, 4), np.float32)
        for i in range(N):
            r_i, i_i = orc.propose_one(anchors, sc[i], de[i], c["img_w"], c["img_h"], c["pre_nms"], post)
            assert int(cnt[i]) == len(i_i), (k, i)
            assert np.array_equal(idx[i, :len(i_i)].astype(np.int64), i_i), (k, i)
            o_rois[i, :len(i_i)] = r_i
        assert np.array_equal(rois.view(np.uint32), o_rois.view(np.uint32)), k
        ob = orc.roi_transform(o_rois.reshape(-1, 4), inds, c["img_h"], c["img_w"], H, W)
        assert np.array_equal(boxes.view(np.uint32), ob.view(np.uint32)), k
        oo, oa = orc.roi_pool_forward(x, ob, 7)
        assert np.array_equal(am, oa), k
        assert np.array_equal(out.view(np.uint32), oo.view(np.uint32)), k
