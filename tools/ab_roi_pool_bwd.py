"""A/B timing of the RoIPool backward paths (frcnn_set_path("roi_pool_bwd", ...))
on the training-step shape (BASELINE configs[4]: 16 images, 128 sampled RoIs
each, 256 x 38 x 38 features): the sampled RoIs are ProposalTarget's draw per
image (as tools/pool_alone.py; --rois first: the first 128 proposals of each image); every path's gradient is checked bit-equal to the first path's.

    python tools/ab_roi_pool_bwd.py [--config cfg5] [--paths ring,plain]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402


def build(config="cfg5", per_image=128, rois_mode="sampled", dev=None):
    """The backward's inputs at the training-step shape: (upstream grad, packed
    boxes, argmax, feature shape)."""
    dev = dev or torch.device("cuda", 0)
    c = synth.CONFIGS[config]
    c, sc, de, x = make_inputs(config, range(c["batch"]), dev)
    N, S = sc.size(0), per_image
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, _, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                               post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
    if rois_mode == "sampled":  # the training step's RoIs: ProposalTarget's 128 per image (as tools/pool_alone.py)
        from replication_faster_rcnn_amd import targets
        from replication_faster_rcnn_amd.utils import rng_state_to_device
        gl = [synth.gt_boxes(c["img_h"], c["img_w"], 32, 0, i) for i in range(N)]
        gb = torch.from_numpy(np.stack([b for b, _ in gl])).to(dev)
        gl_ = torch.from_numpy(np.stack([lb for _, lb in gl])).to(dev)
        st = np.random.get_state()
        np.random.seed(0)
        rng, _ = rng_state_to_device(dev)
        np.random.set_state(st)
        sr = targets.proposal_targets(rois, cnt, gb, gl_, n_sample=S, rng=rng)[0].float().reshape(-1, 4)
    else:
        sr = rois[:, :S].reshape(-1, 4).contiguous()
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(S)
    _, am, boxes = ops.roi_pool_head(x, sr, inds, 7, c["img_h"], c["img_w"], rois_sorted=True)
    g = torch.randn(am.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    return g, boxes, am, tuple(x.shape)


def set_variant(p):
    """A roi_pool_bwd path (auto = the leader kernel for 7-wide bins)."""
    _lib.set_path("roi_pool_bwd", p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--paths", default="ring,plain")
    ap.add_argument("--per-image", type=int, default=128)
    ap.add_argument("--rois", default="sampled", choices=("sampled", "first"),
                    help="sampled: ProposalTarget's draw per image (the bench); first: the top proposals")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    g, boxes, am, xs = build(a.config, a.per_image, a.rois)
    N, C, H, W = xs
    R = am.shape[0]
    alg = 2 * R * C * 49 * 4 + R * 20 + N * C * H * W * 4
    ref, times = None, {p: [] for p in a.paths.split(",")}
    for rnd in range(a.rounds):
        for p in times:
            set_variant(p)
            gi = ops._roi_pool_bwd(g, boxes, am, xs, 1.0)
            if ref is None:
                ref = gi.clone()
            elif rnd == 0:
                assert torch.equal(gi, ref), f"path {p} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops._roi_pool_bwd(g, boxes, am, xs, 1.0)
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / a.iters * 1e3)
    _lib.set_path("roi_pool_bwd", "auto")
    res = {p: {"us_median": float(np.median(t)), "GBps": alg / (np.median(t) * 1e-6) / 1e9,
               "frac": alg / (np.median(t) * 1e-6) / 8e12} for p, t in times.items()}
    print(json.dumps({"config": a.config, "R": R, "alg_bytes": alg, "paths": res}, indent=1))


if __name__ == "__main__":
    main()
