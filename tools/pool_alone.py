"""The bench's dominant kernel by itself, for a standalone rocprofv3 record.

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/pool_alone.py --config cfg2 --launches 60

Builds the bench's inputs for the config (synthetic features, the batch's
proposals), then issues the RoIPool forward of the step (RoI transform + pack +
pool, one launch: nets/heads.py:42-48) -- or for cfg5 the RoIPool backward of a
resident upstream gradient -- `--launches` times back to back on one stream,
the same launch bench.py's `kernel_us_alone` times with HIP events.  Prints the
event-timed mean per launch as JSON, so the rocprofv3 average of the same run
can be checked against it.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import anchors as A, ops, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--launches", type=int, default=60)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[a.config]
    N = 16 if a.config == "cfg5" else c["batch"]
    c, sc, de, x = make_inputs(a.config, range(N), dev)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, _, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                               post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                               feat_w=c["feat_w"])
    post = c["post_nms"]
    if a.config == "cfg5":  # the training step pools the 128 sampled RoIs per image (train.py:86-108)
        import numpy as np
        from replication_faster_rcnn_amd import targets
        from replication_faster_rcnn_amd.utils import rng_state_to_device
        gl = [synth.gt_boxes(c["img_h"], c["img_w"], 32, 0, i) for i in range(N)]
        gb = torch.from_numpy(np.stack([b for b, _ in gl])).to(dev)
        gl_ = torch.from_numpy(np.stack([lb for _, lb in gl])).to(dev)
        np.random.seed(0)
        rng, _ = rng_state_to_device(dev)
        s_roi = targets.proposal_targets(rois, cnt, gb, gl_, n_sample=128, rng=rng)[0]
        post = 128
        rois = s_roi.float()
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(post)
    out, am, boxes = ops.roi_pool_head(x, rois.reshape(-1, 4), inds, 7, c["img_h"], c["img_w"],
                                       rois_sorted=True)
    if a.config == "cfg5":
        g = torch.randn(out.shape, device=dev)
        launch = lambda: ops._roi_pool_bwd(g, boxes, am, tuple(x.shape), 1.0)  # noqa: E731
        kernel = "roi_pool_bwd_lead_kernel (op: prep + lists + kernel)"
    else:
        outs = (out, am, boxes)
        launch = lambda: ops.roi_pool_head(x, rois.reshape(-1, 4), inds, 7, c["img_h"], c["img_w"],  # noqa: E731
                                           rois_sorted=True, out=outs)
        kernel = "roi_pool_fwd (head)"
    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.launches):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.launches * 1e3
    R = boxes.size(0)
    C, H, W = x.shape[1:]
    alg = N * C * H * W * 4 + R * 20 + 2 * R * C * 49 * 4
    print(json.dumps({"config": a.config, "kernel": kernel, "launches": a.launches, "us_per_launch": us,
                      "alg_bytes": alg, "frac_of_8TBps": alg / (us * 1e-6) / 8e12}))


if __name__ == "__main__":
    main()
