"""Dump the bench's RoIPool inputs (the [R,5] feature-map boxes of a config's
proposals) for host-side lane-mapping models.

    python tools/dump_rois.py --config cfg2 --out gpurun_out/rois_cfg2.npy
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[a.config]
    c, sc, de, x = make_inputs(a.config, range(c["batch"]), dev)
    N = sc.size(0)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                 post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                                 feat_w=c["feat_w"])
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
    boxes = ops.roi_transform(rois.view(-1, 4), inds, c["img_h"], c["img_w"], c["feat_h"], c["feat_w"])
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.save(a.out, boxes.cpu().numpy())
    print("saved", a.out, tuple(boxes.shape), "feat", tuple(x.shape))


if __name__ == "__main__":
    main()
