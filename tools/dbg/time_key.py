"""Time the RoIPool forward paths at a config on the current library
(FRCNN_LIB_PATH selects a build): median of interleaved rounds, us."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, ops, synth  # noqa: E402
from replication_faster_rcnn_amd import anchors as A  # noqa: E402

cfg = sys.argv[1]
paths = sys.argv[2].split(",")
tag = sys.argv[3] if len(sys.argv) > 3 else os.environ.get("FRCNN_LIB_PATH", "default")
dev = torch.device("cuda", 0)
c = synth.CONFIGS[cfg]
c, sc, de, x = make_inputs(cfg, range(c["batch"]), dev)
N = sc.size(0)
base = A.generate_anchor_base_device(anchor_scales=c["scales"])
rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                             post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(c["post_nms"])
res = {p: [] for p in paths}
for rnd in range(5):
    for p in paths:
        _lib.set_path("roi_pool_fwd", p)
        ops.roi_pool_head(x, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"], rois_sorted=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.roi_pool_head(x, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"], rois_sorted=True)
        e1.record()
        torch.cuda.synchronize()
        res[p].append(e0.elapsed_time(e1) / 10 * 1e3)
print(tag, cfg, {p: round(float(np.median(v)), 1) for p, v in res.items()})
